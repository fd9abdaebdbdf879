// Small kernels around the block stack: token embedding, key-padding bias, workspace pad
// initialisation.  (FinalLayer + Euler runs as the EULER epilogue of the GEMM, gemm.hip.)
#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {

// out[n][c] = sum_j x[n][j] Wt[j][c] + bias[c] + base[n][c] + pos[l][c] + emb[idx[n]][c]
//             + ipa[b*L + l][c]
// latent_to_emb / cond_to_emb (nn.Linear, K = 21 or 28) + pos_embed + mask_to_emb
// (latent_model.py:242-250) + the IPA prepend broadcast over frames (latent_model.py:255).
// K is tiny, so this is a bandwidth kernel: 8 tokens per block share the x rows in LDS.
__global__ __launch_bounds__(256) void embed_kernel(int N, int T, int L, int C, int K,
                                                    const float* __restrict__ x,
                                                    const float* __restrict__ Wt,
                                                    const float* __restrict__ bias,
                                                    const float* __restrict__ base,
                                                    const float* __restrict__ pos,
                                                    const float* __restrict__ emb,
                                                    const int64_t* __restrict__ idx,
                                                    const float* __restrict__ ipa,
                                                    float* __restrict__ out) {
  constexpr int TOK = 8;
  __shared__ float xs[TOK][64];
  const int n0 = blockIdx.x * TOK;
  for (int i = threadIdx.x; i < TOK * K; i += 256) {
    const int r = i / K, j = i % K, n = n0 + r;
    xs[r][j] = (n < N) ? x[(size_t)n * K + j] : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float acc[TOK];
#pragma unroll
    for (int r = 0; r < TOK; ++r) acc[r] = 0.f;
    for (int j = 0; j < K; ++j) {
      const float w = Wt[(size_t)j * C + c];  // coalesced across the block's channels
#pragma unroll
      for (int r = 0; r < TOK; ++r) acc[r] += xs[r][j] * w;
    }
#pragma unroll
    for (int r = 0; r < TOK; ++r) {
      const int n = n0 + r;
      if (n >= N) break;
      float v = acc[r];
      if (bias) v += bias[c];
      if (base) v += base[(size_t)n * C + c];
      const int l = n % L;
      if (pos) v += pos[(size_t)l * C + c];
      if (emb) v += emb[(size_t)idx[n] * C + c];
      if (ipa) v += ipa[((size_t)(n / (T * L)) * L + l) * C + c];
      out[(size_t)n * C + c] = v;
    }
  }
}

// kbias[b*L + l][t] = 0 where mask[b][t][l] != 0 else -inf  (key_padding_mask = 1 - mask,
// latent_model.py:336, masked_fill(-inf) mha.py:370-376)
__global__ void mask_bias_kernel(int B, int T, int L, const float* __restrict__ mask,
                                 float* __restrict__ kbias) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * T * L) return;
  const int l = i % L, t = (i / L) % T, b = i / (T * L);
  kbias[((size_t)b * L + l) * T + t] = (mask[i] != 0.f) ? 0.f : -INFINITY;
}

// 1.0 in pad column D of every temporal V row (softmax row sum rides in it).
template <typename CT>
__global__ void set_vpad_kernel(CT* v, size_t rows, int D) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < rows) v[i * MDG_DP + D] = (CT)1.0f;
}

hipError_t embed_launch(int N, int T, int L, int C, int K, const float* x, const float* Wt,
                        const float* bias, const float* base, const float* pos, const float* emb,
                        const int64_t* idx, const float* ipa, float* out, hipStream_t s) {
  hipLaunchKernelGGL(embed_kernel, dim3((N + 7) / 8), dim3(256), 0, s, N, T, L, C, K, x, Wt, bias,
                     base, pos, emb, idx, ipa, out);
  return hipGetLastError();
}

hipError_t mask_bias_launch(int B, int T, int L, const float* mask, float* kbias, hipStream_t s) {
  const int n = B * T * L;
  hipLaunchKernelGGL(mask_bias_kernel, dim3((n + 255) / 256), dim3(256), 0, s, B, T, L, mask, kbias);
  return hipGetLastError();
}

hipError_t set_vpad_launch(int dtype, void* v, size_t rows, int D, hipStream_t s) {
  dim3 grid((unsigned)((rows + 255) / 256));
  if (dtype == MDG_BF16)
    hipLaunchKernelGGL(set_vpad_kernel<bf16_t>, grid, dim3(256), 0, s, (bf16_t*)v, rows, D);
  else
    hipLaunchKernelGGL(set_vpad_kernel<float>, grid, dim3(256), 0, s, (float*)v, rows, D);
  return hipGetLastError();
}

}  // namespace mdg
