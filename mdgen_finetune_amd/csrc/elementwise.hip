// Small kernels around the block stack: token embedding, FinalLayer + Euler update,
// key-padding bias, workspace pad initialisation.
#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {

// out[n][c] = sum_j x[n][j] W[c][j] + bias[c] + base[n][c] + pos[l][c] + emb[idx[n]][c]
//             + ipa[b*L + l][c]
// latent_to_emb / cond_to_emb (nn.Linear, K = 21 or 28) + pos_embed + mask_to_emb
// (latent_model.py:242-250) + the IPA prepend broadcast over frames (latent_model.py:255).
// K is tiny, so this is a bandwidth kernel: 8 tokens per block share the x rows in LDS.
__global__ __launch_bounds__(256) void embed_kernel(int N, int T, int L, int C, int K,
                                                    const float* __restrict__ x,
                                                    const float* __restrict__ W,
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
      const float w = W[(size_t)c * K + j];
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

// FinalLayer (layers.py:58-75): v = Linear(LN(h)*(1+scale) + shift), then the Euler update
// x_out = x_in + dt * v (torchdiffeq fixed-grid Euler, integrators.py:106-113) with the
// multiply and add rounded separately, as the reference computes dy then y + dy.
// One wave per token; the [latent][C] weight lives in LDS.
__global__ __launch_bounds__(256) void final_euler_kernel(int N, int rows_per_b, int C, int lat,
                                                          const float* __restrict__ Wf,
                                                          const float* __restrict__ bf,
                                                          const float* __restrict__ mods,
                                                          const float* __restrict__ h,
                                                          const float* __restrict__ x_in,
                                                          float dt, float* x_out, float* v_out) {
  extern __shared__ __attribute__((aligned(16))) float Ws[];
  for (int i = threadIdx.x; i < lat * C; i += 256) Ws[i] = Wf[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nper = C >> 6;
  const float invC = 1.0f / (float)C;
  for (int n = blockIdx.x * 4 + wave; n < N; n += gridDim.x * 4) {
    const float* hr = h + (size_t)n * C;
    float v[8];
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = (e < nper) ? hr[lane + 64 * e] : 0.f;
      s += v[e];
    }
    const float mean = wave_sum(s) * invC;
    float ss = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[e] - mean;
      ss += (e < nper) ? d * d : 0.f;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(ss) * invC + 1e-6f);
    const float* mr = mods + (size_t)(n / rows_per_b) * 2 * C;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (e < nper) {
        const int k = lane + 64 * e;
        v[e] = (v[e] - mean) * rstd * (1.0f + mr[C + k]) + mr[k];
      }
    }
    float mine = 0.f;
    for (int o = 0; o < lat; ++o) {
      float part = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < nper) part += v[e] * Ws[o * C + lane + 64 * e];
      part = wave_sum(part);
      if (lane == o) mine = part;
    }
    if (lane < lat) {
      const float vv = mine + bf[lane];
      const size_t off = (size_t)n * lat + lane;
      if (v_out) v_out[off] = vv;
      if (x_out) x_out[off] = __fadd_rn(x_in[off], __fmul_rn(dt, vv));
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

hipError_t embed_launch(int N, int T, int L, int C, int K, const float* x, const float* W,
                        const float* bias, const float* base, const float* pos, const float* emb,
                        const int64_t* idx, const float* ipa, float* out, hipStream_t s) {
  hipLaunchKernelGGL(embed_kernel, dim3((N + 7) / 8), dim3(256), 0, s, N, T, L, C, K, x, W, bias,
                     base, pos, emb, idx, ipa, out);
  return hipGetLastError();
}

hipError_t final_euler_launch(int N, int rows_per_b, int C, int lat, const float* Wf,
                              const float* bf, const float* mods, const float* h,
                              const float* x_in, float dt, float* x_out, float* v_out,
                              hipStream_t s) {
  const size_t smem = (size_t)lat * C * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&final_euler_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  int grid = (N + 3) / 4;
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(final_euler_kernel, dim3(grid), dim3(256), smem, s, N, rows_per_b, C, lat,
                     Wf, bf, mods, h, x_in, dt, x_out, v_out);
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
