// Small kernels around the block stack: token embedding, LayerNorm + adaLN modulate,
// key-padding bias, workspace pad initialisation.  (FinalLayer + Euler runs as the EULER epilogue of the GEMM, gemm.hip.)
#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {

// out[n][c] = sum_j x[n][j] Wt[j][c] + bias[c] + base[n][c] + pos[l][c] + emb[idx[n]][c]
//             + ipa[b*L + l][c]
// latent_to_emb / cond_to_emb (nn.Linear, K = 21 or 28) + pos_embed + mask_to_emb
// (latent_model.py:242-250) + the IPA prepend broadcast over frames (latent_model.py:255).
// HBM-bound (base read + out write dominate).  Thread (c4, g) of a C/4 x 4 block keeps its
// 4-channel column of W (K x float4) in registers for the whole block and sweeps tokens
// g, g+4, ... of a 64-token tile whose x rows are staged in LDS (broadcast reads), so global
// traffic is one coalesced float4 per optional term per output quad.
constexpr int kEmbedKMax = 32, kEmbedTile = 64;

__global__ __launch_bounds__(512) void embed_kernel(int N, int T, int L, int C, int K,
                                                    const float* __restrict__ x,
                                                    const float* __restrict__ Wt,
                                                    const float* __restrict__ bias,
                                                    const float* __restrict__ base,
                                                    const float* __restrict__ pos,
                                                    const float* __restrict__ emb,
                                                    const int64_t* __restrict__ idx,
                                                    const float* __restrict__ ipa,
                                                    float* __restrict__ out) {
  __shared__ float xs[kEmbedTile * kEmbedKMax];
  const int C4 = C >> 2, tid = threadIdx.x;
  const int c4 = tid % C4, g = tid / C4, c = c4 * 4;
  float4 w[kEmbedKMax];
#pragma unroll
  for (int j = 0; j < kEmbedKMax; ++j)
    w[j] = (j < K) ? *reinterpret_cast<const float4*>(Wt + (size_t)j * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 bb = bias ? *reinterpret_cast<const float4*>(bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int n0 = blockIdx.x * kEmbedTile; n0 < N; n0 += gridDim.x * kEmbedTile) {
    const int nt = min(kEmbedTile, N - n0);
    __syncthreads();
    for (int i = tid; i < nt * K; i += blockDim.x) xs[(i / K) * kEmbedKMax + (i % K)] = x[(size_t)n0 * K + i];
    __syncthreads();
    // 4 tokens per pass (rows g, g+4, g+8, g+12 of the tile): their global operands are all
    // issued before any is consumed
    for (int r0 = g; r0 < nt; r0 += 16) {
      float4 a[4], t0[4], t1[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = min(r0 + 4 * u, nt - 1), n = n0 + r, l = n % L;
        t0[u] = base ? *reinterpret_cast<const float4*>(base + (size_t)n * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        t1[u] = ipa ? *reinterpret_cast<const float4*>(ipa + ((size_t)(n / (T * L)) * L + l) * C + c)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
        if (pos) {
          const float4 t = *reinterpret_cast<const float4*>(pos + (size_t)l * C + c);
          t1[u].x += t.x; t1[u].y += t.y; t1[u].z += t.z; t1[u].w += t.w;
        }
        if (emb) {
          const float4 t = *reinterpret_cast<const float4*>(emb + (size_t)idx[n] * C + c);
          t1[u].x += t.x; t1[u].y += t.y; t1[u].z += t.z; t1[u].w += t.w;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* xr = xs + min(r0 + 4 * u, nt - 1) * kEmbedKMax;
        a[u] = bb;
#pragma unroll
        for (int j = 0; j < kEmbedKMax; ++j) {
          if (j < K) {
            const float xv = xr[j];
            a[u].x += xv * w[j].x; a[u].y += xv * w[j].y; a[u].z += xv * w[j].z; a[u].w += xv * w[j].w;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = r0 + 4 * u;
        if (r < nt) {
          float4 v = a[u];
          v.x += t0[u].x + t1[u].x; v.y += t0[u].y + t1[u].y; v.z += t0[u].z + t1[u].z; v.w += t0[u].w + t1[u].w;
          *reinterpret_cast<float4*>(out + (size_t)(n0 + r) * C + c) = v;
        }
      }
    }
  }
}

// xn[m][k] = CT( LN(h[m])[k] * (1 + scale[b][k]) + shift[b][k] ),  b = m / rows_per_mod
// The no-affine LayerNorm (eps 1e-6) + adaLN modulate in front of every projection of the
// block (latent_model.py:467/475/489, FinalLayer layers.py:73, modulate layers.py:14-15).
// One wave per R = 4 consecutive rows (their 4 x C/64 loads in flight together; the shift /
// scale rows loaded once when the 4 rows share a batch entry).  Each lane holds W
// consecutive channels of every 64W-channel chunk (W = 2 when C % 128 == 0: 256-B bf16
// stores per wave instruction); two wave reductions per row (mean, then the centred sum of
// squares, as torch's two-pass LayerNorm).
template <typename CT, int W>
__global__ __launch_bounds__(256) void ln_mod_kernel(int M, int C, const float* __restrict__ h,
                                                     const float* __restrict__ mods, int mod_stride,
                                                     int rows_per_mod, int shift_off, int scale_off,
                                                     float eps, CT* __restrict__ xn, float* __restrict__ stats) {
  constexpr int E = 8 / W, R = 4;  // C <= 512
  const int lane = threadIdx.x & 63;
  const int m0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (m0 >= M) return;
  const int nE = C / (64 * W);
  float v[R][E][W], sc[E][W], sh[E][W];
  const int b0 = m0 / rows_per_mod;
  const bool shared = (min(m0 + R - 1, M - 1) / rows_per_mod) == b0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float* hr = h + (size_t)min(m0 + r, M - 1) * C;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int k = W * lane + 64 * W * e;
      if (e < nE) {
        if constexpr (W == 2) {
          const float2 a = *reinterpret_cast<const float2*>(hr + k);
          v[r][e][0] = a.x; v[r][e][1] = a.y;
        } else {
          v[r][e][0] = hr[k];
        }
      } else {
#pragma unroll
        for (int j = 0; j < W; ++j) v[r][e][j] = 0.f;
      }
    }
  }
  auto load_mods = [&](int b) {
    const float* mr = mods + (size_t)b * mod_stride;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int k = W * lane + 64 * W * e;
      if (e < nE) {
        if constexpr (W == 2) {
          const float2 x = *reinterpret_cast<const float2*>(mr + scale_off + k);
          const float2 y = *reinterpret_cast<const float2*>(mr + shift_off + k);
          sc[e][0] = x.x; sc[e][1] = x.y; sh[e][0] = y.x; sh[e][1] = y.y;
        } else {
          sc[e][0] = mr[scale_off + k]; sh[e][0] = mr[shift_off + k];
        }
      }
    }
  };
  if (shared) load_mods(b0);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int m = m0 + r;
    if (m >= M) break;
    if (!shared) load_mods(m / rows_per_mod);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int j = 0; j < W; ++j) s += v[r][e][j];
    const float mean = wave_sum(s) / (float)C;
    float ss = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (e < nE)
#pragma unroll
        for (int j = 0; j < W; ++j) {
          const float a = v[r][e][j] - mean;
          ss += a * a;
        }
    const float rs = 1.0f / sqrtf(wave_sum(ss) / (float)C + eps);
    if (stats && lane == 0) *reinterpret_cast<float2*>(stats + 2 * (size_t)m) = make_float2(mean, rs);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (e < nE) {
        const int k = W * lane + 64 * W * e;
        float y[W];
#pragma unroll
        for (int j = 0; j < W; ++j) y[j] = (v[r][e][j] - mean) * rs * (1.0f + sc[e][j]) + sh[e][j];
        CT* o = xn + (size_t)m * C + k;
        if constexpr (W == 2 && is_bf16<CT>()) {
          typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
          bf16x2 pr;
          pr[0] = (bf16_t)y[0];
          pr[1] = (bf16_t)y[1];
          *reinterpret_cast<bf16x2*>(o) = pr;
        } else if constexpr (W == 2) {
          *reinterpret_cast<float2*>(o) = make_float2(y[0], y[1]);
        } else {
          o[0] = (CT)y[0];
        }
      }
    }
  }
}

// kbias[b*L + l][t] = 0 where mask[b][t][l] != 0 else -inf  (key_padding_mask = 1 - mask,
// latent_model.py:336, masked_fill(-inf) mha.py:370-376)
__global__ void mask_bias_kernel(int B, int T, int L, const float* __restrict__ mask,
                                 float* __restrict__ kbias, float* __restrict__ kbias_s) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * T * L) return;
  const int l = i % L, t = (i / L) % T, b = i / (T * L);
  const float v = (mask[i] != 0.f) ? 0.f : -INFINITY;
  kbias[((size_t)b * L + l) * T + t] = v;  // temporal sequences (b, l) over t
  kbias_s[i] = v;                          // spatial sequences (b, t) over l
}

// 1.0 in pad column D of every temporal V row (softmax row sum rides in it).
template <typename CT>
__global__ void set_vpad_kernel(CT* v, size_t rows, int D) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < rows) v[i * dp_of(D) + D] = (CT)1.0f;
}

hipError_t embed_launch(int N, int T, int L, int C, int K, const float* x, const float* Wt,
                        const float* bias, const float* base, const float* pos, const float* emb,
                        const int64_t* idx, const float* ipa, float* out, hipStream_t s) {
  if (K > kEmbedKMax || C % 4 || C > 512) return hipErrorInvalidValue;
  const int tiles = (N + kEmbedTile - 1) / kEmbedTile;
  const int grid = tiles < 2048 ? tiles : 2048;
  hipLaunchKernelGGL(embed_kernel, dim3(grid), dim3(C), 0, s, N, T, L, C, K, x, Wt, bias, base, pos, emb, idx,
                     ipa, out);
  return hipGetLastError();
}

// Token embedding fused with layer 0's spatial LayerNorm (bf16 path, C = 128 * NE):
//   h  = x . W_l2e^T + (base + ipa[b, l])          (fp32, latent_model.py:242-255; same FMA
//        order as embed_kernel: the K products from 0, then the x-independent terms)
//   xn = LN(h) * (1 + scale[b]) + shift[b]         (bf16, eps 1e-6, latent_model.py:467)
// One wave owns 4 rows; lane holds columns 2*lane + 128e (float2, e < NE), so every row is
// read and written with full 512-B wave accesses and the row statistics are two wave
// reductions.  W_l2e^T [K][C] is staged once per block in LDS; x[n][0..K) is one dword per lane
// broadcast by v_readlane.  Every global operand of the 4 rows is issued before any is used.
// Replaces embed_kernel + ln_mod_kernel (49 MB re-read of h gone).
template <int NE, int KC>  // KC: compile-time latent width (0 = runtime K)
__global__ __launch_bounds__(256, 4) void embed_ln_kernel(int N, int TL, int L, int Kr, const float* __restrict__ x,
                                                       const float* __restrict__ Wt, const float* __restrict__ base,
                                                       const float* __restrict__ ipa, const float* __restrict__ mods,
                                                       int mod_stride, int shift_off, int scale_off, float eps,
                                                       float* __restrict__ h, bf16_t* __restrict__ xn) {
  constexpr int C = 128 * NE, R = 4;
  const int K = KC ? KC : Kr;
  extern __shared__ __attribute__((aligned(16))) float wl[];  // [K][C]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float invC = 1.0f / (float)C;
  const int groups = (N + 16 - 1) / 16;
  for (int gi = blockIdx.x; gi < groups; gi += gridDim.x) {
    const int r0 = gi * 16 + wave * R;
    float2 hv[R][NE], uv[R][NE], sv[NE], cv[NE];
    float xv[R];
    // shift / scale of the first row's batch entry; a row of another entry (a group that
    // straddles a trajectory boundary) reloads its own below
    const int b0 = min(r0, N - 1) / TL;
    {
      const float* mr = mods + (size_t)b0 * mod_stride;
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        sv[e] = *reinterpret_cast<const float2*>(mr + scale_off + 2 * lane + 128 * e);
        cv[e] = *reinterpret_cast<const float2*>(mr + shift_off + 2 * lane + 128 * e);
      }
    }
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
      const int n = min(r0 + rr, N - 1), b = n / TL, l = n % L;
      xv[rr] = lane < K ? x[(size_t)n * K + lane] : 0.f;
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const int k = 2 * lane + 128 * e;
        hv[rr][e] = *reinterpret_cast<const float2*>(base + (size_t)n * C + k);
        uv[rr][e] = ipa ? *reinterpret_cast<const float2*>(ipa + ((size_t)b * L + l) * C + k) : make_float2(0.f, 0.f);
      }
    }
    // W_l2e^T is staged after the first group's row loads are issued, so its L2 round trip
    // and the block barrier overlap their HBM latency instead of preceding it
    // (LDS DMA: all of a thread's pieces in flight at once, next to the row loads)
    if (gi == (int)blockIdx.x) {
      typedef __attribute__((address_space(3))) void* lds_ptr_t;
      const int n4 = K * C / 4;
      for (int u = 0; u * 256 < n4; ++u) {
        const int i0 = u * 256 + wave * 64;  // this wave's 64 float4 pieces
        if (i0 + lane < n4)
          __builtin_amdgcn_global_load_lds((const void*)(Wt + 4 * (size_t)(i0 + lane)), (lds_ptr_t)(wl + 4 * i0), 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if (ipa) {
#pragma unroll
      for (int rr = 0; rr < R; ++rr)
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          hv[rr][e].x += uv[rr][e].x;
          hv[rr][e].y += uv[rr][e].y;
        }
    }
    float2 a[R][NE];
#pragma unroll
    for (int rr = 0; rr < R; ++rr)
#pragma unroll
      for (int e = 0; e < NE; ++e) a[rr][e] = make_float2(0.f, 0.f);
    auto kstep = [&](int j) {
      float2 wv[NE];
#pragma unroll
      for (int e = 0; e < NE; ++e) wv[e] = *reinterpret_cast<const float2*>(wl + j * C + 2 * lane + 128 * e);
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const float xs = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv[rr]), j));
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          a[rr][e].x += xs * wv[e].x;
          a[rr][e].y += xs * wv[e].y;
        }
      }
    };
    if constexpr (KC > 0) {
#pragma unroll 7
      for (int j = 0; j < KC; ++j) kstep(j);
    } else {
      for (int j = 0; j < K; ++j) kstep(j);
    }
    float sum[R], ss[R];
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
      float t = 0.f;
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        hv[rr][e].x = a[rr][e].x + hv[rr][e].x;
        hv[rr][e].y = a[rr][e].y + hv[rr][e].y;
        t += hv[rr][e].x + hv[rr][e].y;
      }
      sum[rr] = t;
      if (r0 + rr < N) {
#pragma unroll
        for (int e = 0; e < NE; ++e)
          *reinterpret_cast<float2*>(h + (size_t)(r0 + rr) * C + 2 * lane + 128 * e) = hv[rr][e];
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
      for (int rr = 0; rr < R; ++rr) sum[rr] += __shfl_xor(sum[rr], o, 64);
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
      sum[rr] *= invC;
      float t = 0.f;
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const float d0 = hv[rr][e].x - sum[rr], d1 = hv[rr][e].y - sum[rr];
        t += d0 * d0 + d1 * d1;
      }
      ss[rr] = t;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
      for (int rr = 0; rr < R; ++rr) ss[rr] += __shfl_xor(ss[rr], o, 64);
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
      if (r0 + rr >= N) continue;
      const float rs = 1.0f / sqrtf(ss[rr] * invC + eps);
      const int b = (r0 + rr) / TL;
      if (b != b0) {
        const float* mr = mods + (size_t)b * mod_stride;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          sv[e] = *reinterpret_cast<const float2*>(mr + scale_off + 2 * lane + 128 * e);
          cv[e] = *reinterpret_cast<const float2*>(mr + shift_off + 2 * lane + 128 * e);
        }
      }
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
        bf16x2 pr;
        pr[0] = (bf16_t)((hv[rr][e].x - sum[rr]) * rs * (1.0f + sv[e].x) + cv[e].x);
        pr[1] = (bf16_t)((hv[rr][e].y - sum[rr]) * rs * (1.0f + sv[e].y) + cv[e].y);
        *reinterpret_cast<bf16x2*>(xn + (size_t)(r0 + rr) * C + 2 * lane + 128 * e) = pr;
      }
    }
  }
}

hipError_t embed_ln_launch(int N, int TL, int L, int C, int K, const float* x, const float* Wt, const float* base,
                           const float* ipa, const float* mods, int mod_stride, int shift_off, int scale_off,
                           float eps, float* h, void* xn, hipStream_t s) {
  if (K > 64 || (C != 128 && C != 256 && C != 384 && C != 512)) return hipErrorInvalidValue;
  const int groups = (N + 15) / 16, grid = groups < 65535 ? groups : 65535;
  const size_t smem = (size_t)K * C * 4;
#define MDG_ELN(NE, KC)                                                                                        \
  hipLaunchKernelGGL((embed_ln_kernel<NE, KC>), dim3(grid), dim3(256), smem, s, N, TL, L, K, x, Wt, base, ipa, \
                     mods, mod_stride, shift_off, scale_off, eps, h, (bf16_t*)xn)
  if (C == 384 && K == 21) MDG_ELN(3, 21);        // the tetrapeptide / ATLAS latent
  else if (C == 384 && K == 28) MDG_ELN(3, 28);   // TPS latent
  else if (C == 128) MDG_ELN(1, 0);
  else if (C == 256) MDG_ELN(2, 0);
  else if (C == 384) MDG_ELN(3, 0);
  else MDG_ELN(4, 0);
#undef MDG_ELN
  return hipGetLastError();
}

hipError_t ln_mod_launch(int dtype, int M, int C, const float* h, const float* mods, int mod_stride,
                         int rows_per_mod, int shift_off, int scale_off, float eps, void* xn,
                         hipStream_t s, float* stats) {
  dim3 grid((M + 15) / 16);
#define MDG_LN(CTT, W)                                                                        \
  hipLaunchKernelGGL((ln_mod_kernel<CTT, W>), grid, dim3(256), 0, s, M, C, h, mods, mod_stride, \
                     rows_per_mod, shift_off, scale_off, eps, (CTT*)xn, stats)
  const bool w2 = (C % 128) == 0;
  if (dtype == MDG_BF16) {
    if (w2) MDG_LN(bf16_t, 2); else MDG_LN(bf16_t, 1);
  } else {
    if (w2) MDG_LN(float, 2); else MDG_LN(float, 1);
  }
#undef MDG_LN
  return hipGetLastError();
}

hipError_t mask_bias_launch(int B, int T, int L, const float* mask, float* kbias, float* kbias_s,
                            hipStream_t s) {
  const int n = B * T * L;
  hipLaunchKernelGGL(mask_bias_kernel, dim3((n + 255) / 256), dim3(256), 0, s, B, T, L, mask, kbias, kbias_s);
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
