// Fused GEMM for every projection of the MDGen block:  out = epi( pro(A) . W^T + bias ).
//
//   prologue  A_LNMOD : the whole BM x K row block of the fp32 residual stream is normalised
//                       (no-affine LayerNorm, eps 1e-6, latent_model.py:449/454) — or the
//                       affine LN of IPALayer.ipa_norm — then adaLN-modulated
//                       y*(1+scale[b]) + shift[b] (layers.py:14-15), converted to CT and kept
//                       resident in LDS for the whole K loop (K = C = 384 is small);
//             A_PLAIN : CT activations streamed through LDS with the weights.
//   epilogue  STORE   : + bias, optional exact-erf GELU / SiLU, CT or fp32 store (fc1);
//             GATE_RES: h += gate[b] * (acc + bias)  — gated residual of
//                       latent_model.py:472/486/491 fused into out_proj / fc2;
//             QKV     : + bias, q *= D^-1/2 (mha.py:264; * log2(e) for the exp2 softmax of
//                       the temporal kernel), rotate-half RoPE on q and k (fair-esm rotary,
//                       mha.py:356-357) at position l (spatial) or t (temporal), scattered
//                       into the attention layout the consumer kernel reads.
//
// Tiling (gfx950): 256 threads = 4 waves as 2(M) x 2(N); block tile 64 x BN (BN = 96 for
// C = 384 so a tile holds whole 24-wide heads, 64 for C = 64 test models), K-step 64,
// register-staged double buffer, 16-byte global loads, LDS rows padded by 16 B so the
// 16-lane fragment reads of ds_read_b128 spread over distinct bank slots.  Each wave owns a
// 32 x BN/2 sub-tile = 2 x (BN/32) MFMA 16x16 accumulators.
#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {

template <typename CT, int BN, int AMODE, int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(const mdg_gemm_desc p) {
  constexpr int BM = 64, BK = 64;
  constexpr int VEC = 16 / sizeof(CT);
  constexpr int LDT = BK + VEC;  // streamed tile row stride (elements)
  constexpr int NT = BN / 32;    // 16-wide n-tiles per wave
  constexpr int HALF_N = BN / 2;
  constexpr int LDC = BN + 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int M = p.M, K = p.K;

  CT* As = reinterpret_cast<CT*>(smem);
  CT* Bs;
  int lda_s;
  if constexpr (AMODE == MDG_A_LNMOD) {
    lda_s = K + VEC;
    Bs = As + BM * lda_s;
  } else {
    lda_s = LDT;
    Bs = As + 2 * BM * LDT;
  }

  // ---------------------------------------------------------------- prologue (LN + mod)
  if constexpr (AMODE == MDG_A_LNMOD) {
    const float* A = reinterpret_cast<const float*>(p.A);
    const int nper = K >> 6;
    const float invK = 1.0f / (float)K;
    for (int r = wave; r < BM; r += 4) {
      const int m = m0 + r;
      CT* dst = As + r * lda_s;
      if (m >= M) {
        for (int k = lane; k < K; k += 64) dst[k] = (CT)0.0f;
        continue;
      }
      const float* src = A + (size_t)m * p.lda;
      float v[8];
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = (e < nper) ? src[lane + 64 * e] : 0.f;
        s += v[e];
      }
      const float mean = wave_sum(s) * invK;
      float ss = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dlt = v[e] - mean;
        ss += (e < nper) ? dlt * dlt : 0.f;
      }
      const float rstd = 1.0f / sqrtf(wave_sum(ss) * invK + p.ln_eps);
      const float* mrow = p.mods ? p.mods + (size_t)(m / p.rows_per_mod) * p.mod_stride : nullptr;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (e < nper) {
          const int k = lane + 64 * e;
          float y = (v[e] - mean) * rstd;
          if (p.ln_w) y = y * p.ln_w[k] + p.ln_b[k];
          if (mrow) y = y * (1.0f + mrow[p.scale_off + k]) + mrow[p.shift_off + k];
          dst[k] = (CT)y;
        }
      }
    }
  }

  // ---------------------------------------------------------------- main loop
  const CT* W = reinterpret_cast<const CT*>(p.W);
  const CT* Ap = reinterpret_cast<const CT*>(p.A);
  constexpr int CPR = BK / VEC;                  // 16-B chunks per tile row
  constexpr int BCH = BN * CPR / 256;            // per-thread chunks of the W tile
  constexpr int ACH = (AMODE == MDG_A_PLAIN) ? BM * CPR / 256 : 1;
  uint4 breg[BCH];
  uint4 areg[ACH];

  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int c = 0; c < BCH; ++c) {
      const int idx = tid + c * 256, row = idx / CPR, cc = idx % CPR;
      breg[c] = *reinterpret_cast<const uint4*>(W + (size_t)(n0 + row) * p.ldw + k0 + cc * VEC);
    }
    if constexpr (AMODE == MDG_A_PLAIN) {
#pragma unroll
      for (int c = 0; c < ACH; ++c) {
        const int idx = tid + c * 256, row = idx / CPR, cc = idx % CPR;
        const int m = m0 + row;
        areg[c] = (m < M) ? *reinterpret_cast<const uint4*>(Ap + (size_t)m * p.lda + k0 + cc * VEC)
                          : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_tiles = [&](int buf) {
    CT* bdst = Bs + buf * BN * LDT;
#pragma unroll
    for (int c = 0; c < BCH; ++c) {
      const int idx = tid + c * 256, row = idx / CPR, cc = idx % CPR;
      *reinterpret_cast<uint4*>(bdst + row * LDT + cc * VEC) = breg[c];
    }
    if constexpr (AMODE == MDG_A_PLAIN) {
      CT* adst = As + buf * BM * LDT;
#pragma unroll
      for (int c = 0; c < ACH; ++c) {
        const int idx = tid + c * 256, row = idx / CPR, cc = idx % CPR;
        *reinterpret_cast<uint4*>(adst + row * LDT + cc * VEC) = areg[c];
      }
    }
  };

  f32x4 acc[2][NT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles((kt + 1) * BK);
    const CT* Ab;
    int acol;
    if constexpr (AMODE == MDG_A_PLAIN) {
      Ab = As + cur * BM * LDT;
      acol = 0;
    } else {
      Ab = As;
      acol = kt * BK;
    }
    const CT* Bb = Bs + cur * BN * LDT;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      typename V8<CT>::T a[2], b[NT];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = ld8<CT>(Ab + (wm * 32 + i * 16 + lr) * lda_s + acol + kk + 8 * lg);
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = ld8<CT>(Bb + (wn * HALF_N + j * 16 + lr) * LDT + kk + 8 * lg);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) mma_k32<CT>(acc[i][j], a[i], b[j]);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue via LDS
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * 32 + i * 16 + lg * 4 + r) * LDC + wn * HALF_N + j * 16 + lr] = acc[i][j][r];
  __syncthreads();

  constexpr int C4 = BN / 4;
  for (int idx = tid; idx < BM * C4; idx += 256) {
    const int r = idx / C4, c = (idx % C4) * 4;
    const int m = m0 + r;
    if (m >= M) continue;
    const int n = n0 + c;
    const float* crow = Cs + r * LDC;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = crow[c + e] + (p.bias ? p.bias[n + e] : 0.f);

    if constexpr (EPI == MDG_EPI_STORE) {
      if (p.act == MDG_ACT_GELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
      } else if (p.act == MDG_ACT_SILU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = silu(v[e]);
      }
      if (p.out_f32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + (size_t)m * p.ldo + n) =
            make_float4(v[0], v[1], v[2], v[3]);
      } else {
        st4<CT>(reinterpret_cast<CT*>(p.out) + (size_t)m * p.ldo + n, v[0], v[1], v[2], v[3]);
      }
    } else if constexpr (EPI == MDG_EPI_GATE_RES) {
      float4* R = reinterpret_cast<float4*>(p.resid + (size_t)m * p.ldr + n);
      float4 hv = *R;
      if (p.gate) {
        const float* g = p.gate + (size_t)(m / p.rows_per_mod) * p.mod_stride + p.gate_off + n;
        hv.x += g[0] * v[0]; hv.y += g[1] * v[1]; hv.z += g[2] * v[2]; hv.w += g[3] * v[3];
      } else {
        hv.x += v[0]; hv.y += v[1]; hv.z += v[2]; hv.w += v[3];
      }
      *R = hv;
    } else {  // QKV
      const int Cm = p.N / 3, D = p.D, half = D >> 1;
      const int which = n / Cm, w = n - which * Cm, head = w / D, d = w - head * D;
      const float qs = (which == 0) ? p.qscale : 1.0f;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] *= qs;
      int T = p.T, L = p.L;
      if (p.rope && which < 2) {
        const int pos = (p.qkv_layout == MDG_QKV_SPATIAL) ? (m % L) : ((m / L) % T);
        const float* cs = p.rope + (size_t)pos * half;
        const float* sn = p.rope + (size_t)p.rope_rows * half + (size_t)pos * half;
        float o[4];
        if (d < half) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float pv = (crow[c + half + e] + (p.bias ? p.bias[n + half + e] : 0.f)) * qs;
            o[e] = v[e] * cs[d + e] - pv * sn[d + e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float pv = (crow[c - half + e] + (p.bias ? p.bias[n - half + e] : 0.f)) * qs;
            o[e] = v[e] * cs[d - half + e] + pv * sn[d - half + e];
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = o[e];
      }
      CT* dst;
      if (p.qkv_layout == MDG_QKV_SPATIAL) {
        dst = reinterpret_cast<CT*>(p.qkv_out) + ((size_t)(m * 3 + which) * p.H + head) * MDG_DP + d;
      } else {
        const int TL = T * L, b = m / TL, l = m % L, t = (m / L) % T;
        const int BL = (M / TL) * L, seq = b * L + l;
        dst = reinterpret_cast<CT*>(p.qkv_out) + (size_t)which * BL * p.H * T * MDG_DP +
              ((size_t)(seq * p.H + head) * T + t) * MDG_DP + d;
      }
      st4<CT>(dst, v[0], v[1], v[2], v[3]);
    }
  }
}

template <typename CT, int BN, int AMODE, int EPI>
static size_t smem_bytes(int K) {
  constexpr int BM = 64, BK = 64, VEC = 16 / sizeof(CT), LDT = BK + VEC;
  size_t main = (AMODE == MDG_A_LNMOD)
                    ? (size_t)BM * (K + VEC) * sizeof(CT) + 2ull * BN * LDT * sizeof(CT)
                    : 2ull * BM * LDT * sizeof(CT) + 2ull * BN * LDT * sizeof(CT);
  size_t epi = (size_t)BM * (BN + 4) * sizeof(float);
  return main > epi ? main : epi;
}

template <typename CT, int BN, int AMODE, int EPI>
static hipError_t launch_one(const mdg_gemm_desc& p, hipStream_t s) {
  const size_t smem = smem_bytes<CT, BN, AMODE, EPI>(p.K);
  static bool attr_set = false;  // benign race: idempotent attribute write
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<CT, BN, AMODE, EPI>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  dim3 grid(p.N / BN, (p.M + 63) / 64);
  hipLaunchKernelGGL((gemm_kernel<CT, BN, AMODE, EPI>), grid, dim3(256), smem, s, p);
  return hipGetLastError();
}

template <typename CT, int BN>
static hipError_t dispatch_epi(const mdg_gemm_desc& p, hipStream_t s) {
  if (p.a_mode == MDG_A_LNMOD) {
    switch (p.epi) {
      case MDG_EPI_STORE: return launch_one<CT, BN, MDG_A_LNMOD, MDG_EPI_STORE>(p, s);
      case MDG_EPI_GATE_RES: return launch_one<CT, BN, MDG_A_LNMOD, MDG_EPI_GATE_RES>(p, s);
      default: return launch_one<CT, BN, MDG_A_LNMOD, MDG_EPI_QKV>(p, s);
    }
  }
  switch (p.epi) {
    case MDG_EPI_STORE: return launch_one<CT, BN, MDG_A_PLAIN, MDG_EPI_STORE>(p, s);
    case MDG_EPI_GATE_RES: return launch_one<CT, BN, MDG_A_PLAIN, MDG_EPI_GATE_RES>(p, s);
    default: return launch_one<CT, BN, MDG_A_PLAIN, MDG_EPI_QKV>(p, s);
  }
}

// Returns the block-N tile for this problem, or 0 if unsupported.
int gemm_pick_bn(const mdg_gemm_desc& p) {
  const int cand[2] = {96, 64};
  for (int bn : cand) {
    if (p.N % bn) continue;
    if (p.epi == MDG_EPI_QKV) {
      if (p.N % 3 || (p.N / 3) % bn || bn % p.D) continue;
    }
    return bn;
  }
  return 0;
}

size_t gemm_smem_bytes(const mdg_gemm_desc& p, int bn) {
  const bool bf = p.dtype == MDG_BF16;
  const bool ln = p.a_mode == MDG_A_LNMOD;
  if (bn == 96)
    return bf ? (ln ? smem_bytes<bf16_t, 96, 1, 0>(p.K) : smem_bytes<bf16_t, 96, 0, 0>(p.K))
              : (ln ? smem_bytes<float, 96, 1, 0>(p.K) : smem_bytes<float, 96, 0, 0>(p.K));
  return bf ? (ln ? smem_bytes<bf16_t, 64, 1, 0>(p.K) : smem_bytes<bf16_t, 64, 0, 0>(p.K))
            : (ln ? smem_bytes<float, 64, 1, 0>(p.K) : smem_bytes<float, 64, 0, 0>(p.K));
}

hipError_t gemm_launch(const mdg_gemm_desc& p, int bn, hipStream_t s) {
  if (p.dtype == MDG_BF16) return bn == 96 ? dispatch_epi<bf16_t, 96>(p, s) : dispatch_epi<bf16_t, 64>(p, s);
  return bn == 96 ? dispatch_epi<float, 96>(p, s) : dispatch_epi<float, 64>(p, s);
}

}  // namespace mdg
