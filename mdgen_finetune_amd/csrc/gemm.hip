// Fused GEMM for every projection of the MDGen block:  out = epi( pro(A) . W^T + bias ).
//
//   prologue  A_LNMOD : the block's BM rows of the fp32 residual stream are normalised
//                       (no-affine LayerNorm eps 1e-6, latent_model.py:449/454, FinalLayer
//                       layers.py:62 — or IPALayer's affine ipa_norm), adaLN-modulated
//                       y*(1+scale[b]) + shift[b] (layers.py:14-15), converted to CT and kept
//                       resident in LDS; the block then sweeps a group of N tiles, so the
//                       LayerNorm is computed once per row per group.
//             A_PLAIN : CT activations streamed through LDS with the weights.
//   epilogue  (accumulators -> LDS band stage -> full-row coalesced 8/16-B accesses)
//             STORE   : + bias, optional exact-erf GELU / SiLU, CT or fp32 store (fc1);
//             GATE_RES: h += gate[b] * (acc + bias)  — the gated residual of
//                       latent_model.py:472/486/491 fused into out_proj / fc2;
//             QKV     : + bias, q *= D^-1/2 (mha.py:264; * log2 e for the exp2 softmax of the
//                       temporal kernel), RoPE on q and k at position l (spatial) or t
//                       (temporal), scattered into the attention layout the consumer reads.
//                       The packer stores each q/k head's rows PAIR-INTERLEAVED
//                       (column 2i = dim i, 2i+1 = dim i+D/2): fair-esm's rotate-half partner
//                       (mha.py:356-357) is the neighbouring column of the same 4-column chunk.
//                       q.k dot products are invariant to the shared permutation; V keeps
//                       natural order.
//             EULER   : FinalLayer + Euler update (layers.py:58-75, integrators.py:106-113):
//                       v = acc + bias; x_out = x_in + dt * v for the n_valid real columns.
//
// Tiling (gfx950): 512 threads = 8 waves as WM x WN; block tile BM x BN, K-step 64,
// register-staged double buffer (the next K-step's 16-B global loads are issued before the
// current K-step's MFMAs; one barrier per K-step), outer loop over the block's N tiles with
// the next tile's first K-step prefetched across the epilogue.  Two waves per SIMD let one
// wave's VALU epilogue / LN prologue overlap the other's MFMAs.  LDS rows are padded by 16 B
// so the 16-lane ds_read_b128 fragment reads hit distinct bank slots.
//   configs: LN-resident QKV / fc1 / final  128x128 (2x4 waves), 128x32 (8x1)
//            streamed out_proj / fc2        128x384 (2x4): full output rows, so the activation
//                                           is read from HBM exactly once
//            fp32 parity path               64x32 / 64x96 / 64x128 (4x2)
#include "../../include/mdgen_hip.h"
#include "common.h"

#include <stdlib.h>

namespace mdg {

// kRingWaitNote — every raw s_barrier after which a wave refills a ring slot (LDS DMA) is
// preceded by an explicit s_waitcnt lgkmcnt(0): the compiler may otherwise leave the previous
// step's last ds_reads of THAT slot in flight across the barrier (it moves their MFMAs, and the
// waits guarding them, below it), and an LDS-DMA write issued by another wave after the barrier
// then races those reads.  Found in round 3 by scanning the ISA of every kernel for LDS
// operations pending at a barrier (mlp_rowln_kernel<384, false>, rowln_qkv_kernel); DESIGN.md §4.

constexpr int kThreads = 512;

// x + dt * v rounded twice, as torchdiffeq's Euler step computes it (integrators.py:106-113:
// dt * f, then y0 + that).  hipcc's __fmul_rn / __fadd_rn are plain operations that the
// default -ffp-contract=fast fuses into one v_fma (one rounding); contraction is off here.
__device__ __forceinline__ float euler_update(float x, float dt, float v) {
#pragma clang fp contract(off)
  const float dv = dt * v;
  return x + dv;
}

// floor(a / d) for 0 <= a < 2^24 with a float reciprocal + one-step fix-up
__device__ __forceinline__ int fdiv(int a, int d, float inv) {
  int q = (int)((float)a * inv);
  const int r = a - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

// Epilogue of 4 consecutive output columns n..n+3 of row m (v = the fp32 accumulators).
template <typename CT, int EPI>
__device__ __forceinline__ void epi4(const mdg_gemm_desc& p, int m, int n, float4 v, float invD, float invL,
                                     float invT) {
  const int M = p.M;
  if (p.bias) {
    const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
    v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
  }
  if constexpr (EPI == MDG_EPI_STORE) {
    if (p.act == MDG_ACT_GELU) {
      if (p.aux) st4<CT>(reinterpret_cast<CT*>(p.aux) + (size_t)m * p.ldaux + n, v.x, v.y, v.z, v.w);
      v.x = gelu_erf(v.x); v.y = gelu_erf(v.y); v.z = gelu_erf(v.z); v.w = gelu_erf(v.w);
    } else if (p.act == MDG_ACT_DGELU) {
      const float4 u = ld4f<CT>(reinterpret_cast<const CT*>(p.aux) + (size_t)m * p.ldaux + n);
      v.x *= gelu_grad(u.x); v.y *= gelu_grad(u.y); v.z *= gelu_grad(u.z); v.w *= gelu_grad(u.w);
    } else if (p.act == MDG_ACT_SILU) {
      v.x = silu(v.x); v.y = silu(v.y); v.z = silu(v.z); v.w = silu(v.w);
    }
    if (p.out_f32) *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + (size_t)m * p.ldo + n) = v;
    else st4<CT>(reinterpret_cast<CT*>(p.out) + (size_t)m * p.ldo + n, v.x, v.y, v.z, v.w);
  } else if constexpr (EPI == MDG_EPI_GATE_RES) {
    float4* R = reinterpret_cast<float4*>(p.resid + (size_t)m * p.ldr + n);
    float4 hv = p.resid_in ? *reinterpret_cast<const float4*>(p.resid_in + (size_t)m * p.ldr + n) : *R;
    if (p.aux) st4<CT>(reinterpret_cast<CT*>(p.aux) + (size_t)m * p.ldaux + n, v.x, v.y, v.z, v.w);
    if (p.gate) {
      const float4 g = *reinterpret_cast<const float4*>(
          p.gate + (size_t)(m / p.rows_per_mod) * p.mod_stride + p.gate_off + n);
      hv.x += g.x * v.x; hv.y += g.y * v.y; hv.z += g.z * v.z; hv.w += g.w * v.w;
    } else {
      hv.x += v.x; hv.y += v.y; hv.z += v.z; hv.w += v.w;
    }
    *R = hv;
  } else if constexpr (EPI == MDG_EPI_QKV) {
    // 4 columns = 2 rotate-half pairs of one head (D % 4 == 0, pair-interleaved rows)
    const int Cm = p.N / 3, D = p.D;
    const int which = (n >= Cm) + (n >= 2 * Cm), w = n - which * Cm;
    const int head = fdiv(w, D, invD), cp = w - head * D;
    if (which == 0) {
      v.x *= p.qscale; v.y *= p.qscale; v.z *= p.qscale; v.w *= p.qscale;
    }
    const int ml = fdiv(m, p.L, invL), l = m - ml * p.L;  // m = ml*L + l
    const int mt = fdiv(ml, p.T, invT), t = ml - mt * p.T;  // ml = b*T + t
    if (p.rope && which < 2) {
      const int half = D >> 1, pi = cp >> 1;
      const int pos = (p.qkv_layout == MDG_QKV_SPATIAL) ? l : t;
      const float* cs = p.rope + (size_t)pos * half + pi;
      const float* sn = p.rope + (size_t)p.rope_rows * half + (size_t)pos * half + pi;
      const float c0 = cs[0], s0 = sn[0], c1 = cs[1], s1 = sn[1];
      const float x0 = v.x * c0 - v.y * s0, y0 = v.y * c0 + v.x * s0;
      const float x1 = v.z * c1 - v.w * s1, y1 = v.w * c1 + v.z * s1;
      v.x = x0; v.y = y0; v.z = x1; v.w = y1;
    }
    CT* dst;
    if (p.qkv_layout == MDG_QKV_SPATIAL) {
      dst = reinterpret_cast<CT*>(p.qkv_out) + ((size_t)(m * 3 + which) * p.H + head) * D + cp;
    } else {
      const int BL = (M / (p.T * p.L)) * p.L, seq = mt * p.L + l;
      const int dp = p.qkv_layout == MDG_QKV_TEMPORAL_PACKED ? p.D : dp_of(p.D);
      dst = reinterpret_cast<CT*>(p.qkv_out) + (size_t)which * BL * p.H * p.T * dp +
            ((size_t)(seq * p.H + head) * p.T + t) * dp + cp;
    }
    st4<CT>(dst, v.x, v.y, v.z, v.w);
  } else {  // EULER
    const size_t rowoff = (size_t)m * p.ldo;
    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (n + e < p.n_valid) {
        if (p.v_out) p.v_out[rowoff + n + e] = vv[e];
        float* xo = reinterpret_cast<float*>(p.out);
        if (xo) xo[rowoff + n + e] = euler_update(p.x_in[rowoff + n + e], p.dt, vv[e]);
      }
    }
  }
}

template <typename CT, int BM, int BN, int WM, int AMODE, int EPI>
__global__ __launch_bounds__(kThreads) void gemm_kernel(const mdg_gemm_desc p) {
  constexpr int WN = 8 / WM;
  constexpr int BK = 64;
  constexpr int VEC = 16 / sizeof(CT);
  constexpr int LDT = BK + VEC;
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int CPR = BK / VEC;                // 16-B chunks per tile row
  constexpr int BCH = (BN * CPR + kThreads - 1) / kThreads;
  constexpr int ACH = (AMODE == MDG_A_PLAIN) ? BM * CPR / kThreads : 1;
  constexpr int BAND = BM / WM;                // epilogue rows staged per pass
  constexpr int LDS_ST = BN + 4;
  static_assert(MT >= 1 && NT >= 1 && WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  static_assert(AMODE == MDG_A_LNMOD || (BM * CPR) % kThreads == 0, "A tile / threads");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.y * BM;
  const int M = p.M, K = p.K;
  const int n_tiles = p.N / BN;
  const int tpg = (n_tiles + gridDim.x - 1) / gridDim.x;
  const int nt0 = blockIdx.x * tpg;
  const int nt1 = min(n_tiles, nt0 + tpg);
  if (nt0 >= nt1) return;

  CT* As = reinterpret_cast<CT*>(smem);
  const int lda_s = (AMODE == MDG_A_LNMOD) ? K + VEC : LDT;
  CT* Bs = (AMODE == MDG_A_LNMOD) ? As + BM * lda_s : As + 2 * BM * LDT;
  // band stage: the B double buffer (LNMOD) or the whole A+B ring (PLAIN); both are idle
  // while the epilogue runs (size checked on the host: gemm_plan / stage_fits)
  float* stage = reinterpret_cast<float*>(AMODE == MDG_A_LNMOD ? reinterpret_cast<unsigned char*>(Bs) : smem);

  const CT* W = reinterpret_cast<const CT*>(p.W);
  const CT* Ap = reinterpret_cast<const CT*>(p.A);
  u32x4 breg[BCH];
  u32x4 areg[ACH];

#define MDG_LOAD_TILES(nb_, k0_)                                                                \
  {                                                                                             \
    _Pragma("unroll") for (int c = 0; c < BCH; ++c) {                                           \
      const int idx = tid + c * kThreads, row = idx / CPR, cc = idx % CPR;                      \
      if (BN * CPR % kThreads == 0 || row < BN)                                                 \
        breg[c] = *reinterpret_cast<const u32x4*>(W + (size_t)((nb_) + row) * p.ldw + (k0_) + cc * VEC); \
    }                                                                                           \
    if constexpr (AMODE == MDG_A_PLAIN) {                                                       \
      _Pragma("unroll") for (int c = 0; c < ACH; ++c) {                                         \
        const int idx = tid + c * kThreads, row = idx / CPR, cc = idx % CPR, m = m0 + row;      \
        areg[c] = (m < M) ? *reinterpret_cast<const u32x4*>(Ap + (size_t)m * p.lda + (k0_) + cc * VEC) \
                          : u32x4{0u, 0u, 0u, 0u};                                              \
      }                                                                                         \
    }                                                                                           \
  }
#define MDG_STORE_TILES(buf)                                                                    \
  {                                                                                             \
    CT* bdst = Bs + (buf) * BN * LDT;                                                           \
    _Pragma("unroll") for (int c = 0; c < BCH; ++c) {                                           \
      const int idx = tid + c * kThreads, row = idx / CPR, cc = idx % CPR;                      \
      if (BN * CPR % kThreads == 0 || row < BN)                                                 \
        *reinterpret_cast<u32x4*>(bdst + row * LDT + cc * VEC) = breg[c];                       \
    }                                                                                           \
    if constexpr (AMODE == MDG_A_PLAIN) {                                                       \
      CT* adst = As + (buf) * BM * LDT;                                                         \
      _Pragma("unroll") for (int c = 0; c < ACH; ++c) {                                         \
        const int idx = tid + c * kThreads, row = idx / CPR, cc = idx % CPR;                    \
        *reinterpret_cast<u32x4*>(adst + row * LDT + cc * VEC) = areg[c];                       \
      }                                                                                         \
    }                                                                                           \
  }

  // first K-step of the first N tile in flight while the LayerNorm prologue runs
  MDG_LOAD_TILES(nt0 * BN, 0);

  // ---------------------------------------------------------------- prologue (LN + mod)
  if constexpr (AMODE == MDG_A_LNMOD) {
    const float* A = reinterpret_cast<const float*>(p.A);
    const float invK = 1.0f / (float)K;
    if ((K & 127) == 0) {
      // lane owns columns k = 2*lane + 128*e, e < K/128 <= 4; 4 rows at a time per wave
      const int nE = K >> 7;
      for (int r0 = wave * 4; r0 < BM; r0 += 32) {
        float2 v[4][4], sc[4][4], sh[4][4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int m = min(m0 + r0 + rr, M - 1);
          const float* mrow = p.mods ? p.mods + (size_t)(m / p.rows_per_mod) * p.mod_stride : nullptr;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sc[rr][e] = make_float2(0.f, 0.f);
            sh[rr][e] = make_float2(0.f, 0.f);
            if (e < nE) {
              const int k = 2 * lane + 128 * e;
              v[rr][e] = *reinterpret_cast<const float2*>(A + (size_t)m * p.lda + k);
              if (mrow) {
                sc[rr][e] = *reinterpret_cast<const float2*>(mrow + p.scale_off + k);
                sh[rr][e] = *reinterpret_cast<const float2*>(mrow + p.shift_off + k);
              }
            } else {
              v[rr][e] = make_float2(0.f, 0.f);
            }
          }
        }
        float mean[4], var[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          float s = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) s += v[rr][e].x + v[rr][e].y;
          mean[rr] = s;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) mean[rr] += __shfl_xor(mean[rr], o, 64);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          mean[rr] *= invK;
          float ss = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (e < nE) {
              const float a = v[rr][e].x - mean[rr], b = v[rr][e].y - mean[rr];
              ss += a * a + b * b;
            }
          var[rr] = ss;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) var[rr] += __shfl_xor(var[rr], o, 64);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int r = r0 + rr;
          const bool live = m0 + r < M;
          const float rs = 1.0f / sqrtf(var[rr] * invK + p.ln_eps);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (e < nE) {
              const int k = 2 * lane + 128 * e;
              float y0 = (v[rr][e].x - mean[rr]) * rs, y1 = (v[rr][e].y - mean[rr]) * rs;
              if (p.ln_w) {
                y0 = y0 * p.ln_w[k] + p.ln_b[k];
                y1 = y1 * p.ln_w[k + 1] + p.ln_b[k + 1];
              }
              if (p.mods) {
                y0 = y0 * (1.0f + sc[rr][e].x) + sh[rr][e].x;
                y1 = y1 * (1.0f + sc[rr][e].y) + sh[rr][e].y;
              }
              if (!live) y0 = y1 = 0.f;
              if constexpr (is_bf16<CT>()) {
                typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
                bf16x2 pr;
                pr[0] = (bf16_t)y0;
                pr[1] = (bf16_t)y1;
                *reinterpret_cast<bf16x2*>(As + r * lda_s + k) = pr;
              } else {
                *reinterpret_cast<float2*>(As + r * lda_s + k) = make_float2(y0, y1);
              }
            }
          }
        }
      }
    } else {
      // generic (K % 64 == 0, small test models): one row per wave, scalar columns
      for (int r = wave; r < BM; r += 8) {
        const int m = m0 + r;
        const bool live = m < M;
        const float* src = A + (size_t)(live ? m : M - 1) * p.lda;
        float s = 0.f;
        for (int k = lane; k < K; k += 64) s += src[k];
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        const float mean = s * invK;
        float ss = 0.f;
        for (int k = lane; k < K; k += 64) {
          const float a = src[k] - mean;
          ss += a * a;
        }
        for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o, 64);
        const float rs = 1.0f / sqrtf(ss * invK + p.ln_eps);
        const float* mrow = p.mods ? p.mods + (size_t)((live ? m : M - 1) / p.rows_per_mod) * p.mod_stride : nullptr;
        for (int k = lane; k < K; k += 64) {
          float y = (src[k] - mean) * rs;
          if (p.ln_w) y = y * p.ln_w[k] + p.ln_b[k];
          if (mrow) y = y * (1.0f + mrow[p.scale_off + k]) + mrow[p.shift_off + k];
          As[r * lda_s + k] = (CT)(live ? y : 0.f);
        }
      }
    }
  }

  MDG_STORE_TILES(0);
  __syncthreads();

  const int nk = K / BK;
  const float invD = 1.0f / (float)(p.D > 0 ? p.D : 1);
  const float invL = 1.0f / (float)(p.L > 0 ? p.L : 1);
  const float invT = 1.0f / (float)(p.T > 0 ? p.T : 1);

  for (int nt = nt0; nt < nt1; ++nt) {
    const int n0 = nt * BN;
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) MDG_LOAD_TILES(n0, (kt + 1) * BK)
      else if (nt + 1 < nt1) MDG_LOAD_TILES(n0 + BN, 0)
      const CT* Ab = (AMODE == MDG_A_PLAIN) ? As + cur * BM * LDT : As;
      const int acol = (AMODE == MDG_A_PLAIN) ? 0 : kt * BK;
      const CT* Bb = Bs + cur * BN * LDT;
#pragma unroll
      for (int kk = 0; kk < BK; kk += 32) {
        typename V8<CT>::T a[MT], b[NT];
#pragma unroll
        for (int i = 0; i < MT; ++i) a[i] = ld8<CT>(Ab + (wm * WTM + i * 16 + lr) * lda_s + acol + kk + 8 * lg);
#pragma unroll
        for (int j = 0; j < NT; ++j) b[j] = ld8<CT>(Bb + (wn * WTN + j * 16 + lr) * LDT + kk + 8 * lg);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) mma_k32<CT>(acc[i][j], a[i], b[j]);
      }
      if (kt + 1 < nk) MDG_STORE_TILES(cur ^ 1);
      __syncthreads();
    }

    // ------------------------------------------------------------------ epilogue
    // pass p: waves with wm == p stage their BAND rows x BN into LDS, then all threads sweep
    // full rows with 4-column chunks (16-B fp32 / 8-B bf16 accesses, contiguous per row)
#pragma unroll 1
    for (int pass = 0; pass < WM; ++pass) {
      if (wm == pass) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              stage[(i * 16 + lg * 4 + r) * LDS_ST + wn * WTN + j * 16 + lr] = acc[i][j][r];
      }
      __syncthreads();
      constexpr int C4 = BN / 4;
      for (int idx = tid; idx < BAND * C4; idx += kThreads) {
        const int rb = idx / C4, c = (idx % C4) * 4;
        const int m = m0 + pass * BAND + rb;
        if (m >= M) continue;
        const float4 v = *reinterpret_cast<const float4*>(stage + rb * LDS_ST + c);
        epi4<CT, EPI>(p, m, n0 + c, v, invD, invL, invT);
      }
      __syncthreads();
    }
    if (nt + 1 < nt1) {
      MDG_STORE_TILES(0);  // next N tile's first K-step, loaded before the epilogue
      __syncthreads();
    }
  }
#undef MDG_LOAD_TILES
#undef MDG_STORE_TILES
}

// ---------------------------------------------------------------------------------------
// bf16 streamed-A GEMM for the block's big projections (qkv, out_proj, fc1, fc2 at
// M = B*T*L rows): 128x128 block tile, 4 waves as 2x2 with 64x64 wave tiles (4x4
// accumulators of v_mfma_f32_16x16x32_bf16, 8 fragment reads per 16 MFMAs), K-step 64.
//   staging : global_load_lds (16 B/lane, no VGPR round trip) into two LDS stages; the
//             image is lane-linear per wave instruction (8 rows x 128 B), so the
//             ds_read_b128 bank swizzle (16-B chunk c of row r stored at c ^ ((r>>1)&7))
//             is applied to the per-lane GLOBAL source address and undone on the read.
//             With 16 fragment rows of one lane group on 8 row pairs the read is
//             conflict-free for all four ds_read_b128 lane groups.
//   schedule: one barrier per K-step — wait for stage k, barrier, issue stage k+1's
//             loads, MFMAs on stage k; two blocks per CU hide each other's barriers.
//   order   : XCD-aware bijective remap of the 1-D grid so the N tiles of one M tile run on
//             the same XCD (its L2 serves the A panel re-reads; W stays L2-resident).
//   epilogue: accumulators -> fp32 LDS image of the whole tile -> epi4 on 4-column chunks
//             with full-row coalesced accesses.
constexpr int kB4Threads = 256;
constexpr int kB4Tile = 128;


// Epilogue of one BM x 128 output tile staged in LDS as fp32 [BM][132] (NT threads).
template <int EPI, int NT, int BM>
__device__ __forceinline__ void epi_tile(const mdg_gemm_desc& p, const float* __restrict__ stage, int m0, int n0,
                                         int tid) {
  constexpr int LDS_ST = 128 + 4;
  const int M = p.M;
  // Thread -> (4-column chunk c, rows r0 + RS*u): the chunk is fixed per thread, so every
  // per-column operand (bias, head/which/pair of the QKV scatter) is loaded once, and the
  // per-row global operands (residual, gate, RoPE table) of 8 rows are gathered before any
  // of them is consumed — no load -> store -> load latency chain.
  constexpr int U = (EPI == MDG_EPI_QKV) ? 4 : 8;
  const int c = (tid & 31) * 4, n = n0 + c, r0 = tid >> 5;
  constexpr int RS = NT / 32, RPT = BM / RS;  // row stride, rows per thread
  float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
  if (p.bias) bb = *reinterpret_cast<const float4*>(p.bias + n);
  if constexpr (EPI == MDG_EPI_STORE) {
#pragma unroll
    for (int u0 = 0; u0 < RPT; u0 += U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u] = *reinterpret_cast<const float4*>(stage + (r0 + RS * (u0 + u)) * LDS_ST + c);
        v[u].x += bb.x; v[u].y += bb.y; v[u].z += bb.z; v[u].w += bb.w;
        if (p.act == MDG_ACT_GELU) {
          if (p.aux && m0 + r0 + RS * (u0 + u) < M)
            st4<bf16_t>(reinterpret_cast<bf16_t*>(p.aux) + (size_t)(m0 + r0 + RS * (u0 + u)) * p.ldaux + n, v[u].x,
                        v[u].y, v[u].z, v[u].w);
          v[u].x = gelu_fast(v[u].x); v[u].y = gelu_fast(v[u].y); v[u].z = gelu_fast(v[u].z); v[u].w = gelu_fast(v[u].w);
        } else if (p.act == MDG_ACT_DGELU) {
          const int mm = min(m0 + r0 + RS * (u0 + u), M - 1);
          const float4 a = ld4f<bf16_t>(reinterpret_cast<const bf16_t*>(p.aux) + (size_t)mm * p.ldaux + n);
          v[u].x *= gelu_grad_fast(a.x); v[u].y *= gelu_grad_fast(a.y);
          v[u].z *= gelu_grad_fast(a.z); v[u].w *= gelu_grad_fast(a.w);
        } else if (p.act == MDG_ACT_SILU) {
          v[u].x = silu(v[u].x); v[u].y = silu(v[u].y); v[u].z = silu(v[u].z); v[u].w = silu(v[u].w);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = m0 + r0 + RS * (u0 + u);
        if (m >= M) break;
        if (p.out_f32) *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + (size_t)m * p.ldo + n) = v[u];
        else st4<bf16_t>(reinterpret_cast<bf16_t*>(p.out) + (size_t)m * p.ldo + n, v[u].x, v[u].y, v[u].z, v[u].w);
      }
    }
  } else if constexpr (EPI == MDG_EPI_GATE_RES) {
    const float inv_rpm = 1.0f / (float)p.rows_per_mod;
#pragma unroll
    for (int u0 = 0; u0 < RPT; u0 += U) {
      float4 hv[U], g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = min(m0 + r0 + RS * (u0 + u), M - 1);
        hv[u] = *reinterpret_cast<const float4*>((p.resid_in ? p.resid_in : p.resid) + (size_t)m * p.ldr + n);
        g[u] = make_float4(1.f, 1.f, 1.f, 1.f);
        if (p.gate)
          g[u] = *reinterpret_cast<const float4*>(p.gate + (size_t)fdiv(m, p.rows_per_mod, inv_rpm) * p.mod_stride +
                                                  p.gate_off + n);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = m0 + r0 + RS * (u0 + u);
        if (m >= M) break;
        float4 v = *reinterpret_cast<const float4*>(stage + (r0 + RS * (u0 + u)) * LDS_ST + c);
        v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
        if (p.aux) st4<bf16_t>(reinterpret_cast<bf16_t*>(p.aux) + (size_t)m * p.ldaux + n, v.x, v.y, v.z, v.w);
        float4 h = hv[u];
        if (p.gate) {
          h.x += g[u].x * v.x; h.y += g[u].y * v.y; h.z += g[u].z * v.z; h.w += g[u].w * v.w;
        } else {
          h.x += v.x; h.y += v.y; h.z += v.z; h.w += v.w;
        }
        *reinterpret_cast<float4*>(p.resid + (size_t)m * p.ldr + n) = h;
      }
    }
  } else if constexpr (EPI == MDG_EPI_QKV) {
    const int Cm = p.N / 3, D = p.D, half = D >> 1;
    const int which = (n >= Cm) + (n >= 2 * Cm), w = n - which * Cm;
    const int head = w / D, cp = w - head * D, pi = cp >> 1;
    const float sc = (which == 0) ? p.qscale : 1.0f;
    const bool rope = p.rope && which < 2, spatial = p.qkv_layout == MDG_QKV_SPATIAL;
    const float invL = 1.0f / (float)p.L, invT = 1.0f / (float)p.T;
    const int BL = (M / (p.T * p.L)) * p.L;
    bf16_t* qo = reinterpret_cast<bf16_t*>(p.qkv_out);
    const size_t colS = (size_t)(which * p.H + head) * D + cp;               // spatial: + m*3*H*D
    const int dp = p.qkv_layout == MDG_QKV_TEMPORAL_PACKED ? D : dp_of(D);
    const size_t colT = (size_t)which * BL * p.H * p.T * dp + (size_t)head * p.T * dp + cp;
#pragma unroll
    for (int u0 = 0; u0 < RPT; u0 += U) {
      float2 cs[U], sn[U];
      int pos[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = min(m0 + r0 + RS * (u0 + u), M - 1);
        const int ml = fdiv(m, p.L, invL), l = m - ml * p.L;
        const int t = ml - fdiv(ml, p.T, invT) * p.T;
        pos[u] = spatial ? l : t;
        cs[u] = sn[u] = make_float2(0.f, 0.f);
        if (rope) {
          cs[u] = *reinterpret_cast<const float2*>(p.rope + (size_t)pos[u] * half + pi);
          sn[u] = *reinterpret_cast<const float2*>(p.rope + (size_t)(p.rope_rows + pos[u]) * half + pi);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = m0 + r0 + RS * (u0 + u);
        if (m >= M) break;
        float4 v = *reinterpret_cast<const float4*>(stage + (r0 + RS * (u0 + u)) * LDS_ST + c);
        v.x = (v.x + bb.x) * sc; v.y = (v.y + bb.y) * sc; v.z = (v.z + bb.z) * sc; v.w = (v.w + bb.w) * sc;
        if (rope) {
          const float x0 = v.x * cs[u].x - v.y * sn[u].x, y0 = v.y * cs[u].x + v.x * sn[u].x;
          const float x1 = v.z * cs[u].y - v.w * sn[u].y, y1 = v.w * cs[u].y + v.z * sn[u].y;
          v.x = x0; v.y = y0; v.z = x1; v.w = y1;
        }
        size_t off;
        if (spatial) {
          off = (size_t)m * 3 * p.H * D + colS;
        } else {
          const int ml = fdiv(m, p.L, invL), l = m - ml * p.L;
          const int b = fdiv(ml, p.T, invT), t = ml - b * p.T;
          off = colT + ((size_t)(b * p.L + l) * p.H * p.T + t) * dp;
        }
        st4<bf16_t>(qo + off, v.x, v.y, v.z, v.w);
      }
    }
  } else {
    const float invD = 1.0f / (float)(p.D > 0 ? p.D : 1);
    const float invL = 1.0f / (float)(p.L > 0 ? p.L : 1);
    const float invT = 1.0f / (float)(p.T > 0 ? p.T : 1);
    for (int u = 0; u < RPT; ++u) {
      const int m = m0 + r0 + RS * u;
      if (m >= M) break;
      float4 v = *reinterpret_cast<const float4*>(stage + (r0 + RS * u) * LDS_ST + c);
      epi4<bf16_t, EPI>(p, m, n, v, invD, invL, invT);
    }
  }
}

// Wide-store variant of epi_tile for the bf16 STORE (fc1 + GELU, plain projections) and QKV
// (q|k|v + RoPE scatter, head dim a multiple of 8) epilogues: a thread owns 8 consecutive
// columns (16 threads per 128-column row), so every output store is a 16-B bf16x8 (was 8 B):
// half the store instructions, which bound these epilogues, for the same bytes.
template <int EPI, int NT, int BM>
__device__ __forceinline__ void epi_tile8(const mdg_gemm_desc& p, const float* __restrict__ stage, int m0, int n0,
                                          int tid) {
  constexpr int LDS_ST = 128 + 4;
  const int M = p.M;
  const int c = (tid & 15) * 8, n = n0 + c, r0 = tid >> 4;
  constexpr int RS = NT / 16, RPT = BM / RS, U = 2;
  static_assert(RPT % U == 0, "rows per thread");
  float bb[8];
#pragma unroll
  for (int j = 0; j < 8; j += 4) {
    const float4 b = p.bias ? *reinterpret_cast<const float4*>(p.bias + n + j) : make_float4(0.f, 0.f, 0.f, 0.f);
    bb[j] = b.x; bb[j + 1] = b.y; bb[j + 2] = b.z; bb[j + 3] = b.w;
  }
  auto ld8s = [&](int row, float (&v)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(stage + row * LDS_ST + c);
    const float4 b = *reinterpret_cast<const float4*>(stage + row * LDS_ST + c + 4);
    v[0] = a.x + bb[0]; v[1] = a.y + bb[1]; v[2] = a.z + bb[2]; v[3] = a.w + bb[3];
    v[4] = b.x + bb[4]; v[5] = b.y + bb[5]; v[6] = b.z + bb[6]; v[7] = b.w + bb[7];
  };
  auto st8 = [&](bf16_t* dst, const float (&v)[8]) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16_t)v[j];
    *reinterpret_cast<bf16x8*>(dst) = o;
  };
  if constexpr (EPI == MDG_EPI_STORE) {
    // DGELU: every row's pre-activation piece is loaded up front (one HBM round trip per band
    // instead of one per U-row batch)
    bf16x8 ax[RPT];
    if (p.act == MDG_ACT_DGELU) {
#pragma unroll
      for (int i = 0; i < RPT; ++i)
        ax[i] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16_t*>(p.aux) +
                                                 (size_t)min(m0 + r0 + RS * i, M - 1) * p.ldaux + n);
    }
#pragma unroll
    for (int u0 = 0; u0 < RPT; u0 += U) {
      float v[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = r0 + RS * (u0 + u), m = m0 + row;
        ld8s(row, v[u]);
        if (p.act == MDG_ACT_GELU) {
          if (p.aux && m < M) st8(reinterpret_cast<bf16_t*>(p.aux) + (size_t)m * p.ldaux + n, v[u]);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[u][j] = gelu_fast(v[u][j]);
        } else if (p.act == MDG_ACT_DGELU) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[u][j] *= gelu_grad_fast((float)ax[u0 + u][j]);
        } else if (p.act == MDG_ACT_SILU) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[u][j] = silu(v[u][j]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = m0 + r0 + RS * (u0 + u);
        if (m >= M) break;
        if (p.out_f32) {
          float* o = reinterpret_cast<float*>(p.out) + (size_t)m * p.ldo + n;
          *reinterpret_cast<float4*>(o) = make_float4(v[u][0], v[u][1], v[u][2], v[u][3]);
          *reinterpret_cast<float4*>(o + 4) = make_float4(v[u][4], v[u][5], v[u][6], v[u][7]);
        } else {
          st8(reinterpret_cast<bf16_t*>(p.out) + (size_t)m * p.ldo + n, v[u]);
        }
      }
    }
  } else {  // MDG_EPI_QKV, D % 8 == 0: the 8 columns lie in one head of one of q | k | v
    const int Cm = p.N / 3, D = p.D, half = D >> 1;
    const int which = (n >= Cm) + (n >= 2 * Cm), w = n - which * Cm;
    const int head = w / D, cp = w - head * D, pi = cp >> 1;  // 4 RoPE pairs pi .. pi+3
    const float sc = (which == 0) ? p.qscale : 1.0f;
    const bool rope = p.rope && which < 2, spatial = p.qkv_layout == MDG_QKV_SPATIAL;
    const float invL = 1.0f / (float)p.L, invT = 1.0f / (float)p.T;
    const int BL = (M / (p.T * p.L)) * p.L;
    const int dp = p.qkv_layout == MDG_QKV_TEMPORAL_PACKED ? D : dp_of(D);
    bf16_t* qo = reinterpret_cast<bf16_t*>(p.qkv_out);
    const size_t colS = (size_t)(which * p.H + head) * D + cp;
    const size_t colT = (size_t)which * BL * p.H * p.T * dp + (size_t)head * p.T * dp + cp;
#pragma unroll
    for (int u0 = 0; u0 < RPT; u0 += U) {
      float4 cs[U], sn[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = min(m0 + r0 + RS * (u0 + u), M - 1);
        const int ml = fdiv(m, p.L, invL), l = m - ml * p.L;
        const int t = ml - fdiv(ml, p.T, invT) * p.T;
        const int pos = spatial ? l : t;
        cs[u] = sn[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (rope) {  // cos / sin of pairs pi..pi+3 (16-B aligned: half and pi are multiples of 4)
          cs[u] = *reinterpret_cast<const float4*>(p.rope + (size_t)pos * half + pi);
          sn[u] = *reinterpret_cast<const float4*>(p.rope + (size_t)(p.rope_rows + pos) * half + pi);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = r0 + RS * (u0 + u), m = m0 + row;
        if (m >= M) break;
        float v[8];
        ld8s(row, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= sc;
        if (rope) {
          const float cc[4] = {cs[u].x, cs[u].y, cs[u].z, cs[u].w}, ss[4] = {sn[u].x, sn[u].y, sn[u].z, sn[u].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {  // explicit fma: the fused rowln_qkv epilogue rounds alike
            const float x = v[2 * k], y = v[2 * k + 1];
            v[2 * k] = __builtin_fmaf(x, cc[k], -(y * ss[k]));
            v[2 * k + 1] = __builtin_fmaf(y, cc[k], x * ss[k]);
          }
        }
        size_t off;
        if (spatial) {
          off = (size_t)m * 3 * p.H * D + colS;
        } else {
          const int ml = fdiv(m, p.L, invL), l = m - ml * p.L;
          const int b = fdiv(ml, p.T, invT), t = ml - b * p.T;
          off = colT + ((size_t)(b * p.L + l) * p.H * p.T + t) * dp;
        }
        st8(qo + off, v);
      }
    }
  }
}

// NS: operand ring depth.  2 (default for BK 64): wait for everything, then prefetch one step
// ahead.  3 / 4 (BK 32, the training step's large-M GEMMs, MDG_B4_STAGES): stages issued NS - 1
// steps ahead and a COUNTED vmcnt per step (the next stages' loads stay in flight across the
// barrier), as the 256x128 kernel below; LDS NS x 16 KiB.
template <int EPI, int BK, bool WIDE = false, int NS = 2>  // WIDE: the 16-B-store epilogue (epi_tile8)
__global__ __launch_bounds__(kB4Threads) void gemm_bf16_b4_kernel(const mdg_gemm_desc p) {
  constexpr int BM = kB4Tile, BN = kB4Tile, TILE = BM * BK, LDS_ST = BN + 4;
  constexpr int CPR = BK / 8;      // 16-B chunks per tile row
  constexpr int RPI = 64 / CPR;    // rows per glds wave-instruction (1 KiB)
  constexpr int NLD = 32 / RPI;    // glds per operand per wave (a wave fills 32 rows)
  static_assert(BK == 32 || BK == 64, "BK");
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, lg = lane >> 4;
  const int M = p.M, K = p.K;
  const int n_tiles = p.N / BN, m_tiles = (M + BM - 1) / BM, nwg = n_tiles * m_tiles;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + loc;
  const int mt = wg / n_tiles, nt = wg - mt * n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;

  // chunk swizzle of tile row r: 128-B rows (BK 64) pair up in a 256-B bank row -> c ^ ((r>>1)&7);
  // 64-B rows (BK 32) come four to a bank row -> c ^ ((-(r>>2))&3).  Both make the 16 fragment
  // rows of each ds_read_b128 lane group land on 16 distinct 16-B bank slots.
  auto swz_of = [](int r) { return BK == 64 ? ((r >> 1) & 7) : ((-(r >> 2)) & 3); };
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A);
  const bf16_t* W = reinterpret_cast<const bf16_t*>(p.W);
  const bf16_t* asrc[NLD];
  const bf16_t* bsrc[NLD];
#pragma unroll
  for (int i = 0; i < NLD; ++i) {
    const int row = 32 * wave + RPI * i + lane / CPR;
    const int ch = ((lane % CPR) ^ swz_of(row)) * 8;
    asrc[i] = A + (size_t)min(m0 + row, M - 1) * p.lda + ch;
    bsrc[i] = W + (size_t)(n0 + row) * p.ldw + ch;
  }

#define MDG_B4_LOAD(stage_, k0_)                                                                   \
  {                                                                                                \
    bf16_t* sa = lds + (stage_) * 2 * TILE + (32 * wave) * BK;                                     \
    _Pragma("unroll") for (int i = 0; i < NLD; ++i) {                                              \
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + (k0_)), (lds_ptr_t)(sa + RPI * i * BK), 16, 0, 0); \
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + (k0_)), (lds_ptr_t)(sa + TILE + RPI * i * BK), 16, 0, 0); \
    }                                                                                              \
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  const int swz = swz_of(lr);  // every fragment row this lane reads is lr mod 16
  MDG_B4_LOAD(0, 0);
  if constexpr (NS > 2) {
#pragma unroll
    for (int s0 = 1; s0 < NS - 1; ++s0)
      if (s0 < nk) MDG_B4_LOAD(s0, s0 * BK);
  }
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (NS == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (kt + 1 < nk) MDG_B4_LOAD(cur ^ 1, (kt + 1) * BK);
    } else {
      // stage kt landed for this wave: the loads of the (at most NS - 2) later stages already
      // issued stay outstanding (2 NLD per stage); then every wave's loads + every wave done
      // reading stage kt - 1 (lgkmcnt: its ds_reads retired), whose slot is refilled below
      const int ahead = min(NS - 2, nk - 1 - kt);
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * NLD) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NLD) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + NS - 1 < nk) {
        const int nb = (cur + NS - 1) % NS;
        MDG_B4_LOAD(nb, (kt + NS - 1) * BK);
      }
    }
    const bf16_t* As = lds + cur * 2 * TILE;
    const bf16_t* Bs = As + TILE;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      const int ch = (((kk >> 3) + lg) ^ swz) * 8;
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + lr) * BK + ch);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + j * 16 + lr) * BK + ch);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    cur = (NS == 2) ? (cur ^ 1) : (cur + 1 == NS ? 0 : cur + 1);
  }
#undef MDG_B4_LOAD

  // ------------------------------------------------------------------ epilogue
  // BK 64: the whole tile is staged at once (67.5 KiB, two blocks per CU);
  // BK 32: two 64-row bands (33.8 KiB of LDS in all, four blocks per CU).
  constexpr int BANDS = (BK == 64) ? 1 : 2, BROWS = BM / BANDS;
  float* stage = reinterpret_cast<float*>(smem);
  __syncthreads();  // every wave is done reading the last stage
#pragma unroll
  for (int band = 0; band < BANDS; ++band) {
    if (BANDS == 1 || wm == band) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stage[((BANDS == 1 ? wm * 64 : 0) + i * 16 + lg * 4 + r) * LDS_ST + wn * 64 + j * 16 + lr] = acc[i][j][r];
    }
    __syncthreads();
    if constexpr (WIDE && (EPI == MDG_EPI_STORE || EPI == MDG_EPI_QKV))
      epi_tile8<EPI, kB4Threads, BROWS>(p, stage, m0 + band * BROWS, n0, tid);
    else
      epi_tile<EPI, kB4Threads, BROWS>(p, stage, m0 + band * BROWS, n0, tid);
    if (band + 1 < BANDS) __syncthreads();
  }
}

template <int BK, int NS = 2>
__host__ __device__ constexpr size_t b4_smem() {
  // max(the operand ring, the fp32 epilogue image: the whole tile (BK 64) or a 64-row band)
  return BK == 64 ? (size_t)kB4Tile * (kB4Tile + 4) * 4
                  : (NS * 2 * kB4Tile * BK * 2 > (kB4Tile / 2) * (kB4Tile + 4) * 4
                         ? (size_t)NS * 2 * kB4Tile * BK * 2
                         : (size_t)(kB4Tile / 2) * (kB4Tile + 4) * 4);
}

template <int EPI, int BK, bool WIDE, int NS>
static hipError_t launch_b4_v(const mdg_gemm_desc& p, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_bf16_b4_kernel<EPI, BK, WIDE, NS>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)b4_smem<BK, NS>());
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int nwg = (p.N / kB4Tile) * ((p.M + kB4Tile - 1) / kB4Tile);
  constexpr size_t smem = b4_smem<BK, NS>();
  hipLaunchKernelGGL((gemm_bf16_b4_kernel<EPI, BK, WIDE, NS>), dim3(nwg), dim3(kB4Threads), smem, s, p);
  return hipGetLastError();
}

// operand ring depth of the K-step-32 kernel (MDG_B4_STAGES=2|3|4)
static int b4_stages() {
  static const int v = [] {
    const char* e = getenv("MDG_B4_STAGES");
    const int n = e ? atoi(e) : 2;
    return (n == 3 || n == 4) ? n : 2;
  }();
  return v;
}

template <int EPI, int BK, bool WIDE>
static hipError_t launch_b4_ns(const mdg_gemm_desc& p, hipStream_t s) {
  if constexpr (BK == 32) {
    const int ns = b4_stages();
    if (ns == 3) return launch_b4_v<EPI, BK, WIDE, 3>(p, s);
    if (ns == 4) return launch_b4_v<EPI, BK, WIDE, 4>(p, s);
  }
  return launch_b4_v<EPI, BK, WIDE, 2>(p, s);
}

// the 16-B-store epilogue where its alignment holds (MDG_WIDE_EPI=0: the 8-B one, A/B knob)
template <int EPI, int BK>
static hipError_t launch_b4(const mdg_gemm_desc& p, hipStream_t s) {
  static const bool knob = [] {
    const char* e = getenv("MDG_WIDE_EPI");
    return !(e && e[0] == '0');
  }();
  bool wide = false;
  if constexpr (EPI == MDG_EPI_STORE) wide = p.ldo % 8 == 0 && (!p.aux || p.ldaux % 8 == 0);
  if constexpr (EPI == MDG_EPI_QKV) wide = p.D % 8 == 0;
  if constexpr (EPI == MDG_EPI_STORE || EPI == MDG_EPI_QKV)
    if (wide && knob) return launch_b4_ns<EPI, BK, true>(p, s);
  return launch_b4_ns<EPI, BK, false>(p, s);
}

// ---------------------------------------------------------------------------------------
// Large-M variant: 256x128 block tile, 8 waves as 4x2 (64x64 wave tiles), K-step 64, a
// 3-stage global_load_lds ring with two stages in flight across the (raw) barriers: per
// K-step a wave waits with a COUNTED vmcnt for the stage it is about to read (leaving the
// next stage's 6 loads outstanding), passes the barrier, issues the stage two ahead into
// the buffer every wave finished reading one step earlier, then runs 32 MFMAs.  One block
// per CU (144 KiB of LDS); the 256-row tile halves the L2->LDS bytes per FLOP of 128x128.
constexpr int kB8Threads = 512;
constexpr int kB8M = 256;
constexpr size_t kB8Smem = 3ull * (kB8M + 128) * 64 * 2;  // 147456 B (the fp32 epilogue image, 135168 B, fits)

template <int EPI>
__global__ __launch_bounds__(kB8Threads) void gemm_bf16_b8_kernel(const mdg_gemm_desc p) {
  constexpr int BM = kB8M, BN = 128, BK = 64, ATILE = BM * BK, STAGE = (BM + BN) * BK, LDS_ST = BN + 4;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, lg = lane >> 4;
  const int M = p.M, K = p.K;
  const int n_tiles = p.N / BN, m_tiles = (M + BM - 1) / BM, nwg = n_tiles * m_tiles;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + loc;
  const int mt = wg / n_tiles, nt = wg - mt * n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;

  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A);
  const bf16_t* W = reinterpret_cast<const bf16_t*>(p.W);
  // A: 4 wave-instructions (rows 32*wave + 8i + lane/8); B: 2 (rows 16*wave + 8i + lane/8)
  const bf16_t* asrc[4];
  const bf16_t* bsrc[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 32 * wave + 8 * i + (lane >> 3);
    asrc[i] = A + (size_t)min(m0 + row, M - 1) * p.lda + ((lane & 7) ^ ((row >> 1) & 7)) * 8;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * wave + 8 * i + (lane >> 3);
    bsrc[i] = W + (size_t)(n0 + row) * p.ldw + ((lane & 7) ^ ((row >> 1) & 7)) * 8;
  }

#define MDG_B8_LOAD(stage_, k0_)                                                                   \
  {                                                                                                \
    bf16_t* sa = lds + (stage_) * STAGE;                                                           \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                  \
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + (k0_)),                             \
                                       (lds_ptr_t)(sa + (32 * wave + 8 * i) * BK), 16, 0, 0);       \
    _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                  \
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + (k0_)),                             \
                                       (lds_ptr_t)(sa + ATILE + (16 * wave + 8 * i) * BK), 16, 0, 0); \
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  MDG_B8_LOAD(0, 0);
  if (nk > 1) MDG_B8_LOAD(1, BK);
  const int swz = (lr >> 1) & 7;
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed (this wave's loads) -> barrier (every wave's loads, and every wave
    // finished reading stage kt-1, whose buffer the loads below overwrite)
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring reads retired (see kRingWaitNote)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + 2 < nk) {
      const int nb = (cur == 0) ? 2 : cur - 1;  // (kt + 2) % 3
      MDG_B8_LOAD(nb, (kt + 2) * BK);
    }
    const bf16_t* As = lds + cur * STAGE;
    const bf16_t* Bs = As + ATILE;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      const int ch = (((kk >> 3) + lg) ^ swz) * 8;
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + lr) * BK + ch);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + j * 16 + lr) * BK + ch);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    cur = (cur == 2) ? 0 : cur + 1;
  }
#undef MDG_B8_LOAD

  __syncthreads();
  float* stage = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        stage[(wm * 64 + i * 16 + lg * 4 + r) * LDS_ST + wn * 64 + j * 16 + lr] = acc[i][j][r];
  __syncthreads();
  epi_tile<EPI, kB8Threads, BM>(p, stage, m0, n0, tid);
}

template <int EPI>
static hipError_t launch_b8(const mdg_gemm_desc& p, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_bf16_b8_kernel<EPI>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kB8Smem);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int nwg = (p.N / 128) * ((p.M + kB8M - 1) / kB8M);
  hipLaunchKernelGGL((gemm_bf16_b8_kernel<EPI>), dim3(nwg), dim3(kB8Threads), kB8Smem, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Full-row gated residual + LayerNorm: out_proj / fc2 whose epilogue also produces the next
// projection's normalised, modulated bf16 input, so the stand-alone LN pass (and its 49 MB
// re-read of h) disappears.  Block = 128 rows x all NCOL output columns (the whole row is in
// the block, so the LN statistics are exact), 8 waves as 2 x 4 with 64 x NCOL/4 wave tiles,
// K-step 32, a 4-stage global_load_lds ring with counted vmcnt (one block per CU: the ring
// depth, not a second block, hides the load latency).  Epilogue in four 32-row bands: the
// accumulators are staged in LDS, then each wave owns 4 rows: gather h and gate of its rows,
// h += gate * (acc + bias) (stored), two wave reductions, xn = LN(h)*(1+scale)+shift (bf16).
constexpr int kRowThreads = 512;

// BM 128: 8 waves as 2 x 4, 4-stage ring, one block per CU.  BM 64 (row tiles of 64, twice
// the blocks): 8 waves as 1 x 8, 2-stage ring, two blocks per CU, so one block's HBM-bound
// epilogue (h read/write, xn write) overlaps the other's MFMA main loop.
template <int BM> struct RowCfg;
template <> struct RowCfg<128> { static constexpr int WMW = 2, STAGES = 4; };
template <> struct RowCfg<64> { static constexpr int WMW = 1, STAGES = 2; };
// 32-row tiles (round 5): a lone chain's out_proj (B = 1 window: 125 tiles instead of 32, no
// split-K partials or reduction pass); every wave 32 rows x 48 columns
template <> struct RowCfg<32> { static constexpr int WMW = 1, STAGES = 2; };
// 16-row tiles: a lone chain's out_proj on 250 tiles (B = 1: M = 4 000) instead of 125 on 256 CUs;
// every wave 16 rows x 48 columns, epilogue bands of 16 rows (2 per wave)
template <> struct RowCfg<16> { static constexpr int WMW = 1, STAGES = 2; };

template <int NCOL, int BM>
__host__ __device__ constexpr size_t rowln_smem() {
  return (size_t)RowCfg<BM>::STAGES * (BM + NCOL) * 32 * 2;
}

// The row-LN fast epilogue (BM 128, 8 waves as 2 x 4, the tile spans <= 2 adaLN entries):
// shared by gemm_rowln_kernel and the fused MLP kernel.  acc = the waves' 64 x NCOL/4
// accumulator tiles; h4 = band 0's residual rows (rowln_load_band), already in flight.
// Token row of a row-LN tile's local row r (0 .. 127).  RowsLinear: rows m0 .. m0 + 127 (every
// kernel but one).  RowsFrames: 8 consecutive frames x 16 consecutive residues, r = 16 f + l
// (the fused out_proj + q|k|v for the long residue axis, L % 16 == 0: each (residue, head)
// plane then receives 8 consecutive 48-B rows from one block instead of one row from each of 8
// blocks); rows of frames past the last map to M (invalid: loads clamp, stores skip).
struct RowsLinear {
  int m0;
  __device__ int operator()(int r) const { return m0 + r; }
};
struct RowsFrames {
  int f0, l0, L, nf, M;
  __device__ int operator()(int r) const {
    const int f = f0 + (r >> 4);
    return f < nf ? f * L + l0 + (r & 15) : M;
  }
};

// TRAIN: the residual is read from resid_in (the training forward keeps the sublayer input for
// the backward), the pre-gate value and the LN row statistics are stored (rowln_fast_epilogue_impl)
template <int NCOL, typename RM, bool TRAIN = false>
__device__ __forceinline__ void rowln_load_band(const mdg_gemm_desc& p, RM rows, int u, float4 (&h4)[2][NCOL / 128]) {
  constexpr int NE = NCOL / 128;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, hl = lane & 31;
  const float* src = TRAIN ? p.resid_in : p.resid;
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) {
    const int m = min(rows(u * 32 + wave * 4 + 2 * pr + half), p.M - 1);
    const float* hr = src + (size_t)m * p.ldr + 4 * hl;
#pragma unroll
    for (int e = 0; e < NE; ++e) h4[pr][e] = *reinterpret_cast<const float4*>(hr + 128 * e);
  }
}

// xlds: write the normalised rows (xn) not to p.xn_out but into LDS, as K-slice images of 32
// columns ([NCOL / 32][BM][32] bf16, 16-B chunk c of row r at c ^ ((-(r >> 2)) & 3)): the
// A operand of a following GEMM in the same block.
// stage_band(band, stage) writes the block's fp32 accumulator rows [32 band, 32 band + 32)
// into stage (row stride LDS_ST floats); the kernels differ only in where their accumulators live.
// NREG stage regions: band b is read from region b % NREG, so a caller with NREG = 3 may write
// bands 0-2 at once (at band 0's call; band 3 at its own) and free their registers early.
// LATE_H: h4 is not loaded yet; band 0's residual rows are read right after band 0's staging (a
// caller whose accumulators fill the registers until then).
template <int NCOL, int NREG = 1, bool LATE_H = false, typename StageBand, typename RM = RowsLinear, bool TRAIN = false>
__device__ __forceinline__ void rowln_fast_epilogue_impl(const mdg_gemm_desc& p, StageBand stage_band,
                                                         float4 (&h4)[2][NCOL / 128], unsigned char* smem, RM rows,
                                                         int b_lo, float inv_rpm, bf16_t* xlds = nullptr) {
  // no fp contraction: every kernel that inlines this epilogue (the row-LN GEMM, the fused MLP,
  // the fused out_proj + q|k|v) rounds h and xn identically
#pragma clang fp contract(off)
  constexpr int BM = 128, LDS_ST = NCOL + 4, NE = NCOL / 128;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, hl = lane & 31;
  const int M = p.M;
  const int b_hi = fdiv(min(rows(BM - 1), M - 1), p.rows_per_mod, inv_rpm);
  float* stage = reinterpret_cast<float*>(smem);
  const float invN = 1.0f / (float)NCOL;
  auto load_unit4 = [&](int u, float4 (&hb)[2][NE]) { rowln_load_band<NCOL, RM, TRAIN>(p, rows, u, hb); };
  float* emods = stage + NREG * 32 * LDS_ST;  // [2][3][NCOL]: gate | xn scale | xn shift
  // the caller's smem holds (32 * LDS_ST + 6 * NCOL) floats: the band stage + the adaLN rows
  static_assert(LDS_ST % 4 == 0, "16-B aligned stage rows");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last K-step's ring reads (kRingWaitNote)
  __builtin_amdgcn_s_barrier();  // every wave is done reading the ring (its loads were all waited)
  for (int i = tid; i < 6 * NCOL; i += kRowThreads) {
    const int eb = i / (3 * NCOL), w = (i / NCOL) % 3, k = i % NCOL;
    const size_t b = (size_t)min(b_lo + eb, b_hi);
    float v;
    if (w == 0) v = p.gate ? p.gate[b * p.mod_stride + p.gate_off + k] : 1.0f;
    else if (w == 1) v = p.xn_out ? p.xn_mods[b * p.xn_mod_stride + p.xn_scale_off + k] : 0.0f;
    else v = p.xn_out ? p.xn_mods[b * p.xn_mod_stride + p.xn_shift_off + k] : 0.0f;
    emods[i] = v;
  }
  float4 b4[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e)
    b4[e] = p.bias ? *reinterpret_cast<const float4*>(p.bias + 4 * hl + 128 * e) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  // unrolled: a rolled band loop made the next band's prefetch conditional, and on the merged
  // path the compiler drained it with s_waitcnt vmcnt(0) before the current band's first use
  for (int band = 0; band < BM / 32; ++band) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // previous band's stage reads (and the adaLN rows) are done
    stage_band(band, stage);
    if (LATE_H && band == 0) rowln_load_band<NCOL, RM, TRAIN>(p, rows, 0, h4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const float* bstage = stage + (band % NREG) * 32 * LDS_ST;
    __builtin_amdgcn_s_barrier();
    float4 hn[2][NE];
    if (band + 1 < BM / 32) load_unit4(band + 1, hn);
    float sum[2];
    int eb[2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int m = rows(band * 32 + wave * 4 + 2 * pr + half);
      eb[pr] = fdiv(min(m, M - 1), p.rows_per_mod, inv_rpm) - b_lo;
      const float* srow = bstage + (wave * 4 + 2 * pr + half) * LDS_ST + 4 * hl;
      const float* gr = emods + eb[pr] * 3 * NCOL + 4 * hl;
      float sacc = 0.f;
      const int mrow = rows(band * 32 + wave * 4 + 2 * pr + half);
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const float4 v = *reinterpret_cast<const float4*>(srow + 128 * e);
        const float4 g = *reinterpret_cast<const float4*>(gr + 128 * e);
        if (TRAIN && mrow < M)  // the pre-gate out_proj / fc2 output, saved for the gate's backward
          st4<bf16_t>(reinterpret_cast<bf16_t*>(p.aux) + (size_t)mrow * p.ldaux + 4 * hl + 128 * e, v.x + b4[e].x,
                      v.y + b4[e].y, v.z + b4[e].z, v.w + b4[e].w);
        float4& h = h4[pr][e];
        h.x += g.x * (v.x + b4[e].x);
        h.y += g.y * (v.y + b4[e].y);
        h.z += g.z * (v.z + b4[e].z);
        h.w += g.w * (v.w + b4[e].w);
        sacc += (h.x + h.y) + (h.z + h.w);
      }
      sum[pr] = sacc;
      if (m < M) {
        float* hr = p.resid + (size_t)m * p.ldr + 4 * hl;
#pragma unroll
        for (int e = 0; e < NE; ++e) *reinterpret_cast<float4*>(hr + 128 * e) = h4[pr][e];
      }
    }
    if (p.xn_out) {
      // row sums over each half-wave (32 lanes)
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) sum[pr] += __shfl_xor(sum[pr], o, 64);
      float ss[2];
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        sum[pr] *= invN;  // mean
        float t = 0.f;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const float4 h = h4[pr][e];
          const float a0 = h.x - sum[pr], a1 = h.y - sum[pr], a2 = h.z - sum[pr], a3 = h.w - sum[pr];
          t += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
        }
        ss[pr] = t;
      }
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) ss[pr] += __shfl_xor(ss[pr], o, 64);
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int rl = band * 32 + wave * 4 + 2 * pr + half, m = rows(rl);
        const float rs = 1.0f / sqrtf(ss[pr] * invN + p.ln_eps);
        if (TRAIN && hl == 0 && m < M)  // (mean, rstd) for the LN backward (ln_mod's stats layout)
          *reinterpret_cast<float2*>(p.ln_stats + 2 * (size_t)m) = make_float2(sum[pr], rs);
        const float* mr = emods + eb[pr] * 3 * NCOL + 4 * hl;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const float4 xs = *reinterpret_cast<const float4*>(mr + NCOL + 128 * e);
          const float4 xh = *reinterpret_cast<const float4*>(mr + 2 * NCOL + 128 * e);
          const float4 h = h4[pr][e];
          const float o0 = (h.x - sum[pr]) * rs * (1.0f + xs.x) + xh.x, o1 = (h.y - sum[pr]) * rs * (1.0f + xs.y) + xh.y;
          const float o2 = (h.z - sum[pr]) * rs * (1.0f + xs.z) + xh.z, o3 = (h.w - sum[pr]) * rs * (1.0f + xs.w) + xh.w;
          if (xlds) {
            const int r = rl, col = 4 * hl + 128 * e, cw = col & 31;
            st4<bf16_t>(xlds + (col >> 5) * (BM * 32) + r * 32 + (((cw >> 3) ^ ((-(r >> 2)) & 3)) * 8) + (cw & 7), o0, o1,
                        o2, o3);
          } else if (m < M) {
            st4<bf16_t>(reinterpret_cast<bf16_t*>(p.xn_out) + (size_t)m * NCOL + 4 * hl + 128 * e, o0, o1, o2, o3);
          }
        }
      }
    }
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int e = 0; e < NE; ++e) h4[pr][e] = hn[pr][e];
  }
}

// The 8-wave (2 x 4) accumulator layout of the row-LN GEMM / fused MLP / fused out_proj + qkv:
// wave (wm, wn) holds rows wm * 64 + 16 i + 4 lg + r, columns wn * NCOL / 4 + 16 j + lr.
template <int NCOL, typename RM = RowsLinear, bool TRAIN = false>
__device__ __forceinline__ void rowln_fast_epilogue(const mdg_gemm_desc& p, f32x4 (&acc)[4][NCOL / 64],
                                                    float4 (&h4)[2][NCOL / 128], unsigned char* smem, RM rows,
                                                    int b_lo, float inv_rpm, bf16_t* xlds = nullptr) {
  constexpr int WTN = NCOL / 4, NT = WTN / 16, LDS_ST = NCOL + 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave / 4, wn = wave % 4;
  const int lr = lane & 15, lg = lane >> 4;
  auto stage_band = [&](int band, float* stage) {
    if (wm == (band >> 1)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if ((i >> 1) != (band & 1)) continue;
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stage[((i & 1) * 16 + lg * 4 + r) * LDS_ST + wn * WTN + j * 16 + lr] = acc[i][j][r];
      }
    }
  };
  rowln_fast_epilogue_impl<NCOL, 1, false, decltype(stage_band), RM, TRAIN>(p, stage_band, h4, smem, rows, b_lo, inv_rpm,
                                                                            xlds);
}

// PART: split-K form for small M — block (tile, y) runs K-steps [y nk, (y + 1) nk) and writes its
// fp32 partial tile to (float*)p.aux + y * M * NCOL; mlp_split_reduce_kernel finishes the rows
// TRAIN (BM 128, every tile on the fast epilogue: rows_per_mod >= 128): the training forward's
// out_proj / fc2 — residual read from resid_in, out of place; pre-gate value to aux; LN stats
template <int NCOL, int BM, bool PART = false, bool TRAIN = false>
__global__ __launch_bounds__(kRowThreads, BM <= 64 ? 4 : 1) void gemm_rowln_kernel(const mdg_gemm_desc p) {
  constexpr int kRowStages = RowCfg<BM>::STAGES, WMW = RowCfg<BM>::WMW, WNW = 8 / WMW;
  constexpr int MI = BM >= 64 ? 4 : BM / 16;  // 16-row fragment tiles per wave
  constexpr int BK = 32, WTN = NCOL / WNW, NT = WTN / 16, ATILE = BM * BK, STAGE = (BM + NCOL) * BK;
  constexpr int LDS_ST = NCOL + 4, NE = NCOL / 128;  // float2 column pairs per lane per row
  constexpr int WLD = NCOL / 128;                    // W glds instructions per wave per stage
  constexpr int ALD_WAVES = BM / 16;                 // waves that stage A (one 16-row glds each)
  // epilogue bands of BH rows, RPW per wave; RG of them processed together
  constexpr int BH = BM >= 32 ? 32 : 16, RPW = BH / 8;
  constexpr int RG = ((BM == 64 && NCOL > 256) || BM < 32) ? 2 : 4;
  static_assert(NCOL % 128 == 0 && NCOL <= 512 && WTN % 16 == 0, "NCOL");
  static_assert(32 * LDS_ST * 4 <= kRowStages * STAGE * 2, "band stage fits the ring");
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WNW, wn = wave % WNW;
  const bool has_a = wave < ALD_WAVES;
  const int lr = lane & 15, lg = lane >> 4;
  const int M = p.M, K = p.K;
  // XCD-aware order of the row tiles (neighbouring tiles share nothing but W, which every
  // XCD's L2 holds anyway; the remap keeps consecutive tiles on one XCD for the h / gate rows)
  const int nwg = (M + BM - 1) / BM;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q = nwg >> 3, r8 = nwg & 7;
  const int m0 = ((xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + loc) * BM;

  // 64-B tile rows: chunk c of row r at c ^ ((-(r >> 2)) & 3)
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A);
  const bf16_t* W = reinterpret_cast<const bf16_t*>(p.W);
  const int arow = 16 * wave + (lane >> 2);
  const bf16_t* asrc = A + (size_t)min(m0 + arow, M - 1) * p.lda + (((lane & 3) ^ ((-(arow >> 2)) & 3)) * 8);
  const bf16_t* bsrc[WLD];
#pragma unroll
  for (int i = 0; i < WLD; ++i) {
    const int row = 16 * (wave * WLD + i) + (lane >> 2);
    bsrc[i] = W + (size_t)row * p.ldw + (((lane & 3) ^ ((-(row >> 2)) & 3)) * 8);
  }
#define MDG_ROW_LOAD(stage_, k0_)                                                                   \
  {                                                                                                 \
    bf16_t* sa = lds + (stage_) * STAGE;                                                            \
    if (has_a)                                                                                      \
      __builtin_amdgcn_global_load_lds((const void*)(asrc + (k0_)), (lds_ptr_t)(sa + 16 * wave * BK), 16, 0, 0); \
    _Pragma("unroll") for (int i = 0; i < WLD; ++i)                                                 \
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + (k0_)),                              \
                                       (lds_ptr_t)(sa + ATILE + 16 * (wave * WLD + i) * BK), 16, 0, 0); \
  }

  // Epilogue work unit u = (band u / UPB, row group u % UPB): RG rows of this wave.  Their h and
  // gate rows are loaded one unit AHEAD of use (unit 0 before the main loop, so its HBM
  // latency hides under the K loop; unit u+1 while unit u computes), so the epilogue pays the
  // residual-read latency once instead of once per band.
  constexpr int UPB = RPW / RG, NU = (BM / BH) * UPB;
  const float inv_rpm = 1.0f / (float)p.rows_per_mod;
  // the gate row is per trajectory: one row of it per unit (the unit's first row's entry; a
  // row of another entry, in a unit straddling a trajectory boundary, reloads its own)
  auto load_unit = [&](int u, float2 (&hv)[RG][NE], float2 (&gv)[NE]) {
    const int mu = min(m0 + (u / UPB) * BH + wave * RPW + (u % UPB) * RG, M - 1);
    const float* gr = p.gate ? p.gate + (size_t)fdiv(mu, p.rows_per_mod, inv_rpm) * p.mod_stride + p.gate_off : nullptr;
#pragma unroll
    for (int e = 0; e < NE; ++e)
      gv[e] = gr ? *reinterpret_cast<const float2*>(gr + 2 * lane + 128 * e) : make_float2(1.f, 1.f);
#pragma unroll
    for (int rr = 0; rr < RG; ++rr) {
      const int m = min(mu + rr, M - 1);
      const float* hr = p.resid + (size_t)m * p.ldr;
#pragma unroll
      for (int e = 0; e < NE; ++e) hv[rr][e] = *reinterpret_cast<const float2*>(hr + 2 * lane + 128 * e);
    }
  };
  // Fast epilogue (BM 128, the tile spans <= 2 trajectory entries -- every tile when
  // rows_per_mod >= 128): the adaLN rows go to LDS once and each wave processes its rows as
  // PAIRS, one row per half-wave, 4 consecutive columns per lane, so every h load / store is a
  // 16-B-per-lane access (1 KiB per wave instruction) and every xn store 8 B per lane: half the
  // memory instructions of the float2 layout.  Unit u = (band u, the wave's 4 rows as 2 pairs).
  int b_lo = 0, b_hi = 1 << 30;
  if (BM == 128) {
    b_lo = fdiv(m0, p.rows_per_mod, inv_rpm);
    b_hi = fdiv(min(m0 + BM - 1, M - 1), p.rows_per_mod, inv_rpm);
  }
  const bool fast = BM == 128 && b_hi - b_lo < 2;
  float4 h4[2][NE];
  float2 hv[RG][NE], gv[NE];
  if (!PART) {
    if (fast) rowln_load_band<NCOL, RowsLinear, TRAIN>(p, RowsLinear{m0}, 0, h4);
    else if (BM <= 64) load_unit(0, hv, gv);
  }

  f32x4 acc[MI][NT];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (PART ? K / (int)gridDim.y : K) / BK, kbeg = PART ? (int)blockIdx.y * nk * BK : 0;
  // 32-row tiles (a lone chain's small-M launch, W-stream bound: 24 KiB of W per 2 KiB of A per
  // step): the pieces go global -> VGPRs -> ds_write_b128 into the same LDS image, the next
  // step's loaded under this step's MFMAs (plain loads fill ~3x faster than LDS-DMA per CU,
  // tools/ubench/l2lds.hip)
  constexpr bool VST = BM <= 32;
  u32x4 vr[1 + WLD];
  auto vload = [&](int k0) {
    if (has_a) vr[0] = *reinterpret_cast<const u32x4*>(asrc + k0);
#pragma unroll
    for (int i = 0; i < WLD; ++i) vr[1 + i] = *reinterpret_cast<const u32x4*>(bsrc[i] + k0);
  };
  auto vstore = [&](int st) {
    bf16_t* sa = lds + st * STAGE;
    if (has_a) *reinterpret_cast<u32x4*>(sa + 16 * wave * BK + 8 * lane) = vr[0];
#pragma unroll
    for (int i = 0; i < WLD; ++i) *reinterpret_cast<u32x4*>(sa + ATILE + 16 * (wave * WLD + i) * BK + 8 * lane) = vr[1 + i];
  };
  if constexpr (VST) {
    vload(kbeg);
    vstore(0);
  } else {
#pragma unroll
    for (int s0 = 0; s0 < kRowStages - 1; ++s0)
      if (s0 < nk) MDG_ROW_LOAD(s0, kbeg + s0 * BK);
  }
  const int swz = (-(lr >> 2)) & 3;
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (VST) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this stage's writes, the last stage's reads
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + 1 < nk) vload(kbeg + (kt + 1) * BK);
    } else {
    // stage kt landed: leave the (up to 2) younger stages' loads in flight
    const int younger = min(kRowStages - 2, nk - 1 - kt);
    if (has_a) {
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (1 + WLD)) : "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 + WLD) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * WLD) : "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WLD) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring reads retired (see kRingWaitNote)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + kRowStages - 1 < nk) MDG_ROW_LOAD((kt + kRowStages - 1) % kRowStages, kbeg + (kt + kRowStages - 1) * BK);
    }
    const bf16_t* As = lds + (kt % kRowStages) * STAGE;
    const bf16_t* Bs = As + ATILE;
    const int ch = (lg ^ swz) * 8;
    bf16x8 a[MI], b[NT];
#pragma unroll
    for (int i = 0; i < MI; ++i) a[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + lr) * BK + ch);
#pragma unroll
    for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * WTN + j * 16 + lr) * BK + ch);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    if constexpr (VST)
      if (kt + 1 < nk) vstore((kt + 1) % kRowStages);
  }
#undef MDG_ROW_LOAD

  if constexpr (PART) {
    static_assert(BM == 128 && MI == 4, "split-K form: 128-row tiles");
    float* pp = reinterpret_cast<float*>(p.aux) + (size_t)blockIdx.y * M * NCOL;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + lg * 4 + r;
        if (m < M)
#pragma unroll
          for (int j = 0; j < NT; ++j) pp[(size_t)m * NCOL + wn * WTN + j * 16 + lr] = acc[i][j][r];
      }
    return;
  }

  // ------------------------------------------------------------------ epilogue
  float* stage = reinterpret_cast<float*>(smem);
  const float invN = 1.0f / (float)NCOL;
  float2 bb[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e)
    bb[e] = p.bias ? *reinterpret_cast<const float2*>(p.bias + 2 * lane + 128 * e) : make_float2(0.f, 0.f);
  // The adaLN rows the epilogue needs (gate; the next LayerNorm's scale and shift) of the <= 2
  // trajectory entries a 128-row tile spans go to LDS once, and the per-row loop reads them
  // with ds_read.  (Per-row global loads in exec-masked branches -- the rare row of the next
  // trajectory -- made the compiler drain every outstanding store and prefetch with
  // s_waitcnt vmcnt(0) on every row.)  The band barriers are raw s_barrier after an LDS wait:
  // they order the stage buffer only, so the h / xn stores stay in flight across them.
  if constexpr (BM == 128) {
    static_assert((32 * LDS_ST + 6 * NCOL) * 4 <= kRowStages * STAGE * 2, "adaLN rows fit the ring");
    if (fast) {
      rowln_fast_epilogue<NCOL, RowsLinear, TRAIN>(p, acc, h4, smem, RowsLinear{m0}, b_lo, inv_rpm);
      return;
    }
  }
  if constexpr (TRAIN) return;  // (unreachable: the host takes this route only when every tile is fast)
  if (BM == 128) load_unit(0, hv, gv);  // the rare tile over > 2 entries: no prefetch under the K loop
  __syncthreads();  // all waves are done with the ring
#pragma unroll 1
  for (int band = 0; band < BM / BH; ++band) {
    if (wm == (band >> 1)) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {  // compile-time acc index; the band selects 2 of the 4
        if ((i >> 1) != (band & 1)) continue;
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stage[((i & 1) * 16 + lg * 4 + r) * LDS_ST + wn * WTN + j * 16 + lr] = acc[i][j][r];
      }
    }
    __syncthreads();
    // wave -> rows 4*wave .. 4*wave+3 of the band; every global operand of the 4 rows is
    // gathered before use and the 4 rows' reductions run interleaved (independent chains)
    // rows of this wave in groups of RG (fewer live registers at BM 64, two blocks per CU)
#pragma unroll 1
    for (int g0 = 0; g0 < RPW; g0 += RG) {
      const int u = band * UPB + g0 / RG;
      float2 hn[RG][NE], gn[NE];
      if (u + 1 < NU) load_unit(u + 1, hn, gn);
      const int mb0 = min(m0 + band * BH + wave * RPW + g0, M - 1), mb3 = min(mb0 + RG - 1, M - 1);
      const int b0 = fdiv(mb0, p.rows_per_mod, inv_rpm);
      const bool one_b = fdiv(mb3, p.rows_per_mod, inv_rpm) == b0;  // the 4 rows share a batch entry
      float2 xs[NE], xh[NE];
      if (p.xn_out) {
        const float* mr = p.xn_mods + (size_t)b0 * p.xn_mod_stride;
  #pragma unroll
        for (int e = 0; e < NE; ++e) {
          const int k = 2 * lane + 128 * e;
          xs[e] = *reinterpret_cast<const float2*>(mr + p.xn_scale_off + k);
          xh[e] = *reinterpret_cast<const float2*>(mr + p.xn_shift_off + k);
        }
      }
      float sum[RG];
  #pragma unroll
      for (int rr = 0; rr < RG; ++rr) {
        const float* srow = stage + (wave * RPW + g0 + rr) * LDS_ST;
        float2 g2[NE];
  #pragma unroll
        for (int e = 0; e < NE; ++e) g2[e] = gv[e];
        if (!one_b && p.gate) {  // rare: this row belongs to the next trajectory
          const int br = fdiv(min(m0 + band * BH + wave * RPW + g0 + rr, M - 1), p.rows_per_mod, inv_rpm);
          if (br != b0) {
            const float* gr = p.gate + (size_t)br * p.mod_stride + p.gate_off;
  #pragma unroll
            for (int e = 0; e < NE; ++e) g2[e] = *reinterpret_cast<const float2*>(gr + 2 * lane + 128 * e);
          }
        }
        float s = 0.f;
  #pragma unroll
        for (int e = 0; e < NE; ++e) {
          const float2 v = *reinterpret_cast<const float2*>(srow + 2 * lane + 128 * e);
          hv[rr][e].x += g2[e].x * (v.x + bb[e].x);
          hv[rr][e].y += g2[e].y * (v.y + bb[e].y);
          s += hv[rr][e].x + hv[rr][e].y;
        }
        sum[rr] = s;
        const int m = m0 + band * BH + wave * RPW + g0 + rr;
        if (m < M) {
  #pragma unroll
          for (int e = 0; e < NE; ++e) *reinterpret_cast<float2*>(p.resid + (size_t)m * p.ldr + 2 * lane + 128 * e) = hv[rr][e];
        }
      }
      if (p.xn_out) {
  #pragma unroll
        for (int o = 32; o >= 1; o >>= 1)
  #pragma unroll
          for (int rr = 0; rr < RG; ++rr) sum[rr] += __shfl_xor(sum[rr], o, 64);
        float ss[RG];
  #pragma unroll
        for (int rr = 0; rr < RG; ++rr) {
          sum[rr] *= invN;  // mean
          float t = 0.f;
  #pragma unroll
          for (int e = 0; e < NE; ++e) {
            const float a0 = hv[rr][e].x - sum[rr], a1 = hv[rr][e].y - sum[rr];
            t += a0 * a0 + a1 * a1;
          }
          ss[rr] = t;
        }
  #pragma unroll
        for (int o = 32; o >= 1; o >>= 1)
  #pragma unroll
          for (int rr = 0; rr < RG; ++rr) ss[rr] += __shfl_xor(ss[rr], o, 64);
  #pragma unroll
        for (int rr = 0; rr < RG; ++rr) {
          const int m = m0 + band * BH + wave * RPW + g0 + rr;
          if (m >= M) continue;
          const float rs = 1.0f / sqrtf(ss[rr] * invN + p.ln_eps);
          if (!one_b) {  // rows straddle a batch boundary: this row's own shift / scale
            const float* mr = p.xn_mods + (size_t)fdiv(m, p.rows_per_mod, inv_rpm) * p.xn_mod_stride;
  #pragma unroll
            for (int e = 0; e < NE; ++e) {
              const int k = 2 * lane + 128 * e;
              xs[e] = *reinterpret_cast<const float2*>(mr + p.xn_scale_off + k);
              xh[e] = *reinterpret_cast<const float2*>(mr + p.xn_shift_off + k);
            }
          }
  #pragma unroll
          for (int e = 0; e < NE; ++e) {
            const int k = 2 * lane + 128 * e;
            typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
            bf16x2 pr;
            pr[0] = (bf16_t)((hv[rr][e].x - sum[rr]) * rs * (1.0f + xs[e].x) + xh[e].x);
            pr[1] = (bf16_t)((hv[rr][e].y - sum[rr]) * rs * (1.0f + xs[e].y) + xh[e].y);
            *reinterpret_cast<bf16x2*>(reinterpret_cast<bf16_t*>(p.xn_out) + (size_t)m * NCOL + k) = pr;
          }
        }
      }
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        gv[e] = gn[e];
#pragma unroll
        for (int rr = 0; rr < RG; ++rr) hv[rr][e] = hn[rr][e];
      }
    }
    __syncthreads();
  }
}

template <int NCOL, int BM>
static hipError_t launch_rowln(const mdg_gemm_desc& p, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_rowln_kernel<NCOL, BM>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)rowln_smem<NCOL, BM>());
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_rowln_kernel<NCOL, BM>), dim3((p.M + BM - 1) / BM), dim3(kRowThreads),
                     (rowln_smem<NCOL, BM>()), s, p);
  return hipGetLastError();
}

// the 32-row tile form for a lone chain's small-M out_proj (mdg_denoise_step, chain_alone):
// the fast path's envelope without its tile-height requirement (the general epilogue handles
// tiles over any number of adaLN entries)
bool rowln_bm32_supported(const mdg_gemm_desc& r) {
  return r.dtype == MDG_BF16 && r.a_mode == MDG_A_PLAIN && r.epi == MDG_EPI_GATE_RES && r.N == 384 && r.K % 32 == 0 &&
         r.K > 0 && r.M > 0 && r.resid && !r.resid_in && !r.aux && r.lda % 8 == 0 && r.ldw % 8 == 0 && r.ldr % 2 == 0 &&
         (!r.xn_out || r.xn_mods);
}

// MDG_ROWLN_BM: the small-M row-LN tile height (16 default: 250 tiles at B = 1, 1.846 / 1.823 vs
// 1.813 / 1.816 M frames/s with 32, same box; 32 restores the 125-tile form)
static int rowln_small_bm() {
  static const int v = [] {
    const char* e = getenv("MDG_ROWLN_BM");
    return (e && atoi(e) == 32) ? 32 : 16;
  }();
  return v;
}
hipError_t rowln_bm32_launch(const mdg_gemm_desc& p, hipStream_t s) {
  return rowln_small_bm() == 16 ? launch_rowln<384, 16>(p, s) : launch_rowln<384, 32>(p, s);
}

static hipError_t launch_rowln_train(const mdg_gemm_desc& p, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_rowln_kernel<384, 128, false, true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)rowln_smem<384, 128>());
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_rowln_kernel<384, 128, false, true>), dim3((p.M + 127) / 128), dim3(kRowThreads),
                     (rowln_smem<384, 128>()), s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Fused MLP (latent_model.py:488-491): x += gate_m * fc2(gelu(fc1(xn))) and the next LN, the
// hidden activation never leaving the CU.  Block = 128 token rows (one block per CU, 8 waves),
// the hidden dimension in chunks of 128: per chunk 6 fc1 K-steps of 64 (Hc^T = W1c . xn^T,
// 64 hidden x 32 tokens per wave, acc1) -> bias + GELU -> bf16 chunk Hc [128 tokens][128] in
// LDS -> 4 fc2 K-steps of 32 (acc2 += Hc . W2c^T, 64 tokens x 96 outputs per wave, the row-LN
// layout) -> after the last chunk the row-LN epilogue.  Every K-step's operand slice (xn +
// W1c rows as two 32-wide images, or W2 rows) streams through one 3-slot global_load_lds ring
// with counted vmcnt (4 or 3 pieces per wave per step, one barrier per step).  The fc1 product
// is computed transposed so a lane's accumulator holds 4 consecutive hidden units of one
// token: one 8-B LDS write per 4 GELU outputs.  The K order of both products is the unfused
// GEMMs' (ascending in 32s), so the result equals fc1 then fc2 bit for bit.
struct MlpArgs {
  mdg_gemm_desc f1, f2;
  float* part;  // split form: [nsplit][M][NCOL] fp32 fc2 partials (no epilogue in the kernel)
  int nsplit;   // hidden chunks are divided over gridDim.y = nsplit blocks per row tile
  mdg_gemm_desc r;  // PRE form: the temporal out_proj row-LN GEMM run first (r.xn_out = f1.A)
};
// timing diagnostics only (tools/diag_mlp_attn.sh builds them into separate libraries): 1 = xn
// staged for the first hidden chunk only, 2 = GELU replaced by the identity, 3 = nothing staged
// after the first chunk.  Results are wrong in every diagnostic build.
#ifndef MDG_DIAG_MLP
#define MDG_DIAG_MLP 0
#endif
constexpr int kMlpThreads = 512, kMlpHC = 128, kMlpStages = 3, kMlpSlot = 512 * 32;

__host__ __device__ constexpr size_t mlp_smem(int F, bool vst = false) {
  return (size_t)(vst ? 2 : kMlpStages) * kMlpSlot * 2 + (size_t)128 * kMlpHC * 2 + (size_t)F * 4;
}

// LDS accesses the compiler's wait-count pass does not see.  It makes every LDS access that
// follows a global_load_lds wait for ALL outstanding LDS DMA (s_waitcnt vmcnt(0): it cannot
// tell the ring slots from the other LDS arrays), which drains the ring ahead of the
// epilogues' bias / RoPE reads; these kernels order their LDS by their own barriers instead.
// Each read group is ONE asm statement ending in s_waitcnt lgkmcnt(0), with early-clobber
// outputs: with the wait in a separate statement the compiler copied a destination register
// before the data had arrived.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ __forceinline__ void lds_ld4x4_raw(const float* p0, const float* p1, const float* p2, const float* p3,
                                              f32x4& v0, f32x4& v1, f32x4& v2, f32x4& v3) {
  asm volatile(
      "ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\tds_read_b128 %2, %6\n\tds_read_b128 %3, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
      : "v"(lds_addr(p0)), "v"(lds_addr(p1)), "v"(lds_addr(p2)), "v"(lds_addr(p3)));
}
__device__ __forceinline__ f32x4 lds_ld4_raw(const float* p) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(lds_addr(p)));
  return v;
}
// one float4 + four float2 (the bias and the RoPE cos / sin pairs of two tokens)
__device__ __forceinline__ void lds_ld4_2x4_raw(const float* pb, const float* pc0, const float* ps0, const float* pc1,
                                                const float* ps1, f32x4& b, f32x2& c0, f32x2& s0, f32x2& c1,
                                                f32x2& s1) {
  asm volatile(
      "ds_read_b128 %0, %5\n\tds_read_b64 %1, %6\n\tds_read_b64 %2, %7\n\tds_read_b64 %3, %8\n\t"
      "ds_read_b64 %4, %9\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(b), "=&v"(c0), "=&v"(s0), "=&v"(c1), "=&v"(s1)
      : "v"(lds_addr(pb)), "v"(lds_addr(pc0)), "v"(lds_addr(ps0)), "v"(lds_addr(pc1)), "v"(lds_addr(ps1)));
}
__device__ __forceinline__ void lds_st1_raw(float* p, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 6]
__device__ __forceinline__ void vm_wait_upto6(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
  }
}

// PRE (round 5): the block first runs the temporal attention's out_proj row-LN GEMM on its own
// 128 rows (latent_model.py:486: h += gate_t * out_proj(o), then LN_mlp + modulate -> xn), the
// exact K loop and epilogue of gemm_rowln_kernel<384, 128> on this kernel's 3-slot ring (one
// 32-wide step = 128 o rows + 384 W_o rows = one slot), so h and xn equal the two-launch form bit
// for bit.  The block's h / xn rows are then read back by the MLP below (ring DMA for xn, the
// residual load for h): ordered by a work-group barrier with release / acquire at work-group
// scope (one CU, one L1).  Saves the out_proj launch, its grid tail and the xn HBM round trip.
// VST (round 5; the small-M split form): the operand pieces go global -> VGPRs ->
// ds_write_b128 into the same LDS image instead of global_load_lds, two steps ahead in two
// register sets, two LDS slots.  A split block streams ~576 KiB of operands for 2 hidden chunks
// of 128 rows; LDS-DMA fills ~16 B/clk per CU, plain loads ~3x that (tools/ubench/l2lds.hip).
// (The one-pass form with VST measured equal, round 5 DESIGN §3, and is not instantiated.)
template <int NCOL, bool SPLIT, bool PRE = false, bool VST = false>  // SPLIT: chunks [y * cps, (y + 1) * cps) only, fp32 partials out
__global__ __launch_bounds__(kMlpThreads, 1) void mlp_rowln_kernel(const MlpArgs args) {
  static_assert(NCOL == 384, "the ring slot holds 384 W2 rows");
  static_assert(!(PRE && VST), "the out_proj prologue stages by DMA");
  constexpr int BM = 128, BK = 32, HC = kMlpHC, STAGES = VST ? 2 : kMlpStages, SLOT = kMlpSlot;
  constexpr int WTN = NCOL / 4, NT = WTN / 16, NE = NCOL / 128, LDS_ST = NCOL + 4;
  static_assert((32 * LDS_ST + 6 * NCOL) * 4 <= STAGES * SLOT * 2, "epilogue stage + adaLN rows fit the ring");
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const mdg_gemm_desc& q = args.f1;  // xn, W1, b1
  const mdg_gemm_desc& p = args.f2;  // W2, b2 and the row-LN epilogue
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Hs = ring + STAGES * SLOT;                    // [BM][HC]: 16-B chunk c of row r at c ^ (r & 15)
  float* b1s = reinterpret_cast<float*>(Hs + BM * HC);  // [F]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / 4, wn = wave % 4;    // fc2: 64 tokens x WTN outputs
  const int wah = wave / 4, wat = wave % 4;  // fc1: 64 hidden x 32 tokens
  const int lr = lane & 15, lg = lane >> 4;
  const int M = p.M, F = p.K;
  const int cps = SPLIT ? (F / HC) / args.nsplit : F / HC, j0 = SPLIT ? (int)blockIdx.y * cps : 0;
  const int NS = cps * 10;  // 6 fc1 (K 64) + 4 fc2 (K 32) steps per hidden chunk
  const int nwg = (M + BM - 1) / BM;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int m0 = ((xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc) * BM;

  for (int i = tid; i < F; i += kMlpThreads) b1s[i] = q.bias ? q.bias[i] : 0.f;
  // ring loader: slot row r's 16-B chunk c at c ^ ((-(r >> 2)) & 3); a 16-row piece per glds
  const int cswz = ((lane & 3) ^ ((-(lane >> 4)) & 3)) * 8;
  if constexpr (PRE) {
    static_assert(!SPLIT, "the out_proj prologue runs in the one-pass form");
    const mdg_gemm_desc& r = args.r;
    constexpr int NK = NCOL / BK;
    const int chp = (lg ^ ((-(lr >> 2)) & 3)) * 8;  // r.K == NCOL: 12 steps of 32
    const float inv_rpm_r = 1.0f / (float)r.rows_per_mod;
    float4 h4p[2][NE];
    rowln_load_band<NCOL>(r, RowsLinear{m0}, 0, h4p);  // band 0's residual rows, in flight under the K loop
    // wave w stages slot rows 64 w + 16 i + lane / 4 (i < 4): rows < 128 from o, the rest from W_o
    const bool ow = wave < 2;
    const bf16_t* pbase = reinterpret_cast<const bf16_t*>(ow ? r.A : r.W);
    int poff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int sr = 64 * wave + 16 * i + (lane >> 2);
      poff[i] = (ow ? min(m0 + sr, M - 1) * r.lda : (sr - BM) * r.ldw) + cswz;
    }
    auto pissue = [&](int s) {
      bf16_t* sl = ring + (s % STAGES) * SLOT;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(pbase + s * BK + poff[i]),
                                         (lds_ptr_t)(sl + (64 * wave + 16 * i) * BK), 16, 0, 0);
    };
    f32x4 acc[4][NT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    pissue(0);
    pissue(1);
    for (int s = 0; s < NK; ++s) {
      // step s landed (the residual rows with it at s = 0); step s + 1's 4 pieces stay in flight
      if (s + 1 < NK) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring reads retired (see kRingWaitNote)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s + 2 < NK) pissue(s + 2);
      const bf16_t* As = ring + (s % STAGES) * SLOT;
      const bf16_t* Bs = As + BM * BK;
      bf16x8 a[4], b[NT];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + lr) * BK + chp);
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * WTN + j * 16 + lr) * BK + chp);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    rowln_fast_epilogue<NCOL>(r, acc, h4p, smem, RowsLinear{m0}, fdiv(m0, r.rows_per_mod, inv_rpm_r), inv_rpm_r);
    // the block's h and xn rows are stored before any wave reads them back (the ring's xn DMA,
    // the epilogue's residual load); the stage region is free again for the ring
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  const bf16_t* X = reinterpret_cast<const bf16_t*>(q.A);
  const bf16_t* W1 = reinterpret_cast<const bf16_t*>(q.W);
  const bf16_t* W2 = reinterpret_cast<const bf16_t*>(p.W);
  // fc1 step (k0 = 64 t): two 32-wide images of 256 slot rows each (xn rows, then the chunk's
  // W1 rows): waves 0-3 stage xn rows 16(2w + i) + lane/4, waves 4-7 W1 rows (slot rows
  // 128 + ...), in both images; fc2 step: wave w stages W2 rows 16(3w + i) + lane/4.
  // (Element offsets from wave-uniform bases: one 64-bit address per lane is rebuilt per issue.)
  const bool xw = wave < 4;
  const bf16_t* abase = xw ? X : W1;
  const int ald = xw ? q.lda : q.ldw;
  int aoff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * (2 * (wave & 3) + i) + (lane >> 2);
    aoff[i] = (xw ? min(m0 + r, M - 1) : r) * ald + cswz;
  }
  const int boff = (16 * 3 * wave + (lane >> 2)) * p.ldw + cswz, bstep = 16 * p.ldw;
  constexpr int IMG = 2 * BM * BK;  // one 32-wide image of the fc1 step (xn + W1c rows)
  auto issue = [&](int s) {
    bf16_t* sl = ring + (s % STAGES) * SLOT;
    const int j = j0 + s / 10, t = s % 10;  // hidden chunk, step within it
    if ((MDG_DIAG_MLP == 1 && xw && t < 6 && j > 0) || (MDG_DIAG_MLP == 3 && j > 0)) return;
    if (t < 6) {
      const bf16_t* base = abase + (size_t)t * 2 * BK + (xw ? (size_t)0 : (size_t)j * HC * q.ldw);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          __builtin_amdgcn_global_load_lds((const void*)(base + h * BK + aoff[i]),
                                           (lds_ptr_t)(sl + h * IMG + ((xw ? 0 : BM) + 16 * (2 * (wave & 3) + i)) * BK),
                                           16, 0, 0);
    } else {
      const bf16_t* base = W2 + j * HC + (t - 6) * BK;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(base + boff + i * bstep), (lds_ptr_t)(sl + 16 * (3 * wave + i) * BK),
                                         16, 0, 0);
    }
  };

  // VST: the same pieces (source address, LDS destination) through 16-B register loads; two
  // named register sets picked by the step's parity (a uniform branch; no indexed register
  // array, which the compiler would put in scratch)
  u32x4 vA[4], vB[4];
  // K: the step's kind as a compile-time constant (0: fc1 step, 1: fc2 step)
  auto vload_set = [&](auto K, int s, u32x4(&vr)[4]) __attribute__((always_inline)) {
    const int j = j0 + s / 10, t = s % 10;
    if constexpr (!decltype(K)::value) {
      const bf16_t* base = abase + (size_t)t * 2 * BK + (xw ? (size_t)0 : (size_t)j * HC * q.ldw);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) vr[2 * h + i] = *reinterpret_cast<const u32x4*>(base + h * BK + aoff[i]);
    } else {
      const bf16_t* base = W2 + j * HC + (t - 6) * BK;
#pragma unroll
      for (int i = 0; i < 3; ++i) vr[i] = *reinterpret_cast<const u32x4*>(base + boff + i * bstep);
    }
  };
  auto vload = [&](auto P, auto K, int s) __attribute__((always_inline)) {
    if constexpr (decltype(P)::value) vload_set(K, s, vB);
    else vload_set(K, s, vA);
  };
  auto vcommit_set = [&](auto K, int s, const u32x4(&vr)[4]) __attribute__((always_inline)) {
    bf16_t* sl = ring + (s % STAGES) * SLOT;
    if constexpr (!decltype(K)::value) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          *reinterpret_cast<u32x4*>(sl + h * IMG + ((xw ? 0 : BM) + 16 * (2 * (wave & 3) + i)) * BK + 8 * lane) =
              vr[2 * h + i];
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i) *reinterpret_cast<u32x4*>(sl + 16 * (3 * wave + i) * BK + 8 * lane) = vr[i];
    }
  };
  auto vcommit = [&](auto P, auto K, int s) __attribute__((always_inline)) {
    if constexpr (decltype(P)::value) vcommit_set(K, s, vB);
    else vcommit_set(K, s, vA);
  };

  const int ch = (lg ^ ((-(lr >> 2)) & 3)) * 8;
  f32x4 acc2[4][NT], acc1[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  if constexpr (VST) {  // steps 0 and 1 are fc1 steps
    vload(P0{}, P0{}, 0);
    vcommit(P0{}, P0{}, 0);
    if (1 < NS) vload(P1{}, P0{}, 1);
  } else {
#pragma unroll
    for (int s0 = 0; s0 < STAGES - 1; ++s0)
      if (s0 < NS) issue(s0);
  }
  // DMA: step s landed: leave step s+1's pieces in flight; then refill the slot every wave has
  // finished reading (step s-1's) with step s+2.  VST: slot s % 2 was written before this
  // barrier; step s + 2's pieces are loaded here (into the set step s's pieces left), step
  // s + 1's written after step s's MFMAs (step_end).
  auto step_begin = [&](int s) {
    if constexpr (VST) {  // (the VST loops call vstep_begin below instead)
      return ring + (s % STAGES) * SLOT;
    }
    const int y1 = s + 1 < NS ? ((s + 1) % 10 < 6 ? 4 : 3) : 0;
    vm_wait_upto6(y1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring reads retired (see kRingWaitNote)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + STAGES - 1 < NS) issue(s + STAGES - 1);
    return ring + (s % STAGES) * SLOT;
  };
  if constexpr (VST) {
    // every step of a chunk spelled out with its index as a compile-time constant, so each call
    // site knows the register set (parity) and the kind of the steps it loads and writes
    // (step j * 10 + t: t < 6 fc1, else fc2; the chunk's step count, 10, is even)
    auto vstep_begin = [&](auto P, auto K2, int s) __attribute__((always_inline)) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot writes and ring reads retired
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s + 2 < NS) vload(P, K2, s + 2);  // into the set step s's pieces left
      return ring + (s % STAGES) * SLOT;
    };
    auto step = [&](auto TT, int j) __attribute__((always_inline)) {
      constexpr int t = decltype(TT)::value;
      using P = std::integral_constant<int, t & 1>;
      using Pn = std::integral_constant<int, (t + 1) & 1>;
      using Kn = std::integral_constant<int, ((t + 1) % 10) >= 6 ? 1 : 0>;  // step s + 1's kind
      using K2 = std::integral_constant<int, ((t + 2) % 10) >= 6 ? 1 : 0>;  // step s + 2's kind
      const int s = j * 10 + t;
      const bf16_t* sl = vstep_begin(P{}, K2{}, s);
      if constexpr (t < 6) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          bf16x8 a[4], b[2];
#pragma unroll
          for (int hi = 0; hi < 4; ++hi)
            a[hi] = *reinterpret_cast<const bf16x8*>(sl + h * IMG + (BM + wah * 64 + hi * 16 + lr) * BK + ch);
#pragma unroll
          for (int ti = 0; ti < 2; ++ti)
            b[ti] = *reinterpret_cast<const bf16x8*>(sl + h * IMG + (wat * 32 + ti * 16 + lr) * BK + ch);
#pragma unroll
          for (int hi = 0; hi < 4; ++hi)
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
              acc1[hi][ti] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[hi], b[ti], acc1[hi][ti], 0, 0, 0);
        }
      } else {
        constexpr int kb = t - 6;
        bf16x8 a[4], b[NT];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * 64 + i * 16 + lr;
          a[i] = *reinterpret_cast<const bf16x8*>(Hs + row * HC + (((kb * 4 + lg) ^ (row & 15)) * 8));
        }
#pragma unroll
        for (int jn = 0; jn < NT; ++jn) b[jn] = *reinterpret_cast<const bf16x8*>(sl + (wn * WTN + jn * 16 + lr) * BK + ch);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jn = 0; jn < NT; ++jn) acc2[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[jn], acc2[i][jn], 0, 0, 0);
      }
      if (s + 1 < NS) vcommit(Pn{}, Kn{}, s + 1);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    using I5 = std::integral_constant<int, 5>;
    using I6 = std::integral_constant<int, 6>;
    using I7 = std::integral_constant<int, 7>;
    using I8 = std::integral_constant<int, 8>;
    using I9 = std::integral_constant<int, 9>;
    for (int j = 0; j < NS / 10; ++j) {
      step(I0{}, j);
      step(I1{}, j);
      step(I2{}, j);
      step(I3{}, j);
      step(I4{}, j);
      step(I5{}, j);
      // the chunk's fc1 is complete: + b1, GELU, bf16 -> Hs; restart acc1
      const float* b1c = b1s + (j0 + j) * HC;
      f32x4 b1v[4];
      {
        const float* bp = b1c + wah * 64 + lg * 4;
        lds_ld4x4_raw(bp, bp + 16, bp + 32, bp + 48, b1v[0], b1v[1], b1v[2], b1v[3]);
      }
#pragma unroll
      for (int hi = 0; hi < 4; ++hi)
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) {
          const int hb = wah * 64 + hi * 16 + lg * 4, tok = wat * 32 + ti * 16 + lr;
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (bf16_t)gelu_fast(acc1[hi][ti][r] + b1v[hi][r]);
          *reinterpret_cast<bf16x4*>(Hs + tok * HC + (((hb >> 3) ^ (tok & 15)) * 8) + (hb & 7)) = o;
          acc1[hi][ti] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // Hs complete before the next barrier
      step(I6{}, j);
      step(I7{}, j);
      step(I8{}, j);
      step(I9{}, j);
    }
  } else {
  // (the fc1 and fc2 step bodies are separate loops: one loop with a branch per step made the
  // compiler give the accumulators different registers on the two paths)
  for (int j = 0; j < NS / 10; ++j) {
    for (int t = 0; t < 6; ++t) {
      const bf16_t* sl = step_begin(j * 10 + t);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bf16x8 a[4], b[2];
#pragma unroll
        for (int hi = 0; hi < 4; ++hi)
          a[hi] = *reinterpret_cast<const bf16x8*>(sl + h * IMG + (BM + wah * 64 + hi * 16 + lr) * BK + ch);
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) b[ti] = *reinterpret_cast<const bf16x8*>(sl + h * IMG + (wat * 32 + ti * 16 + lr) * BK + ch);
#pragma unroll
        for (int hi = 0; hi < 4; ++hi)
#pragma unroll
          for (int ti = 0; ti < 2; ++ti) acc1[hi][ti] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[hi], b[ti], acc1[hi][ti], 0, 0, 0);
      }
    }
    // the chunk's fc1 is complete: + b1, GELU, bf16 -> Hs; restart acc1.  (Hs was last read by
    // chunk j - 1's fc2 steps, which every wave finished before this chunk's first barrier.)
    const float* b1c = b1s + (j0 + j) * HC;
    f32x4 b1v[4];
    {
      const float* bp = b1c + wah * 64 + lg * 4;
      lds_ld4x4_raw(bp, bp + 16, bp + 32, bp + 48, b1v[0], b1v[1], b1v[2], b1v[3]);
    }
#pragma unroll
    for (int hi = 0; hi < 4; ++hi)
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
        const int hb = wah * 64 + hi * 16 + lg * 4, tok = wat * 32 + ti * 16 + lr;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[r] = (bf16_t)(MDG_DIAG_MLP == 2 ? acc1[hi][ti][r] + b1v[hi][r] : gelu_fast(acc1[hi][ti][r] + b1v[hi][r]));
        *reinterpret_cast<bf16x4*>(Hs + tok * HC + (((hb >> 3) ^ (tok & 15)) * 8) + (hb & 7)) = o;
        acc1[hi][ti] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // Hs complete before the next barrier
    for (int kb = 0; kb < 4; ++kb) {
      const bf16_t* sl = step_begin(j * 10 + 6 + kb);
      bf16x8 a[4], b[NT];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + lr;
        a[i] = *reinterpret_cast<const bf16x8*>(Hs + row * HC + (((kb * 4 + lg) ^ (row & 15)) * 8));
      }
#pragma unroll
      for (int jn = 0; jn < NT; ++jn) b[jn] = *reinterpret_cast<const bf16x8*>(sl + (wn * WTN + jn * 16 + lr) * BK + ch);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jn = 0; jn < NT; ++jn) acc2[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[jn], acc2[i][jn], 0, 0, 0);
    }
  }
  }
  if constexpr (SPLIT) {
    // this block's fc2 partial sum: 16 consecutive columns (64 B) per 16-lane group and register
    float* pp = args.part + (size_t)blockIdx.y * M * NCOL;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + lg * 4 + r;
        if (m < M)
#pragma unroll
          for (int jn = 0; jn < NT; ++jn) pp[(size_t)m * NCOL + wn * WTN + jn * 16 + lr] = acc2[i][jn][r];
      }
  } else {
    const float inv_rpm = 1.0f / (float)p.rows_per_mod;
    float4 h4[2][NE];
    rowln_load_band<NCOL>(p, RowsLinear{m0}, 0, h4);  // band 0's residual rows
    rowln_fast_epilogue<NCOL>(p, acc2, h4, smem, RowsLinear{m0}, fdiv(m0, p.rows_per_mod, inv_rpm), inv_rpm);
  }
}

// ---------------------------------------------------------------------------------------
// Fused MLP with 256-wide hidden chunks and 64 x 64 fc1 wave tiles (round 6, MDG_MLP_HC=256).
// The kernel above computes each 128-hidden chunk's H^T = W1c . xn^T as 8 wave tiles of 64
// hidden x 32 tokens: 6 LDS fragment reads per 8 MFMAs, and per fc1 K-step of 64 the block reads
// 96 KiB of fragments while its LDS-DMA ring writes 32 KiB (≈ 250 B/clk per CU against the
// 512 cycles of MFMA work of the step, at LDS's 256 B/clk read limit), and the xn tile is
// re-staged for every one of the 12 chunks.  Here a chunk is 256 hidden units: 8 wave tiles of
// 64 hidden x 64 tokens (4 + 4 fragment reads per 16 MFMAs: a third fewer LDS bytes per fc1
// FLOP), xn re-staged 6 times instead of 12, fc1 in K-steps of 32 (one 384-row image per slot:
// 128 xn rows + 256 W1c rows = 24 KiB, the same size as an fc2 step's 384 W2 rows x 32), so
// every step moves 3 LDS-DMA pieces per wave and the ring is 3 x 24 KiB; Hs [128][256] = 64 KiB.
// acc1 is 64 VGPRs (was 32).  The K orders of fc1 (ascending 32-steps) and fc2 (ascending
// hidden) are the other kernel's, so h and xn are bit-identical to it and to fc1-then-fc2.
constexpr int kMlp2HC = 256, kMlp2Slot = 384 * 32;
__host__ __device__ constexpr size_t mlp2_smem(int F) {
  return (size_t)kMlpStages * kMlp2Slot * 2 + (size_t)128 * kMlp2HC * 2 + (size_t)F * 4;
}

template <int NCOL>
__global__ __launch_bounds__(kMlpThreads, 1) void mlp_rowln256_kernel(const MlpArgs args) {
  static_assert(NCOL == 384, "the ring slot holds 384 W2 rows");
  constexpr int BM = 128, BK = 32, HC = kMlp2HC, STAGES = kMlpStages, SLOT = kMlp2Slot;
  constexpr int WTN = NCOL / 4, NT = WTN / 16, NE = NCOL / 128, LDS_ST = NCOL + 4;
  constexpr int NF1 = 12, NF2 = HC / BK, SPC = NF1 + NF2;  // steps per chunk: 12 fc1 + 8 fc2
  static_assert((32 * LDS_ST + 6 * NCOL) * 4 <= STAGES * SLOT * 2, "epilogue stage + adaLN rows fit the ring");
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const mdg_gemm_desc& q = args.f1;  // xn, W1, b1
  const mdg_gemm_desc& p = args.f2;  // W2, b2 and the row-LN epilogue
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Hs = ring + STAGES * SLOT;                    // [BM][HC]: 16-B chunk c of row r at c ^ (r & 15)
  float* b1s = reinterpret_cast<float*>(Hs + BM * HC);  // [F]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / 4, wn = wave % 4;    // fc2: 64 tokens x WTN outputs
  const int wah = wave & 3, wat = wave >> 2;  // fc1: 64 hidden x 64 tokens
  const int lr = lane & 15, lg = lane >> 4;
  const int M = p.M, F = p.K;
  const int NS = (F / HC) * SPC;
  const int nwg = (M + BM - 1) / BM;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int m0 = ((xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc) * BM;

  for (int i = tid; i < F; i += kMlpThreads) b1s[i] = q.bias ? q.bias[i] : 0.f;
  const int cswz = ((lane & 3) ^ ((-(lane >> 4)) & 3)) * 8;
  const bf16_t* X = reinterpret_cast<const bf16_t*>(q.A);
  const bf16_t* W1 = reinterpret_cast<const bf16_t*>(q.W);
  const bf16_t* W2 = reinterpret_cast<const bf16_t*>(p.W);
  // piece i (0..2) of wave w: slot rows 16 (3w + i) + lane / 4; fc1 step: rows < 128 are xn rows
  // (pieces 0..7), the rest W1c rows; fc2 step: W2 rows
  int xoff[3], woff[3];
  bool isx[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int r = 16 * (3 * wave + i) + (lane >> 2);
    isx[i] = r < BM;
    xoff[i] = isx[i] ? min(m0 + r, M - 1) * q.lda + cswz : (r - BM) * q.ldw + cswz;
    woff[i] = r * p.ldw + cswz;
  }
  auto issue = [&](int s) {
    bf16_t* sl = ring + (s % STAGES) * SLOT;
    const int j = s / SPC, t = s % SPC;
    if (t < NF1) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const bf16_t* src = isx[i] ? X + (size_t)t * BK + xoff[i] : W1 + (size_t)j * HC * q.ldw + (size_t)t * BK + xoff[i];
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(sl + 16 * (3 * wave + i) * BK), 16, 0, 0);
      }
    } else {
      const bf16_t* base = W2 + j * HC + (t - NF1) * BK;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(base + woff[i]), (lds_ptr_t)(sl + 16 * (3 * wave + i) * BK), 16,
                                         0, 0);
    }
  };
  const int ch = (lg ^ ((-(lr >> 2)) & 3)) * 8;
  f32x4 acc2[4][NT], acc1[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int s0 = 0; s0 < STAGES - 1; ++s0)
    if (s0 < NS) issue(s0);
  // step s landed (step s + 1's 3 pieces stay in flight); then refill the slot every wave has
  // finished reading (step s - 1's) with step s + 2
  auto step_begin = [&](int s) {
    if (s + 1 < NS) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring reads retired (see kRingWaitNote)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + STAGES - 1 < NS) issue(s + STAGES - 1);
    return ring + (s % STAGES) * SLOT;
  };
  for (int j = 0; j < NS / SPC; ++j) {
    for (int t = 0; t < NF1; ++t) {
      const bf16_t* sl = step_begin(j * SPC + t);
      bf16x8 a[4], b[4];
#pragma unroll
      for (int hi = 0; hi < 4; ++hi) a[hi] = *reinterpret_cast<const bf16x8*>(sl + (BM + wah * 64 + hi * 16 + lr) * BK + ch);
#pragma unroll
      for (int ti = 0; ti < 4; ++ti) b[ti] = *reinterpret_cast<const bf16x8*>(sl + (wat * 64 + ti * 16 + lr) * BK + ch);
#pragma unroll
      for (int hi = 0; hi < 4; ++hi)
#pragma unroll
        for (int ti = 0; ti < 4; ++ti) acc1[hi][ti] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[hi], b[ti], acc1[hi][ti], 0, 0, 0);
    }
    // the chunk's fc1 is complete: + b1, GELU, bf16 -> Hs; restart acc1.  (Hs was last read by
    // chunk j - 1's fc2 steps, which every wave finished before this chunk's first barrier.)
    const float* b1c = b1s + j * HC;
    f32x4 b1v[4];
    {
      const float* bp = b1c + wah * 64 + lg * 4;
      lds_ld4x4_raw(bp, bp + 16, bp + 32, bp + 48, b1v[0], b1v[1], b1v[2], b1v[3]);
    }
#pragma unroll
    for (int hi = 0; hi < 4; ++hi)
#pragma unroll
      for (int ti = 0; ti < 4; ++ti) {
        const int hb = wah * 64 + hi * 16 + lg * 4, tok = wat * 64 + ti * 16 + lr;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16_t)gelu_fast(acc1[hi][ti][r] + b1v[hi][r]);
        *reinterpret_cast<bf16x4*>(Hs + tok * HC + (((hb >> 3) ^ (tok & 15)) * 8) + (hb & 7)) = o;
        acc1[hi][ti] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // Hs complete before the next barrier
    for (int kb = 0; kb < NF2; ++kb) {
      const bf16_t* sl = step_begin(j * SPC + NF1 + kb);
      bf16x8 a[4], b[NT];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + lr;
        a[i] = *reinterpret_cast<const bf16x8*>(Hs + row * HC + (((kb * 4 + lg) ^ (row & 15)) * 8));
      }
#pragma unroll
      for (int jn = 0; jn < NT; ++jn) b[jn] = *reinterpret_cast<const bf16x8*>(sl + (wn * WTN + jn * 16 + lr) * BK + ch);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jn = 0; jn < NT; ++jn) acc2[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[jn], acc2[i][jn], 0, 0, 0);
    }
  }
  const float inv_rpm = 1.0f / (float)p.rows_per_mod;
  float4 h4[2][NE];
  rowln_load_band<NCOL>(p, RowsLinear{m0}, 0, h4);  // band 0's residual rows
  rowln_fast_epilogue<NCOL>(p, acc2, h4, smem, RowsLinear{m0}, fdiv(m0, p.rows_per_mod, inv_rpm), inv_rpm);
}

// ---------------------------------------------------------------------------------------
// Fused MLP, wave-specialised (round 3; large M, one 128-token tile per block, 8 waves).
// The lock-step kernel above runs fc1 -> GELU -> fc2 in every wave, so the GELU's vector issue
// (~3 800 cycles per wave and hidden chunk) sits on the MFMA critical path.  Here the two halves
// of a SIMD's pair of waves do different work at the same time:
//   P waves 0-3 ("producers"): Hc^T = W1c . xn^T for chunk t (32 tokens each, the 128 hidden
//     units of the chunk), + b1, GELU, bf16 -> H[t % 2] in LDS.  Each P wave keeps its 32 xn rows
//     x 384 in registers for the whole kernel (the fc1 B operand: 96 VGPRs), so xn is read from
//     HBM exactly once per tile (the lock-step kernel re-staged it per chunk: 1.11x traffic).
//   Q waves 4-7 ("consumers"): acc2 += H[t-1] . W2c^T for chunk t-1 (128 tokens x 96 outputs
//     each, 192 accumulator VGPRs), then the row-LN epilogue.
// Wave w and w + 4 share SIMD w, so a P wave's GELU issues beside a Q wave's MFMAs.  A chunk is
// 4 phases separated by one block barrier: per phase P does 3 fc1 K-steps of 32 (W1 slice 128
// rows x 96, 24 KiB), Q one fc2 K-step of 32 (W2 slice 384 rows x 32, 24 KiB); both slices of
// phase p+1 stream into the other slot of a 2-slot global_load_lds ring during phase p (6 pieces
// per wave, waited with vmcnt(0) before the phase's barrier).  LDS: H 2 x 32 KiB + ring 2 x 48
// KiB = 160 KiB.  The K orders of both products equal the lock-step kernel's, so h and xn are
// bit-identical to it (tests/test_gpu_kernels.py).
constexpr int kWsThreads = 512, kWsHC = 128, kWsW1Img = 128 * 32;
constexpr int kWsSlot = 3 * kWsW1Img + 384 * 32;                                 // bf16 elements
constexpr size_t kWsSmem = (size_t)2 * 128 * kWsHC * 2 + (size_t)2 * kWsSlot * 2;  // 160 KiB

template <int NCOL>
__global__ __launch_bounds__(kWsThreads, 1) void mlp_ws_kernel(const MlpArgs args) {
  static_assert(NCOL == 384, "the ring's W2 slice holds 384 rows");
  constexpr int BM = 128, HC = kWsHC, BK = 32, NQ = 6, LDS_ST = NCOL + 4;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Hb = reinterpret_cast<bf16_t*>(smem);  // [2][BM][HC]: 16-B chunk c of row r at c ^ (r & 15)
  bf16_t* ring = Hb + 2 * BM * HC;               // [2][kWsSlot]
  const mdg_gemm_desc& q = args.f1;              // xn, W1, b1
  const mdg_gemm_desc& p = args.f2;              // W2, b2 and the row-LN epilogue
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wq = wave & 3;
  const bool isP = wave < 4;
  const int lr = lane & 15, lg = lane >> 4;
  const int M = p.M, F = p.K, NCH = F / HC, NPH = 4 * (NCH + 1);
  const int nwg = (M + BM - 1) / BM;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int m0 = ((xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc) * BM;
  const bf16_t* X = reinterpret_cast<const bf16_t*>(q.A);
  const bf16_t* W1 = reinterpret_cast<const bf16_t*>(q.W);
  const bf16_t* W2 = reinterpret_cast<const bf16_t*>(p.W);
  // ring pieces (16 rows x 64 B each, lane-linear destination, swizzle on the source chunk):
  // P wave wq stages W1 pieces 6wq..6wq+5 (image k3 = id / 8, row block id % 8), Q wave wq W2
  // row blocks 6wq..6wq+5
  // the row swizzle of row 16 rb + prow depends on prow only: one per-lane offset for all pieces
  const int prow = lane >> 2, pch = lane & 3;
  const int ldw = isP ? q.ldw : p.ldw;
  const int voff = prow * ldw + ((pch ^ ((-(prow >> 2)) & 3)) * 8);
  auto issue = [&](int ph) {
    if (ph >= NPH) return;
    bf16_t* sl = ring + (ph & 1) * kWsSlot;
    if (isP) {
      if (ph >= 4 * NCH) return;
      const bf16_t* base = W1 + (size_t)(ph >> 2) * HC * ldw + 96 * (ph & 3) + voff;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int id = 6 * wq + i;
        __builtin_amdgcn_global_load_lds((const void*)(base + 32 * (id >> 3) + 16 * (id & 7) * ldw),
                                         (lds_ptr_t)(sl + (id >> 3) * kWsW1Img + 16 * (id & 7) * BK), 16, 0, 0);
      }
    } else {
      if (ph < 4) return;
      const bf16_t* base = W2 + (size_t)((ph >> 2) - 1) * HC + 32 * (ph & 3) + voff;
#pragma unroll
      for (int i = 0; i < 6; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(base + 16 * (6 * wq + i) * ldw),
                                         (lds_ptr_t)(sl + 3 * kWsW1Img + 16 * (6 * wq + i) * BK), 16, 0, 0);
    }
  };
  const int ch = (lg ^ ((-(lr >> 2)) & 3)) * 8;  // fragment rows are lr mod 16
  issue(0);
  if (isP) {
    // P: the wave's 32 xn rows as the fc1 B operand, k-step kk, token tile ni
    bf16x8 xf[12][2];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const bf16_t* xr = X + (size_t)min(m0 + 32 * wq + 16 * ni + lr, M - 1) * q.lda + 8 * lg;
#pragma unroll
      for (int kk = 0; kk < 12; ++kk) xf[kk][ni] = *reinterpret_cast<const bf16x8*>(xr + 32 * kk);
    }
    f32x4 acc1[8][2];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) acc1[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // (the chunk's 4 phases unrolled: xf is indexed by compile-time k-steps only, so it stays in
    // registers)
    for (int t = 0; t < NCH; ++t) {
#pragma unroll
      for (int sub = 0; sub < 4; ++sub) {
        const int ph = 4 * t + sub;
        asm volatile("" ::: "memory");
        issue(ph + 1);
        const bf16_t* img = ring + (ph & 1) * kWsSlot;
        f32x4 b1v[8];
        if (sub == 3) {
#pragma unroll
          for (int mi = 0; mi < 8; ++mi)
            b1v[mi] = q.bias ? *reinterpret_cast<const f32x4*>(q.bias + t * HC + 16 * mi + 4 * lg)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int k3 = 0; k3 < 3; ++k3) {
#pragma unroll
          for (int mi = 0; mi < 8; ++mi) {
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(img + k3 * kWsW1Img + (16 * mi + lr) * BK + ch);
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc1[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, xf[3 * sub + k3][ni], acc1[mi][ni], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);  // keep the next k-step's fragment reads out of this one
        }
        if (sub == 3) {  // the chunk's fc1 is complete: + b1, GELU, bf16 -> H[t % 2]
          bf16_t* Hs = Hb + (t & 1) * BM * HC;
#pragma unroll
          for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
              const int hb = 16 * mi + 4 * lg, tok = 32 * wq + 16 * ni + lr;
              bf16x4 o;
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = (bf16_t)gelu_fast(acc1[mi][ni][r] + b1v[mi][r]);
              *reinterpret_cast<bf16x4*>(Hs + tok * HC + (((hb >> 3) ^ (tok & 15)) * 8) + (hb & 7)) = o;
              acc1[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            __builtin_amdgcn_sched_barrier(0);  // one tile pair at a time: bounded temporaries
          }
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
    for (int ph = 4 * NCH; ph < NPH; ++ph) {  // the Q waves' last chunk
      asm volatile("" ::: "memory");
      issue(ph + 1);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    const float inv_rpm = 1.0f / (float)p.rows_per_mod;
    float4 h4[2][NCOL / 128];
    auto no_stage = [&](int, float*) {};
    rowln_fast_epilogue_impl<NCOL, 3, true>(p, no_stage, h4, smem, RowsLinear{m0}, fdiv(m0, p.rows_per_mod, inv_rpm),
                                            inv_rpm);
  } else {
    f32x4 acc2[8][NQ];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int nj = 0; nj < NQ; ++nj) acc2[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int ph = 0; ph < 4; ++ph) {  // the P waves' first chunk
      asm volatile("" ::: "memory");
      issue(ph + 1);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    for (int u = 0; u < NCH; ++u) {
#pragma unroll
      for (int sub = 0; sub < 4; ++sub) {
        const int ph = 4 * (u + 1) + sub;
        asm volatile("" ::: "memory");
        issue(ph + 1);
        const bf16_t* Hs = Hb + (u & 1) * BM * HC;
        const bf16_t* img = ring + (ph & 1) * kWsSlot + 3 * kWsW1Img;
        // two halves of 4 token tiles (fewer live fragment registers beside the 192 accumulators)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          bf16x8 a[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = 16 * (4 * hf + i) + lr;
            a[i] = *reinterpret_cast<const bf16x8*>(Hs + row * HC + (((sub * 4 + lg) ^ (row & 15)) * 8));
          }
#pragma unroll
          for (int nj = 0; nj < NQ; ++nj) {
            const bf16x8 b = *reinterpret_cast<const bf16x8*>(img + (96 * wq + 16 * nj + lr) * BK + ch);
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc2[4 * hf + i][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc2[4 * hf + i][nj], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
    const float inv_rpm = 1.0f / (float)p.rows_per_mod;
    float4 h4[2][NCOL / 128];
    // band b = accumulator rows 16 mi + 4 lg + r with mi in {2b, 2b+1}; columns 96 wq + 16 nj + lr.
    // Bands 0-2 go to stage regions 0-2 at band 0 (144 accumulator VGPRs freed before the row
    // work), band 3 to region 0 once band 0 is done
    auto stage_band = [&](int band, float* stage) {
      if (band == 1 || band == 2) return;
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        if (band == 0 ? mi >= 6 : mi < 6) continue;
        float* rg = stage + ((mi >> 1) % 3) * 32 * LDS_ST;
#pragma unroll
        for (int nj = 0; nj < NQ; ++nj)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            rg[((mi & 1) * 16 + lg * 4 + r) * LDS_ST + 96 * wq + 16 * nj + lr] = acc2[mi][nj][r];
      }
    };
    rowln_fast_epilogue_impl<NCOL, 3, true>(p, stage_band, h4, smem, RowsLinear{m0}, fdiv(m0, p.rows_per_mod, inv_rpm),
                                            inv_rpm);
  }
}

// The split MLP's second pass: v = sum of the nsplit fc2 partials (split order), then exactly
// the row-LN epilogue's arithmetic: h += gate * (v + b2), LayerNorm + adaLN modulate -> xn.
// One wave per row, lane = columns 2 lane + 128 e.
// Diagnostic build (MDG_DIAG_ORDER=1, tools/gpu_lane_race.sh "order"): launch-order check of
// the split-MLP reduction -> next layer's fused spatial kernel hand-off.  Per xn buffer (hashed
// slot) the reduction's blocks count their completion after a release fence, and every block of
// the spatial kernel, before its first load, compares that count with the number the stream
// order implies (spatial launch j of a lane follows j reductions of (M + 3) / 4 blocks).
#ifndef MDG_DIAG_ORDER
#define MDG_DIAG_ORDER 0
#endif
#if MDG_DIAG_ORDER
struct OrderSlot {
  unsigned long long key;
  unsigned red, spa, err, worst;
};
__device__ OrderSlot g_order[61];
__device__ __forceinline__ OrderSlot& order_slot(const void* xn) {
  return g_order[((uintptr_t)xn >> 8) % 61];
}
#endif

template <int NCOL>
__global__ __launch_bounds__(256) void mlp_split_reduce_kernel(const mdg_gemm_desc p, const float* __restrict__ part,
                                                               int nsplit) {
#pragma clang fp contract(off)
  constexpr int NE = NCOL / 128;
  const int lane = threadIdx.x & 63, m = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int M = p.M;
#if MDG_DIAG_ORDER
  struct Done {
    const mdg_gemm_desc& p;
    __device__ ~Done() {
      if (!p.xn_out) return;
      __syncthreads();
      if (threadIdx.x == 0) {
        __threadfence();
        OrderSlot& o = order_slot(p.xn_out);
        o.key = (unsigned long long)(uintptr_t)p.xn_out;
        atomicAdd(&o.red, 1u);
      }
    }
  } done_{p};
#endif
  if (m >= M) return;
  const size_t b = (size_t)(m / p.rows_per_mod);
  float2 v[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) v[e] = make_float2(0.f, 0.f);
  for (int s = 0; s < nsplit; ++s)
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const float2 t = *reinterpret_cast<const float2*>(part + ((size_t)s * M + m) * NCOL + 2 * lane + 128 * e);
      v[e].x += t.x;
      v[e].y += t.y;
    }
  float2 h[NE];
  float sum = 0.f;
  float* hr = p.resid + (size_t)m * p.ldr;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int k = 2 * lane + 128 * e;
    const float2 hv = *reinterpret_cast<const float2*>(hr + k);
    const float2 bb = p.bias ? *reinterpret_cast<const float2*>(p.bias + k) : make_float2(0.f, 0.f);
    const float2 gg = p.gate ? *reinterpret_cast<const float2*>(p.gate + b * p.mod_stride + p.gate_off + k)
                             : make_float2(1.f, 1.f);
    h[e].x = hv.x + gg.x * (v[e].x + bb.x);
    h[e].y = hv.y + gg.y * (v[e].y + bb.y);
    sum += h[e].x + h[e].y;
    *reinterpret_cast<float2*>(hr + k) = h[e];
  }
  if (!p.xn_out) return;
  const float invN = 1.0f / (float)NCOL;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
  const float mean = sum * invN;
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const float a0 = h[e].x - mean, a1 = h[e].y - mean;
    ss += a0 * a0 + a1 * a1;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const float rs = 1.0f / sqrtf(ss * invN + p.ln_eps);
  const float* mr = p.xn_mods + b * p.xn_mod_stride;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int k = 2 * lane + 128 * e;
    const float2 xs = *reinterpret_cast<const float2*>(mr + p.xn_scale_off + k);
    const float2 xh = *reinterpret_cast<const float2*>(mr + p.xn_shift_off + k);
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    bf16x2 pr;
    pr[0] = (bf16_t)((h[e].x - mean) * rs * (1.0f + xs.x) + xh.x);
    pr[1] = (bf16_t)((h[e].y - mean) * rs * (1.0f + xs.y) + xh.y);
    *reinterpret_cast<bf16x2*>(reinterpret_cast<bf16_t*>(p.xn_out) + (size_t)m * NCOL + k) = pr;
  }
}

// The split passes' reduction, round 5: a row per half-wave (4 consecutive columns per lane,
// 16-B loads: half the memory instructions of the float2 form), the residual / bias / gate rows
// issued before the partials, the partials unrolled 4 deep.  The partial sum runs in split order
// as before; the gated residual, the row statistics and the LN arithmetic are the row-LN fast
// epilogue's (rowln_fast_epilogue_impl), so a small-M step rounds h and xn as the one-pass
// launches do given the same fc2 / out_proj sums.
template <int NCOL>
__global__ __launch_bounds__(256) void split_reduce_rows_kernel(const mdg_gemm_desc p, const float* __restrict__ part,
                                                                int nsplit) {
#pragma clang fp contract(off)
  constexpr int NE = NCOL / 128;
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int m = blockIdx.x * 8 + (threadIdx.x >> 5);  // 8 rows per block, one per half-wave
  const int M = p.M;
  const int mm = min(m, M - 1);
  const size_t b = (size_t)(mm / p.rows_per_mod);
  float4 h4[NE], b4[NE], g4[NE];
  float* hr = p.resid + (size_t)mm * p.ldr;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int k = 4 * hl + 128 * e;
    h4[e] = *reinterpret_cast<const float4*>(hr + k);
    b4[e] = p.bias ? *reinterpret_cast<const float4*>(p.bias + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    g4[e] = p.gate ? *reinterpret_cast<const float4*>(p.gate + b * p.mod_stride + p.gate_off + k)
                   : make_float4(1.f, 1.f, 1.f, 1.f);
  }
  float4 v[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) v[e] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* pr0 = part + (size_t)mm * NCOL + 4 * hl;
#pragma unroll 4
  for (int sp = 0; sp < nsplit; ++sp)
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const float4 t = *reinterpret_cast<const float4*>(pr0 + (size_t)sp * M * NCOL + 128 * e);
      v[e].x += t.x;
      v[e].y += t.y;
      v[e].z += t.z;
      v[e].w += t.w;
    }
  float sacc = 0.f;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    float4& h = h4[e];
    h.x += g4[e].x * (v[e].x + b4[e].x);
    h.y += g4[e].y * (v[e].y + b4[e].y);
    h.z += g4[e].z * (v[e].z + b4[e].z);
    h.w += g4[e].w * (v[e].w + b4[e].w);
    sacc += (h.x + h.y) + (h.z + h.w);
  }
  if (m < M) {
#pragma unroll
    for (int e = 0; e < NE; ++e) *reinterpret_cast<float4*>(hr + 4 * hl + 128 * e) = h4[e];
  }
  if (!p.xn_out) return;
  const float invN = 1.0f / (float)NCOL;
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) sacc += __shfl_xor(sacc, o, 64);
  const float mean = sacc * invN;
  float t = 0.f;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const float4 h = h4[e];
    const float a0 = h.x - mean, a1 = h.y - mean, a2 = h.z - mean, a3 = h.w - mean;
    t += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
  }
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) t += __shfl_xor(t, o, 64);
  const float rs = 1.0f / sqrtf(t * invN + p.ln_eps);
  if (m >= M) return;
  const float* mr = p.xn_mods + b * p.xn_mod_stride;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int k = 4 * hl + 128 * e;
    const float4 xs = *reinterpret_cast<const float4*>(mr + p.xn_scale_off + k);
    const float4 xh = *reinterpret_cast<const float4*>(mr + p.xn_shift_off + k);
    const float4 h = h4[e];
    st4<bf16_t>(reinterpret_cast<bf16_t*>(p.xn_out) + (size_t)m * NCOL + k, (h.x - mean) * rs * (1.0f + xs.x) + xh.x,
                (h.y - mean) * rs * (1.0f + xs.y) + xh.y, (h.z - mean) * rs * (1.0f + xs.z) + xh.z,
                (h.w - mean) * rs * (1.0f + xs.w) + xh.w);
  }
}

// the split passes' reduction launch (MDG_SPLIT_REDUCE=0 or a diagnostic ORDER build: the
// round-3 float2 kernel)
static hipError_t launch_split_reduce(const mdg_gemm_desc& p, const float* part, int S, hipStream_t s) {
  static const bool rows4 = [] {
    const char* e = getenv("MDG_SPLIT_REDUCE");
    return !(e && e[0] == '0');
  }();
  if (rows4 && !MDG_DIAG_ORDER && p.ldr % 4 == 0 && (!p.xn_out || (p.xn_mod_stride % 4 == 0 && p.xn_scale_off % 4 == 0 &&
                                                                  p.xn_shift_off % 4 == 0)) &&
      (!p.gate || (p.mod_stride % 4 == 0 && p.gate_off % 4 == 0)))
    hipLaunchKernelGGL((split_reduce_rows_kernel<384>), dim3((p.M + 7) / 8), dim3(256), 0, s, p, part, S);
  else
    hipLaunchKernelGGL((mlp_split_reduce_kernel<384>), dim3((p.M + 3) / 4), dim3(256), 0, s, p, part, S);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// FinalLayer + Euler update of the bf16 denoise step (layers.py:58-75 then
// integrators.py:106-113): v = xn . W^T + b, x_out = x_in + dt * v for latent <= 32 columns.
// The generic 64x32 GEMM took ~35 us for 25 MB (six barrier-separated register-staged
// K-steps per 64 rows: latency, not bandwidth).  Here one wave owns 16 token rows and loads
// them straight into its MFMA A fragments, every K at once (one HBM round trip per wave);
// W^T (32 x C, pad rows 0) is staged once per block in LDS (rows padded by 16 B, so the
// 16-lane fragment reads hit distinct bank slots), issued beside the row loads.  The
// v_mfma_f32_16x16x32_bf16 chain runs in ascending K like the generic GEMM's, so v is equal
// to it bit for bit.
template <int KC, bool LDSW>  // LDSW = false: B fragments straight from global memory (L2)
__global__ __launch_bounds__(256) void final_euler_kernel(const mdg_gemm_desc p) {
  constexpr int KS = KC / 32, LDW = KC + 8, WCH = 32 * KC / 8;  // 16-B chunks of W
  constexpr int WPT = (WCH + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16_t Ws[LDSW ? 32 * LDW : 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int M = p.M;
  const int m0 = blockIdx.x * 64 + wave * 16;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A) + (size_t)min(m0 + lr, M - 1) * p.lda + 8 * lg;
  bf16x8 a[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) a[ks] = *reinterpret_cast<const bf16x8*>(A + 32 * ks);
  const bf16_t* W = reinterpret_cast<const bf16_t*>(p.W);
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  if constexpr (LDSW) {
    u32x4 wr[WPT];
#pragma unroll
    for (int u = 0; u < WPT; ++u) {
      const int c = tid + 256 * u;
      if (c < WCH) wr[u] = *reinterpret_cast<const u32x4*>(W + (size_t)(c / (KC / 8)) * p.ldw + 8 * (c % (KC / 8)));
    }
#pragma unroll
    for (int u = 0; u < WPT; ++u) {
      const int c = tid + 256 * u;
      if (c < WCH) *reinterpret_cast<u32x4*>(Ws + (c / (KC / 8)) * LDW + 8 * (c % (KC / 8))) = wr[u];
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(Ws + (16 * nt + lr) * LDW + 32 * ks + 8 * lg);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], b, acc[nt], 0, 0, 0);
      }
    }
  } else {
    const bf16_t* Wl = W + (size_t)lr * p.ldw + 8 * lg;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(Wl + (size_t)16 * nt * p.ldw + 32 * ks);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], b, acc[nt], 0, 0, 0);
      }
    }
  }
  // lane: rows 4 lg + r, column 16 nt + lr
  float* xo = reinterpret_cast<float*>(p.out);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n = 16 * nt + lr;
    if (n >= p.n_valid) continue;
    const float bn = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + 4 * lg + r;
      if (m >= M) continue;
      const size_t o = (size_t)m * p.ldo + n;
      const float v = acc[nt][r] + bn;
      if (p.v_out) p.v_out[o] = v;
      if (xo) xo[o] = euler_update(p.x_in[o], p.dt, v);
    }
  }
}

// bf16 EULER GEMM with plain A, latent <= 32 (N = 32 with the pad rows), C in {128 .. 512}
// (mdg_gemm routes such a descriptor here; MDG_FAST_FINAL=0 keeps the generic GEMM)
bool final_euler_supported(const mdg_gemm_desc& p) {
  return p.dtype == MDG_BF16 && p.a_mode == MDG_A_PLAIN && p.epi == MDG_EPI_EULER && p.N == 32 && p.n_valid <= 32 &&
         (p.K == 128 || p.K == 256 || p.K == 384 || p.K == 512) && p.lda % 8 == 0 && p.ldw % 8 == 0 && p.M > 0 &&
         (p.out || p.v_out);
}

hipError_t final_euler_launch(const mdg_gemm_desc& p, hipStream_t s) {
  const dim3 grid((p.M + 63) / 64);
  // W^T staged in LDS: 9.7 us standalone at M = 32000 (2.6 TB/s) vs 13.5 us with the B
  // fragments read from L2 (MDG_FINAL_LDSW=0) and 15.7 us for the generic 64x32 GEMM
  static const bool ldsw = [] {
    const char* e = getenv("MDG_FINAL_LDSW");
    return !(e && e[0] == '0');
  }();
#define MDG_FE(KC_)                                                                                      \
  if (ldsw) hipLaunchKernelGGL((final_euler_kernel<KC_, true>), grid, dim3(256), 0, s, p);              \
  else hipLaunchKernelGGL((final_euler_kernel<KC_, false>), grid, dim3(256), 0, s, p);
  switch (p.K) {
    case 128: MDG_FE(128) break;
    case 256: MDG_FE(256) break;
    case 384: MDG_FE(384) break;
    default: MDG_FE(512) break;
  }
#undef MDG_FE
  return hipGetLastError();
}

// The fused MLP's shape envelope: bf16, C = 384, F % 128 == 0, fc1 = PLAIN STORE + GELU, fc2 =
// PLAIN GATE_RES whose tiles span <= 2 adaLN entries (rows_per_mod >= 128), no training outputs.
bool mlp_fused_supported(const mdg_gemm_desc& f1, const mdg_gemm_desc& f2) {
  return f1.dtype == MDG_BF16 && f2.dtype == MDG_BF16 && f1.a_mode == MDG_A_PLAIN && f2.a_mode == MDG_A_PLAIN &&
         f1.epi == MDG_EPI_STORE && f1.act == MDG_ACT_GELU && f2.epi == MDG_EPI_GATE_RES && f1.K == 384 &&
         f2.N == 384 && f1.N == f2.K && f1.N % kMlpHC == 0 && f1.N >= kMlpHC && f1.M == f2.M && f1.M > 0 &&
         f2.rows_per_mod >= 128 && f2.resid && !f2.resid_in && !f2.aux && !f1.aux && f1.lda % 8 == 0 &&
         f1.ldw % 8 == 0 && f2.ldw % 8 == 0 && f2.ldr % 4 == 0 && (!f2.xn_out || f2.xn_mods) && mlp_smem(f1.N) <= 160 * 1024;
}

// Hidden-chunk split for small M (< 64 row tiles, a quarter of the CUs: each block would stream
// all of W1 and W2 for one tile): the largest divisor of the chunk count that keeps the grid
// within the cap below; 1 = no split.  MDG_MLP_SPLIT=0 disables it (A/B knob).
int mlp_split_factor(int M, int F) {
  static const bool on = [] {
    const char* e = getenv("MDG_MLP_SPLIT");
    return !(e && e[0] == '0');
  }();
  // MDG_MLP_SPLIT_BLOCKS: grid cap (default 240).  Measured (round 2): 160 gives a two-lane TPS
  // window (25 tiles per lane) 6 pieces instead of 12, +12.7 %, and a B = 1 window 4 instead of
  // 6, -3.6 %; 240 gives 6 and 6.  (240 was held back in round 2 by a rare concurrent-lane
  // divergence; its cause was the fused spatial kernel's misaligned RoPE loads, fixed in round 3,
  // DESIGN.md §4.)
  static const int cap = [] {
    const char* e = getenv("MDG_MLP_SPLIT_BLOCKS");
    return e ? atoi(e) : 240;
  }();
  const int tiles = (M + 127) / 128, nch = F / kMlpHC;
  if (!on || tiles >= 64 || nch < 2) return 1;
  int best = 1;
  for (int d = 2; d <= nch; ++d)
    if (nch % d == 0 && tiles * d <= cap) best = d;
  return best;
}

// MDG_MLP_SPLIT_VST=0: the small-M split MLP stages its operands by LDS-DMA (A/B knob)
static bool mlp_split_vst_on() {
  static const bool on = [] {
    const char* e = getenv("MDG_MLP_SPLIT_VST");
    return !(e && e[0] == '0');
  }();
  return on;
}

// The one-pass (large-M) fused MLP kernel, MDG_MLP_WS: 2 (default, round 6) mlp_ws2_kernel;
// 0 the lock-step mlp_rowln_kernel (round 2; then MDG_MLP_HC=256 selects its 256-wide-chunk
// form); 1 round 3's wave-specialised kernel (measured 168 vs 130 us at M = 32 000: each phase's
// 48 KiB ring slot is issued only one phase ahead of an LDS-DMA fill that takes ~1.1 us, and its
// 65 spilled VGPRs).  All three give bit-identical h and xn.
static int mlp_ws_mode() {
  static const int v = [] {
    const char* e = getenv("MDG_MLP_WS");
    return e ? atoi(e) : 2;
  }();
  return v;
}

// MDG_MLP_HC=256: the one-pass fused MLP on 256-wide hidden chunks with 64 x 64 fc1 wave tiles
// (mlp_rowln256_kernel, round 6; A/B knob)
static bool mlp_hc256_on() {
  static const bool on = [] {
    const char* e = getenv("MDG_MLP_HC");
    return e && atoi(e) == 256;
  }();
  return on;
}

// The out_proj prologue's envelope: r is the fast row-LN path's GEMM (bf16 PLAIN, K = N = 384,
// rows_per_mod >= 128) whose h and xn outputs are exactly the MLP's residual and fc1 input, on
// the MLP's rows, and the MLP runs in its one-pass form.
bool mlp_pre_supported(const mdg_gemm_desc& r, const mdg_gemm_desc& f1, const mdg_gemm_desc& f2) {
  return mlp_fused_supported(f1, f2) && mlp_split_factor(f1.M, f1.N) == 1 && r.dtype == MDG_BF16 &&
         r.a_mode == MDG_A_PLAIN && r.epi == MDG_EPI_GATE_RES && r.N == 384 && r.K == 384 && r.M == f1.M &&
         r.rows_per_mod == f2.rows_per_mod && r.resid == f2.resid && r.ldr == f2.ldr && !r.resid_in && !r.aux &&
         r.xn_out && r.xn_out == f1.A && f1.lda == 384 && r.xn_mods && r.A && r.W && r.lda % 8 == 0 && r.ldw % 8 == 0;
}

// ---------------------------------------------------------------------------------------
// Fused MLP, wave-specialised, round 6 (the default one-pass form; large M, one 128-token tile
// per block).  Waves 0-3 ("P") produce H = GELU(xn W1^T + b1) for 32 tokens each, waves 4-7 ("Q")
// consume it: acc2 += H W2^T for all 128 tokens x 96 outputs each, then the row-LN epilogue.
// Wave w and w + 4 share a SIMD, so one wave's matrix work issues beside the other's vector work.
// Against the round-3 form (mlp_ws_kernel: 65 spilled VGPRs, a 2-slot ring issued one phase
// ahead, the whole chunk's GELU in one phase):
//   * the W2 fragments go straight from L2 to the Q waves' registers by buffer loads (each Q wave
//     reads its own 96 rows of W2 once per tile), one K-step ahead; LDS holds a 3-slot ring of
//     W1 slices (24 KiB each, buffer-to-LDS loads three phases ahead), the double-buffered H
//     (2 x 32 KiB) and b1;
//   * a P wave keeps its 32 xn rows in registers (the fc1 B operand, loaded once) and computes a
//     chunk as two 64-hidden halves over two phases each (6 K-steps of 32 per phase); each half's
//     GELU (packed fp32 math) runs inside the next-but-one phase's K-steps, beside the MFMAs of
//     the other half: half A's in phase 2 of the same chunk, half B's in phase 0 of the next.
//     Q's fc2 steps over H(c - 1) read hidden 0-63 in phases 0-1 of chunk c and 64-127 in
//     phases 2-3.
// Phases: 4 (NCH + 1), one block barrier each.  K orders are the lock-step kernel's (fc1 ascending
// per hidden unit, fc2 ascending over the hidden units) and the GELU is gelu_fast's arithmetic,
// so h and xn are bit-identical to it.  Measured: 115-117 vs 128-129 us standalone at
// M = 32 000, 99 vs 107 us on the bench's activations.
constexpr int kWs2Img = 64 * 32, kWs2Slot = 6 * kWs2Img;  // bf16 elements: 6 K-step images of 64 W1 rows

// GELU of hidden block 16 gm .. + 15 of the chunk held in acc (16 units x 2 token tiles of a P
// wave) + the block's b1 -> bf16 rows of H (16-B chunk c of row r at c ^ (r & 15))
__device__ __forceinline__ void ws2_gelu_block(f32x4 (&acc)[2], const f32x4 b1v, bf16_t* Hs, int gm, int wq, int lr,
                                               int lg) {
  constexpr int HC = 128;
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const int hb = 16 * gm + 4 * lg, tok = 32 * wq + 16 * ni + lr;
    bf16x4 o;
#pragma unroll
    for (int r = 0; r < 4; r += 2) {  // packed pairs (gelu_fast2: bit-identical to gelu_fast)
      const f32x2v g = gelu_fast2(f32x2v{acc[ni][r], acc[ni][r + 1]} + f32x2v{b1v[r], b1v[r + 1]});
      o[r] = (bf16_t)g.x;
      o[r + 1] = (bf16_t)g.y;
    }
    *reinterpret_cast<bf16x4*>(Hs + tok * HC + (((hb >> 3) ^ (tok & 15)) * 8) + (hb & 7)) = o;
    acc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

template <int NCOL>
__global__ __launch_bounds__(kWsThreads, 1) void mlp_ws2_kernel(const MlpArgs args) {
  static_assert(NCOL == 384, "Q waves own 96 output columns each");
  constexpr int BM = 128, HC = 128, BK = 32, NQ = 6, LDS_ST = NCOL + 4, NSLOT = 3;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Hb = reinterpret_cast<bf16_t*>(smem);  // [2][BM][HC]: 16-B chunk c of row r at c ^ (r & 15)
  bf16_t* ring = Hb + 2 * BM * HC;               // [NSLOT][kWs2Slot]
  float* b1s = reinterpret_cast<float*>(ring + NSLOT * kWs2Slot);  // [F] (written before the first barrier)
  const mdg_gemm_desc& q = args.f1;              // xn, W1, b1
  const mdg_gemm_desc& p = args.f2;              // W2, b2 and the row-LN epilogue
  // (wave index through readfirstlane: the role branch and the buffer-load scalar offsets are
  // then known wave-uniform; otherwise every buffer load becomes a waterfall loop)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), wq = wave & 3;
  const bool isP = wave < 4;
  const int lr = lane & 15, lg = lane >> 4;
  const int M = p.M, F = p.K, NCH = F / HC, NPH = 4 * (NCH + 1);
  const int nwg = (M + BM - 1) / BM;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int m0 = ((xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc) * BM;
  const bf16_t* X = reinterpret_cast<const bf16_t*>(q.A);
  const bf16_t* W1 = reinterpret_cast<const bf16_t*>(q.W);
  const bf16_t* W2 = reinterpret_cast<const bf16_t*>(p.W);
  const int ch = (lg ^ ((-(lr >> 2)) & 3)) * 8;  // fragment rows are lr mod 16
  const float inv_rpm = 1.0f / (float)p.rows_per_mod;
  float4 h4[2][NCOL / 128];
  for (int i = tid; i < F; i += kWsThreads) b1s[i] = q.bias ? q.bias[i] : 0.f;
  if (isP) {
    // W1 pieces of phase ph (chunk ph / 4, half (ph & 3) >> 1, K range 192 (ph & 1)): piece
    // id = 6 wq + i -> image k3 = id / 4 (K-step), row block id % 4 (16 of the half's 64 rows)
    const int prow = lane >> 2, pch = lane & 3;
    const __amdgpu_buffer_rsrc_t w1rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)W1, 0, F * q.ldw * (int)sizeof(bf16_t), 0x00020000);
    const int w1lane = (prow * q.ldw + ((pch ^ ((-(prow >> 2)) & 3)) * 8)) * (int)sizeof(bf16_t);
    auto issue = [&](int ph) {  // buffer loads: the piece offsets are scalar, no address VGPRs
      if (ph >= 4 * NCH) return;
      bf16_t* sl = ring + (ph % NSLOT) * kWs2Slot;
      const int base = ((ph >> 2) * HC + 64 * ((ph & 3) >> 1)) * q.ldw + 192 * (ph & 1);
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int id = 6 * wq + i;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            w1rs, (lds_ptr_t)(sl + (id >> 2) * kWs2Img + 16 * (id & 3) * BK), 16, w1lane,
            (base + 32 * (id >> 2) + 16 * (id & 3) * q.ldw) * (int)sizeof(bf16_t), 0, 0);
      }
    };
    // the wave's 32 xn rows as the fc1 B operand: xf[k-step][token tile]
    bf16x8 xf[12][2];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const bf16_t* xr = X + (size_t)min(m0 + 32 * wq + 16 * ni + lr, M - 1) * q.lda + 8 * lg;
#pragma unroll
      for (int kk = 0; kk < 12; ++kk) xf[kk][ni] = *reinterpret_cast<const bf16x8*>(xr + 32 * kk);
    }
    f32x4 acc1[8][2];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) acc1[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    issue(0);
    issue(1);
    issue(2);
    // one P phase: 6 K-steps over the slot's 64 hidden rows (half HB, K half KH), 48 MFMAs.  The
    // next K-step's 4 fragments are read while this one's 8 MFMAs issue (two register sets).
    // GJ >= 0: the GELU of hidden half GJ of chunk cg (not the half accumulating here) runs one
    // 16-unit block per K-step (K-steps 0-3) beside the MFMAs, so the wave's vector and matrix
    // work overlap instead of following each other.
    auto fc1_phase = [&](auto HB, auto KH, auto GJ, int ph, int cg) __attribute__((always_inline)) {
      constexpr int hb0 = 4 * decltype(HB)::value, kk0 = 6 * decltype(KH)::value, gj = decltype(GJ)::value;
      static_assert(gj != decltype(HB)::value, "the GELU half is not the one accumulating");
      const bf16_t* img = ring + (ph % NSLOT) * kWs2Slot + lr * BK + ch;
      bf16_t* Hs = Hb + (cg & 1) * BM * HC;
      f32x4 b1v[4];
      if constexpr (gj >= 0) {
#pragma unroll
        for (int m = 0; m < 4; ++m) b1v[m] = *reinterpret_cast<const f32x4*>(b1s + cg * HC + 16 * (4 * gj + m) + 4 * lg);
      }
      bf16x8 fa[2][4];
#pragma unroll
      for (int m = 0; m < 4; ++m) fa[0][m] = *reinterpret_cast<const bf16x8*>(img + 16 * m * BK);
#pragma unroll
      for (int k3 = 0; k3 < 6; ++k3) {
        if (k3 + 1 < 6) {
#pragma unroll
          for (int m = 0; m < 4; ++m)
            fa[(k3 + 1) & 1][m] = *reinterpret_cast<const bf16x8*>(img + (k3 + 1) * kWs2Img + 16 * m * BK);
        }
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc1[hb0 + m][ni] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[k3 & 1][m], xf[kk0 + k3][ni], acc1[hb0 + m][ni], 0, 0, 0);
        if constexpr (gj >= 0) {
          if (k3 < 4) ws2_gelu_block(acc1[4 * gj + k3], b1v[k3], Hs, 4 * gj + k3, wq, lr, lg);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // phase end: this wave's pieces of phase ph + 1 landed (the outstanding ones are phase ph + 1's
    // and ph + 2's: vmcnt(6) leaves the newer six in flight), LDS ops retired, barrier, then phase
    // ph + 3's pieces into the slot phase ph used (every wave's reads of it retired before the barrier)
    auto phase_end = [&](int ph) __attribute__((always_inline)) {
      if (ph + 2 < 4 * NCH) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(ph + 3);
    };
    // (phase 0's pieces landed before the first barrier; 1's and 2's in flight)
    asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    using In = std::integral_constant<int, -1>;
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    for (int c = 0; c < NCH; ++c) {
      const int ph = 4 * c;
      if (c == 0) fc1_phase(I0{}, I0{}, In{}, ph, 0);
      else fc1_phase(I0{}, I0{}, I1{}, ph, c - 1);  // + half B's GELU of chunk c - 1
      phase_end(ph);
      fc1_phase(I0{}, I1{}, In{}, ph + 1, c);
      phase_end(ph + 1);
      fc1_phase(I1{}, I0{}, I0{}, ph + 2, c);  // + half A's GELU of chunk c
      phase_end(ph + 2);
      fc1_phase(I1{}, I1{}, In{}, ph + 3, c);
      phase_end(ph + 3);
    }
    {  // half B's GELU of the last chunk, then the Q waves' last chunk (barriers only)
      bf16_t* Hs = Hb + ((NCH - 1) & 1) * BM * HC;
#pragma unroll
      for (int m = 4; m < 8; ++m)
        ws2_gelu_block(acc1[m], *reinterpret_cast<const f32x4*>(b1s + (NCH - 1) * HC + 16 * m + 4 * lg), Hs, m, wq,
                       lr, lg);
    }
    for (int ph = 4 * NCH; ph < NPH; ++ph) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    auto no_stage = [&](int, float*) {};
    rowln_fast_epilogue_impl<NCOL, 3, true>(p, no_stage, h4, smem, RowsLinear{m0}, fdiv(m0, p.rows_per_mod, inv_rpm),
                                            inv_rpm);
  } else {
    f32x4 acc2[8][NQ];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int nj = 0; nj < NQ; ++nj) acc2[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
    // W2 B fragments: output row 96 wq + 16 nj + lr, hidden 8 lg .. + 7 of the K-step
    // (buffer loads: one lane offset in a VGPR, the K-step / fragment offset in an SGPR, so the six
    // fragment streams cost no address registers beside the 192 accumulators)
    const __amdgpu_buffer_rsrc_t w2rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)W2, 0, NCOL * p.ldw * (int)sizeof(bf16_t), 0x00020000);
    const int w2lane = ((96 * wq + lr) * p.ldw + 8 * lg) * (int)sizeof(bf16_t);
    auto wfrag = [&](int c, int kb, int nj) __attribute__((always_inline)) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
          w2rs, w2lane, (c * HC + BK * kb + 16 * nj * p.ldw) * (int)sizeof(bf16_t), 0);
      return __builtin_bit_cast(bf16x8, v);
    };
    bf16x8 bw[NQ];
#pragma unroll
    for (int nj = 0; nj < NQ; ++nj) bw[nj] = wfrag(0, 0, nj);
    // P's first chunk: 4 phases without fc2 work (the barriers only)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int ph = 0; ph < 4; ++ph) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    for (int c = 1; c <= NCH; ++c) {
      const bf16_t* Hs = Hb + ((c - 1) & 1) * BM * HC;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        // (no blanket vmcnt wait here: the compiler waits for each W2 fragment right before its
        // first MFMA, so the K-step starts as soon as fragment 0 has landed; +1 % in the bench)
        const int nc = kb < 3 ? c - 1 : c, nkb = (kb + 1) & 3;
        const bool more = kb < 3 || c < NCH;
        // two halves of 4 token tiles; fragment nj is reloaded for the next K-step right after
        // its last MFMA of the second half (no second fragment set beside the 192 accumulators;
        // measured 3 % faster than reloading all six after the K-step)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          bf16x8 a[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = 16 * (4 * hf + i) + lr;
            a[i] = *reinterpret_cast<const bf16x8*>(Hs + row * HC + (((kb * 4 + lg) ^ (row & 15)) * 8));
          }
#pragma unroll
          for (int nj = 0; nj < NQ; ++nj) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc2[4 * hf + i][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bw[nj], acc2[4 * hf + i][nj], 0, 0, 0);
            if (hf == 1 && more) bw[nj] = wfrag(nc, nkb, nj);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
    // band b = accumulator rows 16 mi + 4 lg + r with mi in {2b, 2b+1}; columns 96 wq + 16 nj + lr.
    // Bands 0-2 go to stage regions 0-2 at band 0 (144 accumulator VGPRs freed before the row
    // work), band 3 to region 0 once band 0 is done
    auto stage_band = [&](int band, float* stage) {
      if (band == 1 || band == 2) return;
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        if (band == 0 ? mi >= 6 : mi < 6) continue;
        float* rg = stage + ((mi >> 1) % 3) * 32 * LDS_ST;
#pragma unroll
        for (int nj = 0; nj < NQ; ++nj)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            rg[((mi & 1) * 16 + lg * 4 + r) * LDS_ST + 96 * wq + 16 * nj + lr] = acc2[mi][nj][r];
      }
    };
    rowln_fast_epilogue_impl<NCOL, 3, true>(p, stage_band, h4, smem, RowsLinear{m0}, fdiv(m0, p.rows_per_mod, inv_rpm),
                                            inv_rpm);
  }
}

hipError_t mlp_fused_launch(const mdg_gemm_desc& f1, const mdg_gemm_desc& f2, hipStream_t s, float* part,
                            const mdg_gemm_desc* pre) {
  static bool attr_set = false;
  if (!attr_set) {
    for (const void* k : {reinterpret_cast<const void*>(&mlp_rowln_kernel<384, false>),
                          reinterpret_cast<const void*>(&mlp_rowln_kernel<384, true>),
                          reinterpret_cast<const void*>(&mlp_rowln_kernel<384, false, true>),
                          reinterpret_cast<const void*>(&mlp_rowln_kernel<384, true, false, true>),
                          reinterpret_cast<const void*>(&mlp_ws_kernel<384>),
                          reinterpret_cast<const void*>(&mlp_rowln256_kernel<384>),
                          reinterpret_cast<const void*>(&mlp_ws2_kernel<384>)}) {
      hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
  MlpArgs a;
  a.f1 = f1;
  a.f2 = f2;
  a.part = part;
  a.nsplit = part ? mlp_split_factor(f1.M, f1.N) : 1;
  const int tiles = (f1.M + 127) / 128;
  if (pre) {
    if (!mlp_pre_supported(*pre, f1, f2)) return hipErrorInvalidValue;
    a.r = *pre;
    hipLaunchKernelGGL((mlp_rowln_kernel<384, false, true>), dim3(tiles), dim3(kMlpThreads), mlp_smem(f1.N), s, a);
    return hipGetLastError();
  }
  if (a.nsplit > 1) {
    if (mlp_split_vst_on())
      hipLaunchKernelGGL((mlp_rowln_kernel<384, true, false, true>), dim3(tiles, a.nsplit), dim3(kMlpThreads),
                         mlp_smem(f1.N, true), s, a);
    else
      hipLaunchKernelGGL((mlp_rowln_kernel<384, true>), dim3(tiles, a.nsplit), dim3(kMlpThreads), mlp_smem(f1.N), s, a);
    if (hipError_t e = hipGetLastError()) return e;
    return launch_split_reduce(f2, (const float*)part, a.nsplit, s);
  }
  // (H 64 KiB + the W1 ring 72 KiB + b1: F <= 6 144 for the wave-specialised kernel)
  if (mlp_ws_mode() == 2 && (size_t)2 * 128 * 128 * 2 + (size_t)3 * kWs2Slot * 2 + (size_t)f1.N * 4 <= 160 * 1024) {
    hipLaunchKernelGGL((mlp_ws2_kernel<384>), dim3(tiles), dim3(kWsThreads), 160 * 1024, s, a);
    return hipGetLastError();
  }
  if (mlp_ws_mode() == 1) {
    hipLaunchKernelGGL((mlp_ws_kernel<384>), dim3(tiles), dim3(kWsThreads), kWsSmem, s, a);
    return hipGetLastError();
  }
  if (mlp_hc256_on() && f1.N % kMlp2HC == 0 && mlp2_smem(f1.N) <= 160 * 1024) {
    hipLaunchKernelGGL((mlp_rowln256_kernel<384>), dim3(tiles), dim3(kMlpThreads), mlp2_smem(f1.N), s, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((mlp_rowln_kernel<384, false>), dim3(tiles), dim3(kMlpThreads), mlp_smem(f1.N), s, a);
  return hipGetLastError();
}

// Split-K row-LN GEMM for small M (the out_proj launches of a B = 1 window: 32 row tiles):
// S = the MLP's split factor (a divisor of the 12 K-steps), fp32 partials in `part` ([S][M][384]), then
// the split MLP's reduction pass (sum, + bias, gated residual, LN + modulate -> xn).  Same
// envelope as the fast row-LN path: bf16 PLAIN, K = N = 384, rows_per_mod >= 128, xn out.
bool rowln_splitk_supported(const mdg_gemm_desc& r, int S) {
  return S > 1 && (384 / 32) % S == 0 && r.dtype == MDG_BF16 && r.a_mode == MDG_A_PLAIN &&
         r.epi == MDG_EPI_GATE_RES && r.N == 384 && r.K == 384 && r.rows_per_mod >= 128 && r.resid && !r.resid_in &&
         !r.aux && r.xn_out && r.xn_mods && r.lda % 8 == 0 && r.ldw % 8 == 0 && r.ldr % 4 == 0;
}

hipError_t rowln_splitk_launch(const mdg_gemm_desc& r, hipStream_t s, float* part, int S) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_rowln_kernel<384, 128, true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)rowln_smem<384, 128>());
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  mdg_gemm_desc rp = r;
  rp.aux = part;
  hipLaunchKernelGGL((gemm_rowln_kernel<384, 128, true>), dim3((r.M + 127) / 128, S), dim3(kRowThreads),
                     (rowln_smem<384, 128>()), s, rp);
  if (hipError_t e = hipGetLastError()) return e;
  return launch_split_reduce(r, (const float*)part, S, s);
}

// ---------------------------------------------------------------------------------------
// Spatial out_proj + gated residual + temporal LN, then the temporal q|k|v projection, in one
// kernel (latent_model.py:471-477): LN_t(h) never leaves the CU.  Block = 128 token rows, one
// block per CU.  Phase 1 is gemm_rowln_kernel<384, 128> (4-stage ring, fast epilogue) with the
// normalised rows written into LDS as twelve 32-wide K-slice images; each wave then moves its
// 32 token rows x 384 of them into registers (the MFMA B operand for the whole phase).  Phase 2
// streams W_qkv in 9 chunks of 128 output columns x 3 K-steps of 128 through a 4-slot
// global_load_lds ring (counted vmcnt, one barrier per step); wave = 64 output columns x 32
// tokens, computed transposed (q|k|v^T = W . xn^T) so a lane holds 4 consecutive columns of one
// token: + bias, x qscale (q), RoPE at the frame position (q, k), one 8-B store into the packed
// temporal planes.  The K order is the unfused GEMM's, so q|k|v equal it up to the epilogue's
// fp contraction.  LDS: phase-1 ring [0, 128K) | epilogue stage [0, 58K) + xn images [64K, 160K)
// | phase-2 ring [0, 128K) + RoPE rows of the block's tokens + bias [128K, ...).
struct RqArgs {
  mdg_gemm_desc r, q;
  int frames;  // 1: RowsFrames tiles (q.L % 16 == 0, q.T >= 8), 0: RowsLinear
};
constexpr int kRqThreads = 512;
constexpr int kRqSmem = 160 * 1024;

// s_waitcnt vmcnt(n) for a wave-uniform n in {0, 4, 8, 12, 16} (anything else: vmcnt(0))
__device__ __forceinline__ void vm_wait_4x(int n) {
  switch (n) {
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <bool FRAMES>
__global__ __launch_bounds__(kRqThreads, 1) void rowln_qkv_kernel(const RqArgs args) {
  constexpr int NCOL = 384, BM = 128, BK = 32, STAGES = 4, WTN = NCOL / 4, NT = WTN / 16, NE = NCOL / 128;
  constexpr int STAGE = (BM + NCOL) * BK, ATILE = BM * BK, WLD = NCOL / 128;
  constexpr int NCH = 3 * NCOL / 128, KS = NCOL / BK, QSTEPS = NCH * 3, IMG = 128 * BK, QSLOT = 4 * IMG;
  static_assert(STAGES * STAGE * 2 == 131072 && 4 * QSLOT * 2 == 131072, "rings");
  static_assert((32 * (NCOL + 4) + 6 * NCOL) * 4 <= 65536 && KS * BM * BK * 2 + 65536 == kRqSmem, "LDS plan");
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const mdg_gemm_desc& p = args.r;  // out_proj + gated residual + LN_t
  const mdg_gemm_desc& q = args.q;  // temporal q|k|v
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Xs = reinterpret_cast<bf16_t*>(smem + 65536);
  const int D = q.D, half = D >> 1;
  float* Rs = reinterpret_cast<float*>(smem + 131072);  // [BM][D]: cos | sin of each token's pairs
  float* Bq = Rs + BM * D;                               // [3 * NCOL]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int M = p.M;
  const int nlg = q.L / 16, nf = M / q.L;  // (FRAMES) residue groups per frame, frames
  const int nwg = FRAMES ? ((nf + 7) / 8) * nlg : (M + BM - 1) / BM;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  typedef typename std::conditional<FRAMES, RowsFrames, RowsLinear>::type RM;
  RM rows;
  if constexpr (FRAMES) {
    const int fg = tile / nlg;
    rows = RowsFrames{8 * fg, 16 * (tile - fg * nlg), q.L, nf, M};
  } else {
    rows = RowsLinear{tile * BM};
  }
  const int ch = (lg ^ ((-(lr >> 2)) & 3)) * 8;

  // ---------------------------------------------------------------- phase 1: out_proj row-LN
  {
    const int wm = wave / 4, wn = wave % 4;
    const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A);
    const bf16_t* W = reinterpret_cast<const bf16_t*>(p.W);
    const int arow = 16 * wave + (lane >> 2);
    const bf16_t* asrc = A + (size_t)min(rows(arow), M - 1) * p.lda + (((lane & 3) ^ ((-(arow >> 2)) & 3)) * 8);
    const bf16_t* bsrc[WLD];
#pragma unroll
    for (int i = 0; i < WLD; ++i) {
      const int row = 16 * (wave * WLD + i) + (lane >> 2);
      bsrc[i] = W + (size_t)row * p.ldw + (((lane & 3) ^ ((-(row >> 2)) & 3)) * 8);
    }
    auto load = [&](int st, int k0) {
      bf16_t* sa = lds + st * STAGE;
      __builtin_amdgcn_global_load_lds((const void*)(asrc + k0), (lds_ptr_t)(sa + 16 * wave * BK), 16, 0, 0);
#pragma unroll
      for (int i = 0; i < WLD; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + k0), (lds_ptr_t)(sa + ATILE + 16 * (wave * WLD + i) * BK),
                                         16, 0, 0);
    };
    float4 h4[2][NE];
    rowln_load_band<NCOL>(p, rows, 0, h4);
    f32x4 acc[4][NT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int nk = NCOL / BK;
#pragma unroll
    for (int s0 = 0; s0 < STAGES - 1; ++s0) load(s0, s0 * BK);
    for (int kt = 0; kt < nk; ++kt) {
      const int younger = min(STAGES - 2, nk - 1 - kt);
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (1 + WLD)) : "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 + WLD) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring reads retired (see kRingWaitNote)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + STAGES - 1 < nk) load((kt + STAGES - 1) % STAGES, (kt + STAGES - 1) * BK);
      const bf16_t* As = lds + (kt % STAGES) * STAGE;
      const bf16_t* Bs = As + ATILE;
      bf16x8 a[4], b[NT];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + lr) * BK + ch);
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * WTN + j * 16 + lr) * BK + ch);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    const float inv_rpm = 1.0f / (float)p.rows_per_mod;
    rowln_fast_epilogue<NCOL>(p, acc, h4, smem, rows, fdiv(rows(0), p.rows_per_mod, inv_rpm), inv_rpm, Xs);
  }

  // ---------------------------------------------------------------- phase 2: temporal q|k|v
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // xn images complete; the epilogue stage is free
  const int wah = wave >> 2, wat = wave & 3;  // 64 output columns x 32 tokens
  const int T = q.T, L = q.L;
  const float invL = 1.0f / (float)L, invT = 1.0f / (float)T, invD = 1.0f / (float)D;
  // the RoPE rows of the block's tokens and the bias, into registers first (LDS after the xn
  // images are read), issued before the ring so the ring's pieces stay the youngest loads
  constexpr int RMAX = (BM * 48) / kRqThreads, BMAX = (3 * NCOL + kRqThreads - 1) / kRqThreads;
  const int nR = q.rope ? BM * D : 0;
  float rv[RMAX], bv[BMAX];
  // (unpredicated loads of clamped indices: exec-masked ones made the compiler drain vmcnt)
#pragma unroll
  for (int k = 0; k < RMAX; ++k) rv[k] = 0.f;
  if (nR) {
#pragma unroll
    for (int k = 0; k < RMAX; ++k) {
      const int i = min(tid + k * kRqThreads, nR - 1);
      const int tok = fdiv(i, D, invD), j = i - tok * D, hj = j < half ? j : j - half;
      const int m = min(rows(tok), M - 1), ml = fdiv(m, L, invL), t = ml - fdiv(ml, T, invT) * T;
      rv[k] = q.rope[(size_t)((j < half ? 0 : q.rope_rows) + t) * half + hj];
    }
  }
#pragma unroll
  for (int k = 0; k < BMAX; ++k) bv[k] = q.bias ? q.bias[min(tid + k * kRqThreads, 3 * NCOL - 1)] : 0.f;
  const bf16_t* Wq = reinterpret_cast<const bf16_t*>(q.W);
  const int gimg = wave >> 1;
  const int cswz = ((lane & 3) ^ ((-(lane >> 4)) & 3)) * 8;
  int woff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) woff[i] = (16 * (4 * (wave & 1) + i) + (lane >> 2)) * q.ldw + cswz;
  // step s = (chunk s / 3, K rows 128 (s % 3) ..): image g = wave / 2, 16-row pieces 4 (wave & 1) + i
  auto qissue = [&](int s) {
    const int n = s / 3, kk = s - 3 * n;
    bf16_t* sl = lds + (s & 3) * QSLOT + gimg * IMG;
    const bf16_t* base = Wq + (size_t)n * 128 * q.ldw + (4 * kk + gimg) * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(base + woff[i]), (lds_ptr_t)(sl + 16 * (4 * (wave & 1) + i) * BK), 16,
                                       0, 0);
  };
  qissue(0);
  qissue(1);  // slots 0, 1 = the dead ring / epilogue stage region
  bf16x8 xr[2][KS];
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      xr[ti][ks] = *reinterpret_cast<const bf16x8*>(Xs + ks * (BM * BK) + (wat * 32 + ti * 16 + lr) * BK + ch);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  vm_wait_4x(4);  // step 0's pieces (and the RoPE / bias loads before them) landed
  __builtin_amdgcn_s_barrier();  // every wave holds its xn rows: the image region is free
  asm volatile("" ::: "memory");
#pragma unroll
  for (int k = 0; k < RMAX; ++k) {
    const int i = tid + k * kRqThreads;
    if (i < nR) lds_st1_raw(Rs + i, rv[k]);
  }
#pragma unroll
  for (int k = 0; k < BMAX; ++k) {
    const int i = tid + k * kRqThreads;
    if (i < 3 * NCOL) lds_st1_raw(Bq + i, bv[k]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // before step 1's barrier
  qissue(2);
  qissue(3);

  // per-token plane row offsets: token m = (b T + t) L + l -> ((b L + l) H + head) T + t
  const int H = q.H, BL = (M / (T * L)) * L;
  const size_t plane = (size_t)BL * H * T * D;
  size_t toff[2];
#pragma unroll
  for (int ti = 0; ti < 2; ++ti) {
    const int m = min(rows(wat * 32 + ti * 16 + lr), M - 1);
    const int ml = fdiv(m, L, invL), l = m - ml * L, b = fdiv(ml, T, invT), t = ml - b * T;
    toff[ti] = ((size_t)(b * L + l) * H * T + t) * D;
  }
  const bool full = rows(BM - 1) < M;  // every epilogue store is issued (the counted waits rely on it)
  bf16_t* qo = reinterpret_cast<bf16_t*>(q.qkv_out);
  for (int n = 0; n < NCH; ++n) {
    f32x4 acc[4][2];
#pragma unroll
    for (int hi = 0; hi < 4; ++hi)
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) acc[hi][ti] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
      const int s = 3 * n + kk;
      if (s > 0) {
        // step s landed: leave the younger steps' pieces and (after chunk 0) the previous
        // chunk's 8 stores in flight; then refill the slot step s - 1 used with step s + 3
        const int younger = min(2, QSTEPS - 1 - s);
        vm_wait_4x(4 * younger + (full && n > 0 ? 8 : 0));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring reads retired (see kRingWaitNote)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (s + 3 < QSTEPS) qissue(s + 3);
      }
      const bf16_t* sl = lds + (s & 3) * QSLOT + (wah * 64 + lr) * BK + ch;
      // image g + 1's fragments are read while image g's MFMAs run
      bf16x8 a[2][4];
#pragma unroll
      for (int hi = 0; hi < 4; ++hi) a[0][hi] = *reinterpret_cast<const bf16x8*>(sl + hi * 16 * BK);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (g < 3)
#pragma unroll
          for (int hi = 0; hi < 4; ++hi)
            a[(g + 1) & 1][hi] = *reinterpret_cast<const bf16x8*>(sl + (g + 1) * IMG + hi * 16 * BK);
        __builtin_amdgcn_sched_barrier(0);  // (keeps the scheduler from sinking the reads)
#pragma unroll
        for (int hi = 0; hi < 4; ++hi)
#pragma unroll
          for (int ti = 0; ti < 2; ++ti)
            acc[hi][ti] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[g & 1][hi], xr[ti][4 * kk + g], acc[hi][ti], 0, 0, 0);
      }
    }
    // chunk n = 128 columns of one of q | k | v
    const int which = n / 3;
    const float sc = which == 0 ? q.qscale : 1.0f;
    const bool rope = q.rope && which < 2;
#pragma unroll
    for (int hi = 0; hi < 4; ++hi) {
      const int col0 = n * 128 + wah * 64 + hi * 16 + lg * 4, w = col0 - which * NCOL;
      const int head = fdiv(w, D, invD), cp = w - head * D;
      f32x4 bb;
      f32x2 cc[2], ss[2];
      if (rope) {
        const float* r0 = Rs + (wat * 32 + lr) * D + (cp >> 1);
        const float* r1 = r0 + 16 * D;
        lds_ld4_2x4_raw(Bq + col0, r0, r0 + half, r1, r1 + half, bb, cc[0], ss[0], cc[1], ss[1]);
      } else {
        bb = lds_ld4_raw(Bq + col0);
        cc[0] = cc[1] = ss[0] = ss[1] = f32x2{0.f, 0.f};
      }
      bf16_t* dst = qo + which * plane + (size_t)head * T * D + cp;
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
        const int tok = wat * 32 + ti * 16 + lr;
        float v0 = acc[hi][ti][0] + bb[0], v1 = acc[hi][ti][1] + bb[1], v2 = acc[hi][ti][2] + bb[2],
              v3 = acc[hi][ti][3] + bb[3];
        v0 *= sc; v1 *= sc; v2 *= sc; v3 *= sc;
        if (rope) {
          const f32x2 c2 = cc[ti], s2 = ss[ti];
          // (explicit fma, as epi_tile8: the two paths round alike)
          const float x0 = __builtin_fmaf(v0, c2[0], -(v1 * s2[0])), y0 = __builtin_fmaf(v1, c2[0], v0 * s2[0]);
          const float x1 = __builtin_fmaf(v2, c2[1], -(v3 * s2[1])), y1 = __builtin_fmaf(v3, c2[1], v2 * s2[1]);
          v0 = x0; v1 = y0; v2 = x1; v3 = y1;
        }
        if (full || rows(tok) < M) {
          bf16x4 o;
          o[0] = (bf16_t)v0; o[1] = (bf16_t)v1; o[2] = (bf16_t)v2; o[3] = (bf16_t)v3;
          *reinterpret_cast<bf16x4*>(dst + toff[ti]) = o;
        }
      }
    }
  }
}

// Envelope: bf16; out_proj = PLAIN GATE_RES, K = N = 384, LN output on, tiles over <= 2 adaLN
// entries; q|k|v = the temporal QKV epilogue into packed planes, N = 1152, head_dim D % 8 == 0
// and <= 48 (the RoPE rows of 128 tokens fit next to the ring), no training outputs.
bool rowln_qkv_supported(const mdg_gemm_desc& r, const mdg_gemm_desc& q) {
  return r.dtype == MDG_BF16 && q.dtype == MDG_BF16 && r.a_mode == MDG_A_PLAIN && r.epi == MDG_EPI_GATE_RES &&
         r.K == 384 && r.N == 384 && r.M > 0 && r.rows_per_mod >= 128 && r.resid && !r.resid_in && !r.aux &&
         r.xn_out && r.xn_mods && r.lda % 8 == 0 && r.ldw % 8 == 0 && r.ldr % 4 == 0 && q.epi == MDG_EPI_QKV &&
         q.qkv_layout == MDG_QKV_TEMPORAL_PACKED && q.qkv_out && q.W && q.M == r.M && q.N == 3 * 384 && q.K == 384 &&
         q.ldw % 8 == 0 && !q.aux && q.D > 0 && q.D % 8 == 0 && q.D <= 48 && q.H * q.D == 384 && q.T > 0 && q.L > 0 &&
         r.M % (q.T * q.L) == 0 && (!q.rope || q.rope_rows >= q.T);
}

// MDG_RQ_FRAMES=1: frame tiles (8 frames x 16 residues) for L % 16 == 0 and T >= 8 (a tile
// then spans <= 2 trajectories).  Off by default: at the ATLAS shape (B 1, T 250, L 256) the
// kernel wrote 246.6 vs 257 MB (PMC WRITE_SIZE; h 98.3 + planes 147.5 MB algorithmic — the
// plane rows were not partial-line writes after all) and took 144 vs 139 us (same box).
static bool rq_frames(const mdg_gemm_desc& q) {
  static const bool on = [] {
    const char* e = getenv("MDG_RQ_FRAMES");
    return e && e[0] == '1';
  }();
  return on && q.L % 16 == 0 && q.T >= 8;
}

hipError_t rowln_qkv_launch(const mdg_gemm_desc& r, const mdg_gemm_desc& q, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    for (const void* k : {reinterpret_cast<const void*>(&rowln_qkv_kernel<false>),
                          reinterpret_cast<const void*>(&rowln_qkv_kernel<true>)}) {
      hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kRqSmem);
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
  RqArgs a;
  a.r = r;
  a.q = q;
  a.frames = rq_frames(q) ? 1 : 0;
  if (a.frames) {
    const int nf = r.M / q.L;
    hipLaunchKernelGGL(rowln_qkv_kernel<true>, dim3(((nf + 7) / 8) * (q.L / 16)), dim3(kRqThreads), kRqSmem, s, a);
  } else {
    hipLaunchKernelGGL(rowln_qkv_kernel<false>, dim3((r.M + 127) / 128), dim3(kRqThreads), kRqSmem, s, a);
  }
  return hipGetLastError();
}

// row-tile height of the fused gated-residual + LN GEMM (MDG_ROWLN_BM=64 knob; default 128:
// measured at M = 32000 / 64000, 64-row tiles at two blocks per CU tie on out_proj and lose
// 20 % on fc2 — the extra W re-reads from L2 outweigh the epilogue / main-loop overlap.  Not
// chosen automatically for small M either: its epilogue rounds h 1 ulp differently from the
// 128-row one, which the fused kernels' bit-identity to this GEMM relies on)
static int rowln_bm(int) {
  static const int bm = [] {
    const char* e = getenv("MDG_ROWLN_BM");
    return (e && atoi(e) == 64) ? 64 : 128;
  }();
  return bm;
}

// ---------------------------------------------------------------------------------------
// Spatial q|k|v projection fused with the 4-residue spatial attention (MDG_EPI_ATTN_SPATIAL;
// latent_model.py:466-470 -> mha.py:161-407 with S = L = 4 keys + the bias_k / bias_v row).
// A 128-row tile is 32 whole frames; its 144 output columns are the q | k | v rows of one
// head PAIR (2 x 3 x 24), gathered from the standard packed [3C][C] weight by the loader, so
// the tile holds every operand the pair's attention needs and q|k|v never reaches HBM: the
// epilogue computes softmax(q k^T) v per (frame, head) and writes only o [N][C] (bf16).
//   main loop: 4 waves; wave w owns rows {16w..16w+15} of each 64-row band (frag i = band)
//              and all 9 16-column fragments; K-step 32, double-buffered global_load_lds into
//              a chunk-swizzled image (as gemm_bf16_b4_kernel).
//   epilogue : per band, acc + bias (q also * qscale) -> fp32 LDS [64][148]; then one lane per
//              (frame, head, half of the head dim, residue): RoPE at position l, partial q.k
//              over its 12 dims (the other residues' k / v by DPP quad broadcast, the other
//              half's partial sums by one lane-xor-4 swap), fp32 softmax over the bias key +
//              the unmasked residues, o = P.V, 3 x 8-B bf16 stores.
// Requires bf16, L == 4, D == 24, H even; the unfused QKV GEMM + attn_spatial path covers
// everything else.
constexpr int kSpaThreads = 256;
constexpr int kSpaBN = 144;                                   // 2 heads x q|k|v x 24
constexpr int kSpaLdsSt = kSpaBN + 4;                         // fp32 epilogue row stride
constexpr size_t kSpaStage = (size_t)(128 + kSpaBN) * 32 * 2;  // one K-step's A + B image, 17408 B
// ring of S K-steps (S - 1 in flight while one is read); the epilogue stage reuses it
__host__ __device__ constexpr size_t spa_smem(int S) {
  return (size_t)S * kSpaStage > (size_t)64 * kSpaLdsSt * 4 ? (size_t)S * kSpaStage : (size_t)64 * kSpaLdsSt * 4;
}

template <int I>
__device__ __forceinline__ float quad_bc(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), I | (I << 2) | (I << 4) | (I << 6), 0xF, 0xF, true));
}

// Quad-broadcast FMAs with the DPP riding on the FMA (v_fmac_f32_dpp, src0 read from quad lane j):
// half the VALU of the v_mov_b32_dpp + v_fmac pair the compiler emits for quad_bc(x) * y (it
// does not fold the broadcast).  A DPP source written by a VALU needs two wait states, which
// the hazard recognizer does not provide across inline asm: each block starts with s_nop 1.
// s_j += sum_{c < 6} q[c] * k_j[c]   (k_j = quad lane j's k), c ascending per key
__device__ __forceinline__ void quad_dots6(const float* q, const float* k, float& s0, float& s1, float& s2, float& s3) {
  asm volatile("s_nop 1\n\t"
               "v_fmac_f32_dpp %0, %10, %4 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %1, %10, %4 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %2, %10, %4 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %3, %10, %4 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               "v_fmac_f32_dpp %0, %11, %5 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %1, %11, %5 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %2, %11, %5 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %3, %11, %5 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               "v_fmac_f32_dpp %0, %12, %6 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %1, %12, %6 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %2, %12, %6 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %3, %12, %6 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               "v_fmac_f32_dpp %0, %13, %7 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %1, %13, %7 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %2, %13, %7 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %3, %13, %7 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               "v_fmac_f32_dpp %0, %14, %8 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %1, %14, %8 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %2, %14, %8 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %3, %14, %8 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               "v_fmac_f32_dpp %0, %15, %9 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %1, %15, %9 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %2, %15, %9 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %3, %15, %9 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3)
               : "v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[3]), "v"(q[4]), "v"(q[5]),
                 "v"(k[0]), "v"(k[1]), "v"(k[2]), "v"(k[3]), "v"(k[4]), "v"(k[5]));
}
// o[c] += sum_j p_j * v_j[c] for c < 6, keys j ascending
__device__ __forceinline__ void quad_pv6(float* o, const float* v, float p0, float p1, float p2, float p3) {
  asm volatile("s_nop 1\n\t"
               "v_fmac_f32_dpp %0, %10, %6 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %0, %10, %7 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %0, %10, %8 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %0, %10, %9 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               "v_fmac_f32_dpp %1, %11, %6 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %1, %11, %7 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %1, %11, %8 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %1, %11, %9 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               "v_fmac_f32_dpp %2, %12, %6 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %2, %12, %7 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %2, %12, %8 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %2, %12, %9 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               "v_fmac_f32_dpp %3, %13, %6 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %3, %13, %7 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %3, %13, %8 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %3, %13, %9 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               "v_fmac_f32_dpp %4, %14, %6 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %4, %14, %7 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %4, %14, %8 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %4, %14, %9 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               "v_fmac_f32_dpp %5, %15, %6 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %5, %15, %7 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %5, %15, %8 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" "v_fmac_f32_dpp %5, %15, %9 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
               : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]), "+v"(o[4]), "+v"(o[5])
               : "v"(p0), "v"(p1), "v"(p2), "v"(p3), "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]),
                 "v"(v[5]));
}


// diagnostic builds of the fused spatial kernel (tools/gpu_lane_race.sh, tools/lane_snap.py;
// DESIGN.md §4 "Concurrent-lane divergence"), never set in the product build: 2 = the DPP
// products through the compiler's quad_bc instead of the inline v_fmac_f32_dpp blocks; 8 = each
// band's q|k|v tile also written to p.qkv_out (the spatial q|k|v workspace region, unused on
// this path); 9 = every lane's attention evaluated a second time (same code, the stage address
// made opaque) with both traces logged where the results differ.
#ifndef MDG_DIAG_SPA
#define MDG_DIAG_SPA 0
#endif
#if MDG_DIAG_SPA == 9
__device__ unsigned g_spa_diag[4 + 32 * 128];  // [0] = mismatching lanes, then 32-word records
#endif
// MFMA epilogue (MF = true; opt-in with MDG_SPA_MFMA=1: measured slower than the VALU epilogue,
// 58.9 vs 52.5 us standalone): wave w of band i holds the q|k|v of ITS 16 tokens = 4 whole
// frames in registers (C layout: lane (column lr, group lg) = tokens 4lg..4lg+3), so each wave
// runs its frames' attention alone:
//   1. + bias, q * qscale, RoPE (partner column = the quad neighbour, one DPP move), bf16 ->
//      a wave-private [144 features][16 tokens] LDS image, one 8-B store per fragment;
//   2. per head: S^T = K . Q^T and the bias-key scores sb = bk . Q^T as two 16x16x32 MFMAs
//      (operands by ds_read_b64_tr_b16 from the image, dims 24..31 zeroed), so lane (q, g)
//      holds q's scores against the 4 residues of frame g -- a complete softmax row where
//      g == q / 4 (the block-diagonal frame), nothing to reduce across lanes;
//   3. softmax in those lanes (bias key + the unmasked residues, fp32), the unnormalised P as
//      the B operand of O^T = V^T . P^T (two 16x16x16 MFMAs, V^T by plain 8-B reads of the
//      image), then (O + pb bv) / sum, pb and 1 / sum fetched from the row's lane by one
//      ds_bpermute each, 8-B bf16 stores.
// q, k, v are rounded to bf16 before the attention (as on the unfused route's planes).
constexpr int kSpaImg = kSpaBN * 16;                             // bf16 elements of one wave's image
constexpr int kSpaRtab = 4 * kSpaImg * 2;                        // byte offset of the RoPE table
static_assert(kSpaRtab + 12 * 2 * 4 * 4 <= kSpaStage * 2, "images + RoPE table fit the 2-stage ring");
typedef __attribute__((ext_vector_type(4))) short spa_s4;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

template <int S, bool MF>  // ring depth (K-steps); MF: the MFMA epilogue
#ifndef MDG_SPA_WAVES_MF  // diagnostic builds: waves per SIMD the launch bounds ask for
#define MDG_SPA_WAVES_MF 4
#endif
#ifndef MDG_SPA_WAVES_VALU
#define MDG_SPA_WAVES_VALU 1
#endif
__global__ __launch_bounds__(kSpaThreads, MF ? MDG_SPA_WAVES_MF : MDG_SPA_WAVES_VALU) void gemm_qkv_attn_spatial_kernel(const mdg_gemm_desc p) {
#if MDG_DIAG_ORDER
  if (threadIdx.x == 0) {
    OrderSlot& o = order_slot(p.A);
    const unsigned nwg_ = (unsigned)((p.H / 2) * ((p.M + 127) / 128));
    const unsigned j = atomicAdd(&o.spa, 1u) / nwg_;
    const unsigned red = __hip_atomic_load(&o.red, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned want = j * (unsigned)((p.M + 3) / 4);
    if (red < want) {
      atomicAdd(&o.err, 1u);
      atomicMax(&o.worst, want - red);
    }
  }
  __syncthreads();
#endif
  constexpr int D = 24, HP = 2, BM = 128, BN = kSpaBN, BK = 32, NF = BN / 16, HD = HP * D;
  constexpr int ATILE = BM * BK, STAGE = (BM + BN) * BK, LDS_ST = kSpaLdsSt;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int M = p.M, K = p.K, C = p.H * D;
  const int n_tiles = p.H / HP, m_tiles = (M + BM - 1) / BM, nwg = n_tiles * m_tiles;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = p.ln_eps < 0.f ? (int)blockIdx.x : (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int mt = wg / n_tiles, pair = wg - mt * n_tiles;
  const int m0 = mt * BM;
  // tile column r -> packed weight row: segment r / 48 (q, k, v), head pair `pair`
  auto wrow = [&](int r) { return (r / HD) * C + pair * HD + (r % HD); };

  auto swz_of = [](int r) { return (-(r >> 2)) & 3; };
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A);
  const bf16_t* W = reinterpret_cast<const bf16_t*>(p.W);
  // glds instruction i stages 16 tile rows (64 B each); A: i = wave, wave + 4; B: i = wave,
  // wave + 4, and wave 0 also i = 8
  const bf16_t* asrc[2];
  const bf16_t* bsrc[3];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int row = 16 * (wave + 4 * u) + (lane >> 2);
    asrc[u] = A + (size_t)min(m0 + row, M - 1) * p.lda + (((lane & 3) ^ swz_of(row)) * 8);
  }
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int row = min(16 * (wave + 4 * u) + (lane >> 2), BN - 1);
    bsrc[u] = W + (size_t)wrow(row) * p.ldw + (((lane & 3) ^ swz_of(row)) * 8);
  }
#define MDG_SPA_LOAD(stage_, k0_)                                                                    \
  {                                                                                                  \
    bf16_t* sa = lds + (stage_) * STAGE;                                                             \
    _Pragma("unroll") for (int u = 0; u < 2; ++u)                                                    \
      __builtin_amdgcn_global_load_lds((const void*)(asrc[u] + (k0_)), (lds_ptr_t)(sa + 16 * (wave + 4 * u) * BK), 16, 0, 0); \
    _Pragma("unroll") for (int u = 0; u < 2; ++u)                                                    \
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[u] + (k0_)),                               \
                                       (lds_ptr_t)(sa + ATILE + 16 * (wave + 4 * u) * BK), 16, 0, 0); \
    if (wave == 0)                                                                                   \
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[2] + (k0_)), (lds_ptr_t)(sa + ATILE + 16 * 8 * BK), 16, 0, 0); \
  }

  f32x4 acc[2][NF];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
#pragma unroll
  for (int s0 = 0; s0 < S - 1; ++s0)
    if (s0 < nk) MDG_SPA_LOAD(s0, s0 * BK);
  const int ch = (lg ^ swz_of(lr)) * 8;  // fragment rows are lr mod 16
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % S;
    // step kt landed: leave the younger steps' pieces (4 per step, 5 on wave 0) in flight
    const int younger = min(S - 2, nk - 1 - kt);
    if (S > 2 && younger >= 2) {
      if (wave == 0) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if (S > 2 && younger == 1) {
      if (wave == 0) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (kt + S - 1 < nk) MDG_SPA_LOAD((kt + S - 1) % S, (kt + S - 1) * BK);
    const bf16_t* As = lds + cur * STAGE;
    const bf16_t* Bs = As + ATILE;
    bf16x8 a[2], b[NF];
#pragma unroll
    for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const bf16x8*>(As + (i * 64 + 16 * wave + lr) * BK + ch);
#pragma unroll
    for (int j = 0; j < NF; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Bs + (j * 16 + lr) * BK + ch);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
#undef MDG_SPA_LOAD

  if constexpr (MF) {
    // ---------------------------------------------------------------- MFMA epilogue
    const int gi = lane & 15;
    float* rtab = reinterpret_cast<float*>(smem + kSpaRtab);  // [12 pairs][cos | sin][4 residues]
    bf16_t* img = lds + wave * kSpaImg;                        // [144 features][16 tokens], wave-private
    __syncthreads();                                           // every wave is done reading the ring
    if (p.rope && tid < 12 * 2 * 4) {
      const int pr = tid >> 3, cs = (tid >> 2) & 1, r = tid & 3;
      rtab[tid] = p.rope[(size_t)(cs * p.rope_rows + r) * (D / 2) + pr];
    }
    __syncthreads();
    const bf16x8 z8 = {};
#pragma unroll
    for (int band = 0; band < 2; ++band) {
      // 1. bias, q scale, RoPE at position l = token % 4 (the lane's 4 rows are residues 0..3)
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const float bc = p.bias ? p.bias[wrow(j * 16 + lr)] : 0.f;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (acc[band][j][r] + bc) * (j < 3 ? p.qscale : 1.0f);
        if (j < 6 && p.rope) {
          const int d = (16 * (j % 3) + lr) % D, pr = d >> 1;
          const f32x4 cs = *reinterpret_cast<const f32x4*>(rtab + pr * 8);
          const f32x4 sn = *reinterpret_cast<const f32x4*>(rtab + pr * 8 + 4);
          const float sg = (d & 1) ? 1.0f : -1.0f;  // even dim: x c - y s; odd: x c + y s
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v[r]), 0xB1, 0xF, 0xF, true));
            v[r] = fmaf(y, sg * sn[r], v[r] * cs[r]);
          }
        }
        bf16x4 o4;
#pragma unroll
        for (int r = 0; r < 4; ++r) o4[r] = (bf16_t)v[r];
        *reinterpret_cast<bf16x4*>(img + (16 * j + lr) * 16 + 4 * lg) = o4;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // key validity of this lane's 4 keys (frame lg's residues)
      const int tb = m0 + band * 64 + 16 * wave;  // the wave's first token
      f32x4 km = {1.f, 1.f, 1.f, 1.f};
      if (p.key_mask && tb + 4 * lg < M) km = *reinterpret_cast<const f32x4*>(p.key_mask + tb + 4 * lg);
      const bool own = lg == (lr >> 2);
      const int src = lr + 16 * (lr >> 2);  // the lane holding token lr's softmax row
      const int m = tb + lr;
#pragma unroll
      for (int hh = 0; hh < HP; ++hh) {
        // 2. operands (EXEC full for the transposing reads; lg == 3 = dims 24..31 zeroed after)
        auto tr8 = [&](int fbase) {
          const bf16_t* a0 = img + (fbase + 8 * lg + (gi >> 2)) * 16 + 4 * (gi & 3);
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a0);
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(a0 + 4 * 16));
          bf16x8 r8;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            r8[e] = lo[e];
            r8[4 + e] = hi[e];
          }
          return lg < 3 ? r8 : z8;
        };
        const bf16x8 qf = tr8(hh * D), kf = tr8(HD + hh * D);
        const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
        // the bias key (fair-esm RoPE at position L, kvb) as the A operand of sb = bk . Q^T, and
        // the bias value of this lane's output dims
        const float* kb = p.kvb + (size_t)(pair * HP + hh) * 2 * MDG_DP;
        bf16x8 bkf;
        {
          const f32x4 b0 = *reinterpret_cast<const f32x4*>(kb + 8 * lg), b1 = *reinterpret_cast<const f32x4*>(kb + 8 * lg + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bkf[e] = (bf16_t)(lg < 3 ? b0[e] : 0.f);
            bkf[4 + e] = (bf16_t)(lg < 3 ? b1[e] : 0.f);
          }
        }
        const f32x4 st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf, z4, 0, 0, 0);    // S[q][4lg + r]
        const f32x4 sbt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bkf, qf, z4, 0, 0, 0);  // sb[q]
        // 3. softmax over the bias key + the frame's unmasked residues (mha.py:359-389)
        const float sb = sbt[0];
        float mx = sb;
        bool val[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          val[r] = own && km[r] != 0.f;
          if (val[r]) mx = fmaxf(mx, st[r]);
        }
        const float pb = expf(sb - mx);
        float pr_[4], sum = pb;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pr_[r] = val[r] ? expf(st[r] - mx) : 0.f;
          sum += pr_[r];
        }
        const float inv = 1.0f / sum;
        bf16x4 P;
#pragma unroll
        for (int r = 0; r < 4; ++r) P[r] = (bf16_t)pr_[r];
        const int vrow = 2 * HD + hh * D;
        const bf16x4 va0 = *reinterpret_cast<const bf16x4*>(img + (vrow + lr) * 16 + 4 * lg);
        bf16x4 va1 = {};
        if (lr < D - 16) va1 = *reinterpret_cast<const bf16x4*>(img + (vrow + 16 + lr) * 16 + 4 * lg);
        const spa_s4 Ps = __builtin_bit_cast(spa_s4, P);
        const f32x4 o0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(spa_s4, va0), Ps, z4, 0, 0, 0);
        const f32x4 o1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(spa_s4, va1), Ps, z4, 0, 0, 0);
        const float pbq = __shfl(pb, src, 64), invq = __shfl(inv, src, 64);
        if (m < M) {
          bf16_t* op = reinterpret_cast<bf16_t*>(p.out) + (size_t)m * p.ldo + (pair * HP + hh) * D;
          const f32x4 bv0 = *reinterpret_cast<const f32x4*>(kb + MDG_DP + 4 * lg);
          st4<bf16_t>(op + 4 * lg, (o0[0] + pbq * bv0[0]) * invq, (o0[1] + pbq * bv0[1]) * invq,
                      (o0[2] + pbq * bv0[2]) * invq, (o0[3] + pbq * bv0[3]) * invq);
          if (16 + 4 * lg < D) {
            const f32x4 bv1 = *reinterpret_cast<const f32x4*>(kb + MDG_DP + 16 + 4 * lg);
            st4<bf16_t>(op + 16 + 4 * lg, (o1[0] + pbq * bv1[0]) * invq, (o1[1] + pbq * bv1[1]) * invq,
                        (o1[2] + pbq * bv1[2]) * invq, (o1[3] + pbq * bv1[3]) * invq);
          }
        }
      }
    }
    return;
  }
  // ------------------------------------------------------------------ epilogue
  float bcol[NF], scol[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int r = j * 16 + lr;
    bcol[j] = p.bias ? p.bias[wrow(r)] : 0.f;
    scol[j] = (r < HD) ? p.qscale : 1.0f;  // q = (x Wq + bq) * D^-1/2   (mha.py:263)
  }
  // attention lane map: residue jr (quad lanes), half dh of the head dim, head hh, frame f
  const int jr = tid & 3, dh = (tid >> 2) & 1, hh = (tid >> 3) & 1, f = tid >> 4;
  const int gh = pair * HP + hh, c0 = dh * 12;  // global head; first of the lane's 12 dims
  const float* kbh = p.kvb + (size_t)gh * 2 * MDG_DP;
  float* stage = reinterpret_cast<float*>(smem);
  __syncthreads();  // every wave is done reading the ring
#pragma unroll
  for (int band = 0; band < 2; ++band) {
#pragma unroll
    for (int j = 0; j < NF; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        stage[(16 * wave + lg * 4 + r) * LDS_ST + j * 16 + lr] = (acc[band][j][r] + bcol[j]) * scol[j];
    __syncthreads();
    if (MDG_DIAG_SPA == 8 && p.qkv_out) {  // the band's q|k|v tile (before RoPE) -> [M][H / 2][144] bf16
      for (int i = tid; i < 64 * BN; i += kSpaThreads) {
        const int rr = i / BN, cc = i - rr * BN, mm = m0 + band * 64 + rr;
        if (mm < M) reinterpret_cast<bf16_t*>(p.qkv_out)[(size_t)mm * (p.H / 2) * BN + pair * BN + cc] = (bf16_t)stage[rr * LDS_ST + cc];
      }
    }
    const int row = f * 4 + jr, m = m0 + band * 64 + row;
    // the band's attention for this lane (a lambda so the diagnostic build can evaluate it twice)
    auto attend = [&](auto vol, float (&o)[12], int rowx, unsigned* trace) {
      constexpr bool VOL = decltype(vol)::value;
      typedef typename std::conditional<VOL, const volatile float, const float>::type cf;
      cf* srow = stage + rowx * LDS_ST + hh * D + c0;
      const bool rope = p.rope != nullptr;
      cf* kb = kbh;
      cf* kmask = p.key_mask;
      float q[12], k[12], v[12];
      if constexpr (VOL) {
#pragma unroll
        for (int c = 0; c < 12; ++c) {
          q[c] = srow[c];
          k[c] = srow[HD + c];
          v[c] = srow[2 * HD + c];
        }
      } else {
#pragma unroll
        for (int c = 0; c < 12; c += 4) {
          const float4 a4 = *reinterpret_cast<const float4*>(srow + c);
          const float4 b4 = *reinterpret_cast<const float4*>(srow + HD + c);
          const float4 v4 = *reinterpret_cast<const float4*>(srow + 2 * HD + c);
          q[c] = a4.x; q[c + 1] = a4.y; q[c + 2] = a4.z; q[c + 3] = a4.w;
          k[c] = b4.x; k[c + 1] = b4.y; k[c + 2] = b4.z; k[c + 3] = b4.w;
          v[c] = v4.x; v[c + 1] = v4.y; v[c + 2] = v4.z; v[c + 3] = v4.w;
        }
      }
      if (MDG_DIAG_SPA == 9 && trace) {
        unsigned hq = 0, hk = 0, hv = 0;
#pragma unroll
        for (int c = 0; c < 12; ++c) {
          hq = hq * 31u + __float_as_uint(q[c]); hk = hk * 31u + __float_as_uint(k[c]); hv = hv * 31u + __float_as_uint(v[c]);
        }
        trace[0] = hq; trace[1] = hk; trace[2] = hv;
      }
      if (rope) {  // fair-esm rotate-half on the pair-interleaved columns, position l = jr
        // The lane's 6 cos and 6 sin values start at float (jr * 12 + dh * 6): 8-B aligned, not
        // 16-B.  Read as scalar floats, the compiler merged them into global_load_dwordx4 at that
        // 8-B alignment, and such loads returned wrong data for lanes 48-63 of a wave, rarely and
        // only with another kernel's blocks on the CU (the concurrent-lane divergence of
        // DESIGN.md §4; this change alone: 0 vs 46 divergent replays of 1 200).  Each lane now
        // reads its position's whole 12-float row as three 16-B-aligned float4 and keeps its half.
        constexpr int half = D / 2;
        static_assert(half == 12, "row = 3 float4");
        const float4* rc = reinterpret_cast<const float4*>(p.rope + jr * half);
        const float4* rs = reinterpret_cast<const float4*>(p.rope + (p.rope_rows + jr) * half);
        const float4 c4[3] = {rc[0], rc[1], rc[2]}, s4[3] = {rs[0], rs[1], rs[2]};
        auto pick = [&](const float4 (&r)[3], int e) {  // element e of the 12-float row
          const float4 w = r[e >> 2];
          return (e & 3) == 0 ? w.x : (e & 3) == 1 ? w.y : (e & 3) == 2 ? w.z : w.w;
        };
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const float cs = dh ? pick(c4, 6 + i) : pick(c4, i), sn = dh ? pick(s4, 6 + i) : pick(s4, i);
          const float q0 = q[2 * i], q1 = q[2 * i + 1], k0 = k[2 * i], k1 = k[2 * i + 1];
          q[2 * i] = q0 * cs - q1 * sn; q[2 * i + 1] = q1 * cs + q0 * sn;
          k[2 * i] = k0 * cs - k1 * sn; k[2 * i + 1] = k1 * cs + k0 * sn;
        }
      }
      const float kvalid = (!kmask || kmask[min(m, M - 1)] != 0.f) ? 1.f : 0.f;
      float sb = 0.f, s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
      for (int c = 0; c < 12; ++c) sb += q[c] * kb[c0 + c];
      if (MDG_DIAG_SPA == 2) {
#pragma unroll
        for (int c = 0; c < 12; ++c) {
          s0 = fmaf(quad_bc<0>(k[c]), q[c], s0); s1 = fmaf(quad_bc<1>(k[c]), q[c], s1);
          s2 = fmaf(quad_bc<2>(k[c]), q[c], s2); s3 = fmaf(quad_bc<3>(k[c]), q[c], s3);
        }
      } else {
        quad_dots6(q, k, s0, s1, s2, s3);
        quad_dots6(q + 6, k + 6, s0, s1, s2, s3);
      }
      if (MDG_DIAG_SPA == 9 && trace) {
        trace[3] = __float_as_uint(sb); trace[4] = __float_as_uint(s0); trace[5] = __float_as_uint(s3);
      }
      sb += __shfl_xor(sb, 4, 64); s0 += __shfl_xor(s0, 4, 64); s1 += __shfl_xor(s1, 4, 64);
      s2 += __shfl_xor(s2, 4, 64); s3 += __shfl_xor(s3, 4, 64);
      if (MDG_DIAG_SPA == 9 && trace) {
        trace[6] = __float_as_uint(sb); trace[7] = __float_as_uint(s0); trace[8] = __float_as_uint(s3);
      }
      const float v0 = quad_bc<0>(kvalid), v1 = quad_bc<1>(kvalid), v2 = quad_bc<2>(kvalid), v3 = quad_bc<3>(kvalid);
      float mx = sb;  // the bias key is never masked (mha.py:273-280)
      if (v0 != 0.f) mx = fmaxf(mx, s0);
      if (v1 != 0.f) mx = fmaxf(mx, s1);
      if (v2 != 0.f) mx = fmaxf(mx, s2);
      if (v3 != 0.f) mx = fmaxf(mx, s3);
      const float pb = expf(sb - mx);
      const float p0 = v0 != 0.f ? expf(s0 - mx) : 0.f, p1 = v1 != 0.f ? expf(s1 - mx) : 0.f;
      const float p2 = v2 != 0.f ? expf(s2 - mx) : 0.f, p3 = v3 != 0.f ? expf(s3 - mx) : 0.f;
      const float inv = 1.0f / (pb + p0 + p1 + p2 + p3);
      if (MDG_DIAG_SPA == 9 && trace) {
        trace[9] = __float_as_uint(pb); trace[10] = __float_as_uint(p0); trace[11] = __float_as_uint(inv);
      }
#pragma unroll
      for (int c = 0; c < 12; ++c) o[c] = pb * kb[MDG_DP + c0 + c];
      if (MDG_DIAG_SPA == 2) {
#pragma unroll
        for (int c = 0; c < 12; ++c) {
          o[c] = fmaf(quad_bc<0>(v[c]), p0, o[c]); o[c] = fmaf(quad_bc<1>(v[c]), p1, o[c]);
          o[c] = fmaf(quad_bc<2>(v[c]), p2, o[c]); o[c] = fmaf(quad_bc<3>(v[c]), p3, o[c]);
        }
      } else {
        quad_pv6(o, v, p0, p1, p2, p3);
        quad_pv6(o + 6, v + 6, p0, p1, p2, p3);
      }
#pragma unroll
      for (int c = 0; c < 12; ++c) o[c] *= inv;
    };
    float o[12];
#if MDG_DIAG_SPA == 9
    unsigned tr1[12], tr2[12];
    attend(std::false_type{}, o, row, tr1);
    {  // evaluate again (same code, the stage row address made opaque so every LDS read is
       // reissued) and log any lane whose result differs bit for bit, with both traces
      float o2[12];
      int row2 = row;
      asm volatile("" : "+v"(row2));
      attend(std::false_type{}, o2, row2, tr2);
      int bad = -1;
#pragma unroll
      for (int c = 0; c < 12; ++c)
        if (__float_as_uint(o[c]) != __float_as_uint(o2[c]) && bad < 0) bad = c;
      if (bad >= 0) {
        const unsigned i = atomicAdd(&g_spa_diag[0], 1u);
        if (i < 128) {
          unsigned* e = g_spa_diag + 4 + 32 * i;
          e[0] = blockIdx.x; e[1] = tid; e[2] = band; e[3] = bad;
          e[4] = __float_as_uint(o[bad]); e[5] = __float_as_uint(o2[bad]); e[6] = (unsigned)m; e[7] = pair;
#pragma unroll
          for (int t = 0; t < 12; ++t) { e[8 + t] = tr1[t]; e[20 + t] = tr2[t]; }
        }
      }
    }
#else
    attend(std::false_type{}, o, row, nullptr);
#endif
    if (m < M) {
      bf16_t* op = reinterpret_cast<bf16_t*>(p.out) + (size_t)m * p.ldo + gh * D + c0;
#pragma unroll
      for (int c = 0; c < 12; c += 4) st4<bf16_t>(op + c, o[c], o[c + 1], o[c + 2], o[c + 3]);
    }
    if (band == 0) __syncthreads();  // band 1 overwrites the stage
  }
}

// ring depth: MDG_SPA_STAGES (2, 3 or 4; A/B knob).  Measured standalone at M = 32000: 52.7 /
// 53.5 / 59.5 us: more co-resident blocks (4 per CU at 2 stages) beat a deeper ring
static int spa_stages() {
  static const int st = [] {
    const char* e = getenv("MDG_SPA_STAGES");
    const int v = e ? atoi(e) : 2;
    return (v == 3 || v == 4) ? v : 2;
  }();
  return st;
}

static hipError_t launch_spatial(const mdg_gemm_desc& p0, hipStream_t s) {
  // MDG_SPA_XCD=0: plain block order (diagnostic; carried in the unused ln_eps field)
  static const bool xcd_map = [] {
    const char* e = getenv("MDG_SPA_XCD");
    return !(e && e[0] == '0');
  }();
  // MDG_SPA_MFMA=1: the MFMA epilogue (opt-in: 58.9 vs 52.5 us standalone at one lane's shape,
  // bench -1.4 %, same box) instead of the lane-per-(frame, head) one
  static const bool mf = [] {
    const char* e = getenv("MDG_SPA_MFMA");
    return e && e[0] == '1';
  }();
  mdg_gemm_desc p = p0;
  p.ln_eps = xcd_map ? 0.f : -1.f;
  const int nwg = (p.H / 2) * ((p.M + 127) / 128);
  if (mf) {
    hipLaunchKernelGGL((gemm_qkv_attn_spatial_kernel<2, true>), dim3(nwg), dim3(kSpaThreads), spa_smem(2), s, p);
    return hipGetLastError();
  }
  switch (spa_stages()) {
    case 2: hipLaunchKernelGGL((gemm_qkv_attn_spatial_kernel<2, false>), dim3(nwg), dim3(kSpaThreads), spa_smem(2), s, p); break;
    case 4: {
      static bool attr_set = false;
      if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_qkv_attn_spatial_kernel<4, false>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)spa_smem(4));
        if (e != hipSuccess) return e;
        attr_set = true;
      }
      hipLaunchKernelGGL((gemm_qkv_attn_spatial_kernel<4, false>), dim3(nwg), dim3(kSpaThreads), spa_smem(4), s, p);
      break;
    }
    default: hipLaunchKernelGGL((gemm_qkv_attn_spatial_kernel<3, false>), dim3(nwg), dim3(kSpaThreads), spa_smem(3), s, p); break;
  }
  return hipGetLastError();
}

template <typename CT, int BM, int BN, int WM, int AMODE>
static size_t smem_bytes(int K) {
  constexpr int BK = 64, VEC = 16 / sizeof(CT), LDT = BK + VEC;
  const size_t b = 2ull * BN * LDT * sizeof(CT);
  if (AMODE == MDG_A_LNMOD) return (size_t)BM * (K + VEC) * sizeof(CT) + b;
  return 2ull * BM * LDT * sizeof(CT) + b;
}

template <typename CT, int BM, int BN, int WM, int AMODE>
static bool stage_fits() {
  constexpr int BK = 64, VEC = 16 / sizeof(CT), LDT = BK + VEC;
  const size_t stage = (size_t)(BM / WM) * (BN + 4) * sizeof(float);
  const size_t room = (AMODE == MDG_A_LNMOD) ? 2ull * BN * LDT * sizeof(CT)
                                             : 2ull * BM * LDT * sizeof(CT) + 2ull * BN * LDT * sizeof(CT);
  return stage <= room;
}

constexpr int kCfgB4 = 100, kCfgB8 = 101, kCfgB4K32 = 102, kCfgRow = 103, kCfgSpa = 104, kCfgRowTrain = 105;

struct GemmPlan {
  int cfg;  // index into the config table below; -1 = unsupported
  size_t smem;
  int bm, bn;
};

template <typename CT, int BM, int BN, int WM, int AMODE, int EPI>
static hipError_t launch_one(const mdg_gemm_desc& p, hipStream_t s) {
  const size_t smem = smem_bytes<CT, BM, BN, WM, AMODE>(p.K);
  static bool attr_set = false;  // idempotent attribute write
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<CT, BM, BN, WM, AMODE, EPI>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  // PLAIN: one N tile per block.  LNMOD: a block sweeps a group of N tiles (LayerNorm once per
  // row per group); ~one block per CU is resident anyway, so aim the grid at ~256 blocks.
  const int n_tiles = p.N / BN, m_tiles = (p.M + BM - 1) / BM;
  int groups = n_tiles;
  if (AMODE == MDG_A_LNMOD) {
    int want = (256 + m_tiles - 1) / m_tiles;
    if (want < 1) want = 1;
    if (want > n_tiles) want = n_tiles;
    const int tpg = (n_tiles + want - 1) / want;
    groups = (n_tiles + tpg - 1) / tpg;
  }
  hipLaunchKernelGGL((gemm_kernel<CT, BM, BN, WM, AMODE, EPI>), dim3(groups, m_tiles), dim3(kThreads), smem, s, p);
  return hipGetLastError();
}

template <typename CT, int BM, int BN, int WM, int AM>
static hipError_t dispatch_epi(const mdg_gemm_desc& p, hipStream_t s) {
  switch (p.epi) {
    case MDG_EPI_STORE: return launch_one<CT, BM, BN, WM, AM, MDG_EPI_STORE>(p, s);
    case MDG_EPI_GATE_RES: return launch_one<CT, BM, BN, WM, AM, MDG_EPI_GATE_RES>(p, s);
    case MDG_EPI_QKV: return launch_one<CT, BM, BN, WM, AM, MDG_EPI_QKV>(p, s);
    default: return launch_one<CT, BM, BN, WM, AM, MDG_EPI_EULER>(p, s);
  }
}

// config table: {id, CT, a_mode, BM, BN, WM}
#define MDG_GEMM_CONFIGS(X)    \
  X(0, bf16_t, 1, 128, 128, 2) \
  X(1, bf16_t, 1, 128, 32, 8)  \
  X(2, bf16_t, 1, 64, 128, 4)  \
  X(3, bf16_t, 1, 64, 32, 4)   \
  X(4, bf16_t, 0, 128, 384, 2) \
  X(5, bf16_t, 0, 128, 128, 2) \
  X(6, bf16_t, 0, 64, 384, 4)  \
  X(7, bf16_t, 0, 64, 128, 4)  \
  X(8, bf16_t, 0, 64, 32, 4)   \
  X(9, float, 1, 64, 32, 4)    \
  X(10, float, 0, 64, 96, 4)   \
  X(11, float, 0, 64, 128, 4)  \
  X(12, float, 0, 64, 32, 4)

// Tile plan.  bf16: LN-resident A -> 128x128 (M large) / 64x128; N not a multiple of 128 ->
// BN 32.  Streamed A with N == 384 (out_proj, fc2) -> full-row 128x384 / 64x384, else 128x128.
// fp32 parity path -> 64-row tiles (an fp32 64 x 384 LN block already takes 99 KB of LDS).
GemmPlan gemm_plan(const mdg_gemm_desc& p) {
  GemmPlan g{-1, 0, 0, 0};
  const bool bf = p.dtype == MDG_BF16, ln = p.a_mode == MDG_A_LNMOD;
  const bool big = p.M >= 128 * 128;
  int cfg = -1;
  if (p.epi == MDG_EPI_ATTN_SPATIAL) {  // validated by mdg_gemm: bf16 PLAIN, L 4, D 24, H even
    g.cfg = kCfgSpa;
    g.smem = spa_smem(spa_stages());
    g.bm = 128;
    g.bn = kSpaBN;
    return g;
  }
  const bool ext = p.resid_in || p.aux || p.ln_stats;  // training extensions: epi4 / epi_tile kernels only
  if (bf && p.epi == MDG_EPI_GATE_RES && p.xn_out && p.resid_in && p.aux && p.ln_stats && p.N == 384 &&
      p.K % 64 == 0 && p.lda % 8 == 0 && p.ldw % 8 == 0 && p.ldaux % 4 == 0 && p.rows_per_mod >= 128 &&
      rowln_bm(p.M) == 128) {
    g.cfg = kCfgRowTrain;  // the training forward's out_proj / fc2 + the next LN (row-LN GEMM)
    g.smem = rowln_smem<384, 128>();
    g.bm = 128;
    g.bn = 384;
    return g;
  }
  if (bf && ln) cfg = (p.N % 128 == 0) ? (big ? 0 : 2) : (p.N % 32 == 0 ? (big ? 1 : 3) : -1);
  else if (bf && !ext && p.epi == MDG_EPI_GATE_RES && p.xn_out && p.K % 64 == 0 && p.lda % 8 == 0 && p.ldw % 8 == 0 &&
           (p.N == 128 || p.N == 256 || p.N == 384 || p.N == 512)) {
    g.cfg = kCfgRow;  // full-row gated residual + LayerNorm
    const bool b64 = rowln_bm(p.M) == 64 && p.N <= 384;
#define MDG_ROWSM(n) (b64 ? rowln_smem<n, 64>() : rowln_smem<n, 128>())
    g.smem = p.N == 128 ? MDG_ROWSM(128) : p.N == 256 ? MDG_ROWSM(256) : p.N == 384 ? MDG_ROWSM(384) : MDG_ROWSM(512);
#undef MDG_ROWSM
    g.bm = b64 ? 64 : 128;
    g.bn = p.N;
    return g;
  } else if (bf && p.N % kB4Tile == 0 && p.K % 64 == 0 && p.lda % 8 == 0 && p.ldw % 8 == 0) {
    // MDG_GEMM_TILE=256 / 64 / 32 select the 256x128 3-stage kernel / the 128x128 K-step-64 /
    // K-step-32 kernel (tuning knob); default: K-step 64, or K-step 32 at four blocks per CU when
    // an aux operand rides along (the GELU pre-activation store / DGELU read)
    static const int forced = [] {
      const char* e = getenv("MDG_GEMM_TILE");
      return e ? atoi(e) : 0;
    }();
    if (forced == 256 && !ext) {
      g.cfg = kCfgB8;  // 256x128, 3-stage glds ring
      g.smem = kB8Smem;
      g.bm = kB8M;
    } else if (forced == 64 || (forced == 0 && !p.aux)) {
      // 128x128, K-step 64, two blocks per CU: the default without an aux operand (the
      // training step's input-gradient GEMMs: 45 vs 56 us at N 384, K 1536; the same K order,
      // bit-identical to K-step 32); MDG_GEMM_TILE=32 keeps K-step 32 everywhere
      g.cfg = kCfgB4;
      g.smem = b4_smem<64>();
      g.bm = kB4Tile;
    } else {
      g.cfg = kCfgB4K32;  // 128x128, K-step 32, four blocks per CU
      g.smem = b4_stages() == 4 ? b4_smem<32, 4>() : b4_stages() == 3 ? b4_smem<32, 3>() : b4_smem<32>();
      g.bm = kB4Tile;
    }
    g.bn = 128;
    return g;
  } else if (bf) cfg = (p.N == 384) ? (big ? 4 : 6) : (p.N % 128 == 0 ? (big ? 5 : 7) : (p.N % 32 == 0 ? 8 : -1));
  else if (ln) cfg = (p.N % 32 == 0) ? 9 : -1;
  else cfg = (p.N % 96 == 0) ? 10 : (p.N % 128 == 0 ? 11 : (p.N % 32 == 0 ? 12 : -1));
  if (cfg < 0) return g;
  g.cfg = cfg;
#define MDG_PLAN_CASE(id, CT, AM, BM, BN, WM)            \
  case id:                                             \
    g.smem = smem_bytes<CT, BM, BN, WM, AM>(p.K);      \
    g.bm = BM;                                         \
    g.bn = BN;                                         \
    if (!stage_fits<CT, BM, BN, WM, AM>()) g.cfg = -1; \
    break;
  switch (cfg) { MDG_GEMM_CONFIGS(MDG_PLAN_CASE) }
#undef MDG_PLAN_CASE
  return g;
}

hipError_t gemm_launch(const mdg_gemm_desc& p, const GemmPlan& g, hipStream_t s) {
  if (g.cfg == kCfgSpa) return launch_spatial(p, s);
  if (g.cfg == kCfgRowTrain) return launch_rowln_train(p, s);
  if (g.cfg == kCfgRow) {
    if (g.bm == 64) {
      switch (p.N) {
        case 128: return launch_rowln<128, 64>(p, s);
        case 256: return launch_rowln<256, 64>(p, s);
        case 384: return launch_rowln<384, 64>(p, s);
        default: return launch_rowln<512, 64>(p, s);
      }
    }
    switch (p.N) {
      case 128: return launch_rowln<128, 128>(p, s);
      case 256: return launch_rowln<256, 128>(p, s);
      case 384: return launch_rowln<384, 128>(p, s);
      default: return launch_rowln<512, 128>(p, s);
    }
  }
  if (g.cfg == kCfgB8) {
    switch (p.epi) {
      case MDG_EPI_STORE: return launch_b8<MDG_EPI_STORE>(p, s);
      case MDG_EPI_GATE_RES: return launch_b8<MDG_EPI_GATE_RES>(p, s);
      case MDG_EPI_QKV: return launch_b8<MDG_EPI_QKV>(p, s);
      default: return launch_b8<MDG_EPI_EULER>(p, s);
    }
  }
  if (g.cfg == kCfgB4 || g.cfg == kCfgB4K32) {
    const bool k64 = g.cfg == kCfgB4;
    switch (p.epi) {
      case MDG_EPI_STORE: return k64 ? launch_b4<MDG_EPI_STORE, 64>(p, s) : launch_b4<MDG_EPI_STORE, 32>(p, s);
      case MDG_EPI_GATE_RES: return k64 ? launch_b4<MDG_EPI_GATE_RES, 64>(p, s) : launch_b4<MDG_EPI_GATE_RES, 32>(p, s);
      case MDG_EPI_QKV: return k64 ? launch_b4<MDG_EPI_QKV, 64>(p, s) : launch_b4<MDG_EPI_QKV, 32>(p, s);
      default: return k64 ? launch_b4<MDG_EPI_EULER, 64>(p, s) : launch_b4<MDG_EPI_EULER, 32>(p, s);
    }
  }
#define MDG_LAUNCH_CASE(id, CT, AM, BM, BN, WM) \
  case id:                                    \
    return dispatch_epi<CT, BM, BN, WM, AM>(p, s);
  switch (g.cfg) { MDG_GEMM_CONFIGS(MDG_LAUNCH_CASE) }
#undef MDG_LAUNCH_CASE
  return hipErrorInvalidValue;
}

}  // namespace mdg

#if MDG_DIAG_ORDER
extern "C" int mdg_debug_order_counters(unsigned long long* out, int n) {
  mdg::OrderSlot h[61];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(mdg::g_order), sizeof(h)) != hipSuccess) return -1;
  int k = 0;
  for (int i = 0; i < 61 && k + 5 <= n; ++i)
    if (h[i].key) {
      out[k++] = h[i].key; out[k++] = h[i].red; out[k++] = h[i].spa; out[k++] = h[i].err; out[k++] = h[i].worst;
    }
  return k / 5;
}
#endif

#if MDG_DIAG_SPA == 9
extern "C" int mdg_debug_spa_diag(unsigned* out, int n) {
  if (n < 4 + 32 * 128) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mdg::g_spa_diag), sizeof(unsigned) * (4 + 32 * 128)) == hipSuccess ? 0 : -1;
}
#endif
