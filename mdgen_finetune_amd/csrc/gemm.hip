// Fused GEMM for every projection of the MDGen block:  out = epi( pro(A) . W^T + bias ).
//
//   prologue  A_LNMOD : the whole BM x K row block of the fp32 residual stream is normalised
//                       (no-affine LayerNorm eps 1e-6, latent_model.py:449/454/FinalLayer
//                       layers.py:62 — or IPALayer's affine ipa_norm), adaLN-modulated
//                       y*(1+scale[b]) + shift[b] (layers.py:14-15), converted to CT and kept
//                       resident in LDS; the block then sweeps a group of N tiles, so the
//                       LayerNorm is computed once per row per group.
//             A_PLAIN : CT activations streamed through LDS with the weights.
//   epilogue  (per wave: accumulators -> 4 KiB wave-private LDS stage -> 4 contiguous
//             columns of one row per lane, so every global access is 8-16 B wide)
//             STORE   : + bias, optional exact-erf GELU / SiLU, CT or fp32 store (fc1);
//             GATE_RES: h += gate[b] * (acc + bias)  — the gated residual of
//                       latent_model.py:472/486/491 fused into out_proj / fc2;
//             QKV     : + bias, q *= D^-1/2 (mha.py:264; * log2 e for the exp2 softmax of the
//                       temporal kernel), RoPE on q and k at position l (spatial) or t
//                       (temporal), scattered into the attention layout the consumer reads.
//                       The packer stores each q/k head's rows PAIR-INTERLEAVED
//                       (column 2i = dim i, 2i+1 = dim i+D/2), so fair-esm's rotate-half
//                       partner (mha.py:356-357) sits in the neighbouring lane: one
//                       __shfl_xor(.,1) per element.  q.k dot products are invariant to the
//                       shared permutation; V keeps natural order.
//             EULER   : FinalLayer + Euler update (layers.py:58-75, integrators.py:106-113):
//                       v = acc + bias; x_out = x_in + dt * v for the n_valid real columns.
//
// Tiling (gfx950): 256 threads = 4 waves as 2(M) x 2(N); block tile BM x BN (BM 128 for
// bf16 / 64 for f32; BN 128, 96 or 32), K-step 64, register-staged double buffer with the
// next tile's 16-B global loads issued before the current tile's MFMAs, ONE barrier per
// K-step; the (N-tile, K-step) iteration space of a block is flattened so the prefetch runs
// across N-tile boundaries.  Each wave owns a (BM/2) x (BN/2) sub-tile of 16x16 MFMA
// accumulators.  LDS rows are padded by 16 B so the 16-lane ds_read_b128 fragment reads hit
// distinct bank slots.
#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {

template <typename CT, int BM, int BN, int AMODE, int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(const mdg_gemm_desc p) {
  constexpr int BK = 64;
  constexpr int VEC = 16 / sizeof(CT);
  constexpr int LDT = BK + VEC;
  constexpr int MT = BM / 32, NT = BN / 32;  // 16x16 tiles per wave
  constexpr int HM = BM / 2, HN = BN / 2;
  constexpr int CPR = BK / VEC;              // 16-B chunks per tile row
  constexpr int BCH = BN * CPR / 256;
  constexpr int ACH = (AMODE == MDG_A_PLAIN) ? BM * CPR / 256 : 1;
  static_assert(BN * CPR % 256 == 0 && BM * CPR % 256 == 0, "tile / thread mismatch");
  // epilogue stage [4 waves][16][BN/2+4] fp32: aliases a tile buffer when it fits, else its own
  constexpr int STAGE_B = 4 * 16 * (BN / 2 + 4) * 4;
  constexpr bool STAGE_ALIAS = (AMODE == MDG_A_PLAIN) ? STAGE_B <= 2 * BM * LDT * (int)sizeof(CT)
                                                      : STAGE_B <= BN * LDT * (int)sizeof(CT);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.y * BM;
  const int M = p.M, K = p.K;
  const int n_tiles = p.N / BN;
  const int tpg = (n_tiles + gridDim.x - 1) / gridDim.x;
  const int nt0 = blockIdx.x * tpg;
  const int nt1 = min(n_tiles, nt0 + tpg);
  if (nt0 >= nt1) return;

  constexpr int CPL_Q = HN / 4;      // epilogue columns per lane (4 lanes per row)
  constexpr int LDS_ST = HN + 4;     // stage row stride (floats)
  CT* As = reinterpret_cast<CT*>(smem);
  const int lda_s = (AMODE == MDG_A_LNMOD) ? K + VEC : LDT;
  CT* Bs = (AMODE == MDG_A_LNMOD) ? As + BM * lda_s : As + 2 * BM * LDT;

  // ---------------------------------------------------------------- prologue (LN + mod)
  if constexpr (AMODE == MDG_A_LNMOD) {
    const float* A = reinterpret_cast<const float*>(p.A);
    const float invK = 1.0f / (float)K;
    // lane owns columns k = 2*lane + 128*e (float2), e < 4  (K <= 512)
    for (int r0 = wave * 4; r0 < BM; r0 += 16) {
      float2 v[4][4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int m = m0 + r0 + rr;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 2 * lane + 128 * e;
          v[rr][e] = (m < M && k < K) ? *reinterpret_cast<const float2*>(A + (size_t)m * p.lda + k)
                                      : make_float2(0.f, 0.f);
        }
      }
      float mean[4], rstd[4];
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
        for (int e = 0; e < 4; ++e) {
          const int k = 2 * lane + 128 * e;
          if (k < K) {
            const float a = v[rr][e].x - mean[rr], b = v[rr][e].y - mean[rr];
            ss += a * a + b * b;
          }
        }
        rstd[rr] = ss;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) rstd[rr] += __shfl_xor(rstd[rr], o, 64);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int r = r0 + rr, m = m0 + r;
        const float rs = 1.0f / sqrtf(rstd[rr] * invK + p.ln_eps);
        const float* mrow = (p.mods && m < M) ? p.mods + (size_t)(m / p.rows_per_mod) * p.mod_stride : nullptr;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 2 * lane + 128 * e;
          if (k < K) {
            float y0 = (v[rr][e].x - mean[rr]) * rs, y1 = (v[rr][e].y - mean[rr]) * rs;
            if (p.ln_w) {
              y0 = y0 * p.ln_w[k] + p.ln_b[k];
              y1 = y1 * p.ln_w[k + 1] + p.ln_b[k + 1];
            }
            if (mrow) {
              const float2 sc = *reinterpret_cast<const float2*>(mrow + p.scale_off + k);
              const float2 sh = *reinterpret_cast<const float2*>(mrow + p.shift_off + k);
              y0 = y0 * (1.0f + sc.x) + sh.x;
              y1 = y1 * (1.0f + sc.y) + sh.y;
            }
            if (m >= M) y0 = y1 = 0.f;
            As[r * lda_s + k] = (CT)y0;
            As[r * lda_s + k + 1] = (CT)y1;
          }
        }
      }
    }
  }

  // ---------------------------------------------------------------- main loop
  const CT* W = reinterpret_cast<const CT*>(p.W);
  const CT* Ap = reinterpret_cast<const CT*>(p.A);
  const int nk = K / BK;
  const int total = (nt1 - nt0) * nk;
  u32x4 breg[BCH];  // native vector type: SROA keeps it in registers (HIP's uint4 struct went to scratch)
  u32x4 areg[ACH];

#define MDG_LOAD_TILES(it)                                                                      \
  {                                                                                             \
    const int nb_ = (nt0 + (it) / nk) * BN, k0_ = ((it) % nk) * BK;                             \
    _Pragma("unroll") for (int c = 0; c < BCH; ++c) {                                           \
      const int idx = tid + c * 256, row = idx / CPR, cc = idx % CPR;                           \
      breg[c] = *reinterpret_cast<const u32x4*>(W + (size_t)(nb_ + row) * p.ldw + k0_ + cc * VEC); \
    }                                                                                           \
    if constexpr (AMODE == MDG_A_PLAIN) {                                                       \
      _Pragma("unroll") for (int c = 0; c < ACH; ++c) {                                         \
        const int idx = tid + c * 256, row = idx / CPR, cc = idx % CPR, m = m0 + row;           \
        areg[c] = (m < M) ? *reinterpret_cast<const u32x4*>(Ap + (size_t)m * p.lda + k0_ + cc * VEC) \
                          : u32x4{0u, 0u, 0u, 0u};                                             \
      }                                                                                         \
    }                                                                                           \
  }
#define MDG_STORE_TILES(buf)                                                                    \
  {                                                                                             \
    CT* bdst = Bs + (buf) * BN * LDT;                                                           \
    _Pragma("unroll") for (int c = 0; c < BCH; ++c) {                                           \
      const int idx = tid + c * 256, row = idx / CPR, cc = idx % CPR;                           \
      *reinterpret_cast<u32x4*>(bdst + row * LDT + cc * VEC) = breg[c];                         \
    }                                                                                           \
    if constexpr (AMODE == MDG_A_PLAIN) {                                                       \
      CT* adst = As + (buf) * BM * LDT;                                                         \
      _Pragma("unroll") for (int c = 0; c < ACH; ++c) {                                         \
        const int idx = tid + c * 256, row = idx / CPR, cc = idx % CPR;                         \
        *reinterpret_cast<u32x4*>(adst + row * LDT + cc * VEC) = areg[c];                       \
      }                                                                                         \
    }                                                                                           \
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  MDG_LOAD_TILES(0);
  MDG_STORE_TILES(0);
  __syncthreads();
  for (int it = 0; it < total; ++it) {
    const int cur = it & 1, kt = it % nk;
    if (it + 1 < total) MDG_LOAD_TILES(it + 1);
    const CT* Ab = (AMODE == MDG_A_PLAIN) ? As + cur * BM * LDT : As;
    const int acol = (AMODE == MDG_A_PLAIN) ? 0 : kt * BK;
    const CT* Bb = Bs + cur * BN * LDT;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      typename V8<CT>::T a[MT], b[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = ld8<CT>(Ab + (wm * HM + i * 16 + lr) * lda_s + acol + kk + 8 * lg);
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = ld8<CT>(Bb + (wn * HN + j * 16 + lr) * LDT + kk + 8 * lg);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) mma_k32<CT>(acc[i][j], a[i], b[j]);
    }
    if (it + 1 < total) MDG_STORE_TILES(cur ^ 1);

    if (kt == nk - 1) {
      // ------------------------------------------------------------ epilogue
      // Per wave, per 16-row MFMA tile: accumulators -> wave-private LDS stage -> each lane
      // takes 4 contiguous columns of one row (16-B fp32 / 8-B bf16 global accesses) instead
      // of scattered 2-4 B lane stores.
      const int n0 = (nt0 + it / nk) * BN + wn * HN;
      // the stage aliases tile buffers no longer read: PLAIN (one N tile per block) the A ring,
      // LNMOD the B buffer of the tile just consumed (the next tile's first K-step is in cur^1)
      __syncthreads();
      float* stg = (STAGE_ALIAS ? reinterpret_cast<float*>(AMODE == MDG_A_PLAIN ? As : Bs + cur * BN * LDT)
                                : reinterpret_cast<float*>(Bs + 2 * BN * LDT)) + wave * 16 * LDS_ST;
      const int srow = lane / (HN / CPL_Q), scol0 = (lane % (HN / CPL_Q)) * CPL_Q;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) stg[(lg * 4 + r) * LDS_ST + j * 16 + lr] = acc[i][j][r];
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's stage writes landed
        __builtin_amdgcn_wave_barrier();
        const int m = m0 + wm * HM + i * 16 + srow;
#pragma unroll
        for (int q = 0; q < CPL_Q; q += 4) {
          const int c = scol0 + q, n = n0 + c;
          float4 v = *reinterpret_cast<const float4*>(stg + srow * LDS_ST + c);
          if (p.bias) {
            const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
            v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
          }
          if (m >= M) continue;
          if constexpr (EPI == MDG_EPI_STORE) {
            if (p.act == MDG_ACT_GELU) {
              v.x = gelu_erf(v.x); v.y = gelu_erf(v.y); v.z = gelu_erf(v.z); v.w = gelu_erf(v.w);
            } else if (p.act == MDG_ACT_SILU) {
              v.x = silu(v.x); v.y = silu(v.y); v.z = silu(v.z); v.w = silu(v.w);
            }
            if (p.out_f32) *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + (size_t)m * p.ldo + n) = v;
            else st4<CT>(reinterpret_cast<CT*>(p.out) + (size_t)m * p.ldo + n, v.x, v.y, v.z, v.w);
          } else if constexpr (EPI == MDG_EPI_GATE_RES) {
            float4* R = reinterpret_cast<float4*>(p.resid + (size_t)m * p.ldr + n);
            float4 hv = *R;
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
            const int which = n / Cm, w = n - which * Cm, head = w / D, cp = w - head * D;
            if (which == 0) {
              v.x *= p.qscale; v.y *= p.qscale; v.z *= p.qscale; v.w *= p.qscale;
            }
            if (p.rope && which < 2) {
              const int half = D >> 1, pi = cp >> 1;
              const int pos = (p.qkv_layout == MDG_QKV_SPATIAL) ? (m % p.L) : ((m / p.L) % p.T);
              const float* cs = p.rope + (size_t)pos * half + pi;
              const float* sn = p.rope + (size_t)p.rope_rows * half + (size_t)pos * half + pi;
              const float c0 = cs[0], s0 = sn[0], c1 = cs[1], s1 = sn[1];
              const float x0 = v.x * c0 - v.y * s0, y0 = v.y * c0 + v.x * s0;
              const float x1 = v.z * c1 - v.w * s1, y1 = v.w * c1 + v.z * s1;
              v.x = x0; v.y = y0; v.z = x1; v.w = y1;
            }
            CT* dst;
            if (p.qkv_layout == MDG_QKV_SPATIAL) {
              dst = reinterpret_cast<CT*>(p.qkv_out) + ((size_t)(m * 3 + which) * p.H + head) * MDG_DP + cp;
            } else {
              const int TL = p.T * p.L, bb = m / TL, l = m % p.L, t = (m / p.L) % p.T;
              const int BL = (M / TL) * p.L, seq = bb * p.L + l;
              dst = reinterpret_cast<CT*>(p.qkv_out) + (size_t)which * BL * p.H * p.T * MDG_DP +
                    ((size_t)(seq * p.H + head) * p.T + t) * MDG_DP + cp;
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
                if (xo) xo[rowoff + n + e] = __fadd_rn(p.x_in[rowoff + n + e], __fmul_rn(p.dt, vv[e]));
              }
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
  }
#undef MDG_LOAD_TILES
#undef MDG_STORE_TILES
}

template <typename CT, int BM, int BN, int AMODE>
static size_t smem_bytes(int K) {
  constexpr int BK = 64, VEC = 16 / sizeof(CT), LDT = BK + VEC;
  // the epilogue stage [4 waves][16][BN/2+4] fp32 aliases a tile buffer when it fits
  constexpr size_t stage = 4ull * 16 * (BN / 2 + 4) * 4;
  constexpr bool alias = (AMODE == MDG_A_PLAIN) ? stage <= 2ull * BM * LDT * sizeof(CT)
                                                : stage <= 1ull * BN * LDT * sizeof(CT);
  const size_t b = 2ull * BN * LDT * sizeof(CT) + (alias ? 0 : stage);
  if (AMODE == MDG_A_LNMOD) return (size_t)BM * (K + VEC) * sizeof(CT) + b;
  return 2ull * BM * LDT * sizeof(CT) + b;
}

struct GemmPlan {
  int bm, bn;
  size_t smem;
};

template <typename CT, int BM, int BN, int AMODE, int EPI>
static hipError_t launch_one(const mdg_gemm_desc& p, hipStream_t s) {
  const size_t smem = smem_bytes<CT, BM, BN, AMODE>(p.K);
  static bool attr_set = false;  // idempotent attribute write
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<CT, BM, BN, AMODE, EPI>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  // PLAIN: one N tile per block.  LNMOD: a block sweeps a group of N tiles so the LayerNorm
  // is computed once per row per group; groups chosen so the grid keeps >= ~2 blocks per CU.
  const int n_tiles = p.N / BN, m_tiles = (p.M + BM - 1) / BM;
  int groups = n_tiles;
  if (AMODE == MDG_A_LNMOD) {  // the resident A block allows one block per CU: aim for ~256
    int want = (256 + m_tiles - 1) / m_tiles;
    if (want < 1) want = 1;
    if (want > n_tiles) want = n_tiles;
    const int tpg = (n_tiles + want - 1) / want;
    groups = (n_tiles + tpg - 1) / tpg;
  }
  hipLaunchKernelGGL((gemm_kernel<CT, BM, BN, AMODE, EPI>), dim3(groups, m_tiles), dim3(256), smem, s, p);
  return hipGetLastError();
}

template <typename CT, int BM, int BN>
static hipError_t dispatch_mode(const mdg_gemm_desc& p, hipStream_t s) {
  if (p.a_mode == MDG_A_LNMOD) {
    switch (p.epi) {
      case MDG_EPI_STORE: return launch_one<CT, BM, BN, MDG_A_LNMOD, MDG_EPI_STORE>(p, s);
      case MDG_EPI_GATE_RES: return launch_one<CT, BM, BN, MDG_A_LNMOD, MDG_EPI_GATE_RES>(p, s);
      case MDG_EPI_QKV: return launch_one<CT, BM, BN, MDG_A_LNMOD, MDG_EPI_QKV>(p, s);
      default: return launch_one<CT, BM, BN, MDG_A_LNMOD, MDG_EPI_EULER>(p, s);
    }
  }
  switch (p.epi) {
    case MDG_EPI_STORE: return launch_one<CT, BM, BN, MDG_A_PLAIN, MDG_EPI_STORE>(p, s);
    case MDG_EPI_GATE_RES: return launch_one<CT, BM, BN, MDG_A_PLAIN, MDG_EPI_GATE_RES>(p, s);
    case MDG_EPI_QKV: return launch_one<CT, BM, BN, MDG_A_PLAIN, MDG_EPI_QKV>(p, s);
    default: return launch_one<CT, BM, BN, MDG_A_PLAIN, MDG_EPI_EULER>(p, s);
  }
}

// Tile plan: bf16 BN = 128 where N allows, else 32; f32 BN = 96/128 for streamed A, 32 for the
// LN-resident A (an fp32 64 x 384 block already takes 99 KB of LDS).  BM = 128 for bf16 when
// the grid still fills the chip, else 64.  Returns bn = 0 if unsupported.
GemmPlan gemm_plan(const mdg_gemm_desc& p) {
  GemmPlan g{0, 0, 0};
  const bool bf = p.dtype == MDG_BF16, ln = p.a_mode == MDG_A_LNMOD;
  if (bf) {
    g.bn = (p.N % 128 == 0) ? 128 : (p.N % 32 == 0 ? 32 : 0);
  } else if (ln) {
    g.bn = (p.N % 32 == 0) ? 32 : 0;
  } else {
    g.bn = (p.N % 96 == 0) ? 96 : (p.N % 128 == 0 ? 128 : (p.N % 32 == 0 ? 32 : 0));
  }
  if (!g.bn) return g;
  if (bf) {
    const long tiles128 = (long)((p.M + 127) / 128) * (ln ? 2 : p.N / g.bn);
    g.bm = (p.M >= 128 * 64 && tiles128 >= 256) ? 128 : 64;
    if (g.bm == 128)
      g.smem = ln ? (g.bn == 128 ? smem_bytes<bf16_t, 128, 128, 1>(p.K) : smem_bytes<bf16_t, 128, 32, 1>(p.K))
                  : (g.bn == 128 ? smem_bytes<bf16_t, 128, 128, 0>(p.K) : smem_bytes<bf16_t, 128, 32, 0>(p.K));
    else
      g.smem = ln ? (g.bn == 128 ? smem_bytes<bf16_t, 64, 128, 1>(p.K) : smem_bytes<bf16_t, 64, 32, 1>(p.K))
                  : (g.bn == 128 ? smem_bytes<bf16_t, 64, 128, 0>(p.K) : smem_bytes<bf16_t, 64, 32, 0>(p.K));
  } else {
    g.bm = 64;
    if (ln) g.smem = smem_bytes<float, 64, 32, 1>(p.K);
    else if (g.bn == 96) g.smem = smem_bytes<float, 64, 96, 0>(p.K);
    else if (g.bn == 128) g.smem = smem_bytes<float, 64, 128, 0>(p.K);
    else g.smem = smem_bytes<float, 64, 32, 0>(p.K);
  }
  return g;
}

hipError_t gemm_launch(const mdg_gemm_desc& p, const GemmPlan& g, hipStream_t s) {
  if (p.dtype == MDG_BF16) {
    if (g.bm == 128) return g.bn == 128 ? dispatch_mode<bf16_t, 128, 128>(p, s) : dispatch_mode<bf16_t, 128, 32>(p, s);
    return g.bn == 128 ? dispatch_mode<bf16_t, 64, 128>(p, s) : dispatch_mode<bf16_t, 64, 32>(p, s);
  }
  if (g.bn == 96) return dispatch_mode<float, 64, 96>(p, s);
  if (g.bn == 128) return dispatch_mode<float, 64, 128>(p, s);
  return dispatch_mode<float, 64, 32>(p, s);
}

}  // namespace mdg
