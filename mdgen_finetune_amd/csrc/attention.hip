// Attention kernels of the MDGen block (reference MultiheadAttention rope + bias_kv path,
// mha.py:161-407, called through AttentionWithRoPE latent_model.py:329-338).
//
// Both kernels read Q/K/V written by the QKV-GEMM epilogue (gemm.hip): already biased,
// q-scaled and RoPE-rotated, head_dim D padded to MDG_DP = 32 with zeros.  The learned
// bias_k / bias_v row (appended after projection, mha.py:265-280, never key-padding-masked,
// RoPE-rotated at position S because fair-esm builds its table from k's length S+1) arrives
// pre-rotated in `kvb` [H][2][32] and is handled as a virtual key processed first, so the
// running max is finite before any -inf masked key is seen.
//
//  * attn_temporal: flash-style over the T frames of one (batch, residue) sequence.
//    Swapped product S^T = K Q^T on the matrix cores (16x16x32 bf16 / 16x16x4 f32), so each
//    lane holds 16 keys of ONE query per 64-key chunk: the row max is 15 local fmax + two
//    cross-lane shuffles, and the probabilities P^T are already the B operand of
//    O^T = V^T P^T (the key permutation of that operand is matched by the V^T fragment read,
//    ds_read_b64_tr_b16 of a row-major V tile).  The softmax denominator comes out of the
//    same MFMAs: V's pad column D holds 1.0, so O^T row D = sum_k p_k.  Scores are in
//    log2 units (q was pre-scaled by log2 e) and exponentiated with v_exp_f32; the running
//    max subtraction also rides in the MFMA (K pad column D = 1.0, Q pad element = -offset).
//  * attn_spatial: L+1 keys per query (L = crop = 4): one thread per (token, head), fp32
//    online softmax on the VALU — no MFMA shape fits 4x5 scores.
#include "../../include/mdgen_hip.h"
#include "common.h"

#include <stdlib.h>

namespace mdg {


// DP = padded head dim (MDG_DP for head_dim <= 31, MDG_DP_WIDE up to 63): the QK product runs
// DP / 32 K-steps and O^T has DP / 16 row tiles.
template <typename CT, int DP>
__global__ __launch_bounds__(256) void attn_temporal_kernel(const CT* __restrict__ qkv,
                                                            const float* __restrict__ kbias,
                                                            const float* __restrict__ kvb,
                                                            CT* __restrict__ out, int T, int L,
                                                            int H, int D, int BL, float* __restrict__ lse,
                                                            CT* __restrict__ out_lo = nullptr) {
  constexpr int KC = 64, LDK = DP + 16;  // DP 32: 96-B LDS rows (bf16), conflict-free b128 + tr reads
  constexpr int KS = DP / 32, DT = DP / 16;
  constexpr int VEC = 16 / sizeof(CT);
  constexpr int PIECES = KC * DP / VEC / 256;
  __shared__ __attribute__((aligned(16))) CT Ks[2][KC * LDK];
  __shared__ __attribute__((aligned(16))) CT Vs[2][KC * LDK];
  __shared__ float kbs[2][KC];
  __shared__ int kflag[2];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int seq = blockIdx.z, head = blockIdx.y;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const size_t plane = (size_t)BL * H * T * DP;
  const CT* Qg = qkv + ((size_t)seq * H + head) * T * DP;
  const CT* Kg = Qg + plane;
  const CT* Vg = Qg + 2 * plane;
  const float* kb = kbias + (size_t)seq * T;

  typename V8<CT>::T qf[2][KS];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = q0 + qg * 16 + lr;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[qg][ks] = (q < T) ? ld8<CT>(Qg + (size_t)q * DP + 32 * ks + 8 * lg) : zero8<CT>();
  }

  // virtual bias key first.  The running softmax offset mt (per query, exactly representable
  // in CT) rides in the MFMA: K's pad column D holds 1.0 and Q's pad element D holds -mt, so
  // S^T = K Q^T comes out of the matrix cores already as score - mt and the common case
  // needs one v_exp_f32 per score and nothing else.  mt is only raised (rare path below)
  // when a score exceeds it by more than kGrow (log2 units), so p <= 2^kGrow.
  constexpr float kGrow = 8.0f;
  const int pads = D >> 5, padg = (D & 31) >> 3, pade = D & 7;  // K-step / lane group / element of pad column
  const float* kvh = kvb + head * 2 * DP;
  float mt[2];
  f32x4 o[DT][2];  // [d-tile][q-group]: O^T[d = 16dt + 4lg + i][q = lr]
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    float sb = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) sb += (float)qf[qg][ks][j] * kvh[32 * ks + 8 * lg + j];
    sb += __shfl_xor(sb, 16, 64);
    sb += __shfl_xor(sb, 32, 64);
    mt[qg] = (float)(CT)sb;
    const float pb = __builtin_amdgcn_exp2f(sb - mt[qg]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) o[dt][qg][i] = pb * kvh[DP + dt * 16 + lg * 4 + i];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (ks == pads && lg == padg && j == pade) qf[qg][ks][j] = (CT)(-mt[qg]);
  }

  uint4 kreg[PIECES], vreg[PIECES];
  float kbreg = 0.f;
  auto gload = [&](int c) {
#pragma unroll
    for (int pc = 0; pc < PIECES; ++pc) {
      const int idx = tid + pc * 256, row = idx / (DP / VEC), cc = idx % (DP / VEC);
      const int key = c * KC + row;
      if (key < T) {
        kreg[pc] = *reinterpret_cast<const uint4*>(Kg + (size_t)key * DP + cc * VEC);
        vreg[pc] = *reinterpret_cast<const uint4*>(Vg + (size_t)key * DP + cc * VEC);
      } else {
        kreg[pc] = make_uint4(0, 0, 0, 0);
        vreg[pc] = make_uint4(0, 0, 0, 0);
      }
    }
    if (tid < KC) {
      const int key = c * KC + tid;
      kbreg = (key < T) ? kb[key] : -INFINITY;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int pc = 0; pc < PIECES; ++pc) {
      const int idx = tid + pc * 256, row = idx / (DP / VEC), cc = idx % (DP / VEC);
      *reinterpret_cast<uint4*>(&Ks[buf][row * LDK + cc * VEC]) = kreg[pc];
      *reinterpret_cast<uint4*>(&Vs[buf][row * LDK + cc * VEC]) = vreg[pc];
    }
    if (tid < KC) {
      kbs[buf][tid] = kbreg;
      const bool any = __any(kbreg != 0.f);
      if (tid == 0) kflag[buf] = any ? 1 : 0;
    }
  };

  const int nchunks = (T + KC - 1) / KC;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const int cur = c & 1;
    if (c + 1 < nchunks) gload(c + 1);
    const CT* Kc = Ks[cur];
    const CT* Vc = Vs[cur];

    f32x4 s[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) s[kt][qg] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const typename V8<CT>::T kf = ld8<CT>(Kc + (kt * 16 + lr) * LDK + 32 * ks + 8 * lg);
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) mma_k32<CT>(s[kt][qg], kf, qf[qg][ks]);
      }
    }
    if (kflag[cur]) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float bb = kbs[cur][kt * 16 + lg * 4 + i];
          s[kt][0][i] += bb;
          s[kt][1][i] += bb;
        }
    }
    float mx[2];
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      float m = s[0][qg][0];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) m = fmaxf(m, s[kt][qg][i]);
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      mx[qg] = fmaxf(m, __shfl_xor(m, 32, 64));
    }
    if (__builtin_expect(__any(mx[0] > kGrow || mx[1] > kGrow), 0)) {
      // raise the offset of the queries that outgrew it: rescale O, shift this chunk's scores
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) {
        const float nm = (mx[qg] > kGrow) ? (float)(CT)(mt[qg] + mx[qg]) : mt[qg];
        const float delta = nm - mt[qg];
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        mt[qg] = nm;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[dt][qg][i] *= alpha;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) s[kt][qg][i] -= delta;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (ks == pads && lg == padg && j == pade) qf[qg][ks][j] = (CT)(-nm);
      }
    }
#pragma unroll
    for (int qg = 0; qg < 2; ++qg)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) s[kt][qg][i] = __builtin_amdgcn_exp2f(s[kt][qg][i]);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      typename V8<CT>::T pf[2];
#pragma unroll
      for (int qg = 0; qg < 2; ++qg)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pf[qg][j] = (CT)s[2 * kh][qg][j];
          pf[qg][4 + j] = (CT)s[2 * kh + 1][qg][j];
        }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        typename V8<CT>::T vf;
        if constexpr (is_bf16<CT>()) {
          typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
          const bf16_t* pa = Vc + (32 * kh + 4 * lg + (lr >> 2)) * LDK + dt * 16 + 4 * (lr & 3);
          const bf16_t* pb = pa + 16 * LDK;
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(pa));
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(pb));
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            vf[j] = lo[j];
            vf[4 + j] = hi[j];
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            vf[j] = Vc[(32 * kh + 4 * lg + j) * LDK + dt * 16 + lr];
            vf[4 + j] = Vc[(32 * kh + 16 + 4 * lg + j) * LDK + dt * 16 + lr];
          }
        }
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) mma_k32<CT>(o[dt][qg], vf, pf[qg]);
      }
    }
    if (c + 1 < nchunks) lstore(cur ^ 1);
    __syncthreads();
  }

  // normalise by the row sum carried in O^T row D, write O[token][head*D + d]
  const int dt_s = D >> 4, g_s = (D & 15) >> 2, i_s = D & 3;
  const int C = H * D, b = seq / L, l = seq % L;
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    float mine = 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (dt == dt_s && i == i_s) mine = o[dt][qg][i];
    const float lsum = __shfl(mine, lr + 16 * g_s, 64);
    const float inv = 1.0f / lsum;
    const int q = q0 + qg * 16 + lr;
    if (lse && q < T && lg == 0) lse[((size_t)seq * H + head) * T + q] = mt[qg] + log2f(lsum);
    if (q < T) {
      CT* orow = out + ((size_t)(b * T + q) * L + l) * C + head * D;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int d0 = dt * 16 + lg * 4;
        if (d0 < D) {
          const float v0 = o[dt][qg][0] * inv, v1 = o[dt][qg][1] * inv, v2 = o[dt][qg][2] * inv,
                      v3 = o[dt][qg][3] * inv;
          st4<CT>(orow + d0, v0, v1, v2, v3);
          if (out_lo)  // training: O - CT(O), the backward's delta = dO . (O + O_lo)
            st4<CT>(out_lo + (orow - out) + d0, v0 - (float)(CT)v0, v1 - (float)(CT)v1, v2 - (float)(CT)v2,
                    v3 - (float)(CT)v3);
        }
      }
    }
  }
}

// bf16 temporal attention on 32x32x16 MFMAs.  A block = 8 waves x 32 queries of one
// (sequence, head); K/V stream through LDS in 128-key chunks (register-staged double
// buffer, one barrier per chunk), each chunk processed as two 64-key sub-chunks:
//   S^T (2 tiles of 32 keys x 32 queries) = K Q^T   — lane l holds 16 keys of query l&31
//     (rows (reg&3) + 8(reg>>2) + 4(l>>5)); K is the A operand read by ds_read_b128 from an
//     image whose 16-B chunk c of key row k sits at c ^ ((k>>3)&3) (conflict-free for the
//     four ds_read_b128 lane groups), Q the B operand held in registers;
//   P = exp2(S^T) converted pairwise to bf16 IS the B operand of O^T = V^T P (the
//     accumulator-as-operand map: element j of k-step s is key 16s + 8(j>>2) + 4h + (j&3)),
//     and the matching V^T fragment is two ds_read_b64_tr_b16 of the plain [key][32] image;
//   the softmax offset rides in the QK MFMA (K pad column D = 1, Q pad element = -mt, mt =
//   the bias key's score); the row sum is O^T row D (V pad column = 1).
// Optimistic pass first: the offset is never raised and no score is tested, so the common
// path is one v_exp_f32 and half a v_cvt_pk per score.  P is floating point, so a lagging
// offset costs no precision unless something overflows (a score 128 above the bias key's, or
// the f32 accumulators); the pass ends with a block-wide finiteness test of O^T and, when it
// fails, the block reruns with the growth-tested offset (raised whenever a score outgrows it
// by kGrow), the only path whose P stay bounded.
typedef __attribute__((ext_vector_type(16))) float f32x16;
// timing diagnostics only (tools/diag_mlp_attn.sh): 1 = exp2 replaced by the identity, 2 = no
// K / V chunk restaged after the first.  Results are wrong in every diagnostic build.
#ifndef MDG_DIAG_ATTN
#define MDG_DIAG_ATTN 0
#endif

// One 64-key sub-chunk of the bf16 temporal attention (K / V images of its 64 rows at Kc /
// Vc, key-padding bias at kbsub): S^T = K Q^T (4 MFMAs), growth test / rare offset raise,
// P = exp2(S^T) -> bf16 B operand, O^T += V^T P (4 MFMAs with tr-read V^T fragments).
__device__ __forceinline__ void ta_subchunk(const bf16_t* Kc, const bf16_t* Vc, const float* kbsub, bool masked, bool GROW,
                                            int r, int h, int grow, int gcol, int padS, int padH, int padJ,
                                            bf16x8 (&qf)[2], float& mt, f32x16& o) {
  constexpr int DP = MDG_DP;
  constexpr float kGrow = 8.0f;
  typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
  f32x16 sacc[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int row = kt * 32 + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) sacc[kt][i] = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Kc + row * DP + (((2 * s2 + h) ^ ((row >> 3) & 3)) * 8));
      sacc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s2], sacc[kt], 0, 0, 0);
    }
  }
  if (masked) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[kt][i] += kbsub[kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h];
  }
  float lm = sacc[0][0];
  if (GROW) {  // block-uniform
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) lm = fmaxf(lm, sacc[kt][i]);
  }
  if (GROW && __builtin_expect(__any(lm > kGrow), 0)) {
    const float mx = fmaxf(lm, __shfl_xor(lm, 32, 64));
    const float nm = (mx > kGrow) ? (float)(bf16_t)(mt + mx) : mt;
    const float delta = nm - mt;
    const float alpha = __builtin_amdgcn_exp2f(-delta);
    mt = nm;
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] *= alpha;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[kt][i] -= delta;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (s2 == padS && h == padH && j == padJ) qf[s2][j] = (bf16_t)(-nm);
  }
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        pf[j] = (bf16_t)(MDG_DIAG_ATTN == 1 ? sacc[kt][8 * s2 + j] : __builtin_amdgcn_exp2f(sacc[kt][8 * s2 + j]));
      const bf16_t* vb = Vc + (kt * 32 + 16 * s2 + grow) * DP + gcol;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(vb));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(vb + 8 * DP));
      bf16x8 vf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        vf[j] = lo[j];
        vf[4 + j] = hi[j];
      }
      o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o, 0, 0, 0);
    }
  }
}

// Bias key + offset setup shared by both bf16 temporal kernels: Q fragments (B operand,
// d = 16s + 8h + j), mt = bf16(score of the bias key), O^T = exp2(score_b - mt) * bias_v,
// Q pad element = -mt.
// rs = the planes' row stride: MDG_DP (padded) or D (packed: the 8-column pieces at and after
// column D are not in memory and read as zeros)
__device__ __forceinline__ void ta_setup(const bf16_t* Qg, const float* kvh, int q, int T, int D, int rs, int r,
                                         int h, bf16x8 (&qf)[2], float& mt, f32x16& o) {
  constexpr int DP = MDG_DP;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int pc = 16 * s2 + 8 * h;  // first column of this lane's 8-column piece
    qf[s2] = (q < T && pc < (rs == DP ? DP : D)) ? *reinterpret_cast<const bf16x8*>(Qg + (size_t)q * rs + pc)
                                                 : zero8<bf16_t>();
  }
  float sb = 0.f;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < 8; ++j) sb += (float)qf[s2][j] * kvh[16 * s2 + 8 * h + j];
  sb += __shfl_xor(sb, 32, 64);
  mt = (float)(bf16_t)sb;
  const float pb = __builtin_amdgcn_exp2f(sb - mt);
#pragma unroll
  for (int i = 0; i < 16; ++i) o[i] = pb * kvh[DP + (i & 3) + 8 * (i >> 2) + 4 * h];
  const int padS = D >> 4, padH = (D >> 3) & 1, padJ = D & 7;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (s2 == padS && h == padH && j == padJ) qf[s2][j] = (bf16_t)(-mt);
}

// O = O^T / row sum (O^T row D), stored as O[token][head*D + d]
__device__ __forceinline__ void ta_store(const f32x16& o, bf16_t* out, int q, int T, int L, int H, int D, int seq,
                                         int head, int h, float mt, float* lse, bf16_t* out_lo) {
  const int hD = (D >> 2) & 1, regD = (D & 3) + 4 * (D >> 3);
  float mine = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i == regD) mine = o[i];
  const float other = __shfl_xor(mine, 32, 64);
  const float lsum = (h == hD) ? mine : other;
  const float inv = 1.0f / lsum;
  // log2 of the row's softmax normaliser in the score units of the kernel (q pre-scaled by
  // log2 e): the training backward recomputes P = exp2(S - lse) from it
  if (lse && q < T && h == 0) lse[((size_t)seq * H + head) * T + q] = mt + log2f(lsum);
  if (q < T) {
    const int C = H * D, b = seq / L, l = seq % L;
    bf16_t* orow = out + ((size_t)(b * T + q) * L + l) * C + head * D;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d0 = 8 * g4 + 4 * h;
      if (d0 < D)
        st4<bf16_t>(orow + d0, o[4 * g4] * inv, o[4 * g4 + 1] * inv, o[4 * g4 + 2] * inv, o[4 * g4 + 3] * inv);
    }
    // training: the bf16 rounding residual of O (O = out + out_lo to ~2^-17), so the backward's
    // delta = dO . O matches the fp32 P it recomputes even where the bias key dominates a row
    // (a fully padded sequence: P = [1, 0, ...], true dS = 0)
    if (out_lo) {
      bf16_t* lrow = out_lo + ((size_t)(b * T + q) * L + l) * C + head * D;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 8 * g4 + 4 * h;
        if (d0 < D) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x = o[4 * g4 + e] * inv;
            v[e] = x - (float)(bf16_t)x;
          }
          st4<bf16_t>(lrow + d0, v[0], v[1], v[2], v[3]);
        }
      }
    }
  }
}


template <int kTW, int kTKC, int PD>  // waves per block, keys per LDS chunk, packed head dim (0: padded)
__global__ __launch_bounds__(kTW * 64, 4) void attn_temporal_bf16_kernel(const bf16_t* __restrict__ qkv,
                                                                    const float* __restrict__ kbias,
                                                                    const float* __restrict__ kvb,
                                                                    bf16_t* __restrict__ out, int T, int L,
                                                                    int H, int D, int BL, float* __restrict__ lse,
                                                                    bf16_t* __restrict__ out_lo) {
  constexpr int DP = MDG_DP, KC = kTKC, NTH = kTW * 64;
  constexpr bool PACKED = PD > 0;
  constexpr int RS = PACKED ? PD : DP;  // plane row stride (a compile-time constant either way)
  if constexpr (PACKED) D = PD;
  static_assert(KC * DP / 8 == NTH, "one 16-B K piece and one V piece per thread per chunk");
  __shared__ __attribute__((aligned(16))) bf16_t Ks[2][KC * DP];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[2][KC * DP];
  __shared__ float kbs[2][KC];
  __shared__ int kflag[2][KC / 64];

  __shared__ int s_bad;
  if (threadIdx.x == 0) s_bad = 0;  // published by the first chunk barrier
  // The optimistic pass, and (rarely, block-uniform) the growth-tested rerun.  Every per-thread
  // value is derived from an opaque copy of the thread index inside the attempt loop, so
  // nothing but the loop counter lives across attempts (hoisted addresses spilled).
  for (int attempt = 0;; ++attempt) {
    const bool grow = attempt > 0;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    // XCD-aware order (bijective remap of the 1-D grid): the query blocks of one (sequence,
    // head) are consecutive on one XCD, so its K / V are fetched into that XCD's L2 once
    const int nqb = (T + kTW * 32 - 1) / (kTW * 32), nwg = nqb * H * BL;
    const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, qq = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (qq + 1) : r8 * (qq + 1) + (xcd - r8) * qq) + loc;
    const int qb = wg % nqb, head = (wg / nqb) % H, seq = wg / (nqb * H);
    const int q0 = qb * (kTW * 32) + wave * 32;
    const size_t plane = (size_t)BL * H * T * RS;
    const bf16_t* Qg = qkv + ((size_t)seq * H + head) * T * RS;
    const bf16_t* Kg = Qg + plane;
    const bf16_t* Vg = Qg + 2 * plane;
    const float* kb = kbias + (size_t)seq * T;

    const int q = q0 + r;
    bf16x8 qf[2];
    float mt;
    f32x16 o;
    ta_setup(Qg, kvb + head * 2 * DP, q, T, D, RS, r, h, qf, mt, o);
    const int padS = D >> 4, padH = (D >> 3) & 1, padJ = D & 7;  // Q element holding -mt

    // chunk staging: thread -> key row tid/4, 16-B piece tid%4 of K and of V
    const int srow = tid >> 2, spc = tid & 3;
    u32x4 kreg, vreg;
    float kbreg = 0.f;
    // packed planes: the pieces at and after column D are not in memory.  Their LDS slots (fixed
    // per thread) hold 1.0 at column D for k (softmax offset) and v (row sum), zeros elsewhere --
    // exactly the padded rows' content -- written before the first chunk and never restaged
    // (rows past T are masked by the -inf key bias, so their constant pad is harmless).
    const bool real = !PACKED || spc * 8 < D;
    if (PACKED && !real && !grow) {
      u32x4 synth = u32x4{0u, 0u, 0u, 0u};
      if (spc == (D >> 3)) {
        const int e = D & 7;  // bf16 1.0 = 0x3F80 in half e & 1 of dword e >> 1
#pragma unroll
        for (int w = 0; w < 4; ++w) synth[w] = (w == (e >> 1)) ? (0x3F80u << (16 * (e & 1))) : 0u;
      }
#pragma unroll
      for (int bf = 0; bf < 2; ++bf) {
        *reinterpret_cast<u32x4*>(&Ks[bf][srow * DP + ((spc ^ ((srow >> 3) & 3)) * 8)]) = synth;
        *reinterpret_cast<u32x4*>(&Vs[bf][srow * DP + spc * 8]) = synth;
      }
    }
#define MDG_TA_GLOAD(c_)                                                                      \
  {                                                                                           \
    const int key = (c_) * KC + srow;                                                         \
    kreg = vreg = u32x4{0u, 0u, 0u, 0u};                                                      \
    if (key < T && real) {                                                                    \
      kreg = *reinterpret_cast<const u32x4*>(Kg + (size_t)key * RS + spc * 8);                \
      vreg = *reinterpret_cast<const u32x4*>(Vg + (size_t)key * RS + spc * 8);                \
    }                                                                                         \
    if (tid < KC) {                                                                           \
      const int kk = (c_) * KC + tid;                                                         \
      kbreg = (kk < T) ? kb[kk] : -INFINITY;                                                  \
    }                                                                                         \
  }
#define MDG_TA_LSTORE(buf)                                                                    \
  {                                                                                           \
    if (real) {                                                                               \
      *reinterpret_cast<u32x4*>(&Ks[buf][srow * DP + ((spc ^ ((srow >> 3) & 3)) * 8)]) = kreg; \
      *reinterpret_cast<u32x4*>(&Vs[buf][srow * DP + spc * 8]) = vreg;                        \
    }                                                                                         \
    if (tid < KC) {                                                                           \
      kbs[buf][tid] = kbreg;                                                                  \
      const bool any = __any(kbreg != 0.f);                                                   \
      if (lane == 0) kflag[buf][wave] = any ? 1 : 0;                                          \
    }                                                                                         \
  }

    const int nchunks = (T + KC - 1) / KC;
    // V^T tr-read lane geometry: 16-lane group g reads keys (+4h + i>>2), columns 16(g&1) + 4(i&3)
    const int gi = lane & 15, gcol = 16 * ((lane >> 4) & 1) + 4 * (gi & 3), grow_r = 4 * h + (gi >> 2);
    MDG_TA_GLOAD(0);
    MDG_TA_LSTORE(0);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
      const int cur = c & 1;
      if (c + 1 < nchunks && MDG_DIAG_ATTN != 2) MDG_TA_GLOAD(c + 1);
      int mflag = 0;
#pragma unroll
      for (int f = 0; f < KC / 64; ++f) mflag |= kflag[cur][f];
      const bool masked = mflag != 0;
      const bf16_t* Kc = Ks[cur];
      const bf16_t* Vc = Vs[cur];
#pragma unroll
      for (int sub = 0; sub < KC / 64; ++sub)
        ta_subchunk(Kc + sub * 64 * DP, Vc + sub * 64 * DP, kbs[cur] + sub * 64, masked, grow, r, h, grow_r, gcol,
                    padS, padH, padJ, qf, mt, o);
      if (c + 1 < nchunks && MDG_DIAG_ATTN != 2) MDG_TA_LSTORE(cur ^ 1);
      __syncthreads();
    }
#undef MDG_TA_GLOAD
#undef MDG_TA_LSTORE
    if (!grow) {
      bool bad = false;
#pragma unroll
      for (int i = 0; i < 16; ++i) bad |= !__builtin_isfinite(o[i]);
      if (__any(bad) && lane == 0) s_bad = 1;
      __syncthreads();
    }
    if (grow || !s_bad) {  // block-uniform
      ta_store(o, out, q, T, L, H, D, seq, head, h, mt, lse, out_lo);
      return;
    }
  }
}


// Spatial attention over the L residues of one frame (+ the bias key): q|k|v come unpadded,
// [token][3][H][D] (no MFMA reads them), so each (token, head) thread reads D-element rows.
template <typename CT, int DP>
__global__ __launch_bounds__(256) void attn_spatial_kernel(const CT* __restrict__ qkv,
                                                           const float* __restrict__ kvb,
                                                           const float* __restrict__ mask,
                                                           CT* __restrict__ out, int nf, int L,
                                                           int H, int D) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= nf * L * H) return;
  const int h = idx % H, tok = idx / H, f = tok / L;
  const size_t tstride = 3ull * H * D;
  float q[DP];
  const CT* qp = qkv + (size_t)tok * tstride + h * D;
#pragma unroll
  for (int d = 0; d < DP; d += 4) {
    const float4 v = (d < D) ? ld4f<CT>(qp + d) : make_float4(0.f, 0.f, 0.f, 0.f);
    q[d] = v.x; q[d + 1] = v.y; q[d + 2] = v.z; q[d + 3] = v.w;
  }
  const float* kbh = kvb + h * 2 * DP;
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < DP; ++d) s += q[d] * kbh[d];
  float m = s, lsum = 1.0f;
  float acc[DP];
#pragma unroll
  for (int d = 0; d < DP; ++d) acc[d] = kbh[DP + d];
  for (int j = 0; j < L; ++j) {
    const int kt = f * L + j;
    if (mask && mask[kt] == 0.f) continue;
    const CT* kp = qkv + (size_t)kt * tstride + (size_t)H * D + h * D;
    const CT* vp = kp + (size_t)H * D;
    float sc = 0.f;
#pragma unroll
    for (int d = 0; d < DP; d += 4) {
      if (d < D) {
        const float4 kv = ld4f<CT>(kp + d);
        sc += q[d] * kv.x + q[d + 1] * kv.y + q[d + 2] * kv.z + q[d + 3] * kv.w;
      }
    }
    const float mn = fmaxf(m, sc);
    const float a = expf(m - mn), pj = expf(sc - mn);
    lsum = lsum * a + pj;
#pragma unroll
    for (int d = 0; d < DP; d += 4) {
      if (d < D) {
        const float4 vv = ld4f<CT>(vp + d);
        acc[d] = acc[d] * a + pj * vv.x;
        acc[d + 1] = acc[d + 1] * a + pj * vv.y;
        acc[d + 2] = acc[d + 2] * a + pj * vv.z;
        acc[d + 3] = acc[d + 3] * a + pj * vv.w;
      }
    }
    m = mn;
  }
  const float inv = 1.0f / lsum;
  CT* op = out + (size_t)tok * H * D + h * D;
#pragma unroll
  for (int d = 0; d < DP; d += 4)
    if (d < D) st4<CT>(op + d, acc[d] * inv, acc[d + 1] * inv, acc[d + 2] * inv, acc[d + 3] * inv);
}

// broadcast lane I of every quad (DPP quad_perm(I,I,I,I))
template <int I>
__device__ __forceinline__ float quad_bcast(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), I | (I << 2) | (I << 4) | (I << 6), 0xF, 0xF, true));
}
template <int I, int DM>
__device__ __forceinline__ void qscore(const float (&q)[DM], const float (&k)[DM], float kvalid, float (&sc)[4],
                                       float (&valid)[4]) {
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < DM; ++d) s += q[d] * quad_bcast<I>(k[d]);
  sc[I] = s;
  valid[I] = quad_bcast<I>(kvalid);
}
template <int I, int DM>
__device__ __forceinline__ void qpv(const float (&p)[4], const float (&v)[DM], float (&acc)[DM]) {
#pragma unroll
  for (int d = 0; d < DM; ++d) acc[d] += p[I] * quad_bcast<I>(v[d]);
}

// L == 4 (tetrapeptide crop) fast path: one lane per (frame, head, residue), a quad of lanes
// per (frame, head).  Each lane loads only its own residue's q / k / v rows; the other three
// residues' k and v reach it by DPP quad broadcasts (no LDS, no redundant loads: the
// q|k|v buffer is read from HBM exactly once).  fp32 softmax over the 4 keys + the bias key.
template <typename CT, int DM>
__global__ __launch_bounds__(256) void attn_spatial_quad_kernel(const CT* __restrict__ qkv,
                                                                const float* __restrict__ kvb,
                                                                const float* __restrict__ mask,
                                                                CT* __restrict__ out, int nf, int H, int D) {
  const int DP = dp_of(D);  // kvb row stride
  const int idx = blockIdx.x * 256 + threadIdx.x;   // ((f * H + h) * 4 + j); nf*H*4 % 64 == 0 not assumed
  const int total = nf * H * 4;
  const bool live = idx < total;
  const int j = idx & 3, fh = (live ? idx : total - 1) >> 2, h = fh % H, f = fh / H;
  const int tok = f * 4 + j;
  const size_t tstride = 3ull * H * D;
  const CT* base = qkv + (size_t)tok * tstride + h * D;
  float q[DM], k[DM], v[DM];  // DM = head_dim rounded up to 8 (24 for the default model)
  // 16-B loads (8 bf16): D % 8 == 0 is checked by the launcher for this kernel
#pragma unroll
  for (int d = 0; d < DM; d += 8) {
    typename V8<CT>::T a = zero8<CT>(), b = a, c = a;
    if (d < D) {
      a = ld8<CT>(base + d);
      b = ld8<CT>(base + (size_t)H * D + d);
      c = ld8<CT>(base + 2ull * H * D + d);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      q[d + e] = (float)a[e];
      k[d + e] = (float)b[e];
      v[d + e] = (float)c[e];
    }
  }
  const float kvalid = (!mask || mask[tok] != 0.f) ? 1.f : 0.f;
  const float* kbh = kvb + h * 2 * DP;
  // bias key first (never masked)
  float sb = 0.f;
#pragma unroll
  for (int d = 0; d < DM; ++d) sb += q[d] * kbh[d];
  float sc[4], valid[4];
  qscore<0, DM>(q, k, kvalid, sc, valid);
  qscore<1, DM>(q, k, kvalid, sc, valid);
  qscore<2, DM>(q, k, kvalid, sc, valid);
  qscore<3, DM>(q, k, kvalid, sc, valid);
  float m = sb;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (valid[i] != 0.f) m = fmaxf(m, sc[i]);
  const float pb = expf(sb - m);
  float lsum = pb, p[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p[i] = (valid[i] != 0.f) ? expf(sc[i] - m) : 0.f;
    lsum += p[i];
  }
  float acc[DM];
#pragma unroll
  for (int d = 0; d < DM; ++d) acc[d] = pb * kbh[DP + d];
  qpv<0, DM>(p, v, acc);
  qpv<1, DM>(p, v, acc);
  qpv<2, DM>(p, v, acc);
  qpv<3, DM>(p, v, acc);
  if (!live) return;
  const float inv = 1.0f / lsum;
  CT* op = out + (size_t)tok * H * D + h * D;
#pragma unroll
  for (int d = 0; d < DM; d += 8) {
    if (d < D) {
      typename V8<CT>::T o8;
#pragma unroll
      for (int e = 0; e < 8; ++e) o8[e] = (CT)(acc[d + e] * inv);
      *reinterpret_cast<typename V8<CT>::T*>(op + d) = o8;
    }
  }
}

hipError_t attn_temporal_launch(int dtype, int B, int T, int L, int H, int D, const void* qkv_t,
                                const float* kbias, const float* kvb, void* out, hipStream_t s, float* lse,
                                bool packed, void* out_lo) {
  if (packed && (dtype != MDG_BF16 || D % 8 || D >= MDG_DP)) return hipErrorInvalidValue;
  if (out_lo && dtype != MDG_BF16) return hipErrorInvalidValue;  // (f32 O is exact)
  if (D >= MDG_DP) {  // wide heads (32..63): the generic 16x16 MFMA kernel on 64-column rows
    dim3 grid((T + 127) / 128, H, B * L);
    if (dtype == MDG_BF16)
      hipLaunchKernelGGL((attn_temporal_kernel<bf16_t, MDG_DP_WIDE>), grid, dim3(256), 0, s, (const bf16_t*)qkv_t,
                         kbias, kvb, (bf16_t*)out, T, L, H, D, B * L, lse, (bf16_t*)out_lo);
    else
      hipLaunchKernelGGL((attn_temporal_kernel<float, MDG_DP_WIDE>), grid, dim3(256), 0, s, (const float*)qkv_t,
                         kbias, kvb, (float*)out, T, L, H, D, B * L, lse);
    return hipGetLastError();
  }
  if (dtype == MDG_BF16) {
    // MDG_ATTN_WAVES=4 selects 4-wave blocks with 64-key chunks (tuning knob; default 8 / 128)
    static const int waves = [] {
      const char* e = getenv("MDG_ATTN_WAVES");
      return e ? atoi(e) : 8;
    }();
    if (waves == 4) {
      dim3 grid((unsigned)((T + 127) / 128 * H * B * L));
#define MDG_TA4(PD_)                                                                                     \
  hipLaunchKernelGGL((attn_temporal_bf16_kernel<4, 64, PD_>), grid, dim3(256), 0, s, (const bf16_t*)qkv_t, kbias, \
                     kvb, (bf16_t*)out, T, L, H, D, B * L, lse, (bf16_t*)out_lo)
      if (!packed) MDG_TA4(0); else if (D == 24) MDG_TA4(24); else if (D == 16) MDG_TA4(16); else MDG_TA4(8);
#undef MDG_TA4
    } else {
      dim3 grid((unsigned)((T + 255) / 256 * H * B * L));
#define MDG_TA8(PD_)                                                                                      \
  hipLaunchKernelGGL((attn_temporal_bf16_kernel<8, 128, PD_>), grid, dim3(512), 0, s, (const bf16_t*)qkv_t, kbias, \
                     kvb, (bf16_t*)out, T, L, H, D, B * L, lse, (bf16_t*)out_lo)
      if (!packed) MDG_TA8(0); else if (D == 24) MDG_TA8(24); else if (D == 16) MDG_TA8(16); else MDG_TA8(8);
#undef MDG_TA8
    }
    return hipGetLastError();
  }
  dim3 grid((T + 127) / 128, H, B * L);
  hipLaunchKernelGGL((attn_temporal_kernel<float, MDG_DP>), grid, dim3(256), 0, s, (const float*)qkv_t, kbias, kvb,
                     (float*)out, T, L, H, D, B * L, lse);
  return hipGetLastError();
}

hipError_t attn_spatial_launch(int dtype, int nf, int L, int H, int D, const void* qkv,
                               const float* kvb, const float* mask, void* out, hipStream_t s) {
  if (L == 4 && D % 8 == 0 && D <= 32) {
    dim3 grid((unsigned)(((size_t)nf * H * 4 + 255) / 256));
#define MDG_QUAD(CTT, DM)                                                                                  \
  hipLaunchKernelGGL((attn_spatial_quad_kernel<CTT, DM>), grid, dim3(256), 0, s, (const CTT*)qkv, kvb, mask, \
                     (CTT*)out, nf, H, D)
    if (dtype == MDG_BF16) {
      if (D <= 16) MDG_QUAD(bf16_t, 16); else if (D <= 24) MDG_QUAD(bf16_t, 24); else MDG_QUAD(bf16_t, 32);
    } else {
      if (D <= 16) MDG_QUAD(float, 16); else if (D <= 24) MDG_QUAD(float, 24); else MDG_QUAD(float, 32);
    }
#undef MDG_QUAD
    return hipGetLastError();
  }
  const int total = nf * L * H;
  dim3 grid((total + 255) / 256);
#define MDG_SPA(CTT, DPP)                                                                            \
  hipLaunchKernelGGL((attn_spatial_kernel<CTT, DPP>), grid, dim3(256), 0, s, (const CTT*)qkv, kvb, mask, \
                     (CTT*)out, nf, L, H, D)
  if (dtype == MDG_BF16) {
    if (D < MDG_DP) MDG_SPA(bf16_t, MDG_DP); else MDG_SPA(bf16_t, MDG_DP_WIDE);
  } else {
    if (D < MDG_DP) MDG_SPA(float, MDG_DP); else MDG_SPA(float, MDG_DP_WIDE);
  }
#undef MDG_SPA
  return hipGetLastError();
}

}  // namespace mdg
