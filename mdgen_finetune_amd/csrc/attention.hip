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

namespace mdg {


template <typename CT>
__global__ __launch_bounds__(256) void attn_temporal_kernel(const CT* __restrict__ qkv,
                                                            const float* __restrict__ kbias,
                                                            const float* __restrict__ kvb,
                                                            CT* __restrict__ out, int T, int L,
                                                            int H, int D, int BL) {
  constexpr int DP = MDG_DP, KC = 64, LDK = 48;  // 96-B LDS rows (bf16): conflict-free b128 + tr reads
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

  typename V8<CT>::T qf[2];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = q0 + qg * 16 + lr;
    qf[qg] = (q < T) ? ld8<CT>(Qg + (size_t)q * DP + 8 * lg) : zero8<CT>();
  }

  // virtual bias key first.  The running softmax offset mt (per query, exactly representable
  // in CT) rides in the MFMA: K's pad column D holds 1.0 and Q's pad element D holds -mt, so
  // S^T = K Q^T comes out of the matrix cores already as score - mt and the common case
  // needs one v_exp_f32 per score and nothing else.  mt is only raised (rare path below)
  // when a score exceeds it by more than kGrow (log2 units), so p <= 2^kGrow.
  constexpr float kGrow = 8.0f;
  const int padg = D >> 3, pade = D & 7;  // lane group / element of the pad column
  const float* kvh = kvb + head * 2 * DP;
  float mt[2];
  f32x4 o[2][2];  // [d-tile][q-group]: O^T[d = 16dt + 4lg + i][q = lr]
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    float sb = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) sb += (float)qf[qg][j] * kvh[8 * lg + j];
    sb += __shfl_xor(sb, 16, 64);
    sb += __shfl_xor(sb, 32, 64);
    mt[qg] = (float)(CT)sb;
    const float pb = __builtin_amdgcn_exp2f(sb - mt[qg]);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) o[dt][qg][i] = pb * kvh[DP + dt * 16 + lg * 4 + i];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (lg == padg && j == pade) qf[qg][j] = (CT)(-mt[qg]);
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
      const typename V8<CT>::T kf = ld8<CT>(Kc + (kt * 16 + lr) * LDK + 8 * lg);
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) {
        s[kt][qg] = f32x4{0.f, 0.f, 0.f, 0.f};
        mma_k32<CT>(s[kt][qg], kf, qf[qg]);
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
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[dt][qg][i] *= alpha;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) s[kt][qg][i] -= delta;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (lg == padg && j == pade) qf[qg][j] = (CT)(-nm);
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
      for (int dt = 0; dt < 2; ++dt) {
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
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (dt == dt_s && i == i_s) mine = o[dt][qg][i];
    const float lsum = __shfl(mine, lr + 16 * g_s, 64);
    const float inv = 1.0f / lsum;
    const int q = q0 + qg * 16 + lr;
    if (q < T) {
      CT* orow = out + ((size_t)(b * T + q) * L + l) * C + head * D;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int d0 = dt * 16 + lg * 4;
        if (d0 < D)
          st4<CT>(orow + d0, o[dt][qg][0] * inv, o[dt][qg][1] * inv, o[dt][qg][2] * inv,
                  o[dt][qg][3] * inv);
      }
    }
  }
}

template <typename CT>
__global__ __launch_bounds__(256) void attn_spatial_kernel(const CT* __restrict__ qkv,
                                                           const float* __restrict__ kvb,
                                                           const float* __restrict__ mask,
                                                           CT* __restrict__ out, int nf, int L,
                                                           int H, int D) {
  constexpr int DP = MDG_DP;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= nf * L * H) return;
  const int h = idx % H, tok = idx / H, f = tok / L;
  const size_t tstride = 3ull * H * DP;
  float q[DP];
  const CT* qp = qkv + (size_t)tok * tstride + h * DP;
#pragma unroll
  for (int d = 0; d < DP; d += 4) {
    const float4 v = ld4f<CT>(qp + d);
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
    const CT* kp = qkv + (size_t)kt * tstride + (size_t)H * DP + h * DP;
    const CT* vp = kp + (size_t)H * DP;
    float sc = 0.f;
#pragma unroll
    for (int d = 0; d < DP; d += 4) {
      const float4 kv = ld4f<CT>(kp + d);
      sc += q[d] * kv.x + q[d + 1] * kv.y + q[d + 2] * kv.z + q[d + 3] * kv.w;
    }
    const float mn = fmaxf(m, sc);
    const float a = expf(m - mn), pj = expf(sc - mn);
    lsum = lsum * a + pj;
#pragma unroll
    for (int d = 0; d < DP; d += 4) {
      const float4 vv = ld4f<CT>(vp + d);
      acc[d] = acc[d] * a + pj * vv.x;
      acc[d + 1] = acc[d + 1] * a + pj * vv.y;
      acc[d + 2] = acc[d + 2] * a + pj * vv.z;
      acc[d + 3] = acc[d + 3] * a + pj * vv.w;
    }
    m = mn;
  }
  const float inv = 1.0f / lsum;
  CT* op = out + (size_t)tok * H * D + h * D;
#pragma unroll
  for (int d = 0; d < DP; d += 4)
    if (d < D) st4<CT>(op + d, acc[d] * inv, acc[d + 1] * inv, acc[d + 2] * inv, acc[d + 3] * inv);
}

hipError_t attn_temporal_launch(int dtype, int B, int T, int L, int H, int D, const void* qkv_t,
                                const float* kbias, const float* kvb, void* out, hipStream_t s) {
  dim3 grid((T + 127) / 128, H, B * L);
  if (dtype == MDG_BF16)
    hipLaunchKernelGGL(attn_temporal_kernel<bf16_t>, grid, dim3(256), 0, s,
                       (const bf16_t*)qkv_t, kbias, kvb, (bf16_t*)out, T, L, H, D, B * L);
  else
    hipLaunchKernelGGL(attn_temporal_kernel<float>, grid, dim3(256), 0, s, (const float*)qkv_t,
                       kbias, kvb, (float*)out, T, L, H, D, B * L);
  return hipGetLastError();
}

hipError_t attn_spatial_launch(int dtype, int nf, int L, int H, int D, const void* qkv,
                               const float* kvb, const float* mask, void* out, hipStream_t s) {
  const int total = nf * L * H;
  dim3 grid((total + 255) / 256);
  if (dtype == MDG_BF16)
    hipLaunchKernelGGL(attn_spatial_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)qkv,
                       kvb, mask, (bf16_t*)out, nf, L, H, D);
  else
    hipLaunchKernelGGL(attn_spatial_kernel<float>, grid, dim3(256), 0, s, (const float*)qkv, kvb,
                       mask, (float*)out, nf, L, H, D);
  return hipGetLastError();
}

}  // namespace mdg
