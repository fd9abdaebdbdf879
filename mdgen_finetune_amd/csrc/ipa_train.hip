// Invariant point attention core for the training step (the IPA prepend under loss.backward():
// reference src/mdgen/model/ipa.py:92-255 with c_z = 0, called from latent_model.py:179-214).
//
// The projections (linear_q / _kv / _q_points / _kv_points and the frame application of the
// points) and linear_out stay ordinary autograd ops; between them sits the attention core,
// which eager PyTorch runs as ~25 forward and ~45 backward kernels of a few microseconds each
// on B * L = 32 tokens -- launch-bound, and five IPA layers deep on the step's critical path.
// Here it is one kernel each way, fp32 throughout.  One block (one wave) per (sample, head);
// lane i = query i (L <= 32):
//   logit_ij = wc q_i.k_j - 1/2 hw_h sum_p |qp_ip - kp_jp|^2 + 1e5 (m_i m_j - 1)
//   a_ij = softmax_j(logit_ij)
//   o_i = sum_j a_ij v_j,  og_i = sum_j a_ij vp_j,  ol_i = R_i^T (og_i - t_i),  n_i = sqrt(|ol_i|^2 + eps)
// written as the linear_out input row [o | ol_x | ol_y | ol_z | n] (ipa.py:226-250's concat order).
// Backward (lane i, then lane j over the block's LDS copies):
//   dol = d ol + dn ol / n,  dog_i = R_i dol,  da_ij = do_i.v_j + dog_i.vp_j,
//   dl_ij = a_ij (da_ij - sum_j' a_ij' da_ij'),
//   dq_i = wc sum_j dl_ij k_j,  dqp_i = -hw sum_j dl_ij (qp_i - kp_j),
//   dk_j = wc sum_i dl_ij q_i,  dkp_j = hw sum_i dl_ij (qp_i - kp_j),
//   dv_j = sum_i a_ij do_i,  dvp_j = sum_i a_ij dog_i,
//   d hw_h = -1/2 sum_ij dl_ij sum_p |qp_ip - kp_jp|^2  (per-sample partials: no atomics).
#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {
namespace {

constexpr int kIpaMaxL = 32;       // one wave per (sample, head), lane = residue: the tetrapeptide crop
constexpr int kIpaLongMaxL = 256;  // 33..256 (ATLAS crops): the long kernels below, 256 threads
constexpr float kIpaInf = 1e5f, kIpaEps = 1e-8f;

// flags (mdg_ipa_core_fwd / _bwd): MDG_IPA_LOCAL_POINTS = the points arrive as the raw
// linear_q_points / linear_kv_points rows [x block | y block | z block] of n = H * P points
// (point h * P + p; ipa.py:121-140's split + stack) in the residue's local frame, and the kernel
// applies R x + t (rigid_utils.py:64-86) itself -- the backward returns d raw = R^T d global;
// MDG_IPA_RAW_HW = hw is the raw head_weights parameter, softplus(w) * sqrt(1 / (3 Pq 9/2))
// taken in the kernel (ipa.py:178-183), d hw is returned w.r.t. the raw parameter.
__device__ __forceinline__ void frame_point(const float* raw, int n, int pidx, const float* R, const float* t,
                                            float (&g)[3]) {
  const float p0 = raw[pidx], p1 = raw[n + pidx], p2 = raw[2 * n + pidx];
#pragma unroll
  for (int x = 0; x < 3; ++x) g[x] = (__fmul_rn(R[x * 3], p0) + __fmul_rn(R[x * 3 + 1], p1)) + __fmul_rn(R[x * 3 + 2], p2) + t[x];
}
__device__ __forceinline__ float softplus_f(float w) { return w > 20.f ? w : log1pf(expf(w)); }

template <int CH, int PQ, int PV>
struct IpaShape {
  static constexpr int KV = 2 * CH;          // k | v per head
  static constexpr int PKV = (PQ + PV) * 3;  // k points | v points per head
};

// logits of query row i against every key, softmax -> P[i][*] (LDS); returns nothing
template <int CH, int PQ>
__device__ __forceinline__ void ipa_row_softmax(const float (&q)[CH], const float (&qp)[PQ * 3], float mi, int L,
                                                const float* Ks, const float* KPs, const float* Ms, float wc, float hwh,
                                                float* Prow) {
  float mx = -INFINITY;
  for (int j = 0; j < L; ++j) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < CH; ++d) s += q[d] * Ks[j * CH + d];
    float d2 = 0.f;
#pragma unroll
    for (int p = 0; p < PQ; ++p) {
      float e = 0.f;
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        const float u = qp[3 * p + x] - KPs[j * PQ * 3 + 3 * p + x];
        e += u * u;
      }
      d2 += e * hwh;
    }
    const float lg = s * wc + d2 * -0.5f + kIpaInf * (mi * Ms[j] - 1.0f);
    Prow[j] = lg;
    mx = fmaxf(mx, lg);
  }
  float sum = 0.f;
  for (int j = 0; j < L; ++j) {
    const float e = expf(Prow[j] - mx);
    Prow[j] = e;
    sum += e;
  }
  const float inv = 1.0f / sum;
  for (int j = 0; j < L; ++j) Prow[j] *= inv;
}

template <int CH, int PQ, int PV>
struct IpaSmem {
  float K[kIpaMaxL * CH], V[kIpaMaxL * CH], KP[kIpaMaxL * PQ * 3], VP[kIpaMaxL * PV * 3], M[kIpaMaxL];
  float P[kIpaMaxL * (kIpaMaxL + 1)];
  float R[kIpaMaxL * 9], Tt[kIpaMaxL * 3];  // the sample's frames (MDG_IPA_LOCAL_POINTS)
};

// stage the block's keys (k, v, key points, value points, mask) of sample b, head h (and, for
// local points, the sample's frames first); SM = IpaSmem or IpaLongSmem
template <int CH, int PQ, int PV, typename SM>
__device__ __forceinline__ void ipa_stage_keys(SM& S, int b, int h, int L, int H, const float* kv,
                                               const float* kvp, const float* mask, const float* rots,
                                               const float* trans, int flags) {
  using SH = IpaShape<CH, PQ, PV>;
  for (int e = threadIdx.x; e < L * CH; e += blockDim.x) {
    const int j = e / CH, d = e % CH;
    const float* row = kv + (((size_t)b * L + j) * H + h) * SH::KV;
    S.K[e] = row[d];
    S.V[e] = row[CH + d];
  }
  for (int j = threadIdx.x; j < L; j += blockDim.x) S.M[j] = mask[(size_t)b * L + j];
  if (flags & MDG_IPA_LOCAL_POINTS) {
    for (int e = threadIdx.x; e < L * 9; e += blockDim.x) S.R[e] = ld1(rots + (size_t)b * L * 9 + e);
    for (int e = threadIdx.x; e < L * 3; e += blockDim.x) S.Tt[e] = ld1(trans + (size_t)b * L * 3 + e);
    __syncthreads();
    constexpr int NP = PQ + PV;
    for (int e = threadIdx.x; e < L * NP; e += blockDim.x) {
      const int j = e / NP, p = e % NP;
      float g[3];
      frame_point(kvp + ((size_t)b * L + j) * H * NP * 3, H * NP, h * NP + p, S.R + j * 9, S.Tt + j * 3, g);
      float* dst = p < PQ ? S.KP + j * PQ * 3 + 3 * p : S.VP + j * PV * 3 + 3 * (p - PQ);
#pragma unroll
      for (int x = 0; x < 3; ++x) dst[x] = g[x];
    }
    return;
  }
  for (int e = threadIdx.x; e < L * PQ * 3; e += blockDim.x) {
    const int j = e / (PQ * 3), r = e % (PQ * 3);
    S.KP[e] = kvp[(((size_t)b * L + j) * H + h) * SH::PKV + r];
  }
  for (int e = threadIdx.x; e < L * PV * 3; e += blockDim.x) {
    const int j = e / (PV * 3), r = e % (PV * 3);
    S.VP[e] = kvp[(((size_t)b * L + j) * H + h) * SH::PKV + PQ * 3 + r];
  }
}

__device__ __forceinline__ float ipa_hw(const float* hw, int h, int flags, float pq) {
  return (flags & MDG_IPA_RAW_HW) ? softplus_f(hw[h]) * sqrtf(1.0f / (3.0f * (pq * 9.0f / 2.0f))) : hw[h];
}

template <int CH, int PQ, int PV>
__global__ __launch_bounds__(64) void ipa_core_fwd_kernel(int L, int H, const float* __restrict__ q,
                                                          const float* __restrict__ kv, const float* __restrict__ qpts,
                                                          const float* __restrict__ kvp, const float* __restrict__ mask,
                                                          const float* __restrict__ rots,
                                                          const float* __restrict__ trans,
                                                          const float* __restrict__ hw, float wc,
                                                          float* __restrict__ out, int flags) {
  __shared__ IpaSmem<CH, PQ, PV> S;
  const int b = blockIdx.x / H, h = blockIdx.x % H, i = threadIdx.x;
  ipa_stage_keys<CH, PQ, PV>(S, b, h, L, H, kv, kvp, mask, rots, trans, flags);
  __syncthreads();
  if (i >= L) return;  // (no barrier below)
  const size_t tok = (size_t)b * L + i;
  float qr[CH], qpr[PQ * 3];
#pragma unroll
  for (int d = 0; d < CH; ++d) qr[d] = q[(tok * H + h) * CH + d];
  if (flags & MDG_IPA_LOCAL_POINTS) {
#pragma unroll
    for (int p = 0; p < PQ; ++p) {
      float g[3];
      frame_point(qpts + tok * H * PQ * 3, H * PQ, h * PQ + p, S.R + i * 9, S.Tt + i * 3, g);
#pragma unroll
      for (int x = 0; x < 3; ++x) qpr[3 * p + x] = g[x];
    }
  } else {
#pragma unroll
    for (int r = 0; r < PQ * 3; ++r) qpr[r] = qpts[(tok * H + h) * PQ * 3 + r];
  }
  float* Prow = S.P + i * (kIpaMaxL + 1);
  ipa_row_softmax<CH, PQ>(qr, qpr, S.M[i], L, S.K, S.KP, S.M, wc, ipa_hw(hw, h, flags, (float)PQ), Prow);
  const int W = H * CH + 4 * H * PV;
  float* orow = out + tok * W;
  // o_i
  for (int d = 0; d < CH; ++d) {
    float acc = 0.f;
    for (int j = 0; j < L; ++j) acc += Prow[j] * S.V[j * CH + d];
    orow[h * CH + d] = acc;
  }
  // points: global sum - t_i, then R_i^T, norm
  float R[9], t[3];
#pragma unroll
  for (int e = 0; e < 9; ++e) R[e] = ld1(rots + tok * 9 + e);
#pragma unroll
  for (int e = 0; e < 3; ++e) t[e] = ld1(trans + tok * 3 + e);
  for (int p = 0; p < PV; ++p) {
    float g[3];
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      float acc = 0.f;
      for (int j = 0; j < L; ++j) acc += Prow[j] * S.VP[j * PV * 3 + 3 * p + x];
      g[x] = acc - t[x];
    }
    float l[3], nn = 0.f;
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      l[x] = R[0 * 3 + x] * g[0] + R[1 * 3 + x] * g[1] + R[2 * 3 + x] * g[2];
      nn += l[x] * l[x];
      orow[H * CH + x * H * PV + h * PV + p] = l[x];
    }
    orow[H * CH + 3 * H * PV + h * PV + p] = sqrtf(nn + kIpaEps);
  }
}

template <int CH, int PQ, int PV>
struct IpaBwdSmem {
  IpaSmem<CH, PQ, PV> s;
  float Q[kIpaMaxL * CH], QP[kIpaMaxL * PQ * 3], DO[kIpaMaxL * CH], DOG[kIpaMaxL * PV * 3];
  float DL[kIpaMaxL * (kIpaMaxL + 1)];
  float red[64];
};

template <int CH, int PQ, int PV>
__global__ __launch_bounds__(64) void ipa_core_bwd_kernel(int L, int H, const float* __restrict__ q,
                                                          const float* __restrict__ kv, const float* __restrict__ qpts,
                                                          const float* __restrict__ kvp, const float* __restrict__ mask,
                                                          const float* __restrict__ rots,
                                                          const float* __restrict__ trans,
                                                          const float* __restrict__ hw, float wc,
                                                          const float* __restrict__ dout, float* __restrict__ dq,
                                                          float* __restrict__ dkv, float* __restrict__ dqp,
                                                          float* __restrict__ dkvp, float* __restrict__ dhw_part,
                                                          int flags) {
  using SH = IpaShape<CH, PQ, PV>;
  __shared__ IpaBwdSmem<CH, PQ, PV> S;
  const int b = blockIdx.x / H, h = blockIdx.x % H, i = threadIdx.x;
  const bool local = flags & MDG_IPA_LOCAL_POINTS;
  ipa_stage_keys<CH, PQ, PV>(S.s, b, h, L, H, kv, kvp, mask, rots, trans, flags);
  for (int e = threadIdx.x; e < L * CH; e += blockDim.x) {
    const int j = e / CH, d = e % CH;
    S.Q[e] = q[(((size_t)b * L + j) * H + h) * CH + d];
  }
  if (local) {
    for (int e = threadIdx.x; e < L * PQ; e += blockDim.x) {
      const int j = e / PQ, p = e % PQ;
      float g[3];
      frame_point(qpts + ((size_t)b * L + j) * H * PQ * 3, H * PQ, h * PQ + p, S.s.R + j * 9, S.s.Tt + j * 3, g);
#pragma unroll
      for (int x = 0; x < 3; ++x) S.QP[j * PQ * 3 + 3 * p + x] = g[x];
    }
  } else {
    for (int e = threadIdx.x; e < L * PQ * 3; e += blockDim.x) {
      const int j = e / (PQ * 3), r = e % (PQ * 3);
      S.QP[e] = qpts[(((size_t)b * L + j) * H + h) * PQ * 3 + r];
    }
  }
  __syncthreads();
  const float hwh = ipa_hw(hw, h, flags, (float)PQ);
  float dhw = 0.f;
  if (i < L) {
    const size_t tok = (size_t)b * L + i;
    float qr[CH], qpr[PQ * 3];
#pragma unroll
    for (int d = 0; d < CH; ++d) qr[d] = S.Q[i * CH + d];
#pragma unroll
    for (int r = 0; r < PQ * 3; ++r) qpr[r] = S.QP[i * PQ * 3 + r];
    float* Prow = S.s.P + i * (kIpaMaxL + 1);
    ipa_row_softmax<CH, PQ>(qr, qpr, S.s.M[i], L, S.s.K, S.s.KP, S.s.M, wc, hwh, Prow);
    const int W = H * CH + 4 * H * PV;
    const float* grow = dout + tok * W;
    float R[9], t[3];
#pragma unroll
    for (int e = 0; e < 9; ++e) R[e] = ld1(rots + tok * 9 + e);
#pragma unroll
    for (int e = 0; e < 3; ++e) t[e] = ld1(trans + tok * 3 + e);
    // d o_i -> LDS; d(point outputs) -> d og_i = R_i (d ol + dn ol / n)
    for (int d = 0; d < CH; ++d) S.DO[i * CH + d] = grow[h * CH + d];
    for (int p = 0; p < PV; ++p) {
      float g[3];
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        float acc = 0.f;
        for (int j = 0; j < L; ++j) acc += Prow[j] * S.s.VP[j * PV * 3 + 3 * p + x];
        g[x] = acc - t[x];
      }
      float l[3], nn = 0.f;
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        l[x] = R[0 * 3 + x] * g[0] + R[1 * 3 + x] * g[1] + R[2 * 3 + x] * g[2];
        nn += l[x] * l[x];
      }
      const float n = sqrtf(nn + kIpaEps), dn = grow[H * CH + 3 * H * PV + h * PV + p];
      float dl[3];
#pragma unroll
      for (int x = 0; x < 3; ++x) dl[x] = grow[H * CH + x * H * PV + h * PV + p] + dn * l[x] / n;
#pragma unroll
      for (int x = 0; x < 3; ++x)
        S.DOG[i * PV * 3 + 3 * p + x] = R[x * 3 + 0] * dl[0] + R[x * 3 + 1] * dl[1] + R[x * 3 + 2] * dl[2];
    }
    // da_ij, row dot, dl_ij
    float* DLrow = S.DL + i * (kIpaMaxL + 1);
    float rs = 0.f;
    for (int j = 0; j < L; ++j) {
      float da = 0.f;
#pragma unroll
      for (int d = 0; d < CH; ++d) da += S.DO[i * CH + d] * S.s.V[j * CH + d];
#pragma unroll
      for (int r = 0; r < PV * 3; ++r) da += S.DOG[i * PV * 3 + r] * S.s.VP[j * PV * 3 + r];
      DLrow[j] = da;
      rs += Prow[j] * da;
    }
    float gq[CH], gqp[PQ * 3];
#pragma unroll
    for (int d = 0; d < CH; ++d) gq[d] = 0.f;
#pragma unroll
    for (int r = 0; r < PQ * 3; ++r) gqp[r] = 0.f;
    for (int j = 0; j < L; ++j) {
      const float dlj = Prow[j] * (DLrow[j] - rs);
      DLrow[j] = dlj;
#pragma unroll
      for (int d = 0; d < CH; ++d) gq[d] += dlj * S.s.K[j * CH + d];
      float d2 = 0.f;
#pragma unroll
      for (int r = 0; r < PQ * 3; ++r) {
        const float u = qpr[r] - S.s.KP[j * PQ * 3 + r];
        gqp[r] += dlj * u;
        d2 += u * u;
      }
      dhw += dlj * d2;
    }
    float* dqr = dq + (tok * H + h) * CH;
#pragma unroll
    for (int d = 0; d < CH; ++d) dqr[d] = wc * gq[d];
    if (local) {  // d raw = R_i^T d global, into the raw [x | y | z] blocks
      float* dr = dqp + tok * H * PQ * 3;
      const float* R = S.s.R + i * 9;
#pragma unroll
      for (int p = 0; p < PQ; ++p)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          dr[c * H * PQ + h * PQ + p] =
              -hwh * (R[0 * 3 + c] * gqp[3 * p] + R[1 * 3 + c] * gqp[3 * p + 1] + R[2 * 3 + c] * gqp[3 * p + 2]);
    } else {
      float* dqpr = dqp + (tok * H + h) * PQ * 3;
#pragma unroll
      for (int r = 0; r < PQ * 3; ++r) dqpr[r] = -hwh * gqp[r];
    }
  }
  // d hw_h of this sample: -1/2 sum_ij dl_ij d2_ij
  S.red[threadIdx.x] = dhw;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int k = 0; k < L; ++k) s += S.red[k];
    float d = -0.5f * s;
    if (flags & MDG_IPA_RAW_HW)  // d softplus(w) c / dw = c sigmoid(w)
      d *= sqrtf(1.0f / (3.0f * ((float)PQ * 9.0f / 2.0f))) / (1.0f + expf(-hw[h]));
    dhw_part[(size_t)b * H + h] = d;
  }
  // key side: lane j
  const int j = threadIdx.x;
  if (j >= L) return;
  const size_t tok = (size_t)b * L + j;
  float gk[CH], gv[CH], gkp[PQ * 3], gvp[PV * 3];
#pragma unroll
  for (int d = 0; d < CH; ++d) gk[d] = gv[d] = 0.f;
#pragma unroll
  for (int r = 0; r < PQ * 3; ++r) gkp[r] = 0.f;
#pragma unroll
  for (int r = 0; r < PV * 3; ++r) gvp[r] = 0.f;
  for (int ii = 0; ii < L; ++ii) {
    const float dl = S.DL[ii * (kIpaMaxL + 1) + j], a = S.s.P[ii * (kIpaMaxL + 1) + j];
#pragma unroll
    for (int d = 0; d < CH; ++d) {
      gk[d] += dl * S.Q[ii * CH + d];
      gv[d] += a * S.DO[ii * CH + d];
    }
#pragma unroll
    for (int r = 0; r < PQ * 3; ++r) gkp[r] += dl * (S.QP[ii * PQ * 3 + r] - S.s.KP[j * PQ * 3 + r]);
#pragma unroll
    for (int r = 0; r < PV * 3; ++r) gvp[r] += a * S.DOG[ii * PV * 3 + r];
  }
  float* dkvr = dkv + (tok * H + h) * SH::KV;
#pragma unroll
  for (int d = 0; d < CH; ++d) {
    dkvr[d] = wc * gk[d];
    dkvr[CH + d] = gv[d];
  }
  if (local) {
    constexpr int NP = PQ + PV;
    float* dr = dkvp + tok * H * NP * 3;
    const float* R = S.s.R + j * 9;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const float sc = p < PQ ? hwh : 1.0f;
      const float* gg = p < PQ ? gkp + 3 * p : gvp + 3 * (p - PQ);
#pragma unroll
      for (int c = 0; c < 3; ++c)
        dr[c * H * NP + h * NP + p] = sc * (R[0 * 3 + c] * gg[0] + R[1 * 3 + c] * gg[1] + R[2 * 3 + c] * gg[2]);
    }
    return;
  }
  float* dkvpr = dkvp + (tok * H + h) * SH::PKV;
#pragma unroll
  for (int r = 0; r < PQ * 3; ++r) dkvpr[r] = hwh * gkp[r];
#pragma unroll
  for (int r = 0; r < PV * 3; ++r) dkvpr[PQ * 3 + r] = gvp[r];
}


// ------------------------------------------------------------------------------------------
// Long crops (33 <= L <= 256, ATLAS fine-tuning): one 256-thread block per (sample, head), thread
// i = query i on the query side, thread j = key j on the key side.  The keys (k, v, key / value
// points in the global frame, mask) and the sample's frames sit in LDS (L x 452 B + L x 48 B);
// the L x L softmax and its gradient are never stored: each pass over the keys recomputes the
// logits (56 FMAs), and the key side recomputes a_ij and dl_ij from the query rows' statistics
// (max, 1 / sum, the row dot rs_i) and dog_i that the query side leaves in LDS.
template <int CH, int PQ, int PV>
struct IpaLongSmem {
  float K[kIpaLongMaxL * CH], V[kIpaLongMaxL * CH], KP[kIpaLongMaxL * PQ * 3], VP[kIpaLongMaxL * PV * 3];
  float M[kIpaLongMaxL], R[kIpaLongMaxL * 9], Tt[kIpaLongMaxL * 3];
  float DOG[kIpaLongMaxL * PV * 3], mx[kIpaLongMaxL], isum[kIpaLongMaxL], rs[kIpaLongMaxL];
  float red[256];
};

template <int CH, int PQ, typename SMT>
__device__ __forceinline__ float ipa_logit(const float (&q)[CH], const float (&qp)[PQ * 3], float mi, int j,
                                           const SMT& S, float wc, float hwh, float* d2out = nullptr) {
  float sdot = 0.f;
#pragma unroll
  for (int d = 0; d < CH; ++d) sdot += q[d] * S.K[j * CH + d];
  float d2 = 0.f, raw = 0.f;
#pragma unroll
  for (int p = 0; p < PQ; ++p) {
    float e = 0.f;
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      const float u = qp[3 * p + x] - S.KP[j * PQ * 3 + 3 * p + x];
      e += u * u;
    }
    d2 += e * hwh;
    raw += e;
  }
  if (d2out) *d2out = raw;  // sum_p |qp_ip - kp_jp|^2 (d hw)
  return sdot * wc + d2 * -0.5f + kIpaInf * (mi * S.M[j] - 1.0f);
}

// query i's q and q points (global frame) of head h
template <int CH, int PQ, typename SMT>
__device__ __forceinline__ void ipa_load_query(const float* q, const float* qpts, int b, int i, int L, int H, int h,
                                               bool local, const SMT& S, float (&qr)[CH], float (&qpr)[PQ * 3]) {
  const size_t tok = (size_t)b * L + i;
#pragma unroll
  for (int d = 0; d < CH; ++d) qr[d] = q[(tok * H + h) * CH + d];
  if (local) {
#pragma unroll
    for (int p = 0; p < PQ; ++p) {
      float g[3];
      frame_point(qpts + tok * H * PQ * 3, H * PQ, h * PQ + p, S.R + i * 9, S.Tt + i * 3, g);
#pragma unroll
      for (int x = 0; x < 3; ++x) qpr[3 * p + x] = g[x];
    }
  } else {
#pragma unroll
    for (int r = 0; r < PQ * 3; ++r) qpr[r] = qpts[(tok * H + h) * PQ * 3 + r];
  }
}

// the softmax row statistics of query i: max and 1 / sum (the same exp / sum order as
// ipa_row_softmax)
template <int CH, int PQ, typename SMT>
__device__ __forceinline__ void ipa_row_stats(const float (&qr)[CH], const float (&qpr)[PQ * 3], float mi, int L,
                                              const SMT& S, float wc, float hwh, float& mx, float& isum) {
  mx = -INFINITY;
  for (int j = 0; j < L; ++j) mx = fmaxf(mx, ipa_logit<CH, PQ>(qr, qpr, mi, j, S, wc, hwh));
  float sum = 0.f;
  for (int j = 0; j < L; ++j) sum += expf(ipa_logit<CH, PQ>(qr, qpr, mi, j, S, wc, hwh) - mx);
  isum = 1.0f / sum;
}

template <int CH, int PQ, int PV>
__global__ __launch_bounds__(256) void ipa_core_fwd_long_kernel(int L, int H, const float* __restrict__ q,
                                                                const float* __restrict__ kv,
                                                                const float* __restrict__ qpts,
                                                                const float* __restrict__ kvp,
                                                                const float* __restrict__ mask,
                                                                const float* __restrict__ rots,
                                                                const float* __restrict__ trans,
                                                                const float* __restrict__ hw, float wc,
                                                                float* __restrict__ out, int flags) {
  __shared__ IpaLongSmem<CH, PQ, PV> S;
  const int b = blockIdx.x / H, h = blockIdx.x % H, i = threadIdx.x;
  ipa_stage_keys<CH, PQ, PV>(S, b, h, L, H, kv, kvp, mask, rots, trans, flags);
  __syncthreads();
  if (i >= L) return;  // (no barrier below)
  const size_t tok = (size_t)b * L + i;
  float qr[CH], qpr[PQ * 3];
  ipa_load_query<CH, PQ>(q, qpts, b, i, L, H, h, flags & MDG_IPA_LOCAL_POINTS, S, qr, qpr);
  const float hwh = ipa_hw(hw, h, flags, (float)PQ), mi = S.M[i];
  float mx, isum;
  ipa_row_stats<CH, PQ>(qr, qpr, mi, L, S, wc, hwh, mx, isum);
  float o[CH], og[PV * 3];
#pragma unroll
  for (int d = 0; d < CH; ++d) o[d] = 0.f;
#pragma unroll
  for (int r = 0; r < PV * 3; ++r) og[r] = 0.f;
  for (int j = 0; j < L; ++j) {
    const float a = expf(ipa_logit<CH, PQ>(qr, qpr, mi, j, S, wc, hwh) - mx) * isum;
#pragma unroll
    for (int d = 0; d < CH; ++d) o[d] += a * S.V[j * CH + d];
#pragma unroll
    for (int r = 0; r < PV * 3; ++r) og[r] += a * S.VP[j * PV * 3 + r];
  }
  const int W = H * CH + 4 * H * PV;
  float* orow = out + tok * W;
#pragma unroll
  for (int d = 0; d < CH; ++d) orow[h * CH + d] = o[d];
  const float* R = S.R + i * 9;  // (staged for local points; else from rots below)
  float Rr[9], t[3];
#pragma unroll
  for (int e = 0; e < 9; ++e) Rr[e] = ld1(rots + tok * 9 + e);
#pragma unroll
  for (int e = 0; e < 3; ++e) t[e] = ld1(trans + tok * 3 + e);
  (void)R;
#pragma unroll
  for (int p = 0; p < PV; ++p) {
    float g[3], l[3], nn = 0.f;
#pragma unroll
    for (int x = 0; x < 3; ++x) g[x] = og[3 * p + x] - t[x];
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      l[x] = Rr[0 * 3 + x] * g[0] + Rr[1 * 3 + x] * g[1] + Rr[2 * 3 + x] * g[2];
      nn += l[x] * l[x];
      orow[H * CH + x * H * PV + h * PV + p] = l[x];
    }
    orow[H * CH + 3 * H * PV + h * PV + p] = sqrtf(nn + kIpaEps);
  }
}

template <int CH, int PQ, int PV>
__global__ __launch_bounds__(256) void ipa_core_bwd_long_kernel(
    int L, int H, const float* __restrict__ q, const float* __restrict__ kv, const float* __restrict__ qpts,
    const float* __restrict__ kvp, const float* __restrict__ mask, const float* __restrict__ rots,
    const float* __restrict__ trans, const float* __restrict__ hw, float wc, const float* __restrict__ dout,
    float* __restrict__ dq, float* __restrict__ dkv, float* __restrict__ dqp, float* __restrict__ dkvp,
    float* __restrict__ dhw_part, int flags) {
  using SH = IpaShape<CH, PQ, PV>;
  __shared__ IpaLongSmem<CH, PQ, PV> S;
  const int b = blockIdx.x / H, h = blockIdx.x % H, tid = threadIdx.x;
  const bool local = flags & MDG_IPA_LOCAL_POINTS;
  const int W = H * CH + 4 * H * PV;
  ipa_stage_keys<CH, PQ, PV>(S, b, h, L, H, kv, kvp, mask, rots, trans, flags);
  __syncthreads();
  const float hwh = ipa_hw(hw, h, flags, (float)PQ);
  // ---- query side: thread i
  float dhw = 0.f;
  if (tid < L) {
    const int i = tid;
    const size_t tok = (size_t)b * L + i;
    float qr[CH], qpr[PQ * 3];
    ipa_load_query<CH, PQ>(q, qpts, b, i, L, H, h, local, S, qr, qpr);
    const float mi = S.M[i];
    float mx, isum;
    ipa_row_stats<CH, PQ>(qr, qpr, mi, L, S, wc, hwh, mx, isum);
    // og_i, then d og_i = R_i (d ol + dn ol / n)
    float og[PV * 3];
#pragma unroll
    for (int r = 0; r < PV * 3; ++r) og[r] = 0.f;
    for (int j = 0; j < L; ++j) {
      const float a = expf(ipa_logit<CH, PQ>(qr, qpr, mi, j, S, wc, hwh) - mx) * isum;
#pragma unroll
      for (int r = 0; r < PV * 3; ++r) og[r] += a * S.VP[j * PV * 3 + r];
    }
    const float* grow = dout + tok * W;
    float R[9], t[3];
#pragma unroll
    for (int e = 0; e < 9; ++e) R[e] = ld1(rots + tok * 9 + e);
#pragma unroll
    for (int e = 0; e < 3; ++e) t[e] = ld1(trans + tok * 3 + e);
    float dog[PV * 3];
#pragma unroll
    for (int p = 0; p < PV; ++p) {
      float g[3], l[3], nn = 0.f;
#pragma unroll
      for (int x = 0; x < 3; ++x) g[x] = og[3 * p + x] - t[x];
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        l[x] = R[0 * 3 + x] * g[0] + R[1 * 3 + x] * g[1] + R[2 * 3 + x] * g[2];
        nn += l[x] * l[x];
      }
      const float n = sqrtf(nn + kIpaEps), dn = grow[H * CH + 3 * H * PV + h * PV + p];
      float dl[3];
#pragma unroll
      for (int x = 0; x < 3; ++x) dl[x] = grow[H * CH + x * H * PV + h * PV + p] + dn * l[x] / n;
#pragma unroll
      for (int x = 0; x < 3; ++x) dog[3 * p + x] = R[x * 3 + 0] * dl[0] + R[x * 3 + 1] * dl[1] + R[x * 3 + 2] * dl[2];
    }
    float dor[CH];
#pragma unroll
    for (int d = 0; d < CH; ++d) dor[d] = grow[h * CH + d];
    // rs_i = sum_j a_ij da_ij
    float rs = 0.f;
    for (int j = 0; j < L; ++j) {
      const float a = expf(ipa_logit<CH, PQ>(qr, qpr, mi, j, S, wc, hwh) - mx) * isum;
      float da = 0.f;
#pragma unroll
      for (int d = 0; d < CH; ++d) da += dor[d] * S.V[j * CH + d];
#pragma unroll
      for (int r = 0; r < PV * 3; ++r) da += dog[r] * S.VP[j * PV * 3 + r];
      rs += a * da;
    }
    // dl_ij = a_ij (da_ij - rs_i): dq_i, dqp_i, d hw
    float gq[CH], gqp[PQ * 3];
#pragma unroll
    for (int d = 0; d < CH; ++d) gq[d] = 0.f;
#pragma unroll
    for (int r = 0; r < PQ * 3; ++r) gqp[r] = 0.f;
    for (int j = 0; j < L; ++j) {
      float d2;
      const float a = expf(ipa_logit<CH, PQ>(qr, qpr, mi, j, S, wc, hwh, &d2) - mx) * isum;
      float da = 0.f;
#pragma unroll
      for (int d = 0; d < CH; ++d) da += dor[d] * S.V[j * CH + d];
#pragma unroll
      for (int r = 0; r < PV * 3; ++r) da += dog[r] * S.VP[j * PV * 3 + r];
      const float dlj = a * (da - rs);
#pragma unroll
      for (int d = 0; d < CH; ++d) gq[d] += dlj * S.K[j * CH + d];
#pragma unroll
      for (int r = 0; r < PQ * 3; ++r) gqp[r] += dlj * (qpr[r] - S.KP[j * PQ * 3 + r]);
      dhw += dlj * d2;
    }
    float* dqr = dq + (tok * H + h) * CH;
#pragma unroll
    for (int d = 0; d < CH; ++d) dqr[d] = wc * gq[d];
    if (local) {
      float* dr = dqp + tok * H * PQ * 3;
      const float* Rs = S.R + i * 9;
#pragma unroll
      for (int p = 0; p < PQ; ++p)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          dr[c * H * PQ + h * PQ + p] =
              -hwh * (Rs[0 * 3 + c] * gqp[3 * p] + Rs[1 * 3 + c] * gqp[3 * p + 1] + Rs[2 * 3 + c] * gqp[3 * p + 2]);
    } else {
      float* dqpr = dqp + (tok * H + h) * PQ * 3;
#pragma unroll
      for (int r = 0; r < PQ * 3; ++r) dqpr[r] = -hwh * gqp[r];
    }
    // the key side's view of row i
    S.mx[i] = mx;
    S.isum[i] = isum;
    S.rs[i] = rs;
#pragma unroll
    for (int r = 0; r < PV * 3; ++r) S.DOG[i * PV * 3 + r] = dog[r];
  }
  S.red[tid] = dhw;
  __syncthreads();
  if (tid == 0) {  // d hw_h of this sample, fixed order
    float sacc = 0.f;
    for (int k = 0; k < L; ++k) sacc += S.red[k];
    float d = -0.5f * sacc;
    if (flags & MDG_IPA_RAW_HW) d *= sqrtf(1.0f / (3.0f * ((float)PQ * 9.0f / 2.0f))) / (1.0f + expf(-hw[h]));
    dhw_part[(size_t)b * H + h] = d;
  }
  // ---- key side: thread j, queries i streamed (q_i / q points / d o_i broadcast to the wave)
  const int j = tid;
  if (j >= L) return;  // (no barrier below)
  const size_t tokj = (size_t)b * L + j;
  float gk[CH], gv[CH], gkp[PQ * 3], gvp[PV * 3];
#pragma unroll
  for (int d = 0; d < CH; ++d) gk[d] = gv[d] = 0.f;
#pragma unroll
  for (int r = 0; r < PQ * 3; ++r) gkp[r] = 0.f;
#pragma unroll
  for (int r = 0; r < PV * 3; ++r) gvp[r] = 0.f;
  for (int i = 0; i < L; ++i) {
    float qr[CH], qpr[PQ * 3];
    ipa_load_query<CH, PQ>(q, qpts, b, i, L, H, h, local, S, qr, qpr);
    const float a = expf(ipa_logit<CH, PQ>(qr, qpr, S.M[i], j, S, wc, hwh) - S.mx[i]) * S.isum[i];
    const float* grow = dout + ((size_t)b * L + i) * W + h * CH;
    float da = 0.f;
#pragma unroll
    for (int d = 0; d < CH; ++d) {
      const float g = grow[d];
      da += g * S.V[j * CH + d];
      gv[d] += a * g;
    }
#pragma unroll
    for (int r = 0; r < PV * 3; ++r) {
      const float g = S.DOG[i * PV * 3 + r];
      da += g * S.VP[j * PV * 3 + r];
      gvp[r] += a * g;
    }
    const float dl = a * (da - S.rs[i]);
#pragma unroll
    for (int d = 0; d < CH; ++d) gk[d] += dl * qr[d];
#pragma unroll
    for (int r = 0; r < PQ * 3; ++r) gkp[r] += dl * (qpr[r] - S.KP[j * PQ * 3 + r]);
  }
  float* dkvr = dkv + (tokj * H + h) * SH::KV;
#pragma unroll
  for (int d = 0; d < CH; ++d) {
    dkvr[d] = wc * gk[d];
    dkvr[CH + d] = gv[d];
  }
  if (local) {
    constexpr int NP = PQ + PV;
    float* dr = dkvp + tokj * H * NP * 3;
    const float* R = S.R + j * 9;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const float sc = p < PQ ? hwh : 1.0f;
      const float* gg = p < PQ ? gkp + 3 * p : gvp + 3 * (p - PQ);
#pragma unroll
      for (int c = 0; c < 3; ++c)
        dr[c * H * NP + h * NP + p] = sc * (R[0 * 3 + c] * gg[0] + R[1 * 3 + c] * gg[1] + R[2 * 3 + c] * gg[2]);
    }
    return;
  }
  float* dkvpr = dkvp + (tokj * H + h) * SH::PKV;
#pragma unroll
  for (int r = 0; r < PQ * 3; ++r) dkvpr[r] = hwh * gkp[r];
#pragma unroll
  for (int r = 0; r < PV * 3; ++r) dkvpr[PQ * 3 + r] = gvp[r];
}

}  // namespace

bool ipa_core_supported(int L, int c, int Pq, int Pv) {
  return L >= 1 && L <= kIpaLongMaxL && c == 32 && Pq == 8 && Pv == 8;
}

hipError_t ipa_core_fwd_launch(int B, int L, int H, const float* q, const float* kv, const float* qp, const float* kvp,
                               const float* mask, const float* rots, const float* trans, const float* hw, float wc,
                               float* out, int flags, hipStream_t s) {
  if (L > kIpaMaxL)
    hipLaunchKernelGGL((ipa_core_fwd_long_kernel<32, 8, 8>), dim3(B * H), dim3(256), 0, s, L, H, q, kv, qp, kvp, mask,
                       rots, trans, hw, wc, out, flags);
  else
    hipLaunchKernelGGL((ipa_core_fwd_kernel<32, 8, 8>), dim3(B * H), dim3(64), 0, s, L, H, q, kv, qp, kvp, mask, rots,
                       trans, hw, wc, out, flags);
  return hipGetLastError();
}

hipError_t ipa_core_bwd_launch(int B, int L, int H, const float* q, const float* kv, const float* qp, const float* kvp,
                               const float* mask, const float* rots, const float* trans, const float* hw, float wc,
                               const float* dout, float* dq, float* dkv, float* dqp, float* dkvp, float* dhw_part,
                               int flags, hipStream_t s) {
  if (L > kIpaMaxL)
    hipLaunchKernelGGL((ipa_core_bwd_long_kernel<32, 8, 8>), dim3(B * H), dim3(256), 0, s, L, H, q, kv, qp, kvp, mask,
                       rots, trans, hw, wc, dout, dq, dkv, dqp, dkvp, dhw_part, flags);
  else
    hipLaunchKernelGGL((ipa_core_bwd_kernel<32, 8, 8>), dim3(B * H), dim3(64), 0, s, L, H, q, kv, qp, kvp, mask, rots,
                       trans, hw, wc, dout, dq, dkv, dqp, dkvp, dhw_part, flags);
  return hipGetLastError();
}

}  // namespace mdg
