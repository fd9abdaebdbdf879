// Conditioning precompute kernels (mdg_precompute_cond, capi.hip): the x-independent part of
// LatentMDGenModel.forward, evaluated once per rollout window for all S Euler time points.
//
//   temb_freq_kernel  TimestepEmbedder's sinusoid (layers.py:32-50): [cos(t' f_i) | sin(t' f_i)]
//                     with t' = t * time_multiplier (latent_model.py:252), freqs from the host
//                     table the reference builds on the CPU (layers.py:42-44)
//   cond_scatter      one stacked adaLN GEMM's rows -> the per-step layouts the denoiser reads
//   ipa_init          run_ipa's input (latent_model.py:187-208): aatype embedding, and for TPS
//                     latent_to_emb_f/_r of the relative 7-vectors
//   ipa_attn_kernel   InvariantPointAttention core (ipa.py:108-255, c_z = 0): points to the
//                     global frame, scalar + point logits, square mask, softmax, outputs back to
//                     the local frame, point norms -> the linear_out input row
// The GEMMs (t-MLP, adaLN, IPA projections, linear_out, the IPA layers' MHA and MLP) run on
// mdg_gemm's exact-f32 MFMA tiles.  All arithmetic is fp32; this whole precompute is < 1 % of
// a window's time, so these kernels are written for exactness and generality, not speed.
#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {

__global__ void temb_freq_kernel(int R, int half, float mult, const float* __restrict__ t,
                                 const float* __restrict__ freqs, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * half) return;
  const int r = i / half, k = i - r * half;
  const float arg = (t[r] * mult) * freqs[k];  // (t * multiplier)[:, None].float() * freqs[None]
  out[(size_t)r * 2 * half + k] = cosf(arg);
  out[(size_t)r * 2 * half + half + k] = sinf(arg);
}

// cond_all [S*B][W] (W = nl*9C + 2C + ...) -> mods [lanes][S][nl][B/lanes][9C], mods_final [S][B][2C]
__global__ void cond_scatter_kernel(int S, int B, int nl, int C, int W, int lanes, const float* __restrict__ all,
                                    float* __restrict__ mods, float* __restrict__ mods_final) {
  const int per = nl * 9 * C + 2 * C;  // floats copied per row r
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)S * B * per) return;
  const int r = (int)(i / per), k = (int)(i - (size_t)r * per);
  const int s = r / B, b = r - s * B;
  const float v = all[(size_t)r * W + k];
  if (k < nl * 9 * C) {
    const int layer = k / (9 * C), j = k - layer * 9 * C;
    const int Bl = B / lanes, lane = b / Bl, bl = b - lane * Bl;
    mods[((((size_t)lane * S + s) * nl + layer) * Bl + bl) * 9 * C + j] = v;
  } else {
    mods_final[(size_t)r * 2 * C + (k - nl * 9 * C)] = v;
  }
}

// x[m] (m = r*L + l, r = s*B + b) = [l2e(rel7[b][l])] + [aa_emb[aatype[b][l]]]; mask_rep[m] = mask[b][l]
__global__ void ipa_init_kernel(int R, int B, int L, int C, int mstride, const int64_t* __restrict__ aatype,
                                const float* __restrict__ aa_emb, const float* __restrict__ rel7,
                                const float* __restrict__ w, const float* __restrict__ bias,
                                const float* __restrict__ mask, float* __restrict__ x,
                                float* __restrict__ mask_rep) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)R * L * C) return;
  const int m = (int)(i / C), c = (int)(i - (size_t)m * C);
  const int r = m / L, l = m - r * L, b = r % B;
  float v = 0.f;
  if (rel7) {  // nn.Linear(7, C): bias + sum_k W[c][k] rel[k]
    const float* q = rel7 + ((size_t)b * L + l) * 7;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 7; ++k) acc = fmaf(ld1(w + c * 7 + k), ld1(q + k), acc);
    v = acc + bias[c];
  }
  if (aa_emb) v += aa_emb[aatype[(size_t)b * L + l] * C + c];
  x[i] = v;
  if (mask_rep && c == 0) mask_rep[m] = mask[(size_t)b * mstride + l];
}

__global__ void add_inplace_kernel(size_t n, float* __restrict__ y, const float* __restrict__ x) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] += x[i];
}

// One block (one wave) per (sample r, head h, group of 64 query residues); thread = query
// residue, keys staged in LDS in chunks of 64 with an online softmax.  proj row layout (ldp floats per residue, ipa.py:113-152):
//   q [h*CH + i] | kv [H*CH + h*2CH + {0..CH-1: k, CH..2CH-1: v}] |
//   q_pts raw [3][H*PQ] (x block, y block, z block; point j = h*PQ + p) |
//   kv_pts raw [3][H*(PQ+PV)] (point j = h*(PQ+PV) + p; p < PQ: k, else v)
// out row (ldc floats): o [h*CH + i] | o_pt x [H*PV] | y | z | |o_pt| [H*PV]  (ipa.py:247-253)
template <int CH, int PQ, int PV>
__global__ __launch_bounds__(64) void ipa_attn_kernel(int R, int B, int L, int H, const float* __restrict__ proj,
                                                      int ldp, const float* __restrict__ rots,
                                                      const float* __restrict__ trans, const float* __restrict__ mask,
                                                      const float* __restrict__ head_weights, float* __restrict__ out,
                                                      int ldc) {
  constexpr int KW = 2 * CH + 3 * PQ + 3 * PV;  // floats per staged key
  __shared__ float ks[64][KW + 1];
  __shared__ float mk[64];
  const int nqg = (L + 63) / 64;
  const int r = blockIdx.x / (H * nqg), hq = blockIdx.x - r * (H * nqg), h = hq / nqg, b = r % B, tid = threadIdx.x;
  const int i0 = (hq - h * nqg) * 64;
  const int HPq = H * PQ, HPkv = H * (PQ + PV);
  const int oqp = 3 * H * CH, okvp = oqp + 3 * HPq;
  // softplus(head_weights) * sqrt(1 / (3 * (P_q * 9 / 2)))  (ipa.py:180-185)
  const float hwr = head_weights[h];
  const float hw = (hwr > 20.f ? hwr : log1pf(expf(hwr))) * sqrtf(1.0f / (3.0f * (PQ * 9.0f / 2.0f)));
  const float qk_scale = sqrtf(1.0f / (3.0f * CH));
  const float* rot_b = rots + (size_t)b * L * 9;
  const float* tr_b = trans + (size_t)b * L * 3;
  const float* mask_r = mask + (size_t)r * L;  // sample-replicated frame mask [R][L]

  {
    const int i = i0 + tid;
    const bool qv = i < L;
    const int ii = qv ? i : L - 1;
    const float* prow = proj + ((size_t)r * L + ii) * ldp;
    float q[CH], qp[PQ][3];
#pragma unroll
    for (int c = 0; c < CH; ++c) q[c] = prow[h * CH + c];
    float Ri[3][3], ti[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
      for (int c = 0; c < 3; ++c) Ri[a][c] = ld1(rot_b + (size_t)ii * 9 + a * 3 + c);
      ti[a] = ld1(tr_b + (size_t)ii * 3 + a);
    }
#pragma unroll
    for (int p = 0; p < PQ; ++p) {
      const int j = h * PQ + p;
      const float x = prow[oqp + j], y = prow[oqp + HPq + j], z = prow[oqp + 2 * HPq + j];
#pragma unroll
      for (int a = 0; a < 3; ++a) qp[p][a] = Ri[a][0] * x + Ri[a][1] * y + Ri[a][2] * z + ti[a];  // Rigid.apply
    }
    const float mi = mask_r[ii];
    float mrun = -INFINITY, lrun = 0.f, acc[CH], accp[PV][3];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = 0.f;
#pragma unroll
    for (int p = 0; p < PV; ++p) accp[p][0] = accp[p][1] = accp[p][2] = 0.f;

    for (int j0 = 0; j0 < L; j0 += 64) {
      __syncthreads();
      const int j = j0 + tid;
      if (j < L) {  // stage key j: k, v, k_pts and v_pts in the global frame
        const float* kr = proj + ((size_t)r * L + j) * ldp;
        float* dst = ks[tid];
#pragma unroll
        for (int c = 0; c < 2 * CH; ++c) dst[c] = kr[H * CH + h * 2 * CH + c];
        float Rj[3][3], tj[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
#pragma unroll
          for (int c = 0; c < 3; ++c) Rj[a][c] = ld1(rot_b + (size_t)j * 9 + a * 3 + c);
          tj[a] = ld1(tr_b + (size_t)j * 3 + a);
        }
#pragma unroll
        for (int p = 0; p < PQ + PV; ++p) {
          const int jj = h * (PQ + PV) + p;
          const float x = kr[okvp + jj], y = kr[okvp + HPkv + jj], z = kr[okvp + 2 * HPkv + jj];
#pragma unroll
          for (int a = 0; a < 3; ++a) dst[2 * CH + 3 * p + a] = Rj[a][0] * x + Rj[a][1] * y + Rj[a][2] * z + tj[a];
        }
        mk[tid] = mask_r[j];
      }
      __syncthreads();
      const int nk = min(64, L - j0);
      for (int kk = 0; kk < nk; ++kk) {
        const float* kv = ks[kk];
        float dot = 0.f;
#pragma unroll
        for (int c = 0; c < CH; ++c) dot = fmaf(q[c], kv[c], dot);
        float pt = 0.f;
#pragma unroll
        for (int p = 0; p < PQ; ++p) {
          const float dx = qp[p][0] - kv[2 * CH + 3 * p], dy = qp[p][1] - kv[2 * CH + 3 * p + 1],
                      dz = qp[p][2] - kv[2 * CH + 3 * p + 2];
          pt += (dx * dx + dy * dy + dz * dz) * hw;
        }
        // a = q.k * sqrt(1/(3c)) + (-0.5 * sum_p hw d2) + inf * (m_i m_j - 1)   (ipa.py:162-205)
        const float logit = (dot * qk_scale + pt * (-0.5f)) + 1e5f * (mi * mk[kk] - 1.0f);
        const float mnew = fmaxf(mrun, logit);
        const float corr = expf(mrun - mnew), pw = expf(logit - mnew);
        mrun = mnew;
        lrun = lrun * corr + pw;
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = acc[c] * corr + pw * kv[CH + c];
#pragma unroll
        for (int p = 0; p < PV; ++p)
#pragma unroll
          for (int a = 0; a < 3; ++a) accp[p][a] = accp[p][a] * corr + pw * kv[2 * CH + 3 * (PQ + p) + a];
      }
    }
    if (qv) {
      const float inv = 1.0f / lrun;
      float* orow = out + ((size_t)r * L + i) * ldc;
#pragma unroll
      for (int c = 0; c < CH; ++c) orow[h * CH + c] = acc[c] * inv;
      const int HPv = H * PV, base = H * CH;
#pragma unroll
      for (int p = 0; p < PV; ++p) {
        // Rigid.invert_apply: R^T (p - t)
        const float d0 = accp[p][0] * inv - ti[0], d1 = accp[p][1] * inv - ti[1], d2 = accp[p][2] * inv - ti[2];
        const float lx = Ri[0][0] * d0 + Ri[1][0] * d1 + Ri[2][0] * d2;
        const float ly = Ri[0][1] * d0 + Ri[1][1] * d1 + Ri[2][1] * d2;
        const float lz = Ri[0][2] * d0 + Ri[1][2] * d1 + Ri[2][2] * d2;
        const int j = h * PV + p;
        orow[base + j] = lx;
        orow[base + HPv + j] = ly;
        orow[base + 2 * HPv + j] = lz;
        orow[base + 3 * HPv + j] = sqrtf(lx * lx + ly * ly + lz * lz + 1e-8f);
      }
    }
  }
}

hipError_t temb_freq_launch(int R, int half, float mult, const float* t, const float* freqs, float* out,
                            hipStream_t s) {
  const int n = R * half;
  hipLaunchKernelGGL(temb_freq_kernel, dim3((n + 255) / 256), dim3(256), 0, s, R, half, mult, t, freqs, out);
  return hipGetLastError();
}

hipError_t cond_scatter_launch(int S, int B, int nl, int C, int W, int lanes, const float* all, float* mods,
                               float* mods_final, hipStream_t s) {
  const size_t n = (size_t)S * B * (nl * 9 * C + 2 * C);
  hipLaunchKernelGGL(cond_scatter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, S, B, nl, C, W, lanes,
                     all, mods, mods_final);
  return hipGetLastError();
}

hipError_t ipa_init_launch(int R, int B, int L, int C, int mstride, const int64_t* aatype, const float* aa_emb, const float* rel7,
                           const float* w, const float* bias, const float* mask, float* x, float* mask_rep,
                           hipStream_t s) {
  const size_t n = (size_t)R * L * C;
  hipLaunchKernelGGL(ipa_init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, R, B, L, C, mstride, aatype, aa_emb,
                     rel7, w, bias, mask, x, mask_rep);
  return hipGetLastError();
}

hipError_t add_inplace_launch(size_t n, float* y, const float* x, hipStream_t s) {
  hipLaunchKernelGGL(add_inplace_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, y, x);
  return hipGetLastError();
}

// IPA shapes with a kernel instance; others are refused by the ABI (MDG_E_SHAPE)
bool ipa_attn_supported(int c, int pq, int pv) {
  return (c == 32 && pq == 8 && pv == 8) || (c == 16 && pq == 4 && pv == 8) || (c == 8 && pq == 4 && pv == 4) ||
         (c == 16 && pq == 8 && pv == 8);
}

hipError_t ipa_attn_launch(int R, int B, int L, int H, int c, int pq, int pv, const float* proj, int ldp,
                           const float* rots, const float* trans, const float* mask, const float* head_weights,
                           float* out, int ldc, hipStream_t s) {
  const dim3 grid((unsigned)(R * H * ((L + 63) / 64))), block(64);
#define MDG_IPA(CH_, PQ_, PV_)                                                                              \
  if (c == CH_ && pq == PQ_ && pv == PV_) {                                                                 \
    hipLaunchKernelGGL((ipa_attn_kernel<CH_, PQ_, PV_>), grid, block, 0, s, R, B, L, H, proj, ldp, rots, trans, \
                       mask, head_weights, out, ldc);                                                       \
    return hipGetLastError();                                                                               \
  }
  MDG_IPA(32, 8, 8)
  MDG_IPA(16, 4, 8)
  MDG_IPA(16, 8, 8)
  MDG_IPA(8, 4, 4)
#undef MDG_IPA
  return hipErrorInvalidValue;
}

}  // namespace mdg
