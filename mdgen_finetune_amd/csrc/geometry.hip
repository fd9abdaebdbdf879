// Batch preparation on the device: the rigid-frame offsets and latent assembly of
// NewMDGenWrapper.prep_batch (reference src/mdgen/wrapper.py:283-365), which the reference
// runs in eager PyTorch with a CPU LAPACK eigen-solve per frame (rot_to_quat,
// rigid_utils.py:191-210, via get_offsets, utils.py:7-14).
//
// One thread per token (b, t, l); everything is per-token arithmetic on 48 B of input, so
// the kernel is HBM/latency-bound and tiny next to the denoiser.  Frame-0 (and, for TPS,
// frame-(T-1)) rigids are re-read by the T tokens of a residue and stay in L2.
//
// Quaternion from the relative rotation R: the reference takes the eigenvector of the
// largest eigenvalue of the symmetric K(R) (K = (4 q q^T - I)/3 for an exact rotation).
// Here: Shepperd's column of (3K + I) = 4 q q^T with the largest diagonal, then two power
// steps with (3K + I), whose spectrum is {4, 0, 0, 0} up to R's rounding, so the result is
// that same dominant eigenvector to fp32 rounding; the wrapper's sign fix (real part >= 0,
// wrapper.py:309) removes the eigen-solver's arbitrary sign.
#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {

struct Rig {
  float r[3][3];
  float t[3];
};

__device__ __forceinline__ Rig load_rig(const float* __restrict__ rots, const float* __restrict__ trans, size_t i) {
  Rig g;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
#pragma unroll
    for (int b = 0; b < 3; ++b) g.r[a][b] = ld1(rots + i * 9 + a * 3 + b);
    g.t[a] = ld1(trans + i * 3 + a);
  }
  return g;
}

// ref.invert().compose(x) (rigid_utils.py Rigid.invert / compose): R = Rr^T Rx, t = Rr^T (tx - tr)
__device__ __forceinline__ Rig rel(const Rig& ref, const Rig& x) {
  Rig o;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) o.r[i][j] = ref.r[0][i] * x.r[0][j] + ref.r[1][i] * x.r[1][j] + ref.r[2][i] * x.r[2][j];
    const float a = ref.r[0][i] * x.t[0] + ref.r[1][i] * x.t[1] + ref.r[2][i] * x.t[2];
    const float b = ref.r[0][i] * ref.t[0] + ref.r[1][i] * ref.t[1] + ref.r[2][i] * ref.t[2];
    o.t[i] = a - b;
  }
  return o;
}

__device__ __forceinline__ void rot_to_quat_dev(const float (&r)[3][3], float q[4]) {
  const float xx = r[0][0], xy = r[0][1], xz = r[0][2];
  const float yx = r[1][0], yy = r[1][1], yz = r[1][2];
  const float zx = r[2][0], zy = r[2][1], zz = r[2][2];
  // M = 3K + I (rigid_utils.py:199-206 without the 1/3)
  float m[4][4] = {
      {xx + yy + zz + 1.f, zy - yz, xz - zx, yx - xy},
      {zy - yz, xx - yy - zz + 1.f, xy + yx, xz + zx},
      {xz - zx, xy + yx, yy - xx - zz + 1.f, yz + zy},
      {yx - xy, xz + zx, yz + zy, zz - xx - yy + 1.f},
  };
  int c = 0;
#pragma unroll
  for (int j = 1; j < 4; ++j)
    if (m[j][j] > m[c][c]) c = j;
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = m[i][c];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    float w[4];
    float n2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = m[i][0] * v[0] + m[i][1] * v[1] + m[i][2] * v[2] + m[i][3] * v[3];
      n2 += w[i] * w[i];
    }
    const float inv = rsqrtf(n2);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = w[i] * inv;
  }
  // final normalisation in full precision
  const float n = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = v[i] / n;
}

__global__ void prep_latents_kernel(int B, int T, int L, int lat, int tps, int no_offsets, int cond_mode,
                                    int cond_interval, const float* __restrict__ rots,
                                    const float* __restrict__ trans, const float* __restrict__ torsions,
                                    float* __restrict__ latents, float* __restrict__ x_cond,
                                    int64_t* __restrict__ cond_mask) {
  const size_t n = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t N = (size_t)B * T * L;
  if (n >= N) return;
  const int l = (int)(n % L);
  const size_t bt = n / L;
  const int t = (int)(bt % T);
  const int b = (int)(bt / T);
  bool cond = false;
  if ((cond_mode & MDG_PREP_COND_FIRST) && t == 0) cond = true;
  if ((cond_mode & MDG_PREP_COND_LAST) && t == T - 1) cond = true;
  if (cond_interval > 0 && t % cond_interval == 0) cond = true;
  float* lrow = latents + n * lat;
  float* xrow = x_cond ? x_cond + n * lat : nullptr;
  auto put = [&](int i, float v) {
    st1(lrow + i, v);
    if (xrow) st1(xrow + i, cond ? v : 0.f);
  };
  const Rig x = load_rig(rots, trans, n);
  const int nref = tps ? 2 : 1;
  for (int k = 0; k < nref; ++k) {
    Rig o;
    if (no_offsets && k == 0) {
      o = x;
    } else {
      const size_t ri = ((size_t)b * T + (k == 0 ? 0 : T - 1)) * L + l;
      o = rel(load_rig(rots, trans, ri), x);
    }
    float q[4];
    rot_to_quat_dev(o.r, q);
    const float sg = q[0] < 0.f ? -1.f : 1.f;  // wrapper.py:309
#pragma unroll
    for (int i = 0; i < 4; ++i) put(7 * k + i, q[i] * sg);
#pragma unroll
    for (int i = 0; i < 3; ++i) put(7 * k + 4 + i, o.t[i]);
  }
#pragma unroll
  for (int i = 0; i < 14; ++i) put(7 * nref + i, torsions ? ld1(torsions + n * 14 + i) : 0.f);
  if (cond_mask) cond_mask[n] = cond ? 1 : 0;
}

hipError_t prep_latents_launch(int B, int T, int L, int lat, int tps, int no_offsets, int cond_mode,
                               int cond_interval, const float* rots, const float* trans, const float* torsions,
                               float* latents, float* x_cond, int64_t* cond_mask, hipStream_t s) {
  const size_t N = (size_t)B * T * L;
  hipLaunchKernelGGL(prep_latents_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, B, T, L, lat, tps,
                     no_offsets, cond_mode, cond_interval, rots, trans, torsions, latents, x_cond, cond_mask);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Denoised latents -> atom14 coordinates (wrapper.py:480-505 + geometry.py:62-81, 218-317),
// one thread per token: the offset quaternion (normalised) and translation composed onto the
// token's frame-0 rigid, the 7 torsions normalised to unit (sin, cos), the 8 rigid-group
// frames of the residue type (default frame o torsion rotation, chi2..4 chained onto chi1),
// then each of the 14 atoms = its group's frame applied to the literature position.
__device__ __forceinline__ void mat3_mul(const float (&a)[3][3], const float (&b)[3][3], float (&c)[3][3]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) c[i][j] = a[i][0] * b[0][j] + a[i][1] * b[1][j] + a[i][2] * b[2][j];
}

__global__ void latents_to_atom14_kernel(int B, int T, int L, int lat, int tors_off, int renorm,
                                         const float* __restrict__ samples, const float* __restrict__ ref_rots,
                                         const float* __restrict__ ref_trans, const int64_t* __restrict__ aatype,
                                         const float* __restrict__ default_frames, const int* __restrict__ group_idx,
                                         const float* __restrict__ atom_mask, const float* __restrict__ lit,
                                         float* __restrict__ atom14, float* __restrict__ out_rots,
                                         float* __restrict__ out_trans) {
  const size_t n = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= (size_t)B * T * L) return;
  const int l = (int)(n % L);
  const int b = (int)(n / ((size_t)T * L));
  const float* x = samples + n * lat;
  // Rigid.from_tensor_7(offsets, normalize_quats=True) (rigid_utils.py:155-189 quat -> rot)
  float qa = ld1(x), qb = ld1(x + 1), qc = ld1(x + 2), qd = ld1(x + 3);
  const float x4 = ld1(x + 4), x5 = ld1(x + 5), x6 = ld1(x + 6);
  const float qn = sqrtf(qa * qa + qb * qb + qc * qc + qd * qd);
  qa /= qn; qb /= qn; qc /= qn; qd /= qn;
  const float rr[3][3] = {
      {qa * qa + qb * qb - qc * qc - qd * qd, 2.f * (qb * qc - qa * qd), 2.f * (qb * qd + qa * qc)},
      {2.f * (qb * qc + qa * qd), qa * qa - qb * qb + qc * qc - qd * qd, 2.f * (qc * qd - qa * qb)},
      {2.f * (qb * qd - qa * qc), 2.f * (qc * qd + qa * qb), qa * qa - qb * qb - qc * qc + qd * qd}};
  // frame = frame0 o rel
  const size_t bl = (size_t)b * L + l;
  float r0[3][3], t0[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) r0[i][j] = ld1(ref_rots + bl * 9 + i * 3 + j);
    t0[i] = ld1(ref_trans + bl * 3 + i);
  }
  float R[3][3], Tt[3];
  mat3_mul(r0, rr, R);
#pragma unroll
  for (int i = 0; i < 3; ++i) Tt[i] = r0[i][0] * x4 + r0[i][1] * x5 + r0[i][2] * x6 + t0[i];
  if (out_rots) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) st1(out_rots + n * 9 + i * 3 + j, R[i][j]);
      st1(out_trans + n * 3 + i, Tt[i]);
    }
  }
  int aa = (int)aatype[n];
  aa = aa < 0 ? 0 : (aa > 20 ? 20 : aa);
  // 8 group frames relative to the backbone: default_r o rot_x(alpha)   (geometry.py:283-301)
  float gR[8][3][3], gT[8][3];
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    float sa = 0.f, ca = 1.f;  // backbone group: identity rotation (bb_rot = (0, 1))
    if (g > 0) {
      sa = ld1(x + tors_off + 2 * (g - 1));
      ca = ld1(x + tors_off + 2 * (g - 1) + 1);
      if (renorm) {
        const float nn = sqrtf(sa * sa + ca * ca);
        sa /= nn;
        ca /= nn;
      }
    }
    const float* d = default_frames + ((size_t)aa * 8 + g) * 16;
    // D_R . [[1,0,0],[0,c,-s],[0,s,c]]
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float d0 = d[i * 4 + 0], d1 = d[i * 4 + 1], d2 = d[i * 4 + 2];
      gR[g][i][0] = d0;
      gR[g][i][1] = d1 * ca + d2 * sa;
      gR[g][i][2] = -d1 * sa + d2 * ca;
      gT[g][i] = d[i * 4 + 3];
    }
  }
#pragma unroll
  for (int g = 5; g < 8; ++g) {  // chi2..chi4 chained onto the previous chi frame
    float nr[3][3], nt[3];
    mat3_mul(gR[g - 1], gR[g], nr);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      nt[i] = gR[g - 1][i][0] * gT[g][0] + gR[g - 1][i][1] * gT[g][1] + gR[g - 1][i][2] * gT[g][2] + gT[g - 1][i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) gR[g][i][j] = nr[i][j];
      gT[g][i] = nt[i];
    }
  }
  float* out = atom14 + n * 42;
  for (int a = 0; a < 14; ++a) {
    const int g = group_idx[aa * 14 + a];
    const float m = atom_mask[aa * 14 + a];
    const float* p = lit + ((size_t)aa * 14 + a) * 3;
    const float p0 = ld1(p), p1 = ld1(p + 1), p2 = ld1(p + 2);
    float lr[3][3], lt[3];
    // select the group frame without dynamic register indexing
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      lt[i] = gT[0][i];
#pragma unroll
      for (int j = 0; j < 3; ++j) lr[i][j] = gR[0][i][j];
    }
#pragma unroll
    for (int gg = 1; gg < 8; ++gg)
      if (g == gg) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          lt[i] = gT[gg][i];
#pragma unroll
          for (int j = 0; j < 3; ++j) lr[i][j] = gR[gg][i][j];
        }
      }
    // local = group frame . lit ; global = frame . local
    float loc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) loc[i] = lr[i][0] * p0 + lr[i][1] * p1 + lr[i][2] * p2 + lt[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) st1(out + a * 3 + i, (R[i][0] * loc[0] + R[i][1] * loc[1] + R[i][2] * loc[2] + Tt[i]) * m);
  }
}

hipError_t latents_to_atom14_launch(int B, int T, int L, int lat, int tors_off, int renorm, const float* samples,
                                    const float* ref_rots, const float* ref_trans, const int64_t* aatype,
                                    const float* default_frames, const int* group_idx, const float* atom_mask,
                                    const float* lit, float* atom14, float* out_rots, float* out_trans,
                                    hipStream_t s) {
  const size_t N = (size_t)B * T * L;
  hipLaunchKernelGGL(latents_to_atom14_kernel, dim3((unsigned)((N + 127) / 128)), dim3(128), 0, s, B, T, L, lat,
                     tors_off, renorm, samples, ref_rots, ref_trans, aatype, default_frames, group_idx, atom_mask,
                     lit, atom14, out_rots, out_trans);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// TPS relative frames (latent_model.py:197-199): per residue (b, l) the 7-vectors of
// start^-1 o end and end^-1 o start (Rigid.invert / compose / to_tensor_7), quaternion by the
// same dominant-eigenvector construction as prep_latents, sign fixed to w >= 0 (LAPACK's
// eigh leaves it arbitrary; the reference passes it on unfixed).
__global__ void tps_rel7_kernel(int BL, const float* __restrict__ rots, const float* __restrict__ trans,
                                const float* __restrict__ erots, const float* __restrict__ etrans,
                                float* __restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= BL) return;
  const Rig a = load_rig(rots, trans, n), e = load_rig(erots, etrans, n);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const Rig o = k == 0 ? rel(a, e) : rel(e, a);
    float q[4];
    rot_to_quat_dev(o.r, q);
    const float sg = q[0] < 0.f ? -1.f : 1.f;
    float* row = out + ((size_t)k * BL + n) * 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) st1(row + i, q[i] * sg);
#pragma unroll
    for (int i = 0; i < 3; ++i) st1(row + 4 + i, o.t[i]);
  }
}

hipError_t tps_rel7_launch(int B, int L, const float* rots, const float* trans, const float* erots,
                           const float* etrans, float* out, hipStream_t s) {
  const int BL = B * L;
  hipLaunchKernelGGL(tps_rel7_kernel, dim3((BL + 127) / 128), dim3(128), 0, s, BL, rots, trans, erots, etrans, out);
  return hipGetLastError();
}

}  // namespace mdg
