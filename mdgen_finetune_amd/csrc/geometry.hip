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
    for (int b = 0; b < 3; ++b) g.r[a][b] = rots[i * 9 + a * 3 + b];
    g.t[a] = trans[i * 3 + a];
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
    lrow[i] = v;
    if (xrow) xrow[i] = cond ? v : 0.f;
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
  for (int i = 0; i < 14; ++i) put(7 * nref + i, torsions ? torsions[n * 14 + i] : 0.f);
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

}  // namespace mdg
