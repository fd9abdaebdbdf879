// Training-step glue around the block stack on gfx950: the token embedding's backward and the
// FinalLayer's forward / backward, as library launches instead of ~40 eager PyTorch kernels
// (elementwise adds and modulates over the 32 000 x 384 fp32 residual, their column-sum
// reductions, the LayerNorm backward and three hipBLASLt GEMMs) per training step.
// Reference: LatentMDGenModel.forward (latent_model.py:242-255: latent_to_emb + pos_embed +
// cond_to_emb + mask_to_emb + the IPA prepend broadcast over frames) and FinalLayer
// (layers.py:58-75: no-affine LayerNorm, adaLN modulate, Linear C -> latent) under
// loss.backward() (transport.py:137-222).  All fp32 (the reference's parameter precision).
//
//  * embed_bwd: block = (trajectory b, chunk of frames) x 128 columns; threads 0-127 own one
//    column's latent_to_emb weight-gradient row (K1 accumulators) + the bias column sum + the
//    IPA-prepend gradient of each residue l; threads 128-255 the cond_to_emb row (K2) + the
//    mask_to_emb row sums.  The chunk's x rows are staged in LDS (broadcast reads), dh is read
//    once, coalesced.  Per-chunk partials, then one launch sums them in chunk order
//    (deterministic).  HBM: one pass over dh (49 MB at B=8, T=1000, L=4).
//  * final_fwd: one wave per token row: LN statistics as two wave reductions (6 columns per
//    lane), the modulate, and the 21 output dots from W in LDS, reduced by a halving
//    transpose-sum (32 shuffles for 32 outputs); writes v and (mean, rstd).
//  * final_bwd: one wave per row, rows of one trajectory per block: dxn = dv W, the LN +
//    modulate backward into dh, and per-wave register accumulators of dW (6 columns x 21
//    outputs per lane), dbias, d shift, d scale; block partials summed in order by a reduce
//    launch.
#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {

namespace {

constexpr int kEbFrames = 32, kEbK = 32, kEbLMax = 8, kEbEMax = 4;

struct EbPlan {
  int tch, chunks;  // frame chunks per trajectory, total chunks
  size_t p1, p2, pb, pe, pi, total;  // element offsets of the partial arrays
};

EbPlan eb_plan(int B, int T, int L, int C, int K1, int K2, int E) {
  EbPlan p{};
  p.tch = (T + kEbFrames - 1) / kEbFrames;
  p.chunks = B * p.tch;
  size_t off = 0;
  auto take = [&](size_t n) {
    const size_t o = off;
    off += (n + 63) & ~size_t(63);
    return o;
  };
  p.p1 = take((size_t)p.chunks * C * K1);
  p.p2 = take((size_t)p.chunks * C * (K2 > 0 ? K2 : 0));
  p.pb = take((size_t)p.chunks * C);
  p.pe = take((size_t)p.chunks * C * E);
  p.pi = take((size_t)p.chunks * C * L);
  p.total = off;
  return p;
}

__global__ __launch_bounds__(256) void embed_bwd_kernel(int B, int T, int L, int C, int K1, const float* __restrict__ x1,
                                                        int K2, const float* __restrict__ x2,
                                                        const int64_t* __restrict__ idx, int E,
                                                        const float* __restrict__ dh, float* __restrict__ ws,
                                                        EbPlan pl) {
  // the chunk's x1 and x2 rows, zero-padded to kEbK columns (64 KiB: two blocks per CU)
  __shared__ __attribute__((aligned(16))) float xs[2][kEbFrames * kEbLMax][kEbK];
  const int chunk = blockIdx.x, b = chunk / pl.tch, tc = chunk % pl.tch;
  const int t0 = tc * kEbFrames, nf = min(kEbFrames, T - t0), ntok = nf * L;
  const size_t n0 = ((size_t)b * T + t0) * L;
  const int tid = threadIdx.x, op = tid >> 7, c = blockIdx.y * 128 + (tid & 127);
  const int K = op ? K2 : K1;
  for (int i = tid; i < ntok * kEbK; i += 256) {
    const int r = i / kEbK, k = i % kEbK;
    xs[0][r][k] = k < K1 ? x1[(n0 + r) * K1 + k] : 0.f;
    xs[1][r][k] = (x2 && k < K2) ? x2[(n0 + r) * K2 + k] : 0.f;
  }
  __syncthreads();
  if (c >= C || (op && !x2)) return;
  float acc[kEbK];
#pragma unroll
  for (int k = 0; k < kEbK; ++k) acc[k] = 0.f;
  float cs = 0.f, lsum[kEbLMax], esum[kEbEMax];
#pragma unroll
  for (int u = 0; u < kEbLMax; ++u) lsum[u] = 0.f;
#pragma unroll
  for (int u = 0; u < kEbEMax; ++u) esum[u] = 0.f;
  const float (*X)[kEbK] = xs[op];
  const float* dcol = dh + n0 * C + c;
  // rows in groups of 8 with their dh (and mask index) loads issued up front: one dependent
  // HBM round trip per group instead of per row
  for (int rb = 0; rb < ntok; rb += 8) {
    float gv[8];
    int ev[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      gv[u] = rb + u < ntok ? dcol[(size_t)(rb + u) * C] : 0.f;
      ev[u] = (op && idx && rb + u < ntok) ? (int)idx[n0 + rb + u] : -1;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = rb + u;
      if (r >= ntok) break;
      const int l = r % L;
      const float g = gv[u];
#pragma unroll
      for (int k4 = 0; k4 < kEbK; k4 += 4) {
        if (k4 < K) {
          const float4 xv = *reinterpret_cast<const float4*>(&X[r][k4]);
          acc[k4] = fmaf(g, xv.x, acc[k4]);
          acc[k4 + 1] = fmaf(g, xv.y, acc[k4 + 1]);
          acc[k4 + 2] = fmaf(g, xv.z, acc[k4 + 2]);
          acc[k4 + 3] = fmaf(g, xv.w, acc[k4 + 3]);
        }
      }
      if (op == 0) {
        cs += g;
#pragma unroll
        for (int q = 0; q < kEbLMax; ++q) lsum[q] += (q == l) ? g : 0.f;
      } else if (idx) {
#pragma unroll
        for (int q = 0; q < kEbEMax; ++q) esum[q] += (q == ev[u]) ? g : 0.f;
      }
    }
  }
  {  // [chunk][k][C]: each store instruction writes 64 consecutive floats
    float* P = ws + (op ? pl.p2 : pl.p1) + (size_t)chunk * K * C + c;
#pragma unroll
    for (int k = 0; k < kEbK; ++k)
      if (k < K) P[(size_t)k * C] = acc[k];
  }
  if (op == 0) {
    ws[pl.pb + (size_t)chunk * C + c] = cs;
#pragma unroll
    for (int l = 0; l < kEbLMax; ++l)
      if (l < L) ws[pl.pi + ((size_t)chunk * L + l) * C + c] = lsum[l];
  } else if (idx) {
#pragma unroll
    for (int e = 0; e < kEbEMax; ++e)
      if (e < E) ws[pl.pe + ((size_t)chunk * E + e) * C + c] = esum[e];
  }
}

// Ordered chunk sums, 64 outputs per block: wave q sums chunks [q Z / 4, (q + 1) Z / 4) of its
// lane's output (4 loads in flight), and lane e of wave 0 adds the four in order -- a fixed
// association (deterministic), a quarter of the dependent-load chain of one thread per output.
__device__ __forceinline__ float zsum4(const float* p, size_t zstride, int z0, int z1, float* red) {
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int Z = z1 - z0, a = z0 + q * Z / 4, b = z0 + (q + 1) * Z / 4;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int z = a;
  for (; z + 4 <= b; z += 4) {
    s0 += p[(size_t)z * zstride];
    s1 += p[(size_t)(z + 1) * zstride];
    s2 += p[(size_t)(z + 2) * zstride];
    s3 += p[(size_t)(z + 3) * zstride];
  }
  for (; z < b; ++z) s0 += p[(size_t)z * zstride];
  red[q * 64 + lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  return ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
}

// sums the chunk partials: dw1 [C][K1], dw2 [C][K2], db [C], demb [E][C], dipa [B][L][C] (over
// the chunks of trajectory b); block = 64 outputs x 4 chunk quarters
__global__ __launch_bounds__(256) void embed_bwd_reduce_kernel(int B, int L, int C, int K1, int K2, int E,
                                                               const float* __restrict__ ws, EbPlan pl,
                                                               float* __restrict__ dw1, float* __restrict__ dw2,
                                                               float* __restrict__ db, float* __restrict__ demb,
                                                               float* __restrict__ dipa) {
  __shared__ float red[256];
  const long long n1 = dw1 ? (long long)C * K1 : 0, n2 = dw2 ? (long long)C * K2 : 0, nb = db ? C : 0,
                  ne = demb ? (long long)E * C : 0, ni = dipa ? (long long)B * L * C : 0;
  long long e = (long long)blockIdx.x * 64 + (threadIdx.x & 63);
  const bool wave0 = threadIdx.x < 64;
  // (block-uniform segment: the segment sizes are multiples of 64 when C is, and every block
  // starts a fresh segment range because the launch rounds each segment up to 64 outputs)
  const long long s1 = (n1 + 63) / 64 * 64, s2 = (n2 + 63) / 64 * 64, sb = (nb + 63) / 64 * 64,
                  se = (ne + 63) / 64 * 64;
  if (e < s1) {  // dw1[c][k] from the [chunk][k][C] partials; outputs in partial order (c fastest)
    const bool ok = e < n1;
    const int k = ok ? (int)(e / C) : 0, c = ok ? (int)(e % C) : 0;
    const float v = zsum4(ws + pl.p1 + (size_t)k * C + c, (size_t)K1 * C, 0, pl.chunks, red);
    if (wave0 && ok) dw1[(size_t)c * K1 + k] = v;
    return;
  }
  e -= s1;
  if (e < s2) {
    const bool ok = e < n2;
    const int k = ok ? (int)(e / C) : 0, c = ok ? (int)(e % C) : 0;
    const float v = zsum4(ws + pl.p2 + (size_t)k * C + c, (size_t)K2 * C, 0, pl.chunks, red);
    if (wave0 && ok) dw2[(size_t)c * K2 + k] = v;
    return;
  }
  e -= s2;
  if (e < sb) {
    const bool ok = e < nb;
    const float v = zsum4(ws + pl.pb + (ok ? e : 0), (size_t)C, 0, pl.chunks, red);
    if (wave0 && ok) db[e] = v;
    return;
  }
  e -= sb;
  if (e < se) {
    const bool ok = e < ne;
    const float v = zsum4(ws + pl.pe + (ok ? e : 0), (size_t)E * C, 0, pl.chunks, red);
    if (wave0 && ok) demb[e] = v;
    return;
  }
  e -= se;
  if (e < ni) {
    const int bb = (int)(e / ((long long)L * C)), rem = (int)(e % ((long long)L * C));
    const float v = zsum4(ws + pl.pi + rem, (size_t)L * C, bb * pl.tch, (bb + 1) * pl.tch, red);
    if (wave0) dipa[e] = v;
  }
}

// ------------------------------------------------------------------------------------------
// FinalLayer.  Row layout (C = 384): lane l owns columns 2l + 128 i (i = 0..2) as float2.
constexpr int kFC = 384, kFLat = 32, kFThreads = 256;

__device__ __forceinline__ void row_ld(const float* p, int lane, float (&v)[6]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float2 t = *reinterpret_cast<const float2*>(p + 2 * lane + 128 * i);
    v[2 * i] = t.x;
    v[2 * i + 1] = t.y;
  }
}
__device__ __forceinline__ void row_st(float* p, int lane, const float (&v)[6]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) *reinterpret_cast<float2*>(p + 2 * lane + 128 * i) = make_float2(v[2 * i], v[2 * i + 1]);
}
__device__ __forceinline__ int col_of(int lane, int e) { return 2 * lane + 128 * (e >> 1) + (e & 1); }

// sum over the 64 lanes of 32 per-lane values; lane l ends with the total of output
// j = bits 5..1 of l (lane bit 0 unused: both lanes of a pair hold it)
__device__ __forceinline__ float transpose_sum32(float (&p)[kFLat], int lane) {
#pragma unroll
  for (int step = 0; step < 5; ++step) {
    const int half = 16 >> step, bit = 32 >> step;  // values 2*half -> half; lane bit `bit`
    const bool hi = lane & bit;
#pragma unroll
    for (int j = 0; j < half; ++j) {
      const float keep = hi ? p[j + half] : p[j], give = hi ? p[j] : p[j + half];
      p[j] = keep + __shfl_xor(give, bit, 64);
    }
  }
  return p[0] + __shfl_xor(p[0], 1, 64);
}
__device__ __forceinline__ int transpose_sum_index(int lane) {
  return ((lane >> 5) & 1) << 4 | ((lane >> 4) & 1) << 3 | ((lane >> 3) & 1) << 2 | ((lane >> 2) & 1) << 1 |
         ((lane >> 1) & 1);
}

__device__ __forceinline__ void ln_row(const float (&x)[6], float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 6; ++e) s += x[e];
  mean = wave_sum(s) * (1.0f / kFC);
  float v = 0.f;
#pragma unroll
  for (int e = 0; e < 6; ++e) v += (x[e] - mean) * (x[e] - mean);
  rstd = rsqrtf(wave_sum(v) * (1.0f / kFC) + 1e-6f);
}

// W [LAT][C] staged in LDS and re-read per row as float2 (the compiler would otherwise keep
// all 6 x LAT values of a lane live in VGPRs and drop the kernel to one wave per SIMD); the
// next row's h is loaded while the current one computes.
template <int LAT>
__global__ __launch_bounds__(kFThreads) void final_fwd_kernel(int N, int rows_per_b, const float* __restrict__ h,
                                                              const float* __restrict__ mods,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias, float* __restrict__ v,
                                                              float* __restrict__ stats) {
  __shared__ __attribute__((aligned(16))) float ws_[LAT * kFC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < LAT * kFC; i += kFThreads) ws_[i] = w[i];
  __syncthreads();
  const int jo = transpose_sum_index(lane);
  const float bj = (jo < LAT && bias) ? bias[jo] : 0.f;
  int n = blockIdx.x * 4 + wave;
  const int stride = gridDim.x * 4;
  float xnext[6];
  if (n < N) row_ld(h + (size_t)n * kFC, lane, xnext);
  for (; n < N; n += stride) {
    asm volatile("" ::: "memory");  // W re-read from LDS each row (see above)
    float x[6], sh[6], sc[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) x[e] = xnext[e];
    if (n + stride < N) row_ld(h + (size_t)(n + stride) * kFC, lane, xnext);
    const float* mrow = mods + (size_t)(n / rows_per_b) * 2 * kFC;
    row_ld(mrow, lane, sh);
    row_ld(mrow + kFC, lane, sc);
    float mean, rstd;
    ln_row(x, mean, rstd);
    float xn[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) xn[e] = (x[e] - mean) * rstd * (1.0f + sc[e]) + sh[e];
    float p[kFLat];
#pragma unroll
    for (int j = 0; j < kFLat; ++j) {
      float s = 0.f;
      if (j < LAT) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const float2 wv = *reinterpret_cast<const float2*>(&ws_[j * kFC + 2 * lane + 128 * i]);
          s = fmaf(xn[2 * i], wv.x, s);
          s = fmaf(xn[2 * i + 1], wv.y, s);
        }
      }
      p[j] = s;
    }
    const float out = transpose_sum32(p, lane) + bj;
    if (!(lane & 1) && jo < LAT) v[(size_t)n * LAT + jo] = out;
    if (lane == 0) *reinterpret_cast<float2*>(stats + 2 * (size_t)n) = make_float2(mean, rstd);
  }
}

struct FbPlan {
  int cpb, blocks;  // row chunks per trajectory, blocks
  size_t pw, pb, pm, total;
};
constexpr int kFbRows = 128;  // rows per block (one trajectory's)

FbPlan fb_plan(int N, int rows_per_b, int lat) {
  FbPlan p{};
  const int B = N / rows_per_b;
  p.cpb = (rows_per_b + kFbRows - 1) / kFbRows;
  p.blocks = B * p.cpb;
  p.pw = 0;
  p.pb = p.pw + (size_t)p.blocks * lat * kFC;
  p.pm = p.pb + (size_t)p.blocks * kFLat;
  p.total = p.pm + (size_t)p.blocks * 2 * kFC;
  return p;
}

// LN + modulate backward (one wave per row): dh, and the block's d shift / d scale / dbias
template <int LAT>
__global__ __launch_bounds__(kFThreads) void final_bwd_kernel(int N, int rows_per_b, const float* __restrict__ h,
                                                              const float* __restrict__ stats,
                                                              const float* __restrict__ mods,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ dv, float* __restrict__ dh,
                                                              float* __restrict__ part, FbPlan pl) {
  __shared__ __attribute__((aligned(16))) float ws_[LAT * kFC];
  __shared__ float red[4][kFLat + 2 * kFC];
  __shared__ float dvs[kFbRows * LAT];  // the block's dv rows (broadcast reads; no per-row global loads)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / pl.cpb, ch = blockIdx.x % pl.cpb;
  const int r0 = b * rows_per_b + ch * kFbRows, r1 = min(b * rows_per_b + rows_per_b, r0 + kFbRows);
  for (int i = tid; i < LAT * kFC; i += kFThreads) ws_[i] = w[i];
  for (int i = tid; i < (r1 - r0) * LAT; i += kFThreads) dvs[i] = dv[(size_t)r0 * LAT + i];
  __syncthreads();
  float sh[6], sc[6];
  row_ld(mods + (size_t)b * 2 * kFC, lane, sh);
  row_ld(mods + (size_t)b * 2 * kFC + kFC, lane, sc);
  float gsh[6], gsc[6], gbl = 0.f;  // gbl: dbias of output `lane` (lanes < LAT)
#pragma unroll
  for (int e = 0; e < 6; ++e) gsh[e] = gsc[e] = 0.f;
  float xnext[6];
  int n = r0 + wave;
  if (n < r1) row_ld(h + (size_t)n * kFC, lane, xnext);
  for (; n < r1; n += 4) {
    asm volatile("" ::: "memory");  // W re-read from LDS each row
    float x[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) x[e] = xnext[e];
    if (n + 4 < r1) row_ld(h + (size_t)(n + 4) * kFC, lane, xnext);
    const float2 st = *reinterpret_cast<const float2*>(stats + 2 * (size_t)n);
    const float* dvr = dvs + (n - r0) * LAT;
    if (lane < LAT) gbl += dvr[lane];
    float d[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < LAT; ++j) {
      const float g = dvr[j];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float2 wv = *reinterpret_cast<const float2*>(&ws_[j * kFC + 2 * lane + 128 * i]);
        d[2 * i] = fmaf(g, wv.x, d[2 * i]);
        d[2 * i + 1] = fmaf(g, wv.y, d[2 * i + 1]);
      }
    }
    float xh[6], dxh[6], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      xh[e] = (x[e] - st.x) * st.y;
      gsh[e] += d[e];
      gsc[e] = fmaf(d[e], xh[e], gsc[e]);
      dxh[e] = d[e] * (1.0f + sc[e]);
      s1 += dxh[e];
      s2 += dxh[e] * xh[e];
    }
    s1 = wave_sum(s1) * (1.0f / kFC);
    s2 = wave_sum(s2) * (1.0f / kFC);
    float o[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) o[e] = st.y * (dxh[e] - s1 - xh[e] * s2);
    row_st(dh + (size_t)n * kFC, lane, o);
  }
#pragma unroll
  for (int e = 0; e < 6; ++e) {
    red[wave][col_of(lane, e)] = gsh[e];
    red[wave][kFC + col_of(lane, e)] = gsc[e];
  }
  if (lane < kFLat) red[wave][2 * kFC + lane] = lane < LAT ? gbl : 0.f;
  __syncthreads();
  for (int c = tid; c < 2 * kFC; c += kFThreads)
    part[pl.pm + (size_t)blockIdx.x * 2 * kFC + c] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
  if (tid < kFLat)
    part[pl.pb + (size_t)blockIdx.x * kFLat + tid] =
        ((red[0][2 * kFC + tid] + red[1][2 * kFC + tid]) + red[2][2 * kFC + tid]) + red[3][2 * kFC + tid];
}

// dW[j][c] = sum_n dv[n][j] xn[n][c] (xn recomputed from h and the row statistics): thread =
// column c (LAT accumulators), block = one row chunk of the backward's plan x 128 columns,
// the chunk's dv rows staged in LDS (broadcast reads); partial [block][j][C]
template <int LAT>
__global__ __launch_bounds__(128) void final_dw_kernel(int N, int rows_per_b, const float* __restrict__ h,
                                                       const float* __restrict__ stats,
                                                       const float* __restrict__ mods, const float* __restrict__ dv,
                                                       float* __restrict__ part, FbPlan pl) {
  constexpr int LP = (LAT + 3) & ~3;
  __shared__ __attribute__((aligned(16))) float ds[kFbRows][LP];
  __shared__ float2 sts[kFbRows];
  const int tid = threadIdx.x, c = blockIdx.y * 128 + tid;
  const int b = blockIdx.x / pl.cpb, ch = blockIdx.x % pl.cpb;
  const int r0 = b * rows_per_b + ch * kFbRows, nr = min(rows_per_b - ch * kFbRows, kFbRows);
  for (int i = tid; i < nr * LP; i += 128) {
    const int r = i / LP, j = i % LP;
    ds[r][j] = j < LAT ? dv[(size_t)(r0 + r) * LAT + j] : 0.f;
  }
  for (int r = tid; r < nr; r += 128) sts[r] = *reinterpret_cast<const float2*>(stats + 2 * (size_t)(r0 + r));
  __syncthreads();
  const float sh = mods[(size_t)b * 2 * kFC + c], sc1 = 1.0f + mods[(size_t)b * 2 * kFC + kFC + c];
  float acc[LP];
#pragma unroll
  for (int j = 0; j < LP; ++j) acc[j] = 0.f;
#pragma unroll 4
  for (int r = 0; r < nr; ++r) {
    const float2 st = sts[r];
    const float xn = (h[(size_t)(r0 + r) * kFC + c] - st.x) * st.y * sc1 + sh;
#pragma unroll
    for (int j4 = 0; j4 < LP; j4 += 4) {
      const float4 g = *reinterpret_cast<const float4*>(&ds[r][j4]);
      acc[j4] = fmaf(g.x, xn, acc[j4]);
      acc[j4 + 1] = fmaf(g.y, xn, acc[j4 + 1]);
      acc[j4 + 2] = fmaf(g.z, xn, acc[j4 + 2]);
      acc[j4 + 3] = fmaf(g.w, xn, acc[j4 + 3]);
    }
  }
  float* P = part + pl.pw + (size_t)blockIdx.x * LAT * kFC + c;
#pragma unroll
  for (int j = 0; j < LAT; ++j) P[(size_t)j * kFC] = acc[j];
}

__global__ __launch_bounds__(256) void final_bwd_reduce_kernel(int B, int lat, const float* __restrict__ part,
                                                               FbPlan pl, float* __restrict__ dw,
                                                               float* __restrict__ dbias, float* __restrict__ dmods) {
  __shared__ float red[256];
  const long long nw = (long long)lat * kFC, nm = (long long)B * 2 * kFC;
  const long long sw = (nw + 63) / 64 * 64, sbb = 64;
  long long e = (long long)blockIdx.x * 64 + (threadIdx.x & 63);
  const bool wave0 = threadIdx.x < 64;
  if (e < sw) {
    const bool ok = e < nw;
    const float v = zsum4(part + pl.pw + (ok ? e : 0), (size_t)nw, 0, pl.blocks, red);
    if (wave0 && ok) dw[e] = v;
    return;
  }
  e -= sw;
  if (e < sbb) {
    const bool ok = e < lat;
    const float v = zsum4(part + pl.pb + (ok ? e : 0), (size_t)kFLat, 0, pl.blocks, red);
    if (wave0 && ok && dbias) dbias[e] = v;
    return;
  }
  e -= sbb;
  if (e < nm) {
    const int bb = (int)(e / (2 * kFC)), c = (int)(e % (2 * kFC));
    const float v = zsum4(part + pl.pm + c, (size_t)2 * kFC, bb * pl.cpb, (bb + 1) * pl.cpb, red);
    if (wave0) dmods[e] = v;
  }
}

}  // namespace

size_t embed_bwd_ws_bytes(int B, int T, int L, int C, int K1, int K2, int E) {
  return eb_plan(B, T, L, C, K1, K2, E).total * sizeof(float) + 256;
}

hipError_t embed_bwd_launch(int B, int T, int L, int C, int K1, const float* x1, int K2, const float* x2,
                            const int64_t* idx, int E, const float* dh, float* dw1, float* dw2, float* db, float* demb,
                            float* dipa, float* ws, hipStream_t s) {
  const EbPlan pl = eb_plan(B, T, L, C, K1, x2 ? K2 : 0, E);
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(pl.chunks, (C + 127) / 128), dim3(256), 0, s, B, T, L, C, K1, x1,
                     x2 ? K2 : 0, x2, idx, E, dh, ws, pl);
  if (hipError_t e = hipGetLastError()) return e;
  auto r64 = [](long long v) { return (v + 63) / 64 * 64; };
  const long long n = r64(dw1 ? (long long)C * K1 : 0) + r64(dw2 && x2 ? (long long)C * K2 : 0) + r64(db ? C : 0) +
                      r64(demb && idx ? (long long)E * C : 0) + (dipa ? (long long)B * L * C : 0);
  hipLaunchKernelGGL(embed_bwd_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, B, L, C, K1,
                     x2 ? K2 : 0, E, ws, pl, dw1, x2 ? dw2 : nullptr, db, idx ? demb : nullptr, dipa);
  return hipGetLastError();
}

hipError_t final_fwd_train_launch(int N, int rows_per_b, int lat, const float* h, const float* mods, const float* w,
                                  const float* bias, float* v, float* stats, hipStream_t s) {
  // W (LAT x 384 fp32) is staged per block: enough rows per block to amortise it (~16 per wave)
  const int grid = min((N + 3) / 4, 512);
  if (lat == 21)
    hipLaunchKernelGGL(final_fwd_kernel<21>, dim3(grid), dim3(kFThreads), 0, s, N, rows_per_b, h, mods, w, bias, v, stats);
  else if (lat == 28)
    hipLaunchKernelGGL(final_fwd_kernel<28>, dim3(grid), dim3(kFThreads), 0, s, N, rows_per_b, h, mods, w, bias, v, stats);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

size_t final_bwd_ws_bytes(int N, int rows_per_b, int lat) { return fb_plan(N, rows_per_b, lat).total * sizeof(float) + 256; }

hipError_t final_bwd_train_launch(int N, int rows_per_b, int lat, const float* h, const float* stats, const float* mods,
                                  const float* w, const float* dv, float* dh, float* dw, float* dbias, float* dmods,
                                  float* ws, hipStream_t s) {
  const FbPlan pl = fb_plan(N, rows_per_b, lat);
#define MDG_FB(LAT_)                                                                                                  \
  hipLaunchKernelGGL(final_bwd_kernel<LAT_>, dim3(pl.blocks), dim3(kFThreads), 0, s, N, rows_per_b, h, stats, mods, w, \
                     dv, dh, ws, pl);                                                                                 \
  hipLaunchKernelGGL(final_dw_kernel<LAT_>, dim3(pl.blocks, kFC / 128), dim3(128), 0, s, N, rows_per_b, h, stats, mods, \
                     dv, ws, pl)
  if (lat == 21) {
    MDG_FB(21);
  } else if (lat == 28) {
    MDG_FB(28);
  } else {
    return hipErrorInvalidValue;
  }
#undef MDG_FB
  if (hipError_t e = hipGetLastError()) return e;
  const int B = N / rows_per_b;
  const long long n = ((long long)lat * kFC + 63) / 64 * 64 + 64 + (long long)B * 2 * kFC;
  hipLaunchKernelGGL(final_bwd_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, B, lat, ws, pl, dw,
                     dbias, dmods);
  return hipGetLastError();
}

}  // namespace mdg
