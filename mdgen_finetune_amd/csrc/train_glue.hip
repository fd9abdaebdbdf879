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
//  * final_fwd: 64 rows per block, W in LDS: LN statistics as two wave reductions (6 columns
//    per lane) and the modulate into LDS, then one thread per (row, output group) for the 21
//    output dots (W reads are LDS broadcasts); writes v and (mean, rstd).
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
  // the chunk's x1 and x2 rows, zero-padded to kEbK columns: [2][kEbFrames L][kEbK] (dynamic:
  // 32 KiB at L = 4, four blocks per CU)
  extern __shared__ __attribute__((aligned(16))) float xs_[];
  const int chunk = blockIdx.x, b = chunk / pl.tch, tc = chunk % pl.tch;
  const int t0 = tc * kEbFrames, nf = min(kEbFrames, T - t0), ntok = nf * L;
  float (*xs0)[kEbK] = reinterpret_cast<float (*)[kEbK]>(xs_);
  float (*xs1)[kEbK] = reinterpret_cast<float (*)[kEbK]>(xs_ + (size_t)kEbFrames * L * kEbK);
  const size_t n0 = ((size_t)b * T + t0) * L;
  const int tid = threadIdx.x, op = tid >> 7, c = blockIdx.y * 128 + (tid & 127);
  const int K = op ? K2 : K1;
#pragma unroll 4  // (global loads in flight before their LDS stores)
  for (int i = tid; i < ntok * kEbK; i += 256) {
    const int r = i / kEbK, k = i % kEbK;
    xs0[r][k] = k < K1 ? x1[(n0 + r) * K1 + k] : 0.f;
    xs1[r][k] = (x2 && k < K2) ? x2[(n0 + r) * K2 + k] : 0.f;
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
  const float (*X)[kEbK] = op ? xs1 : xs0;
  const float* dcol = dh + n0 * C + c;
  auto row = [&](int r, float g, int e) {
    const int l = r % L;
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
      for (int q = 0; q < kEbEMax; ++q) esum[q] += (q == e) ? g : 0.f;
    }
  };
  // rows in groups of 8 whose dh (and mask index) loads are issued before any of them is used:
  // one dependent HBM round trip per group instead of per row
  constexpr int G = 8;
  int rr = 0;
  for (; rr + G <= ntok; rr += G) {
    float g[G];
    int e[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      g[j] = dcol[(size_t)(rr + j) * C];
      e[j] = (op && idx) ? (int)idx[n0 + rr + j] : -1;
    }
#pragma unroll
    for (int j = 0; j < G; ++j) row(rr + j, g[j], e[j]);
  }
  for (; rr < ntok; ++rr) row(rr, dcol[(size_t)rr * C], (op && idx) ? (int)idx[n0 + rr] : -1);
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

// 64 rows per block, W [LAT][C] staged in LDS once per block.  Phase 1: wave w LN-modulates
// rows w, w + 4, ... (eight h rows loaded together per pass) into LDS.  Phase 2: thread = (row r,
// output group g = wave) dots row r with W rows g, g + 4, ...: the W reads are wave-uniform LDS
// broadcasts (W read per thread from L2 cost 87 us a step at 32 rows per block).
constexpr int kFfRows = 64, kFfPad = kFC + 4;
template <int LAT>
constexpr size_t ff_smem() { return ((size_t)kFfRows * kFfPad + (size_t)LAT * kFC) * sizeof(float); }
template <int LAT>
__global__ __launch_bounds__(kFThreads) void final_fwd_kernel(int N, int rows_per_b, const float* __restrict__ h,
                                                              const float* __restrict__ mods,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias, float* __restrict__ v,
                                                              float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) float ff_[];
  float* xs = ff_;                      // [kFfRows][kFfPad]
  float* wsm = ff_ + kFfRows * kFfPad;  // [LAT][kFC]
  constexpr int RW = 8;                 // rows per wave per pass
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * kFfRows;
#pragma unroll 4
  for (int i = tid; i < LAT * kFC / 4; i += kFThreads)
    reinterpret_cast<float4*>(wsm)[i] = reinterpret_cast<const float4*>(w)[i];
  // the modulation rows of the block's first trajectory, reloaded only where the rows cross into
  // the next one (rows_per_b = T L >> 64: at most once per block)
  int cur_b = min(r0, N - 1) / rows_per_b;
  float sh[6], sc[6];
  row_ld(mods + (size_t)cur_b * 2 * kFC, lane, sh);
  row_ld(mods + (size_t)cur_b * 2 * kFC + kFC, lane, sc);
  for (int pass = 0; pass < kFfRows / (4 * RW); ++pass) {
    float x[RW][6];
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const int n = r0 + pass * 4 * RW + wave + 4 * i;
      if (n < N) row_ld(h + (size_t)n * kFC, lane, x[i]);
    }
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const int rr = pass * 4 * RW + wave + 4 * i, n = r0 + rr;
      if (n >= N) break;
      const int bb = n / rows_per_b;
      if (bb != cur_b) {  // (wave-uniform)
        cur_b = bb;
        row_ld(mods + (size_t)bb * 2 * kFC, lane, sh);
        row_ld(mods + (size_t)bb * 2 * kFC + kFC, lane, sc);
      }
      float mean, rstd;
      ln_row(x[i], mean, rstd);
      float xn[6];
#pragma unroll
      for (int e = 0; e < 6; ++e) xn[e] = (x[i][e] - mean) * rstd * (1.0f + sc[e]) + sh[e];
      row_st(xs + rr * kFfPad, lane, xn);
      if (lane == 0) *reinterpret_cast<float2*>(stats + 2 * (size_t)n) = make_float2(mean, rstd);
    }
  }
  __syncthreads();
  constexpr int NJ = (LAT + 3) / 4;
  const int r = tid & 63, g = wave, n = r0 + r;
  float acc[NJ];
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) acc[jj] = 0.f;
  const float4* xr = reinterpret_cast<const float4*>(xs + r * kFfPad);
  const float4* wr = reinterpret_cast<const float4*>(wsm);
#pragma unroll 4
  for (int k4 = 0; k4 < kFC / 4; ++k4) {
    const float4 xv = xr[k4];
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int j = g + 4 * jj;
      if (j < LAT) {
        const float4 wv = wr[j * (kFC / 4) + k4];
        acc[jj] = fmaf(xv.x, wv.x, acc[jj]);
        acc[jj] = fmaf(xv.y, wv.y, acc[jj]);
        acc[jj] = fmaf(xv.z, wv.z, acc[jj]);
        acc[jj] = fmaf(xv.w, wv.w, acc[jj]);
      }
    }
  }
  if (n < N) {
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int j = g + 4 * jj;
      if (j < LAT) v[(size_t)n * LAT + j] = acc[jj] + (bias ? bias[j] : 0.f);
    }
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
#pragma unroll 8
  for (int i = tid; i < LAT * kFC; i += kFThreads) ws_[i] = w[i];
#pragma unroll 4
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

// ------------------------------------------------------------------------------------------
// The flow-matching plan and loss of Transport.training_losses (transport.py:137-222, velocity
// model; path.py:81-191): one pass each instead of ~25 small eager kernels per step.
//   plan (per element of trajectory b, t = t[b]):
//     GVP:    u = (t * pi) / 2, a = sin u, s = cos u, da = (pi / 2) cos u, ds = (-pi / 2) sin u
//     Linear: a = t, s = 1 - t, da = 1, ds = -1
//     xt = a x1 + s x0, ut = da x1 + ds x0  (products rounded, then the sum: torch's order)
//   loss_b = sum (out - ut)^2 m / sum m over trajectory b's T x L x K elements (mean_flat,
//   transport.py:12-16; the mask may be a broadcast view: element strides); backward
//   d out = 2 (out - ut) m g_b / den_b.
constexpr int kGvpChunk = 8192;  // elements per partial-sum block

__global__ __launch_bounds__(256) void gvp_plan_kernel(long long npb, long long total, int path, const float* __restrict__ t,
                                                       const float* __restrict__ x0, const float* __restrict__ x1,
                                                       float* __restrict__ xt, float* __restrict__ ut) {
#pragma clang fp contract(off)
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const float tb = t[e / npb];
  const float a0 = x0[e], a1 = x1[e];
  if (path == 0) {  // GVP
    const float u = (tb * 3.14159265358979323846f) / 2.0f;
    const float sa = sinf(u), ca = cosf(u);
    const float da = 1.57079632679489661923f * ca, ds = -1.57079632679489661923f * sa;
    xt[e] = __fadd_rn(__fmul_rn(sa, a1), __fmul_rn(ca, a0));
    ut[e] = __fadd_rn(__fmul_rn(da, a1), __fmul_rn(ds, a0));
  } else {  // Linear
    xt[e] = __fadd_rn(__fmul_rn(tb, a1), __fmul_rn(1.0f - tb, a0));
    ut[e] = __fadd_rn(a1, -a0);
  }
}

struct GvpDims {
  int B, T, L, K;
  long long ms[4];  // mask element strides (b, t, l, k)
};
__device__ __forceinline__ float gvp_mask(const float* m, const GvpDims& d, long long e) {
  const int k = (int)(e % d.K);
  const long long r = e / d.K;
  const int l = (int)(r % d.L);
  const long long r2 = r / d.L;
  const int tt = (int)(r2 % d.T), b = (int)(r2 / d.T);
  return m[b * d.ms[0] + tt * d.ms[1] + l * d.ms[2] + k * d.ms[3]];
}

// partial sums of (num, den) over chunk `blockIdx.x` of trajectory blockIdx.y, block tree order
__global__ __launch_bounds__(256) void gvp_loss_part_kernel(GvpDims d, const float* __restrict__ out,
                                                            const float* __restrict__ ut, const float* __restrict__ m,
                                                            float* __restrict__ part) {
  __shared__ float rn[256], rd[256];
  const long long npb = (long long)d.T * d.L * d.K;
  const int b = blockIdx.y;
  const long long c0 = (long long)blockIdx.x * kGvpChunk, c1 = min(npb, c0 + kGvpChunk);
  float sn = 0.f, sd = 0.f;
  for (long long i = c0 + threadIdx.x; i < c1; i += 256) {
    const long long e = (long long)b * npb + i;
    const float df = out[e] - ut[e], mk = gvp_mask(m, d, e);
    sn += (df * df) * mk;
    sd += mk;
  }
  rn[threadIdx.x] = sn;
  rd[threadIdx.x] = sd;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      rn[threadIdx.x] += rn[threadIdx.x + w];
      rd[threadIdx.x] += rd[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[((size_t)b * gridDim.x + blockIdx.x) * 2] = rn[0];
    part[((size_t)b * gridDim.x + blockIdx.x) * 2 + 1] = rd[0];
  }
}

__global__ void gvp_loss_final_kernel(int B, int nch, const float* __restrict__ part, float* __restrict__ loss,
                                      float* __restrict__ den) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float sn = 0.f, sd = 0.f;
  for (int c = 0; c < nch; ++c) {
    sn += part[((size_t)b * nch + c) * 2];
    sd += part[((size_t)b * nch + c) * 2 + 1];
  }
  loss[b] = sn / sd;
  den[b] = sd;
}

__global__ __launch_bounds__(256) void gvp_loss_bwd_kernel(GvpDims d, long long total, const float* __restrict__ out,
                                                           const float* __restrict__ ut, const float* __restrict__ m,
                                                           const float* __restrict__ g, const float* __restrict__ den,
                                                           float* __restrict__ dout) {
#pragma clang fp contract(off)
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int b = (int)(e / ((long long)d.T * d.L * d.K));
  const float gb = g[b] / den[b];
  dout[e] = (gb * gvp_mask(m, d, e)) * 2.0f * (out[e] - ut[e]);
}

}  // namespace

size_t embed_bwd_ws_bytes(int B, int T, int L, int C, int K1, int K2, int E) {
  return eb_plan(B, T, L, C, K1, K2, E).total * sizeof(float) + 256;
}

hipError_t embed_bwd_launch(int B, int T, int L, int C, int K1, const float* x1, int K2, const float* x2,
                            const int64_t* idx, int E, const float* dh, float* dw1, float* dw2, float* db, float* demb,
                            float* dipa, float* ws, hipStream_t s) {
  const EbPlan pl = eb_plan(B, T, L, C, K1, x2 ? K2 : 0, E);
  const size_t smem = (size_t)2 * kEbFrames * L * kEbK * sizeof(float);
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(pl.chunks, (C + 127) / 128), dim3(256), smem, s, B, T, L, C, K1, x1,
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
  const int grid = (N + kFfRows - 1) / kFfRows;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&final_fwd_kernel<21>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)ff_smem<21>());
    if (e == hipSuccess)
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&final_fwd_kernel<28>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)ff_smem<28>());
    if (e != hipSuccess) return e;
    attr = true;
  }
  if (lat == 21)
    hipLaunchKernelGGL(final_fwd_kernel<21>, dim3(grid), dim3(kFThreads), ff_smem<21>(), s, N, rows_per_b, h, mods, w,
                       bias, v, stats);
  else if (lat == 28)
    hipLaunchKernelGGL(final_fwd_kernel<28>, dim3(grid), dim3(kFThreads), ff_smem<28>(), s, N, rows_per_b, h, mods, w,
                       bias, v, stats);
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

hipError_t gvp_plan_launch(int B, long long npb, int path, const float* t, const float* x0, const float* x1, float* xt,
                           float* ut, hipStream_t s) {
  const long long total = (long long)B * npb;
  hipLaunchKernelGGL(gvp_plan_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, npb, total, path, t, x0,
                     x1, xt, ut);
  return hipGetLastError();
}

static GvpDims gvp_dims(int B, int T, int L, int K, const int64_t* ms) {
  GvpDims d;
  d.B = B, d.T = T, d.L = L, d.K = K;
  for (int i = 0; i < 4; ++i) d.ms[i] = ms[i];
  return d;
}

size_t gvp_loss_ws_bytes(int B, long long npb) {
  const long long nch = (npb + kGvpChunk - 1) / kGvpChunk;
  return (size_t)B * nch * 2 * sizeof(float) + 256;
}

hipError_t gvp_loss_fwd_launch(int B, int T, int L, int K, const float* out, const float* ut, const float* mask,
                               const int64_t* ms, float* loss, float* den, float* ws, hipStream_t s) {
  const GvpDims d = gvp_dims(B, T, L, K, ms);
  const long long npb = (long long)T * L * K;
  const int nch = (int)((npb + kGvpChunk - 1) / kGvpChunk);
  hipLaunchKernelGGL(gvp_loss_part_kernel, dim3(nch, B), dim3(256), 0, s, d, out, ut, mask, ws);
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(gvp_loss_final_kernel, dim3((B + 63) / 64), dim3(64), 0, s, B, nch, (const float*)ws, loss, den);
  return hipGetLastError();
}

hipError_t gvp_loss_bwd_launch(int B, int T, int L, int K, const float* out, const float* ut, const float* mask,
                               const int64_t* ms, const float* g, const float* den, float* dout, hipStream_t s) {
  const GvpDims d = gvp_dims(B, T, L, K, ms);
  const long long total = (long long)B * T * L * K;
  hipLaunchKernelGGL(gvp_loss_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, d, total, out, ut,
                     mask, g, den, dout);
  return hipGetLastError();
}

}  // namespace mdg
