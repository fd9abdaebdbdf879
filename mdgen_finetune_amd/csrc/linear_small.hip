// Few-row fp32 linears of the training step's conditioning, forward and backward, on library
// kernels instead of hipBLASLt GEMMs plus eager concatenations, splits and activations.
// Reference call sites (all under loss.backward(), transport.py:137-222):
//   * TimestepEmbedder.mlp (layers.py:17-55): Linear(256, C) -> SiLU -> Linear(C, C) on B rows;
//   * every adaLN_modulation (SiLU -> Linear) of the model (latent_model.py:341-493, the 6C / 9C
//     rows of the IPA layers and blocks and FinalLayer's 2C, layers.py:58-75) on the same B rows
//     of c: one launch over ALL of them (77C = 29 568 weight rows) without concatenating the
//     weights or splitting the output;
//   * the IPA projections linear_q | linear_kv | linear_q_points | linear_kv_points (ipa.py:92-
//     140) on the B*L residue tokens (one launch for the four), and linear_out (ipa.py:250).
//
// A "segmented" linear: nseg nn.Linear layers that share the input x [M][K] (optionally
// x' = SiLU(x)), each with its own weight [n_i][K], bias, output [M][ldy_i] and, backward,
// dy [M][lddy_i], dW [n_i][K], db [n_i].  The segments form one virtual weight of sum n_i rows;
// tiles map their rows to segments.
//
// Every product is one tile routine, C[r][c] = sum_j A(r, j) B(j, c) over 32 x 64 tiles, j in
// steps of 32 staged through LDS, 256 threads x (2 rows x 4 columns), exact fp32 FMAs in
// ascending j:
//   forward   r = m, c = n, j = k:  y[m][n]   = b[n] + sum_k x'[m][k] W[n][k]
//   dW        r = n, c = k, j = m:  dW[n][k]  = sum_m dy[m][n] x'[m][k]     (+ db[n] = sum_m dy[m][n])
//   dX part   r = m, c = k, j = n:  P[ch][m][k] = sum_{n in chunk ch} dy[m][n] W[n][k]
// and a reduce launch sums the dX partials in chunk order (deterministic) times SiLU'(x).
#include "../../include/mdgen_hip.h"
#include "common.h"

#include <algorithm>

namespace mdg {
namespace {

constexpr int kSlMaxM = 32;   // token rows per block (grid.y covers more)
constexpr int kSlMaxK = 1024;  // input width (32 x' rows staged in LDS: 128 KiB)
constexpr int kSlChunk = 128;  // dX: weight rows per block (row groups of it give the partials)

struct SegMap {
  int nseg, total;
  int start[MDG_SEG_MAX + 1];
};

// Segment of weight row n and per-segment fields picked by it.  The kernel-argument arrays are
// only ever read at constant indices (scalar loads into SGPRs): the segment count is a sum of
// compares and a pick is a select chain, where a per-lane dynamic index would turn every lookup
// into a chain of dependent vector loads from the argument segment.
__device__ __forceinline__ int seg_of(const SegMap& sm, int n) {
  int s = 0;
#pragma unroll
  for (int i = 1; i < MDG_SEG_MAX; ++i) s += (i < sm.nseg && n >= sm.start[i]) ? 1 : 0;
  return s;
}
template <class T, int N>
__device__ __forceinline__ T pk(const T (&arr)[N], int s) {
  T v = arr[0];
#pragma unroll
  for (int i = 1; i < MDG_SEG_MAX; ++i)
    if (s == i) v = arr[i];
  return v;
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float dsilu_f(float x) {
  const float s = 1.0f / (1.0f + expf(-x));
  return s * (1.0f + x * (1.0f - s));
}

// x' rows [m0, m0 + mc) of the block -> LDS [mc][K] (SiLU applied), float4 per thread step
__device__ __forceinline__ void sl_stage_x(float* xs, const float* x, int ldx, int m0, int mc, int K, int act) {
  const int k4 = K >> 2;
  #pragma unroll 4  // (four global loads in flight before their LDS stores)
  for (int e = threadIdx.x; e < mc * k4; e += blockDim.x) {
    const int m = e / k4, c = (e - m * k4) * 4;
    float4 v = *reinterpret_cast<const float4*>(x + (size_t)(m0 + m) * ldx + c);
    if (act == MDG_ACT_SILU) v = make_float4(silu_f(v.x), silu_f(v.y), silu_f(v.z), silu_f(v.w));
    *reinterpret_cast<float4*>(xs + m * K + c) = v;
  }
}

struct SlFwdArgs {
  int M, K, ldx, act;
  const float* x;
  SegMap sm;
  const float* w[MDG_SEG_MAX];
  const float* b[MDG_SEG_MAX];
  float* y[MDG_SEG_MAX];
  int ldy[MDG_SEG_MAX];
  const float* resid[MDG_SEG_MAX];
  int ldr[MDG_SEG_MAX];
};

// Forward.  Block = 64 weight rows (n) x up to 32 token rows; wave w owns rows n0 + 16w + (lane &
// 15), lane >> 4 picks a quarter of every 16-wide k chunk: each lane streams float4 pieces of
// ITS weight row (4 lanes cover 64 contiguous bytes) against the x' rows in LDS (same address
// within a 16-lane group: broadcast), 32 accumulators; the k quarters are summed by two lane
// swaps at the end.
//
// KS = 4 (few-row linears, too few 64-row blocks to fill the chip): 16 weight rows per block and
// the four waves interleave over k as well; their sums are added in wave order through LDS.
template <int MT, int KS>
__global__ __launch_bounds__(256) void sl_fwd_kernel(const SlFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float xs[];  // [MT][K]
  __shared__ float red[KS == 4 ? 3 * 16 * (MT + 1) : 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nl = lane & 15, kq = lane >> 4;
  const int m0 = blockIdx.y * MT, mc = min(MT, a.M - m0);
  sl_stage_x(xs, a.x, a.ldx, m0, mc, a.K, a.act);
  const int n = KS == 1 ? blockIdx.x * 64 + 16 * wave + nl : blockIdx.x * 16 + nl;
  const bool live = n < a.sm.total;
  const int s = live ? seg_of(a.sm, n) : 0, nr = live ? n - pk(a.sm.start, s) : 0;
  const float* wr = pk(a.w, s) + (size_t)nr * a.K;
  // the first weight piece is requested before the x' staging barrier, and each next one while
  // the current one is used (one exposed load latency per row instead of one per k step)
  const int kstep = 16 * KS, k0 = 4 * kq + (KS == 1 ? 0 : 16 * wave);
  float4 wn = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live && k0 < a.K) wn = *reinterpret_cast<const float4*>(wr + k0);
  __syncthreads();
  float acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = 0.f;
  if (live) {
    for (int k = k0; k < a.K; k += kstep) {
      const float4 w4 = wn;
      if (k + kstep < a.K) wn = *reinterpret_cast<const float4*>(wr + k + kstep);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if (m < mc) {
          const float4 x4 = *reinterpret_cast<const float4*>(xs + m * a.K + k);
          acc[m] = fmaf(x4.x, w4.x, acc[m]);
          acc[m] = fmaf(x4.y, w4.y, acc[m]);
          acc[m] = fmaf(x4.z, w4.z, acc[m]);
          acc[m] = fmaf(x4.w, w4.w, acc[m]);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    acc[m] += __shfl_xor(acc[m], 16, 64);
    acc[m] += __shfl_xor(acc[m], 32, 64);
  }
  if constexpr (KS == 4) {
    if (wave > 0 && kq == 0)
#pragma unroll
      for (int m = 0; m < MT; ++m) red[((wave - 1) * 16 + nl) * (MT + 1) + m] = acc[m];
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int m = 0; m < MT; ++m)
      acc[m] = ((acc[m] + red[nl * (MT + 1) + m]) + red[(16 + nl) * (MT + 1) + m]) + red[(32 + nl) * (MT + 1) + m];
  }
  if (!live || kq != 0) return;
  const float bias = pk(a.b, s) ? pk(a.b, s)[nr] : 0.f;
  float* yr = pk(a.y, s) + nr;
  const float* rr = pk(a.resid, s) ? pk(a.resid, s) + nr : nullptr;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if (m < mc) {
      float v = acc[m] + bias;
      if (rr) v = rr[(size_t)(m0 + m) * pk(a.ldr, s)] + v;
      yr[(size_t)(m0 + m) * pk(a.ldy, s)] = v;
    }
  }
}

struct SlBwdArgs {
  int M, K, ldx, act;
  const float* x;
  SegMap sm;
  const float* w[MDG_SEG_MAX];
  const float* dy[MDG_SEG_MAX];
  int lddy[MDG_SEG_MAX];
  float* dw[MDG_SEG_MAX];
  float* db[MDG_SEG_MAX];
  int n_dw_blocks;  // blocks [0, n_dw_blocks): 64 weight rows of dW / db each; the rest: dX chunks
  int chunks, chunk;  // dX: blocks, weight rows per block (<= kSlChunk)
  float* part;  // [chunks][M][K]
};

// Backward, two block roles in one launch (tokens in chunks of 32):
//   dW block: 64 weight rows x 32 float4 columns (one column pass of the row block); thread
//     (column tk = t & 31, row group tn = t >> 5) owns rows tn + 8 j; per token m one dy
//     broadcast from LDS and one x' float4 from LDS: dW[n][k] = sum_m dy[m][n] x'[m][k], db[n] =
//     sum_m dy[m][n] (column pass 0; m ascending, exact fp32 FMAs).
//   dX block: a chunk of weight rows; thread = (float4 column group, row group), register
//     accumulators for every token; per weight row one coalesced float4 of W and the M dy
//     values from LDS: P[chunk, group][m][k] = sum_{n in the group's rows} dy[m][n] W[n][k].
// Row pointers come from per-block LDS tables built once (see rrow_ / rdy_).
template <int MT>  // dX token chunk (8 for M <= 8, else 32)
__global__ __launch_bounds__(256) void sl_bwd_kernel(const SlBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm_[];
  // per-block row tables: segment fields copied at constant indices, then one lookup per row of
  // the block (W or dW row pointer, dy column pointer and stride, db pointer)
  __shared__ int st_[MDG_SEG_MAX + 1], ld_[MDG_SEG_MAX];
  __shared__ const float* sw_[MDG_SEG_MAX];
  __shared__ const float* sdy_[MDG_SEG_MAX];
  __shared__ float* sdw_[MDG_SEG_MAX];
  __shared__ float* sdb_[MDG_SEG_MAX];
  __shared__ const float* rrow_[kSlChunk];  // dX: W row; dW: dW row (nullptr: no row / no dW)
  __shared__ const float* rdy_[kSlChunk];   // dy column of the row (nullptr: no row)
  __shared__ int rld_[kSlChunk];
  __shared__ float* rdb_[64];
  const int t = threadIdx.x;
  const bool dwrole = (int)blockIdx.x < a.n_dw_blocks;
  if (t == 0) {
#pragma unroll
    for (int i = 0; i < MDG_SEG_MAX; ++i) {
      st_[i] = a.sm.start[i];
      ld_[i] = a.lddy[i];
      sw_[i] = a.w[i];
      sdy_[i] = a.dy[i];
      sdw_[i] = a.dw[i];
      sdb_[i] = a.db[i];
    }
    st_[MDG_SEG_MAX] = a.sm.start[MDG_SEG_MAX];
  }
  __syncthreads();
  {
    const int base = dwrole ? (int)blockIdx.x / ((a.K / 4 + 31) / 32) * 64 : (blockIdx.x - a.n_dw_blocks) * a.chunk;
    const int rows = dwrole ? 64 : a.chunk;
    if (t < rows) {
      const int n = base + t;
      const bool live = n < a.sm.total;
      int sg = 0;
#pragma unroll
      for (int i = 1; i < MDG_SEG_MAX; ++i) sg += (i < a.sm.nseg && n >= st_[i]) ? 1 : 0;
      const int nr = n - st_[sg];
      rdy_[t] = live ? sdy_[sg] + nr : nullptr;
      rld_[t] = ld_[sg];
      if (dwrole) {
        rrow_[t] = live && sdw_[sg] ? sdw_[sg] + (size_t)nr * a.K : nullptr;
        rdb_[t] = live && sdb_[sg] ? sdb_[sg] + nr : nullptr;
      } else {
        rrow_[t] = live ? sw_[sg] + (size_t)nr * a.K : nullptr;
      }
    }
  }
  __syncthreads();
  if (dwrole) {
    // 64 weight rows x 32 float4 columns (column pass cp of the row block); the token chunk's x'
    // slice [32][32 float4] and dy tile [32][64] are staged in LDS
    float4* xs = reinterpret_cast<float4*>(sm_);  // [32][32]
    float* dys = sm_ + kSlMaxM * 32 * 4;          // [32][64]
    const int ncp = (a.K / 4 + 31) / 32, cp = blockIdx.x % ncp;
    const int tk = t & 31, tn = t >> 5, c = cp * 32 + tk;
    const bool col_ok = c < a.K / 4;
    float dbacc = 0.f;  // cp == 0, thread t < 64: db of the block's weight row t
    float4 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int mb = 0; mb < a.M; mb += kSlMaxM) {  // token chunks, m ascending overall
      const int mc = min(kSlMaxM, a.M - mb);
      __syncthreads();
      #pragma unroll 4  // (four global loads in flight before their LDS stores)
      for (int e = t; e < mc * 32; e += 256) {
        const int m = e >> 5, cc = cp * 32 + (e & 31);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (cc < a.K / 4) {
          v = *reinterpret_cast<const float4*>(a.x + (size_t)(mb + m) * a.ldx + 4 * cc);
          if (a.act == MDG_ACT_SILU) v = make_float4(silu_f(v.x), silu_f(v.y), silu_f(v.z), silu_f(v.w));
        }
        xs[e] = v;
      }
      #pragma unroll 4  // (four global loads in flight before their LDS stores)
      for (int e = t; e < mc * 64; e += 256) {
        const int m = e >> 6, cc = e & 63;
        const float* col = rdy_[cc];
        dys[m * 64 + cc] = col ? col[(size_t)(mb + m) * rld_[cc]] : 0.f;
      }
      __syncthreads();
      if (cp == 0 && t < 64)
        for (int m = 0; m < mc; ++m) dbacc += dys[m * 64 + t];
      for (int m = 0; m < mc; ++m) {
        const float4 xv = xs[m * 32 + tk];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = dys[m * 64 + tn + 8 * j];
          acc[j].x = fmaf(d, xv.x, acc[j].x);
          acc[j].y = fmaf(d, xv.y, acc[j].y);
          acc[j].z = fmaf(d, xv.z, acc[j].z);
          acc[j].w = fmaf(d, xv.w, acc[j].w);
        }
      }
    }
    if (col_ok) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float* dwr = const_cast<float*>(rrow_[tn + 8 * j]);
        if (dwr) *reinterpret_cast<float4*>(dwr + 4 * c) = acc[j];
      }
    }
    if (cp == 0 && t < 64 && rdb_[t]) *rdb_[t] = dbacc;  // db, m ascending
    return;
  }
  // dX partial of one chunk of kSlChunk weight rows, token chunks of 32: thread = (float4 column
  // group cg, row group rg); row group rg takes rows rg, rg + RG, ... of the chunk, four at a time
  // with their weight loads issued together (row pointers computed per row, no loop-carried
  // address), and writes its own partial P[chunk * RG + rg][m][k] (the reduce sums them in order)
  const int ch = blockIdx.x - a.n_dw_blocks;
  const int j0 = ch * a.chunk, nc = min(a.chunk, a.sm.total - j0);
  float* dys = sm_;  // [kSlChunk][32]
  const int k4 = a.K >> 2, RG = 256 / k4, cg = t % k4, rg = t / k4;
  const bool act_t = rg < RG;
  float* P = a.part + (size_t)(ch * RG + (act_t ? rg : 0)) * a.M * a.K;
  auto wrow = [&](int jj) { return reinterpret_cast<const float4*>(rrow_[jj]) + cg; };
  for (int mb = 0; mb < a.M; mb += MT) {
    const int mc = min(MT, a.M - mb);
    __syncthreads();
    #pragma unroll 4  // (four global loads in flight before their LDS stores)
    for (int e = t; e < nc * mc; e += 256) {
      const int jj = e / mc, m = e - jj * mc;
      dys[jj * MT + m] = rdy_[jj][(size_t)(mb + m) * rld_[jj]];
    }
    __syncthreads();
    if (!act_t) continue;
    float4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = make_float4(0.f, 0.f, 0.f, 0.f);
    auto use = [&](int jj, const float4 w4) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if (m < mc) {
          const float d = dys[jj * MT + m];
          acc[m].x = fmaf(d, w4.x, acc[m].x);
          acc[m].y = fmaf(d, w4.y, acc[m].y);
          acc[m].z = fmaf(d, w4.z, acc[m].z);
          acc[m].w = fmaf(d, w4.w, acc[m].w);
        }
      }
    };
    int jj = rg;
    for (; jj + 3 * RG < nc; jj += 4 * RG) {
      const float4 w0 = *wrow(jj), w1 = *wrow(jj + RG), w2 = *wrow(jj + 2 * RG), w3 = *wrow(jj + 3 * RG);
      use(jj, w0);
      use(jj + RG, w1);
      use(jj + 2 * RG, w2);
      use(jj + 3 * RG, w3);
    }
    for (; jj < nc; jj += RG) use(jj, *wrow(jj));
#pragma unroll
    for (int m = 0; m < MT; ++m)
      if (m < mc) *reinterpret_cast<float4*>(P + (size_t)(mb + m) * a.K + 4 * cg) = acc[m];
  }
}

// dx[m][k] = (sum over the Z partials, in a fixed order) * SiLU'(x) (act SILU) or as is; 64
// outputs per block, the four waves take a quarter of the partials each and wave 0 adds the four
__global__ __launch_bounds__(256) void sl_dx_reduce_kernel(int M, int K, int Z, const float* __restrict__ part,
                                                           const float* __restrict__ x, int ldx, int act,
                                                           float* __restrict__ dx, int lddx) {
  __shared__ float red[256];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  const bool ok = e < M * K;
  const size_t zs = (size_t)M * K;
  const int za = q * Z / 4, zb = (q + 1) * Z / 4;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (ok) {
    const float* p = part + e;
    int z = za;
    for (; z + 4 <= zb; z += 4) {
      s0 += p[(size_t)z * zs];
      s1 += p[(size_t)(z + 1) * zs];
      s2 += p[(size_t)(z + 2) * zs];
      s3 += p[(size_t)(z + 3) * zs];
    }
    for (; z < zb; ++z) s0 += p[(size_t)z * zs];
  }
  red[threadIdx.x] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (q != 0 || !ok) return;
  float s = ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
  const int m = e / K, k = e - m * K;
  if (act == MDG_ACT_SILU) s *= dsilu_f(x[(size_t)m * ldx + k]);
  dx[(size_t)m * lddx + k] = s;
}

}  // namespace

namespace {
bool seg_map(const mdg_seg_linear* s, SegMap& sm) {
  if (!s || s->nseg < 1 || s->nseg > MDG_SEG_MAX) return false;
  sm.nseg = s->nseg;
  int tot = 0;
  for (int i = 0; i < s->nseg; ++i) {
    if (s->n[i] <= 0) return false;
    sm.start[i] = tot;
    tot += s->n[i];
  }
  for (int i = s->nseg; i <= MDG_SEG_MAX; ++i) sm.start[i] = tot;
  sm.total = tot;
  return true;
}
}  // namespace

int seg_total(const mdg_seg_linear* s) {
  SegMap sm;
  return seg_map(s, sm) ? sm.total : -1;
}

static int sl_row_groups(int K) { return 256 / (K >> 2); }
// dX rows per block: kSlChunk when that still gives >= 128 blocks, else 32 (few-row linears)
static int sl_chunk(int total) { return total >= 128 * kSlChunk ? kSlChunk : 32; }

size_t seg_linear_ws_bytes(int M, int K, int total) {
  const int chunks = (total + sl_chunk(total) - 1) / sl_chunk(total);
  return (size_t)chunks * sl_row_groups(K) * M * K * sizeof(float);
}

bool seg_linear_shape_ok(int M, int K) { return M > 0 && K > 0 && K % 4 == 0 && K <= kSlMaxK; }

hipError_t seg_linear_fwd_launch(int M, int K, const float* x, int ldx, int act, const mdg_seg_linear* s,
                                 hipStream_t st) {
  SegMap sm;
  if (!seg_map(s, sm)) return hipErrorInvalidValue;
  SlFwdArgs a{};
  a.M = M, a.K = K, a.ldx = ldx, a.act = act, a.x = x, a.sm = sm;
  for (int i = 0; i < sm.nseg; ++i) {
    a.w[i] = s->w[i], a.b[i] = s->b[i], a.y[i] = s->y[i], a.ldy[i] = s->ldy[i];
    a.resid[i] = s->resid[i], a.ldr[i] = s->ldr[i];
  }
  // 64 weight rows per block, or 16 with the waves splitting K when that leaves < 256 blocks
  const bool ks = (sm.total + 63) / 64 * ((M + kSlMaxM - 1) / kSlMaxM) < 256;
  const unsigned nx = (unsigned)(ks ? (sm.total + 15) / 16 : (sm.total + 63) / 64);
  if (M <= 8) {
    const size_t smem = (size_t)8 * K * sizeof(float);
    if (ks)
      hipLaunchKernelGGL((sl_fwd_kernel<8, 4>), dim3(nx, 1), dim3(256), smem, st, a);
    else
      hipLaunchKernelGGL((sl_fwd_kernel<8, 1>), dim3(nx, 1), dim3(256), smem, st, a);
  } else {
    const size_t smem = (size_t)kSlMaxM * K * sizeof(float);
    static bool attr = false;
    if (!attr) {
      for (const void* f : {reinterpret_cast<const void*>(&sl_fwd_kernel<kSlMaxM, 1>),
                            reinterpret_cast<const void*>(&sl_fwd_kernel<kSlMaxM, 4>)}) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kSlMaxM * kSlMaxK * 4);
        if (e != hipSuccess) return e;
      }
      attr = true;
    }
    const dim3 grid(nx, (M + kSlMaxM - 1) / kSlMaxM);
    if (ks)
      hipLaunchKernelGGL((sl_fwd_kernel<kSlMaxM, 4>), grid, dim3(256), smem, st, a);
    else
      hipLaunchKernelGGL((sl_fwd_kernel<kSlMaxM, 1>), grid, dim3(256), smem, st, a);
  }
  return hipGetLastError();
}

hipError_t seg_linear_bwd_launch(int M, int K, const float* x, int ldx, int act, const mdg_seg_linear* s, float* dx,
                                 int lddx, float* ws, hipStream_t st) {
  SegMap sm;
  if (!seg_map(s, sm)) return hipErrorInvalidValue;
  SlBwdArgs a{};
  a.M = M, a.K = K, a.ldx = ldx, a.act = act, a.x = x, a.sm = sm;
  bool any_w = false;
  for (int i = 0; i < sm.nseg; ++i) {
    a.w[i] = s->w[i], a.dy[i] = s->dy[i], a.lddy[i] = s->lddy[i], a.dw[i] = s->dw[i], a.db[i] = s->db[i];
    any_w = any_w || s->dw[i] || s->db[i];
  }
  a.chunk = sl_chunk(sm.total);
  a.chunks = dx ? (sm.total + a.chunk - 1) / a.chunk : 0;
  a.n_dw_blocks = any_w ? (sm.total + 63) / 64 * ((K / 4 + 31) / 32) : 0;
  a.part = ws;
  const size_t smem = std::max((size_t)(kSlMaxM * 32 * 4 + kSlMaxM * 64) * 4, (size_t)kSlChunk * kSlMaxM * 4);
  const int nblk = a.n_dw_blocks + a.chunks;
  if (nblk > 0) {
    if (M <= 8)
      hipLaunchKernelGGL(sl_bwd_kernel<8>, dim3(nblk), dim3(256), smem, st, a);
    else
      hipLaunchKernelGGL(sl_bwd_kernel<kSlMaxM>, dim3(nblk), dim3(256), smem, st, a);
  }
  if (dx)
    hipLaunchKernelGGL(sl_dx_reduce_kernel, dim3((M * K + 63) / 64), dim3(256), 0, st, M, K, a.chunks * sl_row_groups(K),
                       (const float*)ws, x, ldx, act, dx, lddx);
  return hipGetLastError();
}

}  // namespace mdg
