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

namespace mdg {
namespace {

constexpr int kSlR = 32, kSlC = 64, kSlJ = 32, kSlThreads = 256, kSlChunk = 256;  // dX: weight rows per partial

struct SegMap {
  int nseg, total;
  int start[MDG_SEG_MAX + 1];
};

__device__ __forceinline__ int seg_of(const SegMap& sm, int n) {
  int s = 0;
#pragma unroll 1
  while (s + 1 < sm.nseg && n >= sm.start[s + 1]) ++s;
  return s;
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float dsilu_f(float x) {
  const float s = 1.0f / (1.0f + expf(-x));
  return s * (1.0f + x * (1.0f - s));
}

// C tile [r0, r0 + 32) x [c0, c0 + 64) += sum_{j in [j0, j1)} A(r, j) B(j, c), accumulated in acc.
// getA(r, j) / getB(j, c) return 0 outside the operands.  A_JFAST: consecutive threads stage
// consecutive j of A (A contiguous in j) instead of consecutive r; B_JFAST likewise for B.
template <bool A_JFAST, bool B_JFAST, typename GA, typename GB>
__device__ __forceinline__ void sl_tile(float (&acc)[2][4], int r0, int c0, int j0, int j1, GA getA, GB getB,
                                        float (*As)[kSlJ + 1], float (*Bs)[kSlC + 1]) {
  const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  for (int jb = j0; jb < j1; jb += kSlJ) {
#pragma unroll
    for (int u = 0; u < kSlR * kSlJ / kSlThreads; ++u) {
      const int e = tid + u * kSlThreads;
      const int r = A_JFAST ? e / kSlJ : e % kSlR, j = A_JFAST ? e % kSlJ : e / kSlR;
      As[r][j] = jb + j < j1 ? getA(r0 + r, jb + j) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kSlJ * kSlC / kSlThreads; ++u) {
      const int e = tid + u * kSlThreads;
      const int j = B_JFAST ? e % kSlJ : e / kSlC, c = B_JFAST ? e / kSlJ : e % kSlC;
      Bs[j][c] = jb + j < j1 ? getB(jb + j, c0 + c) : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int j = 0; j < kSlJ; ++j) {
      const float a0 = As[tr][j], a1 = As[tr + 16][j];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float b = Bs[j][tc + 16 * q];
        acc[0][q] = fmaf(a0, b, acc[0][q]);
        acc[1][q] = fmaf(a1, b, acc[1][q]);
      }
    }
    __syncthreads();
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

// grid (n tiles of 64, m tiles of 32)
__global__ __launch_bounds__(kSlThreads) void sl_fwd_kernel(const SlFwdArgs a) {
  __shared__ float As[kSlR][kSlJ + 1];
  __shared__ float Bs[kSlJ][kSlC + 1];
  const int c0 = blockIdx.x * kSlC, r0 = blockIdx.y * kSlR;
  float acc[2][4] = {};
  auto getA = [&](int m, int k) -> float {
    if (m >= a.M) return 0.f;
    const float v = a.x[(size_t)m * a.ldx + k];
    return a.act == MDG_ACT_SILU ? silu_f(v) : v;
  };
  auto getB = [&](int k, int n) -> float {
    if (n >= a.sm.total) return 0.f;
    const int s = seg_of(a.sm, n);
    return a.w[s][(size_t)(n - a.sm.start[s]) * a.K + k];
  };
  sl_tile<true, true>(acc, r0, c0, 0, a.K, getA, getB, As, Bs);
  const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n = c0 + tc + 16 * q;
    if (n >= a.sm.total) continue;
    const int s = seg_of(a.sm, n), nl = n - a.sm.start[s];
    const float bias = a.b[s] ? a.b[s][nl] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = r0 + tr + 16 * i;
      if (m >= a.M) continue;
      float v = acc[i][q] + bias;
      if (a.resid[s]) v = a.resid[s][(size_t)m * a.ldr[s] + nl] + v;
      a.y[s][(size_t)m * a.ldy[s] + nl] = v;
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
  int n_dw_blocks;  // blocks [0, n_dw_blocks): dW tiles (n tiles x k tiles); the rest: dX partial tiles
  int k_tiles, m_tiles, chunks;
  float* part;  // [chunks][M][K]
};

__global__ __launch_bounds__(kSlThreads) void sl_bwd_kernel(const SlBwdArgs a) {
  __shared__ float As[kSlR][kSlJ + 1];
  __shared__ float Bs[kSlJ][kSlC + 1];
  const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;
  float acc[2][4] = {};
  auto dy_at = [&](int m, int n) -> float {  // dy of virtual row n at token m (0 outside)
    if (m >= a.M || n >= a.sm.total) return 0.f;
    const int s = seg_of(a.sm, n);
    return a.dy[s][(size_t)m * a.lddy[s] + (n - a.sm.start[s])];
  };
  if ((int)blockIdx.x < a.n_dw_blocks) {
    // dW tile: r = n (32 weight rows), c = k (64 input columns), j = m
    const int nt = blockIdx.x / a.k_tiles, kt = blockIdx.x % a.k_tiles;
    const int r0 = nt * kSlR, c0 = kt * kSlC;
    auto getA = [&](int n, int m) { return dy_at(m, n); };
    auto getB = [&](int m, int k) -> float {
      if (k >= a.K) return 0.f;
      const float v = a.x[(size_t)m * a.ldx + k];
      return a.act == MDG_ACT_SILU ? silu_f(v) : v;
    };
    sl_tile<false, false>(acc, r0, c0, 0, a.M, getA, getB, As, Bs);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = r0 + tr + 16 * i;
      if (n >= a.sm.total) continue;
      const int s = seg_of(a.sm, n), nl = n - a.sm.start[s];
      if (a.dw[s])
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k = c0 + tc + 16 * q;
          if (k < a.K) a.dw[s][(size_t)nl * a.K + k] = acc[i][q];
        }
    }
    // db[n] = sum_m dy[m][n]: the k-tile-0 blocks, one thread per weight row, m ascending
    if (kt == 0 && threadIdx.x < kSlR) {
      const int n = r0 + threadIdx.x;
      if (n < a.sm.total) {
        const int s = seg_of(a.sm, n);
        if (a.db[s]) {
          float sum = 0.f;
          for (int m = 0; m < a.M; ++m) sum += dy_at(m, n);
          a.db[s][n - a.sm.start[s]] = sum;
        }
      }
    }
    return;
  }
  // dX partial tile: r = m, c = k, j = n over one chunk of kSlChunk weight rows
  const int t = blockIdx.x - a.n_dw_blocks;
  const int kt = t % a.k_tiles, mt = (t / a.k_tiles) % a.m_tiles, ch = t / (a.k_tiles * a.m_tiles);
  const int r0 = mt * kSlR, c0 = kt * kSlC, j0 = ch * kSlChunk, j1 = min(j0 + kSlChunk, a.sm.total);
  auto getA = [&](int m, int n) { return dy_at(m, n); };
  auto getB = [&](int n, int k) -> float {
    if (k >= a.K) return 0.f;
    const int s = seg_of(a.sm, n);
    return a.w[s][(size_t)(n - a.sm.start[s]) * a.K + k];
  };
  sl_tile<true, false>(acc, r0, c0, j0, j1, getA, getB, As, Bs);
  float* P = a.part + (size_t)ch * a.M * a.K;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = r0 + tr + 16 * i;
    if (m >= a.M) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = c0 + tc + 16 * q;
      if (k < a.K) P[(size_t)m * a.K + k] = acc[i][q];
    }
  }
}

// dx[m][k] = (sum over chunks, in order) * SiLU'(x) (act SILU) or as is
__global__ __launch_bounds__(256) void sl_dx_reduce_kernel(int M, int K, int chunks, const float* __restrict__ part,
                                                           const float* __restrict__ x, int ldx, int act,
                                                           float* __restrict__ dx, int lddx) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= M * K) return;
  const int m = e / K, k = e - m * K;
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += part[(size_t)c * M * K + e];
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

size_t seg_linear_ws_bytes(int M, int K, int total) {
  const int chunks = (total + kSlChunk - 1) / kSlChunk;
  return (size_t)chunks * M * K * sizeof(float);
}

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
  dim3 grid((sm.total + kSlC - 1) / kSlC, (M + kSlR - 1) / kSlR);
  hipLaunchKernelGGL(sl_fwd_kernel, grid, dim3(kSlThreads), 0, st, a);
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
  a.k_tiles = (K + kSlC - 1) / kSlC;
  a.m_tiles = (M + kSlR - 1) / kSlR;
  a.chunks = dx ? (sm.total + kSlChunk - 1) / kSlChunk : 0;
  a.n_dw_blocks = any_w ? ((sm.total + kSlR - 1) / kSlR) * a.k_tiles : 0;
  a.part = ws;
  const int nblk = a.n_dw_blocks + a.chunks * a.k_tiles * a.m_tiles;
  if (nblk > 0) hipLaunchKernelGGL(sl_bwd_kernel, dim3(nblk), dim3(kSlThreads), 0, st, a);
  if (dx)
    hipLaunchKernelGGL(sl_dx_reduce_kernel, dim3((M * K + 255) / 256), dim3(256), 0, st, M, K, a.chunks,
                       (const float*)ws, x, ldx, act, dx, lddx);
  return hipGetLastError();
}

}  // namespace mdg
