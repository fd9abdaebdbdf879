// Weight and bias gradients of the block's linear layers (the backward of nn.Linear inside
// LatentMDGenLayer, latent_model.py:456-493 under loss.backward(), transport.py:137-222):
//     dW[m][k] = sum_n dY[n][m] X[n][k]        db[m] = sum_n dY[n][m]
// over the N token rows.  Both operands are token-major ([N][features], as the forward saved
// them and the backward produced them), so the reduction runs along the SLOW axis of both.
//
// bf16 (the training default): one block = a 128 x 128 tile of dW and one chunk of tokens
// (split over gridDim.z; each split writes an fp32 partial, mdg_wgrad sums the partials in
// split order, so the result is deterministic).  Per K-step of 32 tokens the block stages a
// [32 tokens][128 features] image of each operand through a 3-slot global_load_lds ring
// (256-B rows, 16-B chunk c of row r at c ^ (((r&3)<<2) | ((r>>2)&3)), the XOR applied to the
// per-lane SOURCE address since LDS-DMA writes lane-linearly) and every MFMA operand is read
// TRANSPOSED out of it with ds_read_b64_tr_b16: lane 4q+p of a 16-lane group supplies row q
// (a token), columns 4p..4p+3; lane i receives column i of the 4 rows — the token axis lands
// in the registers, which is the k axis of v_mfma_f32_32x32x16_bf16 for BOTH operands (the k
// order inside a step is the same permutation for A and B, so the sum is unchanged).
// 4 waves, each a 64 x 64 quarter (2 x 2 tiles of 32 x 32, 64 accumulator VGPRs).
//
// fp32 (the parity path): a plain 64 x 64 LDS-tiled FMA kernel, same split / reduce.
#include <utility>

#include "common.h"

namespace mdg {

namespace {

constexpr int kWgThreads = 256, kWgTile = 128, kWgBK = 32, kWgStages = 3;
constexpr int kWgImg = kWgBK * kWgTile;  // bf16 elements of one operand image
constexpr int kWgSlot = 2 * kWgImg;      // dY image + X image

__device__ __forceinline__ int wg_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
// element offset of (token row r, feature column c) in an image
__device__ __forceinline__ int wg_off(int r, int c) { return r * kWgTile + (((c >> 3) ^ wg_swz(r)) << 3) + (c & 7); }

struct WgArgs {
  const void* dy;
  const void* x;
  float* part;   // [S][M][K] fp32 (S == 1 with direct = true: dW itself)
  float* cpart;  // [S][M] fp32 column sums of dY per split (the bias gradient; null: none)
  int N, M, K, ldy, ldx, ldp, chunk;
  int gx, gy, gz;  // M tiles, K tiles, token splits (the bf16 kernels' 1-D grid is gx * gy * gz)
};

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Block -> (M tile, K tile, token split) with every tile of one token split on the SAME XCD:
// the 1-D grid is dispatched round-robin over the 8 XCDs, so the remap hands each XCD a
// contiguous range of (split, tile) indices, split-major.  The blocks of a split stream the
// same token rows of dY and X at about the same time, and that XCD's L2 serves the re-reads
// (the 3-D grid spread a split's tiles over all 8 L2s: 4x the algorithmic HBM bytes).
__device__ __forceinline__ void wg_tile_of(int gx, int gy, int gz, int& mt, int& kt, int& z) {
  const int nwg = gx * gy * gz;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, q = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + loc;
  z = wg / (gx * gy);
  const int t = wg - z * gx * gy;
  kt = t / gx;
  mt = t - kt * gx;
}

__device__ __forceinline__ void wg_vm_wait(int n) {
  if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The 8-token A or B operand of one 32 x 32 x 16 MFMA: features cbase + (lane & 31), the
// k-step's tokens {16 s2 + 4h + q} and {16 s2 + 8 + 4h + q} (h = lane >> 5, q = 0..3).
__device__ __forceinline__ bf16x8 wg_frag(const bf16_t* img, int cbase, int s2, int lane) {
  const int h = lane >> 5, gi = lane & 15;
  const int col = cbase + 16 * ((lane >> 4) & 1) + 4 * (gi & 3);
  const int row = 16 * s2 + 4 * h + (gi >> 2);
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + wg_off(row, col)));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + wg_off(row + 8, col)));
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = lo[j];
    r[4 + j] = hi[j];
  }
  return r;
}

template <int NS>  // operand ring depth (3: the default; MDG_WGRAD_STAGES=4 / 5 for A/B)
__global__ __launch_bounds__(kWgThreads, 2) void wgrad_bf16_kernel(const WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int mt, kt, z;
  wg_tile_of(a.gx, a.gy, a.gz, mt, kt, z);
  const int m0 = mt * kWgTile, k0 = kt * kWgTile;
  const int nbeg = z * a.chunk;
  const int nsteps = (min(a.N, nbeg + a.chunk) - nbeg) / kWgBK;
  const bf16_t* DY = reinterpret_cast<const bf16_t*>(a.dy);
  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.x);
  // loader: piece j (0..3) of wave w = image j >> 1, token rows 4 (2w + (j & 1)) + lane / 16,
  // chunk position lane & 15 holding logical chunk (lane & 15) ^ swz(row); columns past the
  // matrix edge are clamped into it (they only feed dW entries that are never stored)
  const int r_lo = lane >> 4, cpos = lane & 15;
  size_t src[4];
  int dst[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int img = j >> 1, rb = 4 * (2 * wave + (j & 1)), r = rb + r_lo;
    const int lim = img ? a.K : a.M;
    const int col = min((img ? k0 : m0) + 8 * (cpos ^ wg_swz(r)), lim - 8);
    src[j] = (size_t)(nbeg + r) * (img ? a.ldx : a.ldy) + col;
    dst[j] = img * kWgImg + rb * kWgTile;
  }
  auto issue = [&](int s) {
    bf16_t* sl = ring + (s % NS) * kWgSlot;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bf16_t* base = (j >> 1) ? X : DY;
      const size_t step = (size_t)s * kWgBK * ((j >> 1) ? a.ldx : a.ldy);
      __builtin_amdgcn_global_load_lds((const void*)(base + src[j] + step), (lds_ptr_t)(sl + dst[j]), 16, 0, 0);
    }
  };
  const int wm = wave >> 1, wk = wave & 1;
  f32x16 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][u][i] = 0.f;

  // bias gradient: the blocks of the first K tile also sum their dY fragments over the tokens
  // (waves wk == 0 hold every feature of the M tile once): 8 tokens per lane and k-step, the
  // two lane halves combined at the end.  No separate column-sum pass over dY.
  const bool csum = a.cpart != nullptr && kt == 0 && wk == 0;
  float cs[2] = {0.f, 0.f};
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < nsteps) issue(s0);
  for (int s = 0; s < nsteps; ++s) {
    // step s landed (the NS - 2 later steps' pieces stay in flight, 4 per step); every wave's
    // reads of step s-1 are retired (lgkmcnt) before the barrier, so the slot can be refilled
    // with step s + NS - 1
    const int ahead = min(NS - 2, nsteps - 1 - s);
    if (ahead >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + NS - 1 < nsteps) issue(s + NS - 1);
    const bf16_t* A = ring + (s % NS) * kWgSlot;
    const bf16_t* B = A + kWgImg;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) af[t] = wg_frag(A, 64 * wm + 32 * t, s2, lane);
#pragma unroll
      for (int u = 0; u < 2; ++u) bfr[u] = wg_frag(B, 64 * wk + 32 * u, s2, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t], bfr[u], acc[t][u], 0, 0, 0);
      if (csum) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          float v = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) v += (float)af[t][j];
          cs[t] += v;
        }
      }
    }
  }
  if (csum) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float v = cs[t] + __shfl_xor(cs[t], 32, 64);
      const int m = m0 + 64 * wm + 32 * t + lane;
      if (lane < 32 && m < a.M) a.cpart[(size_t)z * a.M + m] = v;
    }
  }
  // D[m][k]: k = lane & 31, m = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  float* P = a.part + (size_t)z * a.M * a.ldp;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = k0 + 64 * wk + 32 * u + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 64 * wm + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < a.M && k < a.K) P[(size_t)m * a.ldp + k] = acc[t][u][r];
      }
    }
}

// Register-staged variant (round 6, MDG_WGRAD_VST = NR in 2..4): the same tile, images, swizzle
// and MFMA sequence, but each step's 4 pieces per wave come global -> VGPRs (global_load_dwordx4
// from the swizzled source address) -> ds_write_b128 at the piece's lane-linear LDS position (the
// place LDS-DMA would write them), NR steps ahead in NR register sets, into a 2-slot LDS ring.
// The DMA stream fills LDS at ≈ 16 B/clk per CU (tools/ubench/l2lds.hip), plain 16-B loads at
// ≈ 46–63; this kernel moves 16 KiB per 32-token step for 512 MFMA cycles per SIMD (64 B/clk
// per CU at the full MFMA rate), and its counters show 66 % of wave cycles parked.  Same K order,
// same results bit for bit.
template <typename F, int... I>
__device__ __forceinline__ void wg_unroll(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}

template <int NR>
__global__ __launch_bounds__(kWgThreads, 2) void wgrad_bf16_vst_kernel(const WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);  // [2][kWgSlot]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int mt, kt, z;
  wg_tile_of(a.gx, a.gy, a.gz, mt, kt, z);
  const int m0 = mt * kWgTile, k0 = kt * kWgTile;
  const int nbeg = z * a.chunk;
  const int nsteps = (min(a.N, nbeg + a.chunk) - nbeg) / kWgBK;
  const bf16_t* DY = reinterpret_cast<const bf16_t*>(a.dy);
  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.x);
  const int r_lo = lane >> 4, cpos = lane & 15;
  size_t src[4];
  int dst[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int img = j >> 1, rb = 4 * (2 * wave + (j & 1)), r = rb + r_lo;
    const int lim = img ? a.K : a.M;
    const int col = min((img ? k0 : m0) + 8 * (cpos ^ wg_swz(r)), lim - 8);
    src[j] = (size_t)(nbeg + r) * (img ? a.ldx : a.ldy) + col;
    dst[j] = img * kWgImg + rb * kWgTile + 8 * lane;  // this lane's 16 B of the piece
  }
  u32x4 R[NR][4];
  auto load = [&](int st, u32x4(&rr)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bf16_t* base = (j >> 1) ? X : DY;
      const size_t step = (size_t)st * kWgBK * ((j >> 1) ? a.ldx : a.ldy);
      rr[j] = *reinterpret_cast<const u32x4*>(base + src[j] + step);
    }
  };
  auto commit = [&](int st, const u32x4(&rr)[4]) __attribute__((always_inline)) {
    bf16_t* sl = ring + (st & 1) * kWgSlot;
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<u32x4*>(sl + dst[j]) = rr[j];
  };
  // wait until at most `ahead` later steps' loads (4 per step) are still in flight
  auto vm_wait_steps = [&](int ahead) __attribute__((always_inline)) {
    if (ahead >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  const int wm = wave >> 1, wk = wave & 1;
  f32x16 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][u][i] = 0.f;
  const bool csum = a.cpart != nullptr && kt == 0 && wk == 0;
  float cs[2] = {0.f, 0.f};
  // prologue: steps 0 .. NR - 1 in flight; step 0 written to slot 0; step NR into the freed set
#pragma unroll
  for (int k = 0; k < NR; ++k)
    if (k < nsteps) load(k, R[k]);
  vm_wait_steps(min(NR - 1, nsteps - 1));
  if (nsteps > 0) commit(0, R[0]);
  if (NR < nsteps) load(NR, R[0]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // step s (slot s & 1 complete): its MFMAs; then step s + 1's registers (set (s + 1) % NR, the
  // oldest loads in flight) into slot (s + 1) & 1 — last read in step s - 1, before the barrier
  // that ended it — and step s + 1 + NR's loads into that set; barrier
  for (int s0 = 0; s0 < nsteps; s0 += NR) {
    // the NR steps of a round spelled out with u a compile-time constant, so each knows its
    // register set (an indexed register array would go to scratch)
    wg_unroll(std::make_integer_sequence<int, NR>{}, [&](auto U) __attribute__((always_inline)) {
      constexpr int u = decltype(U)::value;
      const int s = s0 + u;
      if (s < nsteps) {
        const bf16_t* A = ring + (s & 1) * kWgSlot;
        const bf16_t* B = A + kWgImg;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 af[2], bfr[2];
#pragma unroll
          for (int t = 0; t < 2; ++t) af[t] = wg_frag(A, 64 * wm + 32 * t, s2, lane);
#pragma unroll
          for (int v = 0; v < 2; ++v) bfr[v] = wg_frag(B, 64 * wk + 32 * v, s2, lane);
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int v = 0; v < 2; ++v) acc[t][v] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t], bfr[v], acc[t][v], 0, 0, 0);
          if (csum) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              float vs = 0.f;
#pragma unroll
              for (int j = 0; j < 8; ++j) vs += (float)af[t][j];
              cs[t] += vs;
            }
          }
        }
        if (s + 1 < nsteps) {
          constexpr int nxt = (u + 1) % NR;
          vm_wait_steps(min(NR - 1, nsteps - 2 - s));
          commit(s + 1, R[nxt]);
          if (s + 1 + NR < nsteps) load(s + 1 + NR, R[nxt]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
      }
    });
  }
  if (csum) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float v = cs[t] + __shfl_xor(cs[t], 32, 64);
      const int m = m0 + 64 * wm + 32 * t + lane;
      if (lane < 32 && m < a.M) a.cpart[(size_t)z * a.M + m] = v;
    }
  }
  float* P = a.part + (size_t)z * a.M * a.ldp;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int k = k0 + 64 * wk + 32 * v + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 64 * wm + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < a.M && k < a.K) P[(size_t)m * a.ldp + k] = acc[t][v][r];
      }
    }
}

// Wide-tile variant (round 4): block tile TM x TK = 64 WMT x 64 WKT, wave tile 32 WMT x 32 WKT
// (2 x 2 waves), same ring / swizzle / transposing reads.  A 128 x 64 wave tile reads 6 operand
// fragments per 8 MFMAs instead of 4 per 4 (a quarter fewer LDS bytes per FLOP) and the block
// stages 24 KiB per 32 tokens for twice the FLOPs of the 128 x 128 tile; taken for the MLP
// weights (fc1: dW [F][C], fc2: dW [C][F]) whose dims are multiples of 256 on one side.
template <int WMT, int WKT>
__global__ __launch_bounds__(kWgThreads, 2) void wgrad_bf16_wide_kernel(const WgArgs a) {
  constexpr int TM = 64 * WMT, TK = 64 * WKT, IMG_A = kWgBK * TM, SLOT = kWgBK * (TM + TK);
  constexpr int PW = WMT + WKT;  // 1-KiB LDS-DMA pieces per wave per step
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int mt, kt, z;
  wg_tile_of(a.gx, a.gy, a.gz, mt, kt, z);
  const int m0 = mt * TM, k0 = kt * TK;
  const int nbeg = z * a.chunk;
  const int nsteps = (min(a.N, nbeg + a.chunk) - nbeg) / kWgBK;
  const bf16_t* DY = reinterpret_cast<const bf16_t*>(a.dy);
  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.x);
  // piece j of the block (j = PW wave + i): image A (dY, TM wide) for j < TM / 16, then image B
  // (X, TK wide); in an image of width TW a piece covers 512 / TW token rows, lane -> row
  // j' (512 / TW) + lane / (TW / 8), physical chunk lane % (TW / 8) holding logical chunk
  // (lane % (TW / 8)) ^ swz(row)
  size_t src[PW];
  int dst[PW];
  bool isx[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int j = PW * wave + i;
    const bool bimg = j >= TM / 16;
    const int TW = bimg ? TK : TM, cpr = TW / 8, jj = bimg ? j - TM / 16 : j;
    const int r = jj * (64 / cpr) + lane / cpr, cpos = lane % cpr;
    const int lim = bimg ? a.K : a.M;
    const int col = min((bimg ? k0 : m0) + 8 * (cpos ^ wg_swz(r)), lim - 8);
    src[i] = (size_t)(nbeg + r) * (bimg ? a.ldx : a.ldy) + col;
    dst[i] = (bimg ? IMG_A : 0) + jj * (64 / cpr) * TW;
    isx[i] = bimg;
  }
  auto issue = [&](int st) {
    bf16_t* sl = ring + (st % kWgStages) * SLOT;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const bf16_t* base = isx[i] ? X : DY;
      const size_t step = (size_t)st * kWgBK * (isx[i] ? a.ldx : a.ldy);
      __builtin_amdgcn_global_load_lds((const void*)(base + src[i] + step), (lds_ptr_t)(sl + dst[i]), 16, 0, 0);
    }
  };
  auto frag = [&](const bf16_t* img, int TW, int cbase, int s2) {
    const int h = lane >> 5, gi = lane & 15;
    const int col = cbase + 16 * ((lane >> 4) & 1) + 4 * (gi & 3);
    const int row = 16 * s2 + 4 * h + (gi >> 2);
    auto off = [&](int rr, int cc) { return rr * TW + (((cc >> 3) ^ wg_swz(rr)) << 3) + (cc & 7); };
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + off(row, col)));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + off(row + 8, col)));
    bf16x8 r8;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r8[j] = lo[j];
      r8[4 + j] = hi[j];
    }
    return r8;
  };
  const int wm = wave >> 1, wk = wave & 1;
  f32x16 acc[WMT][WKT];
#pragma unroll
  for (int t = 0; t < WMT; ++t)
#pragma unroll
    for (int u = 0; u < WKT; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][u][i] = 0.f;
  const bool csum = a.cpart != nullptr && kt == 0 && wk == 0;
  float cs[WMT];
#pragma unroll
  for (int t = 0; t < WMT; ++t) cs[t] = 0.f;
  for (int s0 = 0; s0 < kWgStages - 1; ++s0)
    if (s0 < nsteps) issue(s0);
  for (int st = 0; st < nsteps; ++st) {
    if (st + 1 < nsteps) {
      if constexpr (PW == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (st + kWgStages - 1 < nsteps) issue(st + kWgStages - 1);
    const bf16_t* A = ring + (st % kWgStages) * SLOT;
    const bf16_t* B = A + IMG_A;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 af[WMT], bfr[WKT];
#pragma unroll
      for (int t = 0; t < WMT; ++t) af[t] = frag(A, TM, 32 * WMT * wm + 32 * t, s2);
#pragma unroll
      for (int u = 0; u < WKT; ++u) bfr[u] = frag(B, TK, 32 * WKT * wk + 32 * u, s2);
#pragma unroll
      for (int t = 0; t < WMT; ++t)
#pragma unroll
        for (int u = 0; u < WKT; ++u) acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t], bfr[u], acc[t][u], 0, 0, 0);
      if (csum) {
#pragma unroll
        for (int t = 0; t < WMT; ++t) {
          float v = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) v += (float)af[t][j];
          cs[t] += v;
        }
      }
    }
  }
  if (csum) {
#pragma unroll
    for (int t = 0; t < WMT; ++t) {
      const float v = cs[t] + __shfl_xor(cs[t], 32, 64);
      const int m = m0 + 32 * WMT * wm + 32 * t + lane;
      if (lane < 32 && m < a.M) a.cpart[(size_t)z * a.M + m] = v;
    }
  }
  float* P = a.part + (size_t)z * a.M * a.ldp;
#pragma unroll
  for (int t = 0; t < WMT; ++t)
#pragma unroll
    for (int u = 0; u < WKT; ++u) {
      const int k = k0 + 32 * WKT * wk + 32 * u + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 32 * WMT * wm + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < a.M && k < a.K) P[(size_t)m * a.ldp + k] = acc[t][u][r];
      }
    }
}

// fp32 parity path: 64 x 64 tile, 16 tokens per LDS step, 4 x 4 outputs per thread.
__global__ __launch_bounds__(256) void wgrad_f32_kernel(const WgArgs a) {
  __shared__ float As[16][64], Bs[16][64];
  const int tid = threadIdx.x, tm = tid >> 4, tk = tid & 15;
  const int m0 = blockIdx.x * 64, k0 = blockIdx.y * 64, z = blockIdx.z;
  const int nbeg = z * a.chunk, nend = min(a.N, nbeg + a.chunk);
  const float* DY = reinterpret_cast<const float*>(a.dy);
  const float* X = reinterpret_cast<const float*>(a.x);
  float acc[4][4] = {};
  for (int n = nbeg; n < nend; n += 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, r = e >> 6, c = e & 63;
      const bool ok = n + r < nend;
      As[r][c] = (ok && m0 + c < a.M) ? DY[(size_t)(n + r) * a.ldy + m0 + c] : 0.f;
      Bs[r][c] = (ok && k0 + c < a.K) ? X[(size_t)(n + r) * a.ldx + k0 + c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[r][tm + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[r][tk + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
  float* P = a.part + (size_t)z * a.M * a.ldp;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + tm + 16 * i, k = k0 + tk + 16 * j;
      if (m < a.M && k < a.K) P[(size_t)m * a.ldp + k] = acc[i][j];
    }
}

// Column sums of dY over a token chunk: thread = 8 consecutive columns (one 16-B bf16 load /
// two float4), 4 waves over interleaved rows, reduced through LDS -> part[z][M].
template <typename CT>
__global__ __launch_bounds__(256) void colsum_kernel(const CT* __restrict__ dy, int N, int M, int ldy, int chunk,
                                                     float* __restrict__ part) {
  __shared__ float red[4][64 * 8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = (blockIdx.x * 64 + lane) * 8, z = blockIdx.y;
  const int nbeg = z * chunk, nend = min(N, nbeg + chunk);
  float s[8] = {};
  if (c0 < M) {
    for (int n = nbeg + wave; n < nend; n += 4) {
      const CT* p = dy + (size_t)n * ldy + c0;
      if constexpr (is_bf16<CT>()) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += (float)v[j];
      } else {
        const float4 v0 = reinterpret_cast<const float4*>(p)[0], v1 = reinterpret_cast<const float4*>(p)[1];
        s[0] += v0.x; s[1] += v0.y; s[2] += v0.z; s[3] += v0.w;
        s[4] += v1.x; s[5] += v1.y; s[6] += v1.z; s[7] += v1.w;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = s[j];
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 8; e += 256) {
    const int c = blockIdx.x * 512 + e;
    if (c < M) part[(size_t)z * M + c] = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
  }
}

// dW[m][k] (ld ldo) = sum over z in order of part[z][m][k] (ld K, 4 columns per thread), and in
// the same launch db[m] = sum over z of cpart[z][m] (the threads past dW's quads)
__global__ __launch_bounds__(256) void split_sum_wb_kernel(const float* __restrict__ part, int S, int M, int K,
                                                           float* __restrict__ out, int ldo,
                                                           const float* __restrict__ cpart, float* __restrict__ db) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long nq = (long long)M * (K >> 2);
  if (e < nq) {
    const int m = (int)(e / (K >> 2)), k = 4 * (int)(e % (K >> 2));
    const size_t zs = (size_t)M * K;
    const float* p = part + (size_t)m * K + k;
    float4 s = *reinterpret_cast<const float4*>(p);
#pragma unroll 8  // (the loads of 8 splits in flight; the adds keep z order)
    for (int z = 1; z < S; ++z) {
      const float4 v = *reinterpret_cast<const float4*>(p + z * zs);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    *reinterpret_cast<float4*>(out + (size_t)m * ldo + k) = s;
  } else if (db && e - nq < M) {
    const int m = (int)(e - nq);
    float s = cpart[m];
#pragma unroll 8
    for (int z = 1; z < S; ++z) s += cpart[(size_t)z * M + m];
    db[m] = s;
  }
}

// out[m][k] (ld ldo) = sum over z in order of part[z][m][k] (ld ldp)
__global__ __launch_bounds__(256) void split_sum_kernel(const float* __restrict__ part, int S, int M, int K, int ldp,
                                                        float* __restrict__ out, int ldo) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)M * K) return;
  const int m = (int)(e / K), k = (int)(e % K);
  const size_t zs = (size_t)M * ldp;
  const float* p = part + (size_t)m * ldp + k;
  float s = p[0];
#pragma unroll 8
  for (int z = 1; z < S; ++z) s += p[z * zs];
  out[(size_t)m * ldo + k] = s;
}

}  // namespace

// Split plan shared by the workspace query and the launch.
struct WgPlan {
  int S, chunk, cs_S, cs_chunk;
  size_t part_elems, cs_elems;
  int wide;  // bf16 tile: 0 = 128 x 128, 1 = 256 x 128 (WMT 4), 2 = 128 x 256 (WKT 4)
};

// MDG_WGRAD_WIDE=1: the wide tiles for the MLP weights (opt-in: the token split doubles with half
// the tiles, and the partial round trip eats the per-FLOP gain; 16.48 vs 16.28 ms per training
// step, same box); MDG_WGRAD_BLOCKS: target block count of the token split (default 768 = 3 per CU:
// training step 11.30-11.39 ms vs 11.61-11.68 at 512, 11.44-11.49 at 640, 11.82-11.91 at 1 024,
// 12.0 at 384, same box, round 5)
static int wgrad_wide_enabled() {
  static const int v = [] {
    const char* e = getenv("MDG_WGRAD_WIDE");
    return e ? atoi(e) : 0;
  }();
  return v;
}
static int wgrad_stages() {
  static const int v = [] {
    const char* e = getenv("MDG_WGRAD_STAGES");
    const int n = e ? atoi(e) : 3;
    return (n == 4 || n == 5) ? n : 3;
  }();
  return v;
}
static int wgrad_vst() {  // MDG_WGRAD_VST = 2..4: the register-staged kernel with that many steps in flight
  static const int v = [] {
    const char* e = getenv("MDG_WGRAD_VST");
    const int n = e ? atoi(e) : 0;
    return (n >= 2 && n <= 4) ? n : 0;
  }();
  return v;
}
static int wgrad_target_blocks() {
  static const int v = [] {
    const char* e = getenv("MDG_WGRAD_BLOCKS");
    const int b = e ? atoi(e) : 768;
    return b > 0 ? b : 768;
  }();
  return v;
}

WgPlan wgrad_plan(int dtype, int N, int M, int K, bool need_w, bool need_b) {
  WgPlan p{};
  if (dtype == MDG_BF16 && wgrad_wide_enabled())
    p.wide = (M % 256 == 0 && K % 128 == 0) ? 1 : (K % 256 == 0 && M % 128 == 0) ? 2 : 0;
  const int tm = dtype == MDG_BF16 ? (p.wide == 1 ? 256 : kWgTile) : 64;
  const int tk = dtype == MDG_BF16 ? (p.wide == 2 ? 256 : kWgTile) : 64;
  const int tiles = ((M + tm - 1) / tm) * ((K + tk - 1) / tk);
  const int quantum = dtype == MDG_BF16 ? kWgBK : 16;
  const int nq = (N + quantum - 1) / quantum;
  // ~3 blocks per CU over the 256 CUs, each split at least 8 K-steps long.  The block count
  // stays AT MOST the target (resident blocks per CU x 256): rounding the split count up put the
  // last few blocks in a second round, which then took as long as the first (w2: 540 blocks,
  // 78 us; at 504 blocks the grid is one round)
  const int target = wgrad_target_blocks();
  int S = need_w ? max(1, target / tiles) : 1;
  S = max(1, min(S, nq / 8));
  p.chunk = ((nq + S - 1) / S) * quantum;
  p.S = (N + p.chunk - 1) / p.chunk;
  p.part_elems = need_w ? (size_t)p.S * M * K : 0;
  if (need_b && need_w && dtype == MDG_BF16) {  // column sums fused into the wgrad blocks
    p.cs_chunk = p.chunk;
    p.cs_S = p.S;
    p.cs_elems = (size_t)p.S * M;
    return p;
  }
  const int cblocks = (M + 511) / 512;
  int cs = need_b ? max(1, min(256 / cblocks, N / 64)) : 0;
  p.cs_chunk = need_b ? (N + cs - 1) / cs : 0;
  p.cs_S = need_b ? (N + p.cs_chunk - 1) / p.cs_chunk : 0;
  p.cs_elems = need_b ? (size_t)p.cs_S * M : 0;
  return p;
}

hipError_t wgrad_launch(int dtype, int N, int M, int K, const void* dy, int ldy, const void* x, int ldx, float* dw,
                        int lddw, float* db, float* ws, hipStream_t s) {
  const WgPlan p = wgrad_plan(dtype, N, M, K, dw != nullptr, db != nullptr);
  const bool fused_b = db && dw && dtype == MDG_BF16;
  if (dw) {
    WgArgs a;
    a.dy = dy; a.x = x; a.N = N; a.M = M; a.K = K; a.ldy = ldy; a.ldx = ldx; a.chunk = p.chunk;
    const bool direct = p.S == 1;
    a.part = direct ? dw : ws;
    a.ldp = direct ? lddw : K;
    float* cp = ws + (p.S > 1 ? p.part_elems : 0);
    a.cpart = fused_b ? (direct ? db : cp) : nullptr;
    if (dtype == MDG_BF16 && p.wide) {
      constexpr int smem = kWgStages * kWgBK * (256 + 128) * 2;
      static bool attr = false;
      if (!attr) {
        for (const void* k : {reinterpret_cast<const void*>(&wgrad_bf16_wide_kernel<4, 2>),
                              reinterpret_cast<const void*>(&wgrad_bf16_wide_kernel<2, 4>)}) {
          hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
          if (e != hipSuccess) return e;
        }
        attr = true;
      }
      a.gx = p.wide == 1 ? M / 256 : M / 128;
      a.gy = p.wide == 1 ? K / 128 : K / 256;
      a.gz = p.S;
      const dim3 grid((unsigned)(a.gx * a.gy * a.gz));
      if (p.wide == 1)
        hipLaunchKernelGGL((wgrad_bf16_wide_kernel<4, 2>), grid, dim3(kWgThreads), smem, s, a);
      else
        hipLaunchKernelGGL((wgrad_bf16_wide_kernel<2, 4>), grid, dim3(kWgThreads), smem, s, a);
    } else if (dtype == MDG_BF16) {
      static bool attr = false;
      if (!attr) {
        const void* ks[3] = {reinterpret_cast<const void*>(&wgrad_bf16_kernel<3>),
                             reinterpret_cast<const void*>(&wgrad_bf16_kernel<4>),
                             reinterpret_cast<const void*>(&wgrad_bf16_kernel<5>)};
        for (int i = 0; i < 3; ++i) {
          hipError_t e = hipFuncSetAttribute(ks[i], hipFuncAttributeMaxDynamicSharedMemorySize, (3 + i) * kWgSlot * 2);
          if (e != hipSuccess) return e;
        }
        attr = true;
      }
      a.gx = (M + 127) / 128;
      a.gy = (K + 127) / 128;
      a.gz = p.S;
      const dim3 grid((unsigned)(a.gx * a.gy * a.gz));
      const int ns = wgrad_stages(), vst = wgrad_vst();
      if (vst == 2) hipLaunchKernelGGL(wgrad_bf16_vst_kernel<2>, grid, dim3(kWgThreads), 2 * kWgSlot * 2, s, a);
      else if (vst == 3) hipLaunchKernelGGL(wgrad_bf16_vst_kernel<3>, grid, dim3(kWgThreads), 2 * kWgSlot * 2, s, a);
      else if (vst == 4) hipLaunchKernelGGL(wgrad_bf16_vst_kernel<4>, grid, dim3(kWgThreads), 2 * kWgSlot * 2, s, a);
      else if (ns == 5) hipLaunchKernelGGL(wgrad_bf16_kernel<5>, grid, dim3(kWgThreads), 5 * kWgSlot * 2, s, a);
      else if (ns == 4) hipLaunchKernelGGL(wgrad_bf16_kernel<4>, grid, dim3(kWgThreads), 4 * kWgSlot * 2, s, a);
      else hipLaunchKernelGGL(wgrad_bf16_kernel<3>, grid, dim3(kWgThreads), 3 * kWgSlot * 2, s, a);
    } else {
      hipLaunchKernelGGL(wgrad_f32_kernel, dim3((M + 63) / 64, (K + 63) / 64, p.S), dim3(256), 0, s, a);
    }
    if (hipError_t e = hipGetLastError()) return e;
    if (!direct && fused_b) {
      const long long n = (long long)M * (K / 4) + M;
      hipLaunchKernelGGL(split_sum_wb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float*)ws, p.S,
                         M, K, dw, lddw, (const float*)cp, db);
      return hipGetLastError();
    }
    if (!direct) {
      const long long n = (long long)M * (K / 4);
      hipLaunchKernelGGL(split_sum_wb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float*)ws, p.S,
                         M, K, dw, lddw, nullptr, nullptr);
      if (hipError_t e = hipGetLastError()) return e;
    }
    if (fused_b) return hipSuccess;  // direct: the kernel wrote db itself
  }
  if (db) {
    float* cp = ws + (p.S > 1 ? p.part_elems : 0);
    const dim3 grid((M + 511) / 512, p.cs_S);
    if (dtype == MDG_BF16)
      hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)dy, N, M, ldy, p.cs_chunk, cp);
    else
      hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, s, (const float*)dy, N, M, ldy, p.cs_chunk, cp);
    if (hipError_t e = hipGetLastError()) return e;
    hipLaunchKernelGGL(split_sum_kernel, dim3((M + 255) / 256), dim3(256), 0, s, (const float*)cp, p.cs_S, 1, M, M, db,
                       M);
    if (hipError_t e = hipGetLastError()) return e;
  }
  return hipSuccess;
}

size_t wgrad_ws_bytes(int dtype, int N, int M, int K, bool need_w, bool need_b) {
  const WgPlan p = wgrad_plan(dtype, N, M, K, need_w, need_b);
  return ((p.S > 1 ? p.part_elems : 0) + p.cs_elems) * sizeof(float) + 256;
}

}  // namespace mdg
