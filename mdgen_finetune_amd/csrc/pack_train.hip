// Weight packing and gradient unpacking of the HIP training layer (train_hip._HipLayerFn), one
// launch each per layer and step.  Done with PyTorch ops they were ~75 small kernels per layer
// (concatenations, row gathers for the q / k pair interleave, casts, transposes for the input-
// gradient GEMMs, the bias-key RoPE rotation and its transpose, the adaLN partial sums):
// 390 launches and 2.9 ms of a 20 ms training step on MI355X (profiles/r03_train_kernels.md).
//
// pack   (forward):  wqkv[i] = CT [3C][C] rows q | k | v, q and k rows pair-interleaved per head
//                    (row 2j = dim j, 2j+1 = dim j + D/2) when RoPE is on; its transpose; bqkv[i];
//                    wo[i], w1, w2 as CT and transposed; kvb[i] = [H][2][DP] (DP = MDG_HEAD_STRIDE(D):
//                    32, or 64 for head_dim 32..63): bias_k RoPE-rotated at
//                    the bias key's position S (fair-esm: x cos + rotate_half(x) sin) in the
//                    interleaved order, bias_v with 1.0 in pad column D.
// unpack (backward): the packed-order fp32 q|k|v weight / bias gradients back to q_proj / k_proj /
//                    v_proj order; bias-key gradient partials summed over parts, un-interleaved and
//                    rotated back (the transpose of the rotation); the adaLN gradient [B][9C]
//                    (latent_model.py:459-461 chunk order) and the out_proj / fc2 bias gradients
//                    from the LN/gate-backward per-block partials.
#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {
namespace {

// natural (q_proj row order) index of packed row r of one head-major q or k block
__device__ __forceinline__ int nat_of_packed(int r, int D) {
  const int h = r / D, j = r - h * D;
  return h * D + ((j & 1) ? (j >> 1) + D / 2 : (j >> 1));
}
__device__ __forceinline__ int packed_of_nat(int n, int D) {
  const int h = n / D, j = n - h * D, half = D / 2;
  return h * D + (j < half ? 2 * j : 2 * (j - half) + 1);
}

// One 32 x 32 tile of a weight: source row gathered by `src_row`, written cast to CT row-major
// and transposed, both coalesced (the transpose goes through LDS); the whole pack launch takes
// ~12 us per layer (rocprofv3, B = 8 training step).
template <typename CT, typename SrcRow>
__device__ __forceinline__ void pack_tile(float (*tile)[33], SrcRow src_row, void* dst, void* dst_t, int R, int K,
                                          int r0, int k0) {
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8 threads
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = r0 + ty + 8 * u, k = k0 + tx;
    const float v = (r < R && k < K) ? src_row(r)[k] : 0.f;
    tile[ty + 8 * u][tx] = v;
    if (r < R && k < K) reinterpret_cast<CT*>(dst)[(size_t)r * K + k] = (CT)v;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = k0 + ty + 8 * u, r = r0 + tx;
    if (r < R && k < K) reinterpret_cast<CT*>(dst_t)[(size_t)k * R + r] = (CT)tile[tx][ty + 8 * u];
  }
  __syncthreads();
}

template <typename CT, typename SrcRow>
__device__ __forceinline__ void pack_matrix(float (*tile)[33], SrcRow src_row, void* dst, void* dst_t, int R, int K) {
  const int tr = (R + 31) / 32, tk = (K + 31) / 32;
  for (int t = blockIdx.x; t < tr * tk; t += gridDim.x) pack_tile<CT>(tile, src_row, dst, dst_t, R, K, (t / tk) * 32,
                                                                      (t % tk) * 32);
}

template <typename CT>
__global__ __launch_bounds__(256) void pack_kernel(const mdg_train_pack p) {
#pragma clang fp contract(off)
  __shared__ float tile[32][33];
  const int C = p.C, D = p.D, F = p.F, H = p.H, half = D / 2;
  const int job = blockIdx.y;
  const int stride = gridDim.x * blockDim.x;
  const int t0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (job < 2) {  // q|k|v weight of attention `job`
    const int i = job;
    auto row = [&](int r) -> const float* {
      if (r < C) return p.wq[i] + (size_t)(p.rope ? nat_of_packed(r, D) : r) * C;
      if (r < 2 * C) return p.wk[i] + (size_t)(p.rope ? nat_of_packed(r - C, D) : r - C) * C;
      return p.wv[i] + (size_t)(r - 2 * C) * C;
    };
    pack_matrix<CT>(tile, row, p.wqkv[i], p.wqkv_t[i], 3 * C, C);
  } else if (job < 4) {  // out_proj weight
    const int i = job - 2;
    pack_matrix<CT>(tile, [&](int r) { return p.wo[i] + (size_t)r * C; }, p.wo_p[i], p.wo_t[i], C, C);
  } else if (job == 4) {  // fc1 [F][C]
    pack_matrix<CT>(tile, [&](int r) { return p.w1 + (size_t)r * C; }, p.w1_p, p.w1_t, F, C);
  } else if (job == 5) {  // fc2 [C][F]
    pack_matrix<CT>(tile, [&](int r) { return p.w2 + (size_t)r * F; }, p.w2_p, p.w2_t, C, F);
  } else {  // q|k|v bias and the bias key / value rows of attention job - 6
    const int i = job - 6;
    for (int e = t0; e < 3 * C; e += stride) {
      float v;
      if (e < C) v = p.bq[i][p.rope ? nat_of_packed(e, D) : e];
      else if (e < 2 * C) v = p.bk[i][p.rope ? nat_of_packed(e - C, D) : e - C];
      else v = p.bv[i][e - 2 * C];
      p.bqkv[i][e] = v;
    }
    const float* tab = p.rope_tab[i];
    const int S = p.rope_pos[i], rows = p.rope_rows[i];
    const int DP = dp_of(D);
    for (int e = t0; e < H * 2 * DP; e += stride) {
      const int h = e / (2 * DP), which = (e / DP) & 1, d = e % DP;
      float v = 0.f;
      if (which == 1) {
        v = d < D ? p.bias_v[i][h * D + d] : (d == D ? 1.0f : 0.f);
      } else if (d < D) {
        if (p.rope) {
          const int j = (d & 1) ? (d >> 1) + half : (d >> 1);  // natural dim of interleaved column d
          const float* kb = p.bias_k[i] + h * D;
          const float c = tab[S * half + (j % half)], s = tab[rows * half + S * half + (j % half)];
          const float rot = j < half ? -kb[j + half] : kb[j - half];
          v = __fadd_rn(__fmul_rn(kb[j], c), __fmul_rn(rot, s));
        } else {
          v = p.bias_k[i][h * D + d];
        }
      }
      p.kvb[i][e] = v;
    }
  }
}

__global__ __launch_bounds__(256) void unpack_kernel(const mdg_train_unpack u) {
#pragma clang fp contract(off)
  const int C = u.C, D = u.D, H = u.H, B = u.B, nb = u.nblk, half = D / 2;
  const int job = blockIdx.y;
  const int stride = gridDim.x * blockDim.x;
  const int t0 = blockIdx.x * blockDim.x + threadIdx.x;
  const bool vec = job < 2 && C % 4 == 0 &&
                   ((reinterpret_cast<uintptr_t>(u.gwqkv[job & 1]) | reinterpret_cast<uintptr_t>(u.gq[job & 1]) |
                     reinterpret_cast<uintptr_t>(u.gk[job & 1]) | reinterpret_cast<uintptr_t>(u.gv[job & 1])) & 15) == 0;
  if (vec) {  // q|k|v weight + bias gradients of attention `job`, natural row order:
    // float4 pieces, four per thread loaded before any is stored (the loads of a scalar loop
    // could not pass its stores: 13 dependent round trips per thread)
    const int i = job, C4 = C / 4, total = 3 * C * C4;
    constexpr int U = 4;
    for (int e0 = t0; e0 < total; e0 += U * stride) {
      float4 v[U];
      int nn_[U], blk_[U], k4_[U], r_[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int e = min(e0 + j * stride, total - 1);
        const int n = e / C4, k4 = e - n * C4;
        const int blk = n / C, nn = n - blk * C;
        const int r = blk * C + (blk < 2 && u.rope ? packed_of_nat(nn, D) : nn);
        v[j] = *reinterpret_cast<const float4*>(u.gwqkv[i] + (size_t)r * C + 4 * k4);
        nn_[j] = nn, blk_[j] = blk, k4_[j] = k4, r_[j] = r;
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (e0 + j * stride >= total) break;
        const int blk = blk_[j], nn = nn_[j];
        float* dst = blk == 0 ? u.gq[i] : blk == 1 ? u.gk[i] : u.gv[i];
        *reinterpret_cast<float4*>(dst + (size_t)nn * C + 4 * k4_[j]) = v[j];
        if (k4_[j] == 0) {
          float* db = blk == 0 ? u.gbq[i] : blk == 1 ? u.gbk[i] : u.gbv[i];
          db[nn] = u.gbqkv[i][r_[j]];
        }
      }
    }
  } else if (job < 2) {  // (C % 4 != 0 or unaligned) one element per step
    const int i = job;
    for (int e = t0; e < 3 * C * C; e += stride) {
      const int n = e / C, k = e - n * C;  // natural row n of [q; k; v]
      const int blk = n / C, nn = n - blk * C;
      const int r = blk * C + (blk < 2 && u.rope ? packed_of_nat(nn, D) : nn);
      const float v = u.gwqkv[i][(size_t)r * C + k];
      float* dst = blk == 0 ? u.gq[i] : blk == 1 ? u.gk[i] : u.gv[i];
      dst[(size_t)nn * C + k] = v;
      if (k == 0) {
        const float bv = u.gbqkv[i][r];
        float* db = blk == 0 ? u.gbq[i] : blk == 1 ? u.gbk[i] : u.gbv[i];
        db[nn] = bv;
      }
    }
  } else if (job < 4) {  // bias_k / bias_v gradients of attention job - 2: block h < H sums head
    // h's [parts][2][DP] slots (the 4 waves take every 4th slot, added in wave order; a lane owns
    // columns lane, lane + 64 .. of the 2 DP; fp64 sums: the slots nearly cancel), then applies
    // the rotation's transpose from LDS
    const int i = job - 2, np = u.parts[i], h = blockIdx.x, DP = dp_of(D);
    if (h >= H) return;
    __shared__ double red[4][2 * MDG_DP_WIDE];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int col = lane; col < 2 * DP; col += 64) {
      const float* bp = u.bpart[i] + (size_t)h * np * 2 * DP + col;  // [H][parts][2][DP]
      // 16 slots in flight per lane (the spatial backward leaves 500 per head at B = 8, T = 1000)
      constexpr int NA = 16;
      double a[NA];
#pragma unroll
      for (int j = 0; j < NA; ++j) a[j] = 0.0;
      int q = w;
      for (; q + 4 * (NA - 1) < np; q += 4 * NA) {
#pragma unroll
        for (int j = 0; j < NA; ++j) a[j] += bp[(size_t)(q + 4 * j) * 2 * DP];
      }
      for (; q < np; q += 4) a[0] += bp[(size_t)q * 2 * DP];
#pragma unroll
      for (int st = NA / 2; st >= 1; st >>= 1)
#pragma unroll
        for (int j = 0; j < st; ++j) a[j] += a[j + st];
      red[w][col] = a[0];
    }
    __syncthreads();
    auto g = [&](int which, int d) {
      const int e = which * DP + d;
      return (float)(((red[0][e] + red[1][e]) + red[2][e]) + red[3][e]);
    };
    const float* tab = u.rope_tab[i];
    const int S = u.rope_pos[i], rows = u.rope_rows[i];
    for (int j = threadIdx.x; j < D; j += blockDim.x) {
      const int e = h * D + j;
      u.gbias_v[i][e] = g(1, j);
      if (!u.rope) {
        u.gbias_k[i][e] = g(0, j);
        continue;
      }
      // gradient w.r.t. the rotated bias key, natural order; then the transpose of x c + rot(x) s
      const int jp = j < half ? j + half : j - half;
      const float gr = g(0, j < half ? 2 * j : 2 * (j - half) + 1);
      const float grp = g(0, jp < half ? 2 * jp : 2 * (jp - half) + 1);
      const float c = tab[S * half + (j % half)], sp = tab[rows * half + S * half + (jp % half)];
      const float z = __fmul_rn(grp, sp);
      u.gbias_k[i][e] = __fadd_rn(__fmul_rn(gr, c), j < half ? z : -z);
    }
  } else if (job == 4) {  // adaLN gradient [B][9C]
    // chunk -> (part tensor, row): shift_l, scale_l | gate_l | shift_t, scale_t | gate_t | shift_m,
    // scale_m | gate_m  (latent_model.py:459-461).  One thread per element, its nb row-block
    // partials loaded 8 at a time into 8 independent sums (every load of a thread in flight
    // together; consecutive threads read consecutive columns), combined in a fixed tree.
    const int src[9] = {0, 0, 1, 1, 1, 2, 2, 2, 3}, row[9] = {0, 1, 2, 0, 1, 2, 0, 1, 2};
    for (int e0 = t0; e0 < B * 9 * C; e0 += stride) {
      const int b = e0 / (9 * C), ck = e0 - b * 9 * C, c9 = ck / C, k = ck - c9 * C;
      const float* pp = u.part[src[c9]] + ((size_t)b * nb * 4 + row[c9]) * C + k;  // slot q at + q 4C
      float a[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = 0.f;
      int q = 0;
#pragma unroll 2
      for (; q + 8 <= nb; q += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += pp[(size_t)(q + j) * 4 * C];
      for (; q < nb; ++q) a[0] += pp[(size_t)q * 4 * C];
      u.dmods[e0] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    }
  } else {  // out_proj (spatial, temporal) and fc2 bias gradients: row 3 of part_s / part_t / part_m
    // 32 lanes per element over its B x nb partials (16 each at B = 8, T = 1000), 8 loads in
    // flight per lane, then a shuffle tree (a serial sum per 8 lanes was the launch's long pole)
    const int g = t0 & 31, n = B * nb;
    for (int e0 = t0 >> 5; e0 < 3 * C; e0 += stride >> 5) {
      const int w = e0 / C, k = e0 - w * C;
      const float* pp = u.part[w + 1] + 3 * C + k;  // (b, q) slot i = b nb + q at + i 4C
      float a[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = 0.f;
      int i = g;
#pragma unroll 2
      for (; i + 32 * 7 < n; i += 32 * 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += pp[(size_t)(i + 32 * j) * 4 * C];
      for (; i < n; i += 32) a[0] += pp[(size_t)i * 4 * C];
      float s = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) s += __shfl_xor(s, o, 64);
      if (g == 0) (w == 0 ? u.gbo[0] : w == 1 ? u.gbo[1] : u.gb2)[k] = s;
    }
  }
}

}  // namespace

hipError_t train_pack_launch(const mdg_train_pack& p, hipStream_t s) {
  const dim3 grid(256, 8);
  if (p.dtype == MDG_BF16) hipLaunchKernelGGL(pack_kernel<bf16_t>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(pack_kernel<float>, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t train_unpack_launch(const mdg_train_unpack& u, hipStream_t s) {
  hipLaunchKernelGGL(unpack_kernel, dim3(144, 6), dim3(256), 0, s, u);
  return hipGetLastError();
}

}  // namespace mdg
