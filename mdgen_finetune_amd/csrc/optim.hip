// The optimizer step of the graphed training step as three library launches over a device table
// of tensors: the reference's Lightning loop clips the global gradient norm (clip_grad_norm_,
// gradient_clip_val in train.py:52) and steps Adam / AdamW (wrapper.py:167-173).  torch's
// foreach norm + multiplies + fused Adam took ~0.55 ms of multi-tensor launches per step at
// 34 M parameters (profiles/r04_train_kernels.md); here one pass reads g for the norm and one
// pass reads p, g, m, v and writes p, m, v (28 B per parameter, the HBM floor of the update).
//
//   adam_norm_part: block = one chunk of kAdamChunk elements of one tensor: sum of g^2 (float4
//     loads, four accumulators, wave + fixed-order block reduction) -> part[chunk]
//   adam_norm_final: one block: parts summed in a fixed order -> norm, clip coefficient, every
//     tensor's step += 1
//   adam_update: block = one chunk: the Adam / AdamW update with the clipped gradient.
// Deterministic: every sum has a fixed order independent of scheduling.
#include "../../include/mdgen_hip.h"
#include "common.h"

#include <cmath>
#include <cstring>

namespace mdg {
namespace {

constexpr int kAdamChunk = 16384;  // elements per block (64 KiB of each array)

struct AdamTab {
  const mdg_adam_tensor* t;
  const int* ct;  // chunk -> tensor
  const int* ci;  // chunk -> chunk index within the tensor
};
__device__ __forceinline__ AdamTab adam_tab(const void* table, int nt, int nc) {
  AdamTab a;
  a.t = reinterpret_cast<const mdg_adam_tensor*>(table);
  a.ct = reinterpret_cast<const int*>(a.t + nt);
  a.ci = a.ct + nc;
  return a;
}

// fixed-order sum over the 256 threads of a block (wave reductions, then the 4 waves in order)
__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

__device__ __forceinline__ bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

__global__ __launch_bounds__(256) void adam_norm_part_kernel(int nt, int nc, const void* table, float* part) {
  __shared__ float red[4];
  const AdamTab tab = adam_tab(table, nt, nc);
  const int ti = tab.ct[blockIdx.x];
  const mdg_adam_tensor& T = tab.t[ti];
  const float* g = T.g;
  const long long n = T.n, s0 = (long long)tab.ci[blockIdx.x] * kAdamChunk;
  const int len = (int)min((long long)kAdamChunk, n - s0);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (al16(g)) {
    const float4* g4 = reinterpret_cast<const float4*>(g + s0);
    const int n4 = len >> 2;
    for (int i = threadIdx.x; i < n4; i += 256) {
      const float4 v = g4[i];
      a0 = fmaf(v.x, v.x, a0);
      a1 = fmaf(v.y, v.y, a1);
      a2 = fmaf(v.z, v.z, a2);
      a3 = fmaf(v.w, v.w, a3);
    }
    for (int i = 4 * n4 + threadIdx.x; i < len; i += 256) a0 = fmaf(g[s0 + i], g[s0 + i], a0);
  } else {
    for (int i = threadIdx.x; i < len; i += 256) a0 = fmaf(g[s0 + i], g[s0 + i], a0);
  }
  const float s = block_sum256((a0 + a1) + (a2 + a3), red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(1024) void adam_norm_final_kernel(int nt, int nc, const void* table, float* ws,
                                                               float max_norm, float* gnorm) {
  __shared__ float red[16];
  const AdamTab tab = adam_tab(table, nt, nc);
  float s = 0.f;
  for (int i = threadIdx.x; i < nc; i += 1024) s += ws[i];
  s = wave_sum(s);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < 16; ++w) tot += red[w];
    const float norm = sqrtf(tot);
    // torch.nn.utils.clip_grad_norm_: coef = max_norm / (norm + 1e-6), clamped to 1
    ws[nc] = max_norm > 0.f ? fminf(max_norm / (norm + 1e-6f), 1.0f) : 1.0f;
    if (gnorm) *gnorm = norm;
  }
  for (int i = threadIdx.x; i < nt; i += 1024) *tab.t[i].step += 1.0f;
}

__global__ __launch_bounds__(256) void adam_update_kernel(int nt, int nc, const void* table, const float* ws, double lr,
                                                          double b1d, double b2d, double epsd, double wdd,
                                                          int decoupled) {
  const AdamTab tab = adam_tab(table, nt, nc);
  const int ti = tab.ct[blockIdx.x];
  const mdg_adam_tensor& T = tab.t[ti];
  float* p = T.p;
  const float* g = T.g;
  float* m = T.m;
  float* v = T.v;
  const long long n = T.n, s0 = (long long)tab.ci[blockIdx.x] * kAdamChunk;
  const int len = (int)min((long long)kAdamChunk, n - s0);
  const float coef = ws[nc];
  // the arithmetic of torch's fused Adam (ATen fused_adam_utils.cuh adam_math): bias corrections
  // in double from the fp32 step, handed over as fp32; the moments formed in double from the
  // double hyper-parameters and rounded once; denom + eps in double; the parameter update in fp32
  const double st = (double)*T.step;
  const float bc1 = (float)(1.0 - pow(b1d, st)), bc2s = (float)sqrt(1.0 - pow(b2d, st));
  const float step_size = (float)(lr / (double)bc1);
  auto upd = [&](float& pp, float gg, float& mm, float& vv) {
    float gc = gg * coef;  // clip_grad_norm_'s in-place multiply
    if (wdd != 0.0) {
      if (decoupled) pp = (float)((double)pp - lr * wdd * (double)pp);
      else gc = (float)((double)gc + (double)pp * wdd);
    }
    mm = (float)(b1d * (double)mm + (1.0 - b1d) * (double)gc);
    vv = (float)(b2d * (double)vv + (1.0 - b2d) * (double)gc * (double)gc);
    const float denom = (float)((double)(sqrtf(vv) / bc2s) + epsd);
    pp -= step_size * mm / denom;
  };
  p += s0, g += s0, m += s0, v += s0;
  int done = 0;
  if (al16(p) && al16(g) && al16(m) && al16(v)) {
    const int n4 = len >> 2;
    for (int i = threadIdx.x; i < n4; i += 256) {
      float4 pv = reinterpret_cast<float4*>(p)[i], mv = reinterpret_cast<float4*>(m)[i],
             vv = reinterpret_cast<float4*>(v)[i];
      const float4 gv = reinterpret_cast<const float4*>(g)[i];
      upd(pv.x, gv.x, mv.x, vv.x);
      upd(pv.y, gv.y, mv.y, vv.y);
      upd(pv.z, gv.z, mv.z, vv.z);
      upd(pv.w, gv.w, mv.w, vv.w);
      reinterpret_cast<float4*>(p)[i] = pv;
      reinterpret_cast<float4*>(m)[i] = mv;
      reinterpret_cast<float4*>(v)[i] = vv;
    }
    done = 4 * n4;
  }
  for (int i = done + threadIdx.x; i < len; i += 256) {
    float pp = p[i], mm = m[i], vv = v[i];
    upd(pp, g[i], mm, vv);
    p[i] = pp, m[i] = mm, v[i] = vv;
  }
}

}  // namespace

int adam_chunks(int nt, const mdg_adam_tensor* t) {
  long long nc = 0;
  for (int i = 0; i < nt; ++i) {
    if (t[i].n <= 0) return -1;
    nc += (t[i].n + kAdamChunk - 1) / kAdamChunk;
  }
  return nc > (1 << 30) ? -1 : (int)nc;
}

size_t adam_table_bytes(int nt, int nc) { return (size_t)nt * sizeof(mdg_adam_tensor) + (size_t)2 * nc * sizeof(int); }

void adam_table_build(int nt, int nc, const mdg_adam_tensor* t, void* table) {
  std::memcpy(table, t, (size_t)nt * sizeof(mdg_adam_tensor));
  int* ct = reinterpret_cast<int*>(reinterpret_cast<mdg_adam_tensor*>(table) + nt);
  int* ci = ct + nc;
  int c = 0;
  for (int i = 0; i < nt; ++i)
    for (long long k = 0; k * kAdamChunk < t[i].n; ++k, ++c) ct[c] = i, ci[c] = (int)k;
}

size_t adam_ws_bytes(int nc) { return ((size_t)(nc + 1) * sizeof(float) + 255) / 256 * 256; }

hipError_t adam_step_launch(int nt, int nc, const void* table, double lr, double b1, double b2, double eps, double wd,
                            int decoupled, double max_norm, float* gnorm, float* ws, hipStream_t s) {
  hipLaunchKernelGGL(adam_norm_part_kernel, dim3(nc), dim3(256), 0, s, nt, nc, table, ws);
  hipLaunchKernelGGL(adam_norm_final_kernel, dim3(1), dim3(1024), 0, s, nt, nc, table, ws, (float)max_norm, gnorm);
  hipLaunchKernelGGL(adam_update_kernel, dim3(nc), dim3(256), 0, s, nt, nc, table, (const float*)ws, lr, b1, b2, eps, wd,
                     decoupled);
  return hipGetLastError();
}

}  // namespace mdg
