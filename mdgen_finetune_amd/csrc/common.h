// Shared device helpers for the MDGen denoiser kernels (gfx950 / CDNA4 only).
//
// Compute-type convention: every kernel is templated on CT, the operand type fed to the
// matrix cores — `float` (exact-f32 MFMA v_mfma_f32_16x16x4_f32: the fp32 parity path) or
// `__bf16` (v_mfma_f32_16x16x32_bf16: the performance path).  Accumulation, softmax,
// LayerNorm statistics and the residual stream are always fp32.
//
// Fragment convention (one 16x16 output tile, K = 32 per step): lane l holds 8 consecutive
// K-elements  [8*(l>>4), 8*(l>>4)+8)  of row (l & 15) for both the A and the B operand.
// For bf16 that is exactly the 16x16x32 operand map; for f32 the 8 elements feed 8
// consecutive 16x16x4 MFMAs (MFMA j reads element j of every lane, i.e. k = 8g + j for lane
// group g), which sums the same 32 products.  The C/D map is the same for both:
//   row = 4*(l>>4) + i (i = register 0..3), col = l & 15.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/mdgen_hip.h"

typedef __bf16 bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) float f32x8;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

template <typename CT> struct V8;
template <> struct V8<bf16_t> { using T = bf16x8; };
template <> struct V8<float> { using T = f32x8; };

template <typename CT> __device__ __forceinline__ constexpr bool is_bf16() {
  return std::is_same<CT, bf16_t>::value;
}

// 8 consecutive CT elements from a 16-byte aligned address (LDS or global).
template <typename CT>
__device__ __forceinline__ typename V8<CT>::T ld8(const CT* p) {
  if constexpr (is_bf16<CT>()) {
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    const float4 a = reinterpret_cast<const float4*>(p)[0];
    const float4 b = reinterpret_cast<const float4*>(p)[1];
    f32x8 r;
    r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
    r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
    return r;
  }
}

template <typename CT>
__device__ __forceinline__ typename V8<CT>::T zero8() {
  typename V8<CT>::T r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (CT)0.0f;
  return r;
}

// acc += A(16x32) * B(32x16) in the fragment convention above.
template <typename CT>
__device__ __forceinline__ void mma_k32(f32x4& acc, const typename V8<CT>::T& a,
                                        const typename V8<CT>::T& b) {
  if constexpr (is_bf16<CT>()) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
  }
}

// Store 4 fp32 values as 4 CT (8 B for bf16, 16 B for f32); p must be aligned accordingly.
template <typename CT>
__device__ __forceinline__ void st4(CT* p, float a, float b, float c, float d) {
  if constexpr (is_bf16<CT>()) {
    bf16x4 v;
    v[0] = (bf16_t)a; v[1] = (bf16_t)b; v[2] = (bf16_t)c; v[3] = (bf16_t)d;
    *reinterpret_cast<bf16x4*>(p) = v;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
  }
}

// Store 8 CT (16 B for bf16, 32 B for f32); p aligned accordingly.
template <typename CT>
__device__ __forceinline__ void st8(CT* p, const typename V8<CT>::T& v) {
  if constexpr (is_bf16<CT>()) {
    *reinterpret_cast<bf16x8*>(p) = v;
  } else {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
}

template <typename CT>
__device__ __forceinline__ float4 ld4f(const CT* p) {
  if constexpr (is_bf16<CT>()) {
    const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
    return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
  } else {
    return *reinterpret_cast<const float4*>(p);
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float gelu_erf(float x) {
  // exact-erf GELU (reference layers.py:78-85)
  return x * 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
}

// exact-erf GELU via erfc(a) = t*poly(t)*exp(-a^2), t = 1/(1 + p a)  (Abramowitz & Stegun
// 7.1.26, |error| <= 1.5e-7 absolute on erf): 1 rcp + 1 exp + 6 FMAs instead of the
// multi-range ocml erff.  Used where the result is rounded to bf16.
__device__ __forceinline__ float gelu_fast(float x) {
  const float a = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float q = fmaf(1.061405429f, t, -1.453152027f);
  q = fmaf(q, t, 1.421413741f);
  q = fmaf(q, t, -0.284496736f);
  q = fmaf(q, t, 0.254829592f);
  q *= t * __builtin_amdgcn_exp2f(-a * a * 1.4426950408889634f);  // erfc(|x|/sqrt2)
  return x >= 0.f ? x * (1.0f - 0.5f * q) : x * (0.5f * q);
}

// gelu_fast on two values with packed fp32 math (v_pk_mul / v_pk_fma / v_pk_add: two lanes'
// worth of work per instruction; the reciprocal and exp2 stay scalar).  The same IEEE operations
// in the same order as gelu_fast, so the results are bit-identical to it (1 - 0.5 q: 0.5 q is
// exact, so the fused and the separate forms round alike).
typedef __attribute__((ext_vector_type(2))) float f32x2v;
__device__ __forceinline__ f32x2v gelu_fast2(f32x2v x) {
#pragma clang fp contract(off)
  const f32x2v a = __builtin_elementwise_abs(x) * 0.70710678118654752440f;
  const f32x2v d = __builtin_elementwise_fma(f32x2v{0.3275911f, 0.3275911f}, a, f32x2v{1.0f, 1.0f});
  const f32x2v t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2v q = __builtin_elementwise_fma(f32x2v{1.061405429f, 1.061405429f}, t, f32x2v{-1.453152027f, -1.453152027f});
  q = __builtin_elementwise_fma(q, t, f32x2v{1.421413741f, 1.421413741f});
  q = __builtin_elementwise_fma(q, t, f32x2v{-0.284496736f, -0.284496736f});
  q = __builtin_elementwise_fma(q, t, f32x2v{0.254829592f, 0.254829592f});
  const f32x2v s = ((-a) * a) * 1.4426950408889634f;
  const f32x2v e = {__builtin_amdgcn_exp2f(s.x), __builtin_amdgcn_exp2f(s.y)};
  q = q * (t * e);
  const f32x2v h = 0.5f * q;
  const f32x2v p = 1.0f - h;
  const f32x2v m = {x.x >= 0.f ? p.x : h.x, x.y >= 0.f ? p.y : h.y};
  return x * m;
}

// d/dx of the exact-erf GELU: Phi(x) + x phi(x)  (the training backward of layers.py:78-85)
__device__ __forceinline__ float gelu_grad(float x) {
  return 0.5f * (1.0f + erff(x * 0.70710678118654752440f)) + x * 0.39894228040143267794f * expf(-0.5f * x * x);
}

// the same with Phi from the A&S erfc of gelu_fast (bf16 path: the derivative of what the
// forward computed)
__device__ __forceinline__ float gelu_grad_fast(float x) {
  const float a = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float q = fmaf(1.061405429f, t, -1.453152027f);
  q = fmaf(q, t, 1.421413741f);
  q = fmaf(q, t, -0.284496736f);
  q = fmaf(q, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-a * a * 1.4426950408889634f);  // exp(-x^2/2)
  q *= t * e;                                                             // erfc(|x|/sqrt2)
  const float phi_cdf = x >= 0.f ? 1.0f - 0.5f * q : 0.5f * q;
  return phi_cdf + x * 0.39894228040143267794f * e;
}

__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// row stride of the padded attention operands (planes, bias_kv rows) for head dim D
__host__ __device__ constexpr int dp_of(int D) { return MDG_HEAD_STRIDE(D); }

// One dword from / to an address that is only 4-B aligned (rows of 3-, 7-, 9-, 14- or 21-float
// records).  A relaxed workgroup-scope atomic is a plain global_load_dword / global_store_dword,
// but the load-store vectoriser never merges it, so no dwordx2/x3/x4 access is formed at an
// alignment below its size ("Concurrent-lane divergence").
__device__ __forceinline__ float ld1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
