// Microbenchmark (diagnostic, not product): the L2 -> LDS fill rate of global_load_lds_dwordx4
// with every CU streaming, as a function of the bytes each block keeps in flight.  One block of
// 512 threads per CU; each step every thread issues PIECES 16-B loads into ring slot (step %
// DEPTH); the wave waits until only the younger DEPTH - 1 steps are outstanding.  The source is a
// window of `window` bytes (L2-resident when small), offset per block and step.
#include <hip/hip_runtime.h>

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int DEPTH, int PIECES>
__global__ __launch_bounds__(512, 1) void l2lds_kernel(const char* __restrict__ src, unsigned long long wmask,
                                                        int steps, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int SLOT = 512 * 16 * PIECES;
  const int tid = threadIdx.x;
  for (int s = 0; s < steps; ++s) {
    const unsigned long long base = ((unsigned long long)blockIdx.x * 7919ull + (unsigned long long)s * SLOT) & wmask;
    char* sl = lds + (s % DEPTH) * SLOT;
#pragma unroll
    for (int p = 0; p < PIECES; ++p) {
      const unsigned long long off = (base + (unsigned long long)(p * 512 + tid) * 16) & wmask;
      __builtin_amdgcn_global_load_lds((const void*)(src + off), (lds_ptr_t)(sl + (p * 512 + (tid & ~63)) * 16), 16, 0, 0);
    }
    if (s >= DEPTH - 1) {
      // steps s - DEPTH + 2 .. s may stay in flight
      if constexpr (DEPTH == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES) : "memory");
      else if constexpr (DEPTH == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PIECES) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(7 * PIECES) : "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0 && lds[blockIdx.x & 1023] == 123) sink[0] = 1;
}

// the same stream into VGPRs (global_load_dwordx4), optionally written on to LDS (ds_write_b128)
template <int DEPTH, int PIECES, bool TOLDS>
__global__ __launch_bounds__(512, 1) void l2vgpr_kernel(const char* __restrict__ src, unsigned long long wmask,
                                                         int steps, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int SLOT = 512 * 16 * PIECES;
  const int tid = threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  uint4 r[DEPTH][PIECES];
  for (int s0 = 0; s0 < steps; s0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const unsigned long long base = ((unsigned long long)blockIdx.x * 7919ull + (unsigned long long)(s0 + d) * SLOT) & wmask;
#pragma unroll
      for (int p = 0; p < PIECES; ++p)
        r[d][p] = *reinterpret_cast<const uint4*>(src + ((base + (unsigned long long)(p * 512 + tid) * 16) & wmask & ~15ull));
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int p = 0; p < PIECES; ++p) {
        if (TOLDS) *reinterpret_cast<uint4*>(lds + (d % 2) * SLOT + (p * 512 + tid) * 16) = r[d][p];
        else { acc.x ^= r[d][p].x; acc.y ^= r[d][p].y; acc.z ^= r[d][p].z; acc.w ^= r[d][p].w; }
      }
  }
  __syncthreads();
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345 || (tid == 0 && lds[blockIdx.x & 1023] == 123)) sink[0] = 1;
}

extern "C" int l2vgpr_run(const void* src, unsigned long long window, int steps, int tolds, int blocks, int* sink,
                          float* ms) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const size_t smem = 2 * 512 * 16 * 4;
  auto launch = [&]() -> hipError_t {
    if (tolds) {
      (void)hipFuncSetAttribute((const void*)&l2vgpr_kernel<4, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      hipLaunchKernelGGL((l2vgpr_kernel<4, 4, true>), dim3(blocks), dim3(512), smem, 0, (const char*)src, window - 1, steps, sink);
    } else {
      hipLaunchKernelGGL((l2vgpr_kernel<4, 4, false>), dim3(blocks), dim3(512), 0, 0, (const char*)src, window - 1, steps, sink);
    }
    return hipGetLastError();
  };
  if (launch() != hipSuccess) return 1;
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < 5; ++i)
    if (launch() != hipSuccess) return 1;
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(ms, a, b);
  *ms /= 5;
  return 0;
}

extern "C" int l2lds_run(const void* src, unsigned long long window, int steps, int depth, int pieces, int blocks,
                         int* sink, float* ms) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const size_t smem = (size_t)depth * 512 * 16 * pieces;
  auto launch = [&]() -> hipError_t {
#define L2L(D, P)                                                                                          \
  if (depth == D && pieces == P) {                                                                        \
    hipFuncSetAttribute((const void*)&l2lds_kernel<D, P>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
    hipLaunchKernelGGL((l2lds_kernel<D, P>), dim3(blocks), dim3(512), smem, 0, (const char*)src, window - 1, steps, sink); \
    return hipGetLastError();                                                                              \
  }
    L2L(2, 2) L2L(2, 4) L2L(4, 2) L2L(4, 4) L2L(8, 2) L2L(8, 4)
#undef L2L
    return hipErrorInvalidValue;
  };
  if (smem > 160 * 1024) return 2;
  if (launch() != hipSuccess) return 1;
  hipEventRecord(a, 0);
  for (int i = 0; i < 5; ++i)
    if (launch() != hipSuccess) return 1;
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  hipEventElapsedTime(ms, a, b);
  *ms /= 5;
  hipEventDestroy(a);
  hipEventDestroy(b);
  return 0;
}
