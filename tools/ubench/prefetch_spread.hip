// prefetch_spread.hip -- does a CU overlap in-flight loads with its own VALU
// work, and does it matter how the loads are issued?  Timing-only
// microbenchmark (never shipped).  The compute phase has a workgroup barrier
// (no memory fence) every 8 elements, so the waves run in lockstep as they do
// in the NTT.
//
// Persistent grid (one 512-thread workgroup per CU) over 8192 jobs of 128 KiB
// (32 u64 per thread, element t + 512 k).  Per job: `spin` float64 FMAs per
// element on the current registers, then store them.
//   mode 0: the next job is loaded after the store (no overlap possible)
//   mode 1: the next job's 32 loads are issued in one burst before the compute
//   mode 2: the next job's loads are spread through the compute (one load
//           after each element's FMA chain)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint64_t u64;

__device__ __forceinline__ double spin_d(double d, int spin) {
  for (int i = 0; i < spin; ++i) d = __builtin_fma(d, 1.0000001, 0.5);
  return d;
}

template <int MODE>
__global__ void __launch_bounds__(512) k_job(const u64* __restrict__ src, u64* __restrict__ dst, int njob, int spin) {
  const int t = threadIdx.x;
  u64 a[32], b[32];
  int job = blockIdx.x;
  if (job >= njob) return;
#pragma unroll
  for (int k = 0; k < 32; ++k) a[k] = src[(size_t)job * 16384 + t + 512 * k];
  for (; job < njob; job += gridDim.x) {
    const int next = job + gridDim.x < njob ? job + gridDim.x : job;
    const u64* np = src + (size_t)next * 16384 + t;
    if (MODE == 1) {
#pragma unroll
      for (int k = 0; k < 32; ++k) b[k] = np[512 * k];
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      a[k] = (u64)spin_d((double)(a[k] & 0xfffff), spin) ^ a[k];
      if (MODE == 2) b[k] = np[512 * k];
      // lockstep waves like the NTT's exchanges: a barrier without a memory fence
      if ((k & 7) == 7) {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    }
    u64* o = dst + (size_t)job * 16384 + t;
#pragma unroll
    for (int k = 0; k < 32; ++k) o[512 * k] = a[k];
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 32; ++k) a[k] = np[512 * k];
    } else {
#pragma unroll
      for (int k = 0; k < 32; ++k) a[k] = b[k];
    }
  }
}

int main() {
  const int njob = 8192;
  u64 *s, *d;
  hipMalloc(&s, (size_t)njob * 16384 * 8);
  hipMalloc(&d, (size_t)njob * 16384 * 8);
  hipMemset(s, 1, (size_t)njob * 16384 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int spin : {0, 25, 50, 100}) {
    for (int mode = 0; mode < 3; ++mode) {
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(k_job<0>, dim3(256), dim3(512), 0, 0, s, d, njob, spin);
        if (mode == 1) hipLaunchKernelGGL(k_job<1>, dim3(256), dim3(512), 0, 0, s, d, njob, spin);
        if (mode == 2) hipLaunchKernelGGL(k_job<2>, dim3(256), dim3(512), 0, 0, s, d, njob, spin);
      };
      for (int i = 0; i < 2; ++i) launch();
      hipEventRecord(e0, 0);
      for (int i = 0; i < 5; ++i) launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1000.0 / 5;
      printf("mode %d spin %4d : %8.1f us/launch  %6.2f us per 256 jobs  %7.1f GB/s\n", mode, spin, us,
             us / (njob / 256.0), 2.0 * 131072.0 * njob / (us * 1e-6) / 1e9);
    }
  }
  return 0;
}
