// half_wg.hip -- does splitting a limb over two 512-thread workgroups (two
// per CU, each reading the whole limb and writing its half) overlap memory
// with compute better than one 1024-thread workgroup per limb?
// Timing-only microbenchmark (never shipped).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint64_t u64;

__device__ __forceinline__ double spin_d(double d, int spin) {
  for (int i = 0; i < spin; ++i) d = __builtin_fma(d, 1.0000001, 0.5);
  return d;
}

// one 1024-thread WG per limb: 32 loads, spin, 32 stores (the current shape)
__global__ void __launch_bounds__(1024) full_wg(u64* __restrict__ src, u64* __restrict__ dst, int spin) {
  const int t = threadIdx.x;
  const u64* p = src + (size_t)blockIdx.x * 32768;
  u64* o = dst + (size_t)blockIdx.x * 32768;
  double a[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) a[k] = (double)(p[t + 1024 * k] & 0xfffff);
#pragma unroll
  for (int k = 0; k < 32; ++k) a[k] = spin_d(a[k], spin);
#pragma unroll
  for (int k = 0; k < 32; ++k) o[t + 1024 * k] = (u64)a[k];
}

// two 512-thread WGs per limb (blocks b, b+8 of a 16-block group share an XCD):
// each loads both halves (element e and e + 2^14), combines them, spins, and
// writes its half
__global__ void __launch_bounds__(512) half_wg(u64* __restrict__ src, u64* __restrict__ dst, int spin) {
  const int t = threadIdx.x;
  const int grp = blockIdx.x / 16, r = blockIdx.x % 16;
  const int h = r / 8, job = grp * 8 + (r % 8);
  const u64* p = src + (size_t)job * 32768;
  u64* o = dst + (size_t)job * 32768 + h * 16384;
  double a[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const double lo = (double)(p[t + 512 * k] & 0xfffff), hi = (double)(p[16384 + t + 512 * k] & 0xfffff);
    a[k] = h ? lo - hi : lo + hi;
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) a[k] = spin_d(a[k], spin);
#pragma unroll
  for (int k = 0; k < 32; ++k) o[t + 512 * k] = (u64)a[k];
}

int main() {
  const int jobs = 4096;
  u64 *s, *d;
  hipMalloc(&s, (size_t)jobs * 32768 * 8);
  hipMalloc(&d, (size_t)jobs * 32768 * 8);
  hipMemset(s, 1, (size_t)jobs * 32768 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int spin : {0, 25, 50, 100}) {
    for (int mode = 0; mode < 2; ++mode) {
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(full_wg, dim3(jobs), dim3(1024), 0, 0, s, d, spin);
        else hipLaunchKernelGGL(half_wg, dim3(2 * jobs), dim3(512), 0, 0, s, d, spin);
      };
      for (int i = 0; i < 3; ++i) launch();
      hipEventRecord(e0, 0);
      for (int i = 0; i < 10; ++i) launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 100.0;
      printf("%s spin %4d : %8.1f us/launch  %6.1f us per 256 limbs  %7.1f GB/s (16N/limb)\n",
             mode ? "half_wg" : "full_wg", spin, us, us / 16, 16.0 * 32768 * jobs / (us * 1e-6) / 1e9);
    }
  }
  return 0;
}
