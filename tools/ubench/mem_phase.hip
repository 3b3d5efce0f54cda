// mem_phase.hip -- how long does one CU take to stream a 256 KiB limb in and
// out (the NTT's memory phase), and does it overlap other CUs' compute?
// Timing-only microbenchmark (never shipped).
//
// kernel: 1024 threads; each thread loads 32 u64 (element t + 1024 k, the
// one-pass NTT's layout), spins `spin` VALU iterations on them (a stand-in for
// the butterflies), stores them back.  Grid G workgroups over G limbs.
//   G <= 256      : one round, per-CU time at G concurrent CUs
//   G = 4096      : 16 rounds, steady state
//   mode 1: 16-B loads/stores (two consecutive elements per access)
//   mode 2: persistent (256 WGs loop over the limbs; next limb loaded right
//           after the stores are issued)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>

typedef uint64_t u64;

__device__ __forceinline__ u64 spin_op(u64 x, int spin) {
  double d = (double)(x & 0xffffff);
  for (int i = 0; i < spin; ++i) d = __builtin_fma(d, 1.0000001, 0.5);
  return x ^ (u64)(d > 1e300);
}

template <int MODE>
__global__ void __launch_bounds__(1024) mem_kernel(u64* __restrict__ buf, int nlimb, int spin) {
  const int t = threadIdx.x;
  for (int j = blockIdx.x; j < nlimb; j += (MODE == 2 ? gridDim.x : nlimb)) {
    u64* p = buf + (size_t)j * 32768;
    u64 a[32];
    if (MODE == 1) {
#pragma unroll
      for (int k = 0; k < 32; k += 2) {
        const ulonglong2 v = *(const ulonglong2*)(p + t * 32 + k);
        a[k] = v.x;
        a[k + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 32; ++k) a[k] = p[t + 1024 * k];
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) a[k] = spin_op(a[k], spin);
    if (MODE == 1) {
#pragma unroll
      for (int k = 0; k < 32; k += 2) *(ulonglong2*)(p + t * 32 + k) = make_ulonglong2(a[k], a[k + 1]);
    } else {
#pragma unroll
      for (int k = 0; k < 32; ++k) p[t + 1024 * k] = a[k];
    }
    if (MODE != 2) break;
  }
}

int main() {
  const int maxl = 4096;
  u64* d;
  hipMalloc(&d, (size_t)maxl * 32768 * 8);
  hipMemset(d, 1, (size_t)maxl * 32768 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](int mode, int G, int nl, int spin) {
    auto launch = [&]() {
      if (mode == 0) hipLaunchKernelGGL(mem_kernel<0>, dim3(G), dim3(1024), 0, 0, d, nl, spin);
      if (mode == 1) hipLaunchKernelGGL(mem_kernel<1>, dim3(G), dim3(1024), 0, 0, d, nl, spin);
      if (mode == 2) hipLaunchKernelGGL(mem_kernel<2>, dim3(G), dim3(1024), 0, 0, d, nl, spin);
    };
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(e0, 0);
    const int reps = 10;
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    const double rounds = (double)nl / 256.0;
    printf("mode %d G %5d limbs %5d spin %5d : %8.1f us/launch  %6.1f us per 256 limbs  %7.1f GB/s\n", mode, G, nl,
           spin, us, us / (rounds < 1 ? 1 : rounds), 16.0 * 32768 * nl / (us * 1e-6) / 1e9);
  };
  for (int mode = 0; mode < 2; ++mode) {
    for (int G : {16, 64, 128, 256}) run(mode, G, G, 0);
    run(mode, 4096, 4096, 0);
  }
  for (int spin : {0, 50, 100, 200, 400}) {
    run(0, 256, 256, spin);
    run(0, 4096, 4096, spin);
    run(2, 256, 4096, spin);
  }
  hipFree(d);
  return 0;
}
