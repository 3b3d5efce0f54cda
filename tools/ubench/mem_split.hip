// mem_split.hip -- which half of the NTT's memory phase caps one CU at
// ~20-26 GB/s (profiles/r02_ubench_mem_phase.txt): the 256 KiB of loads or
// the 256 KiB of stores?  Timing-only microbenchmark (never shipped).
//
// 1024-thread workgroup per limb (N = 2^15 u64), element t + 1024 k (the
// one-pass NTT's coalesced layout) or 16-B accesses (2 consecutive elements).
//   mode 0: load 32 u64 per thread, store one u64 (xor) per thread
//   mode 1: store 32 u64 per thread (computed from t)
//   mode 2: load + store (the NTT's memory phase)
//   mode 3: store only, non-temporal
//   mode 4: load + non-temporal store
//   mode 5/6/7: as 0/1/2 with 16-B accesses
// G workgroups over G limbs: G = 16 (HBM idle: per-CU cap), 256 (one round), 4096.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint64_t u64;

template <int MODE>
__global__ void __launch_bounds__(1024) k_mem(u64* __restrict__ src, u64* __restrict__ dst, u64* __restrict__ sink) {
  const int t = threadIdx.x;
  const u64* p = src + (size_t)blockIdx.x * 32768;
  u64* o = dst + (size_t)blockIdx.x * 32768;
  u64 a[32];
  constexpr bool W16 = MODE >= 5;
  constexpr int M = W16 ? MODE - 5 : MODE;
  if (M == 0 || M == 2 || M == 4) {
    if (W16) {
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
  } else {
#pragma unroll
    for (int k = 0; k < 32; ++k) a[k] = (u64)t * 2654435761u + k;
  }
  if (M == 0) {
    u64 x = 0;
#pragma unroll
    for (int k = 0; k < 32; ++k) x ^= a[k];
    sink[(size_t)blockIdx.x * 1024 + t] = x;
    return;
  }
  if (W16) {
#pragma unroll
    for (int k = 0; k < 32; k += 2) *(ulonglong2*)(o + t * 32 + k) = make_ulonglong2(a[k] + 1, a[k + 1] + 1);
  } else if (M == 3 || M == 4) {
#pragma unroll
    for (int k = 0; k < 32; ++k) __builtin_nontemporal_store(a[k] + 1, o + t + 1024 * k);
  } else {
#pragma unroll
    for (int k = 0; k < 32; ++k) o[t + 1024 * k] = a[k] + 1;
  }
}

int main() {
  const int maxl = 4096;
  u64 *s, *d, *sink;
  hipMalloc(&s, (size_t)maxl * 32768 * 8);
  hipMalloc(&d, (size_t)maxl * 32768 * 8);
  hipMalloc(&sink, (size_t)maxl * 1024 * 8);
  hipMemset(s, 1, (size_t)maxl * 32768 * 8);
  hipMemset(d, 1, (size_t)maxl * 32768 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"load-only", "store-only", "load+store", "store-only nt", "load+store nt",
                         "load-only 16B", "store-only 16B", "load+store 16B"};
  auto run = [&](int mode, int G) {
    auto launch = [&]() {
      switch (mode) {
        case 0: hipLaunchKernelGGL(k_mem<0>, dim3(G), dim3(1024), 0, 0, s, d, sink); break;
        case 1: hipLaunchKernelGGL(k_mem<1>, dim3(G), dim3(1024), 0, 0, s, d, sink); break;
        case 2: hipLaunchKernelGGL(k_mem<2>, dim3(G), dim3(1024), 0, 0, s, d, sink); break;
        case 3: hipLaunchKernelGGL(k_mem<3>, dim3(G), dim3(1024), 0, 0, s, d, sink); break;
        case 4: hipLaunchKernelGGL(k_mem<4>, dim3(G), dim3(1024), 0, 0, s, d, sink); break;
        case 5: hipLaunchKernelGGL(k_mem<5>, dim3(G), dim3(1024), 0, 0, s, d, sink); break;
        case 6: hipLaunchKernelGGL(k_mem<6>, dim3(G), dim3(1024), 0, 0, s, d, sink); break;
        case 7: hipLaunchKernelGGL(k_mem<7>, dim3(G), dim3(1024), 0, 0, s, d, sink); break;
      }
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
    const int M = mode >= 5 ? mode - 5 : mode;
    const double bytes = (M == 2 || M == 4 ? 16.0 : 8.0) * 32768;  // per limb
    const double rounds = G > 256 ? G / 256.0 : 1.0;
    printf("%-15s G %5d : %8.1f us/launch  %6.1f us per round  %7.1f GB/s chip  %6.1f GB/s per CU\n", names[mode], G,
           us, us / rounds, bytes * G / (us * 1e-6) / 1e9, bytes / (us / rounds * 1e-6) / 1e9);
  };
  // an empty-ish launch for the fixed cost
  for (int mode = 0; mode < 8; ++mode)
    for (int G : {16, 256, 4096}) run(mode, G);
  hipFree(s);
  hipFree(d);
  hipFree(sink);
  return 0;
}
