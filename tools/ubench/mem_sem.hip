// mem_sem.hip -- can the NTT's memory and compute phases overlap ACROSS CUs if
// the number of CUs in their memory phase at once is capped?
// Timing-only microbenchmark (never shipped).
//
// Persistent grid of 256 workgroups x 1024 threads walks `nlimb` 256 KiB limbs
// in the one-pass NTT's layout (thread t holds elements t + 1024 k, k < 32).
// Per job: [acquire] store the previous job's limb, load this job's limb,
// wait for the loads [release], then a lockstep compute phase (`spin` FP64
// FMAs per element in blocks of 4 elements with a workgroup barrier between
// blocks, like the NTT's exchanges).  The semaphore is one counter per XCD
// (workgroups go round-robin over the 8 XCDs), `limit` memory phases per XCD
// (0 = no semaphore).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint64_t u64;

// FIFO ticket semaphore per XCD: sem[x*64] = next ticket, sem[x*64+32] = tickets served;
// a workgroup holding ticket t enters once t < served + limit.  Bounded poll (the
// kernel always ends; a workgroup that gives up only admits one extra holder).
__device__ __forceinline__ void sem_acquire(unsigned* s, int limit) {
  if (threadIdx.x == 0) {
    const unsigned t = atomicAdd(s, 1u);
    for (int tries = 0; tries < (1 << 20); ++tries) {
      const unsigned served = __hip_atomic_load(s + 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)(t - served) < limit) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}
__device__ __forceinline__ void sem_release(unsigned* s) {
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(s + 32, 1u);
}

__global__ void __launch_bounds__(1024) job_kernel(u64* __restrict__ buf, int nlimb, int spin, int limit,
                                                   unsigned* sem, int stagger) {
  const int t = threadIdx.x;
  if (blockIdx.x & 8)  // the stagger alternative: half of each XCD's CUs start late
    for (int i = 0; i < stagger; ++i) __builtin_amdgcn_s_sleep(127);
  unsigned* s = sem + (blockIdx.x & 7) * 64;
  u64 a[32];
  int prev = -1;
  for (int j = blockIdx.x; j < nlimb; j += gridDim.x) {
    if (limit > 0) sem_acquire(s, limit);
    if (prev >= 0) {
      u64* q = buf + (size_t)prev * 32768;
#pragma unroll
      for (int k = 0; k < 32; ++k) q[t + 1024 * k] = a[k];
    }
    const u64* p = buf + (size_t)j * 32768;
#pragma unroll
    for (int k = 0; k < 32; ++k) a[k] = p[t + 1024 * k];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (limit > 0) sem_release(s);
    else __syncthreads();
#pragma unroll
    for (int k = 0; k < 32; k += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        double d = (double)(a[k + u] & 0xffffff);
        for (int i = 0; i < spin; ++i) d = __builtin_fma(d, 1.0000001, 0.5);
        a[k + u] ^= (u64)(d > 1e300);
      }
      __syncthreads();
    }
    prev = j;
  }
  if (prev >= 0) {
    if (limit > 0) sem_acquire(s, limit);
    u64* q = buf + (size_t)prev * 32768;
#pragma unroll
    for (int k = 0; k < 32; ++k) q[t + 1024 * k] = a[k];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (limit > 0) sem_release(s);
  }
}

int main() {
  const int nl = 4096;
  u64* d;
  unsigned* sem;
  hipMalloc(&d, (size_t)nl * 32768 * 8);
  hipMemset(d, 1, (size_t)nl * 32768 * 8);
  hipMalloc(&sem, 8 * 64 * sizeof(unsigned));
  hipMemset(sem, 0, 8 * 64 * sizeof(unsigned));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  auto run = [&](int G, int spin, int limit, int stagger) {
    for (int i = 0; i < 2; ++i)
      hipLaunchKernelGGL(job_kernel, dim3(G), dim3(1024), 0, 0, d, nl, spin, limit, sem, stagger);
    hipEventRecord(e0, 0);
    const int reps = 5;
    for (int i = 0; i < reps; ++i)
      hipLaunchKernelGGL(job_kernel, dim3(G), dim3(1024), 0, 0, d, nl, spin, limit, sem, stagger);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    printf("G %3d spin %4d limit/XCD %3d stagger %3d : %8.1f us/launch  %6.1f us per job per CU  %6.1f us per 256 limbs  "
           "%7.1f GB/s\n", G, spin, limit, stagger, us, us / ((double)nl / G), us / (nl / 256.0),
           16.0 * 32768 * nl / (us * 1e-6) / 1e9);
    fflush(stdout);
  };
  printf("CUs %d, %d limbs of 256 KiB, persistent grid G\n", ncu, nl);
  // per-CU memory phase against the number of CUs streaming at once
  for (int G : {8, 16, 32, 64, 128, 192, 256}) run(G, 0, 0, 0);
  for (int spin : {0, 40, 80}) {
    for (int limit : {0, 24, 16, 12, 8, 6, 4}) run(ncu, spin, limit, 0);
    for (int stagger : {2, 5}) run(ncu, spin, 0, stagger);
  }
  unsigned h[8 * 64];
  hipMemcpy(h, sem, sizeof(h), hipMemcpyDeviceToHost);
  printf("tickets next - served per XCD (must be 0):");
  for (int x = 0; x < 8; ++x) printf(" %d", (int)(h[x * 64] - h[x * 64 + 32]));
  printf("\n");
  hipFree(d);
  hipFree(sem);
  return 0;
}
