// clock_probe.hip -- the shader clock a kernel actually runs at, from
// s_memtime (shader clock) against s_memrealtime (constant 100 MHz), for
// full-chip FP64, 64-bit integer multiply-add and HBM-streaming loads (the
// NTT's three ingredients), at 1024-thread workgroups, one per CU.
// Timing-only microbenchmark (never shipped).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint64_t u64;

template <int MODE>
__global__ void __launch_bounds__(1024) probe(u64* __restrict__ out, u64* __restrict__ buf, int iters) {
  const u64 t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const int t = threadIdx.x;
  u64 acc = 0;
  if (MODE == 0) {  // FP64: 8 independent FMA chains
    double d[8];
    for (int i = 0; i < 8; ++i) d[i] = t + i;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = __builtin_fma(d[i], 1.0000001, 0.5);
    for (int i = 0; i < 8; ++i) acc += (u64)d[i];
  } else if (MODE == 1) {  // 64-bit integer multiply-add pieces (v_mad_u64_u32)
    u64 x[8];
    for (int i = 0; i < 8; ++i) x[i] = t * 2654435761u + i;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = (u64)(unsigned)x[i] * 0x9e3779b9u + (x[i] >> 32);
    for (int i = 0; i < 8; ++i) acc += x[i];
  } else if (MODE == 2) {  // streaming loads + stores, 256 KiB per workgroup per pass
    u64* p = buf + (size_t)blockIdx.x * 32768;
    for (int it = 0; it < iters; ++it) {
      u64 a[32];
#pragma unroll
      for (int k = 0; k < 32; ++k) a[k] = p[t + 1024 * k];
#pragma unroll
      for (int k = 0; k < 32; ++k) p[t + 1024 * k] = a[k] + 1;
    }
  } else {  // mostly idle: s_sleep
    for (int it = 0; it < iters; ++it) __builtin_amdgcn_s_sleep(64);
  }
  const u64 t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    out[blockIdx.x * 3 + 0] = t1 - t0;
    out[blockIdx.x * 3 + 1] = r1 - r0;
    out[blockIdx.x * 3 + 2] = acc;
  }
}

int main() {
  const int G = 256;
  u64 *out, *buf;
  (void)hipMalloc(&out, G * 3 * 8);
  (void)hipMalloc(&buf, (size_t)G * 32768 * 8);
  (void)hipMemset(buf, 0, (size_t)G * 32768 * 8);
  const char* names[] = {"fp64 fma", "int mad", "hbm stream", "s_sleep"};
  const int iters[] = {200000, 200000, 200, 20000};
  for (int mode = 0; mode < 4; ++mode) {
    for (int grid : {16, 256}) {
      for (int rep = 0; rep < 2; ++rep) {
        switch (mode) {
          case 0: hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(1024), 0, 0, out, buf, iters[mode]); break;
          case 1: hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(1024), 0, 0, out, buf, iters[mode]); break;
          case 2: hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(1024), 0, 0, out, buf, iters[mode]); break;
          case 3: hipLaunchKernelGGL(probe<3>, dim3(grid), dim3(1024), 0, 0, out, buf, iters[mode]); break;
        }
        (void)hipDeviceSynchronize();
      }
      u64 h[G * 3];
      (void)hipMemcpy(h, out, grid * 3 * 8, hipMemcpyDeviceToHost);
      double mhz = 0, us = 0;
      for (int b = 0; b < grid; ++b) {
        mhz += (double)h[3 * b] / ((double)h[3 * b + 1] / 100.0);
        us += h[3 * b + 1] / 100.0;
      }
      printf("%-11s grid %3d: shader clock %7.1f MHz (memtime/memrealtime), %8.1f us per workgroup\n", names[mode],
             grid, mhz / grid, us / grid);
    }
  }
  return 0;
}
