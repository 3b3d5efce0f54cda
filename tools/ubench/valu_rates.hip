// Microbenchmark: issue rate of 64-bit integer multiply pieces vs FP64 on gfx950.
// Each thread runs 8 independent chains; reports wave-instructions per cycle per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096
template <int OP>
__global__ void __launch_bounds__(256) k(uint64_t* out, uint64_t seed) {
  uint64_t a[8];
  double d[8];
  uint32_t u[8];
  for (int i = 0; i < 8; ++i) { a[i] = seed * (threadIdx.x + i + 1); d[i] = (double)(a[i] & 0xfffffff); u[i] = (uint32_t)a[i]; }
  const uint64_t m = seed | 1;
  const uint32_t m32 = (uint32_t)m;
  const double dm = 1.0000001;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) { uint64_t r; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(u[i]), "v"(m32)); }
      if (OP == 1) { asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(m32)); }
      if (OP == 2) { asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[i]) : "v"(m32)); }
      if (OP == 3) { asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(dm)); }
      if (OP == 4) { asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(m32)); }
      if (OP == 5) { asm volatile("v_rndne_f64 %0, %0" : "+v"(d[i])); }
      if (OP == 6) { asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(dm)); }
      if (OP == 7) { asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(a[(i+1)&7])); }
      if (OP == 8) { asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[i]) : "v"(u[i])); asm volatile("" : "+v"(u[i])); }
    }
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s += a[i] + (uint64_t)d[i] + u[i];
  if (s == 42) out[0] = s;
}

int main() {
  uint64_t* out; hipMalloc(&out, 8);
  const char* names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_fma_f64", "v_add_u32", "v_rndne_f64", "v_mul_f64", "v_lshl_add_u64", "v_cvt_f64_u32"};
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  int cus = p.multiProcessorCount; double clk = p.clockRate * 1e3;
  for (int op = 0; op < 9; ++op) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int blocks = cus * 8;  // 8 blocks x 256 threads per CU = 32 waves/CU
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      switch (op) {
        case 0: hipLaunchKernelGGL(k<0>, blocks, 256, 0, 0, out, 7); break;
        case 1: hipLaunchKernelGGL(k<1>, blocks, 256, 0, 0, out, 7); break;
        case 2: hipLaunchKernelGGL(k<2>, blocks, 256, 0, 0, out, 7); break;
        case 3: hipLaunchKernelGGL(k<3>, blocks, 256, 0, 0, out, 7); break;
        case 4: hipLaunchKernelGGL(k<4>, blocks, 256, 0, 0, out, 7); break;
        case 5: hipLaunchKernelGGL(k<5>, blocks, 256, 0, 0, out, 7); break;
        case 6: hipLaunchKernelGGL(k<6>, blocks, 256, 0, 0, out, 7); break;
        case 7: hipLaunchKernelGGL(k<7>, blocks, 256, 0, 0, out, 7); break;
        case 8: hipLaunchKernelGGL(k<8>, blocks, 256, 0, 0, out, 7); break;
      }
      hipEventRecord(e1); hipEventSynchronize(e1);
    }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double waveinstr = (double)blocks * 4 * ITERS * 8;  // 4 waves per block
    double per_cu_cycle = waveinstr / cus / (ms * 1e-3 * clk);
    printf("%-16s %8.3f ms  wave-instr/cycle/CU = %.3f  (cycles per wave-instr per SIMD = %.2f)\n", names[op], ms, per_cu_cycle, 4.0 / per_cu_cycle);
  }
  printf("CUs %d clock %.0f MHz\n", cus, clk / 1e6);
  return 0;
}
