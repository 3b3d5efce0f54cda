// ubench_valu.hip -- issue throughput of the VALU instructions the modular
// arithmetic is built from, on gfx950 (the cost model behind the choice of
// integer vs float64 paths in ntt_arith.h / kernels.hip).
//
// Each kernel runs ITER iterations of 8 independent chains of one instruction
// (inline asm, so the compiler can neither fold nor reschedule them) on a full
// grid; the result is wave-instructions per SIMD-cycle relative to a 32-bit add.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o tools/_ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);     \
      return 1;                                                            \
    }                                                                      \
  } while (0)

constexpr int ITER = 4096;

#define CHAIN8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

__global__ void k_add_u32(unsigned* out, unsigned seed) {
  unsigned a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + seed;
  const unsigned b = seed * 3 + 1;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  unsigned r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_lo_u32(unsigned* out, unsigned seed) {
  unsigned a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + seed;
  const unsigned b = seed * 3 + 1;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  unsigned r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_hi_u32(unsigned* out, unsigned seed) {
  unsigned a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + seed;
  const unsigned b = seed * 3 + 1;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_mul_hi_u32 %0, %1, %0" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  unsigned r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_u32_u24(unsigned* out, unsigned seed) {
  unsigned a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + seed;
  const unsigned b = seed * 3 + 1;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(a[i]) : "v"(b));
    CHAIN8(S)
#undef S
  }
  unsigned r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad_u64_u32(unsigned* out, unsigned seed) {
  uint64_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + seed;
  const unsigned b = seed * 3 + 1, c = seed ^ 0x5555;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c) : "vcc");
    CHAIN8(S)
#undef S
  }
  uint64_t r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(r ^ (r >> 32));
}

__global__ void k_fma_f64(unsigned* out, unsigned seed) {
  double a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + seed;
  const double b = 0.999 + seed * 1e-9, c = 1e-3;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_fma_f64 %0, %1, %0, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    CHAIN8(S)
#undef S
  }
  double r = 0;
  for (int i = 0; i < 8; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)r;
}

__global__ void k_fma_f32(unsigned* out, unsigned seed) {
  float a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + seed;
  const float b = 0.999f, c = 1e-3f;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_fma_f32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    CHAIN8(S)
#undef S
  }
  float r = 0;
  for (int i = 0; i < 8; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)r;
}

__global__ void k_cvt_f64_u32(unsigned* out, unsigned seed) {
  double a[8];
  unsigned x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i + seed, a[i] = 0;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(a[i]) : "v"(x[i]));
    CHAIN8(S)
#undef S
  }
  double r = 0;
  for (int i = 0; i < 8; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)r;
}

__global__ void k_add_co_u32(unsigned* out, unsigned seed) {
  unsigned a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + seed;
  const unsigned b = seed * 3 + 1;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_add_co_u32 %0, vcc, %1, %0" : "+v"(a[i]) : "v"(b) : "vcc");
    CHAIN8(S)
#undef S
  }
  unsigned r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_lshl_b64(unsigned* out, unsigned seed) {
  uint64_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + seed;
  const unsigned sh = seed & 1;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(a[i]) : "v"(sh));
    CHAIN8(S)
#undef S
  }
  uint64_t r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(r ^ (r >> 32));
}

__global__ void k_cmp_u64(unsigned* out, unsigned seed) {
  uint64_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + seed;
  const uint64_t b = seed * 7ull;
  unsigned cnt = 0;
  for (int it = 0; it < ITER; ++it) {
#define S(i) asm volatile("v_cmp_ge_u64 vcc, %0, %1" : : "v"(a[i]), "v"(b) : "vcc");
    CHAIN8(S)
#undef S
  }
  uint64_t r = cnt;
  for (int i = 0; i < 8; ++i) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(r ^ (r >> 32));
}

typedef void (*Kern)(unsigned*, unsigned);

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const double clk = p.clockRate * 1e3;  // Hz
  const int block = 256, blocks = cus * 8;  // 8 waves per SIMD
  unsigned* out;
  CHK(hipMalloc(&out, (size_t)blocks * block * 4));
  struct {
    const char* name;
    Kern k;
  } ks[] = {{"v_add_u32", k_add_u32},         {"v_add_co_u32", k_add_co_u32},   {"v_mul_lo_u32", k_mul_lo_u32},
            {"v_mul_hi_u32", k_mul_hi_u32},   {"v_mul_u32_u24", k_mul_u32_u24}, {"v_mad_u64_u32", k_mad_u64_u32},
            {"v_fma_f32", k_fma_f32},         {"v_fma_f64", k_fma_f64},         {"v_cvt_f64_u32", k_cvt_f64_u32},
            {"v_lshlrev_b64", k_lshl_b64},    {"v_cmp_ge_u64", k_cmp_u64}};
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  printf("CUs %d, clock %.0f MHz, grid %d x %d, %d instructions per lane per kernel\n", cus, clk / 1e6, blocks, block,
         ITER * 8);
  double base = 0;
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(block), 0, 0, out, 1u);  // warm-up
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(block), 0, 0, out, 1u);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    const double waves = (double)blocks * block / 64;
    const double winst = waves * ITER * 8;                 // wave-instructions
    const double simd_cycles = best * 1e-3 * clk * cus * 4;  // SIMD-cycles available
    const double cyc_per = simd_cycles / winst;            // SIMD cycles per wave-instruction
    if (base == 0) base = cyc_per;
    printf("%-16s %8.3f ms  %6.2f SIMD-cycles per wave-instruction  (%.2fx v_add_u32)\n", k.name, best, cyc_per,
           cyc_per / base);
  }
  CHK(hipFree(out));
  return 0;
}
