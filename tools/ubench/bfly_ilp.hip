// bfly_ilp.hip -- compute-only throughput of the float64 NTT butterfly network
// on registers: 1024 threads x 32 values (4 waves/SIMD) vs 512 threads x 64
// values (2 waves/SIMD), with G butterflies per scheduling region (G = 1: one
// dependent chain at a time per wave; G = 2/4: interleaved chains).
// Timing-only microbenchmark (never shipped).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define PIN(x, y) asm volatile("" : "+v"(x), "+v"(y))

__device__ __forceinline__ void ct(double& X, double& Y, double w, double q, double qinv) {
  const double h = Y * w;
  const double l = __builtin_fma(Y, w, -h);
  const double k = __builtin_rint(h * qinv);
  const double r = __builtin_fma(-k, q, h) + l;
  const double x = X;
  X = x + r;
  Y = x - r;
}

template <int E, int G>
__global__ void __launch_bounds__(32768 / E) net(double* out, const double* tw, int rounds) {
  const double q = 1099511627689.0, qinv = 1.0 / q;
  double a[E];
#pragma unroll
  for (int k = 0; k < E; ++k) a[k] = (double)((threadIdx.x * 131 + k * 7) % 1000003);
  constexpr int LB = E == 32 ? 5 : 6;
  for (int r = 0; r < rounds; ++r) {
#pragma unroll
    for (int s = 0; s < LB; ++s) {
      const double w = tw[(r * 8 + s) & 255] + (double)(threadIdx.x & 7);
#pragma unroll
      for (int p = 0; p < E / 2; p += G) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int pr = p + g;
          const int k0 = ((pr >> s) << (s + 1)) | (pr & ((1 << s) - 1));
          PIN(a[k0], a[k0 | (1 << s)]);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int pr = p + g;
          const int k0 = ((pr >> s) << (s + 1)) | (pr & ((1 << s) - 1));
          ct(a[k0], a[k0 | (1 << s)], w, q, qinv);
        }
      }
    }
  }
  double acc = 0;
#pragma unroll
  for (int k = 0; k < E; ++k) acc += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int E, int G>
void run(double* out, double* tw, int rounds) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 4096, threads = 32768 / E;
  for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((net<E, G>), dim3(blocks), dim3(threads), 0, 0, out, tw, rounds);
  hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((net<E, G>), dim3(blocks), dim3(threads), 0, 0, out, tw, rounds);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double bfly = (double)blocks * 16384.0 * (E == 32 ? 5 : 6) * rounds;  // butterflies per launch
  const double us = ms * 1e3 / 5;
  // a 2^15-point NTT is 15 * 16384 butterflies: time per 256 limbs
  printf("E=%d G=%d: %8.1f us/launch  %6.2f us per 256 limb-NTTs (15 stages)\n", E, G, us,
         us / (bfly / (15.0 * 16384.0)) * 256);
}

int main() {
  double *out, *tw;
  hipMalloc(&out, 4096 * 1024 * 8);
  hipMalloc(&tw, 256 * 8);
  hipMemset(tw, 0, 256 * 8);
  run<32, 1>(out, tw, 6);
  run<32, 2>(out, tw, 6);
  run<32, 4>(out, tw, 6);
  run<64, 1>(out, tw, 5);
  run<64, 2>(out, tw, 5);
  run<64, 4>(out, tw, 5);
  run<64, 8>(out, tw, 5);
  return 0;
}
