// ntt.hip -- batched negacyclic NTT / INTT over 64-bit primes for gfx950.
//
// Restates the Lattigo v6 ring NTT reached from every op in
// /root/reference/orion/backend/lattigo/evaluator.go:
// forward = Cooley-Tukey, natural order in, bit-reversed out, twiddle for the
// butterfly group i of the stage with m groups = psi^bitrev(m+i); inverse =
// Gentleman-Sande with psi^-1 and a final N^-1.
//
// MI355X design (one limb per workgroup, register resident):
//   * N/32 threads per workgroup, 32 u64 per thread held in VGPRs (64 VGPRs);
//     N = 2^15 -> 1024 threads, the whole 256 KiB limb is on one CU and is
//     read from / written to HBM exactly once (16*N algorithmic bytes).
//   * 5 radix-2 stages per "round" run entirely in registers (a radix-32
//     butterfly network); between rounds the limb is re-distributed through
//     LDS in two 32-bit halves (N*4 B + padding = 132 KiB for N = 2^15), with
//     a one-word-per-32 pad that makes every exchange bank-conflict free.
//   * Harvey lazy butterflies with Shoup twiddles: values stay in [0, 4q)
//     (forward) / [0, 2q) (inverse) between stages; one u64 x u64 -> hi
//     product per butterfly.  Twiddles are {w, w'} pairs, 16-B loads.
#include "common.h"

namespace {

template <int LOGN>
struct NttGeom {
  static constexpr int N = 1 << LOGN;
  static constexpr int T = N / 32;  // threads
  static constexpr int B0 = LOGN - 5;
};

__device__ __forceinline__ int lds_pad(int e) { return e + (e >> 5); }

// One limb is addressed through a buffer descriptor built from wave-uniform
// values: element k*2^B0 + t is voffset t*8 plus a per-k SGPR/immediate
// offset, so the 32 loads/stores need no per-element VGPR addresses (hipcc
// otherwise keeps 32 64-bit addresses live from the load to the store and
// spills them).  The descriptor's range check also confines the kernel to
// its limb.
__device__ __forceinline__ u64 buf_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ void buf_ld2(__amdgpu_buffer_rsrc_t r, u64& x, u64& y, int voff, int soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  x = ((u64)v[1] << 32) | v[0];
  y = ((u64)v[3] << 32) | v[2];
}
__device__ __forceinline__ void buf_st2(__amdgpu_buffer_rsrc_t r, u64 x, u64 y, int voff, int soff) {
  __attribute__((ext_vector_type(4))) unsigned v = {(unsigned)x, (unsigned)(x >> 32), (unsigned)y,
                                                   (unsigned)(y >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, 0);
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, u64 v, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), r,
                                        voff, soff, 0);
}

// element index held in slot k of thread t for the round whose 5 k-bits start at bit B
template <int B>
__device__ __forceinline__ int elem(int t, int k) {
  return ((t >> B) << (B + 5)) | (k << B) | (t & ((1 << B) - 1));
}

// Redistribute a[] from window BOLD to window BNEW through LDS, one 32-bit
// half at a time (the whole limb does not fit in 160 KiB of LDS as u64).
// The halves live in two u32 arrays so the exchange never needs more than
// the 64 VGPRs of the data itself.
// LDS word of element e is pad(e) = e + (e >> 5).  With e = T | (k << B) (disjoint
// fields) this splits into a per-thread base and a compile-time per-slot offset,
// so every ds_read/ds_write is base VGPR + immediate.
template <int B>
__device__ __forceinline__ int lds_base(int t) {
  const int T = ((t >> B) << (B + 5)) | (t & ((1 << B) - 1));
  return T + (T >> 5);
}
template <int B>
__host__ __device__ constexpr int lds_off(int k) {
  return (k << B) + ((k << B) >> 5);
}

template <int BOLD, int BNEW>
__device__ __forceinline__ void exchange(u64 (&a)[32], u32* lds, int t) {
  u32 lo[32], hi[32];
  u32* const wr = lds + lds_base<BOLD>(t);
  u32* const rd = lds + lds_base<BNEW>(t);
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    lo[k] = (u32)a[k];
    hi[k] = (u32)(a[k] >> 32);
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) wr[lds_off<BOLD>(k)] = lo[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; ++k) lo[k] = rd[lds_off<BNEW>(k)];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; ++k) wr[lds_off<BOLD>(k)] = hi[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; ++k) hi[k] = rd[lds_off<BNEW>(k)];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; ++k) a[k] = ((u64)hi[k] << 32) | lo[k];
}

// keeps the scheduler from hoisting every twiddle load of a round (which
// would need 124 extra VGPRs and spill): twiddles are loaded group by group.
#define NTT_FENCE() __builtin_amdgcn_sched_barrier(0)
// An empty volatile asm that "redefines" a butterfly's two inputs: volatile
// asm statements stay in program order, so no butterfly can be hoisted above
// its predecessors by IR-level code motion (which sched_barrier cannot stop).
#define PIN(x, y) asm volatile("" : "+v"(x), "+v"(y))

#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(1))) ulonglong2* gtw_ptr;  // global (not flat) twiddle loads
#else
typedef const ulonglong2* gtw_ptr;
#endif

// Forward CT stages for bits DHI..DLO (all inside the window starting at B).
// The 16 butterflies of a stage are issued in fenced groups of 4 so that at
// most 4 are in flight per thread (64 VGPRs hold the data, the rest must
// cover temporaries: the kernel has to fit 128 VGPRs at 1024 threads).
__device__ __forceinline__ ulonglong2 tw_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return make_ulonglong2(((u64)v[1] << 32) | v[0], ((u64)v[3] << 32) | v[2]);
}

template <int LOGN, int B, int DHI, int DLO>
__device__ __forceinline__ void fwd_round(u64 (&a)[32], __amdgpu_buffer_rsrc_t w, u64 q, int t) {
  const u64 q2 = q << 1;
  const int thigh = t >> B;
#pragma unroll
  for (int d = DHI; d >= DLO; --d) {
    const int dk = d - B;
    const int m = (1 << LOGN) >> (d + 1);
    ulonglong2 W;
#pragma unroll
    for (int pr = 0; pr < 16; ++pr) {
      const int khi = pr >> dk, klo = pr & ((1 << dk) - 1);
      if (klo == 0) W = tw_ld(w, (thigh << (4 - dk)) * 16, (m + khi) * 16);
      const int k0 = (khi << (dk + 1)) | klo;
      const int k1 = k0 | (1 << dk);
      PIN(a[k0], a[k1]);
      u64 X = a[k0];
      X = X >= q2 ? X - q2 : X;
      const u64 T = shoup_lazy(a[k1], W.x, W.y, q);
      a[k0] = X + T;
      a[k1] = X - T + q2;
      if ((pr & 3) == 3) NTT_FENCE();
    }
  }
}

// Inverse GS stages for bits DLO..DHI.
template <int LOGN, int B, int DLO, int DHI>
__device__ __forceinline__ void inv_round(u64 (&a)[32], __amdgpu_buffer_rsrc_t w, u64 q, int t) {
  const u64 q2 = q << 1;
  const int thigh = t >> B;
#pragma unroll
  for (int d = DLO; d <= DHI; ++d) {
    const int dk = d - B;
    const int m = (1 << LOGN) >> (d + 1);
    ulonglong2 W;
#pragma unroll
    for (int pr = 0; pr < 16; ++pr) {
      const int khi = pr >> dk, klo = pr & ((1 << dk) - 1);
      if (klo == 0) W = tw_ld(w, (thigh << (4 - dk)) * 16, (m + khi) * 16);
      const int k0 = (khi << (dk + 1)) | klo;
      const int k1 = k0 | (1 << dk);
      PIN(a[k0], a[k1]);
      const u64 X = a[k0], Y = a[k1];
      u64 S = X + Y;
      S = S >= q2 ? S - q2 : S;
      a[k0] = S;
      a[k1] = shoup_lazy(X - Y + q2, W.x, W.y, q);
      if ((pr & 1) == 1) NTT_FENCE();
    }
  }
}

__device__ __forceinline__ u64* job_ptr(const LimbSet& s, int job, int& mod) {
  const int b = job % s.nbatch;
  const int r = job / s.nbatch;
  const int l = r % s.nlimb;
  const int c = r / s.nlimb;
  // the limb tables are indexed dynamically; force the results to be
  // wave-uniform (SGPR) so every element address is SGPR base + lane offset
  mod = __builtin_amdgcn_readfirstlane(s.mod[l]);
  const int pos = __builtin_amdgcn_readfirstlane(s.pos[l]);
  const long long off = c * s.comp_stride + pos * s.limb_stride + b * s.batch_stride;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(off & 0xffffffffll));
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(off >> 32));
  return s.p + (long long)(((unsigned long long)hi << 32) | lo);
}

// Round windows: LOGN=15 -> bits [10,15), [5,10), [0,5); LOGN=14 -> [9,14),[4,9),[0,5)
// (last round only bits 3..0); LOGN=13 -> [8,13),[3,8),[0,5) (bits 2..0).
template <int LOGN>
__global__ void __launch_bounds__(NttGeom<LOGN>::T) ntt_fwd_kernel(LimbSet s, const DeviceTables* __restrict__ tb) {
  constexpr int N = 1 << LOGN, B0 = LOGN - 5, B1 = LOGN - 10;
  extern __shared__ u32 lds[];
  const int t = threadIdx.x;
  int mod;
  u64* __restrict__ p = job_ptr(s, blockIdx.x, mod);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, N * 8, 0x00020000);
  const u64 q = tb->mc[mod].q;
  const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)tb->fwd[mod], 0, (1 << LOGN) * 16, 0x00020000);
  u64 a[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) a[k] = buf_ld(rs, t * 8, (k << B0) * 8);
  fwd_round<LOGN, B0, LOGN - 1, B0>(a, w, q, t);
  exchange<B0, B1>(a, lds, t);
  fwd_round<LOGN, B1, B0 - 1, B1>(a, w, q, t);
  exchange<B1, 0>(a, lds, t);
  fwd_round<LOGN, 0, B1 - 1, 0>(a, w, q, t);
  const u64 q2 = q << 1;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    u64 x = a[k];
    x = x >= q2 ? x - q2 : x;
    a[k] = x >= q ? x - q : x;
  }
  // window 0: thread t holds elements 32t .. 32t+31 -> 16-byte stores
#pragma unroll
  for (int k = 0; k < 32; k += 2) buf_st2(rs, a[k], a[k + 1], t * 256, k * 8);
}

template <int LOGN>
__global__ void __launch_bounds__(NttGeom<LOGN>::T) ntt_inv_kernel(LimbSet s, const DeviceTables* __restrict__ tb) {
  constexpr int B0 = LOGN - 5, B1 = LOGN - 10;
  extern __shared__ u32 lds[];
  const int t = threadIdx.x;
  int mod;
  u64* __restrict__ p = job_ptr(s, blockIdx.x, mod);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, (1 << LOGN) * 8, 0x00020000);
  const ModConst mc = tb->mc[mod];
  const u64 q = mc.q;
  const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)tb->inv[mod], 0, (1 << LOGN) * 16, 0x00020000);
  u64 a[32];
#pragma unroll
  for (int k = 0; k < 32; k += 2) buf_ld2(rs, a[k], a[k + 1], t * 256, k * 8);
  inv_round<LOGN, 0, 0, B1 - 1>(a, w, q, t);
  exchange<0, B1>(a, lds, t);
  inv_round<LOGN, B1, B1, B0 - 1>(a, w, q, t);
  exchange<B1, B0>(a, lds, t);
  inv_round<LOGN, B0, B0, LOGN - 1>(a, w, q, t);
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    u64 x = shoup_lazy(a[k], mc.ninv, mc.ninv_s, q);
    buf_st(rs, x >= q ? x - q : x, t * 8, (k << B0) * 8);
    if ((k & 3) == 3) NTT_FENCE();
  }
}

template <int LOGN>
void launch_ntt(const LimbSet& s, const DeviceTables* tb, bool inverse, hipStream_t st) {
  constexpr int N = 1 << LOGN;
  const int jobs = s.ncomp * s.nlimb * s.nbatch;
  if (jobs == 0) return;
  const size_t lds = (size_t)(N + N / 32) * sizeof(u32);
  if (inverse)
    hipLaunchKernelGGL(ntt_inv_kernel<LOGN>, dim3(jobs), dim3(NttGeom<LOGN>::T), lds, st, s, tb);
  else
    hipLaunchKernelGGL(ntt_fwd_kernel<LOGN>, dim3(jobs), dim3(NttGeom<LOGN>::T), lds, st, s, tb);
}

}  // namespace

// host entry: in-place NTT (inverse=false) or INTT of every limb in s
int orion_launch_ntt(int logN, const LimbSet& s, const DeviceTables* tb, bool inverse, hipStream_t st) {
  switch (logN) {
    case 13: launch_ntt<13>(s, tb, inverse, st); return 0;
    case 14: launch_ntt<14>(s, tb, inverse, st); return 0;
    case 15: launch_ntt<15>(s, tb, inverse, st); return 0;
    default: return -1;
  }
}

// allow >64 KiB dynamic LDS for the N = 2^15 kernels
int orion_ntt_init() {
  hipError_t e1 = hipFuncSetAttribute((const void*)ntt_fwd_kernel<15>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (32768 + 1024) * 4);
  hipError_t e2 = hipFuncSetAttribute((const void*)ntt_inv_kernel<15>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (32768 + 1024) * 4);
  hipError_t e3 = hipFuncSetAttribute((const void*)ntt_fwd_kernel<14>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (16384 + 512) * 4);
  hipError_t e4 = hipFuncSetAttribute((const void*)ntt_inv_kernel<14>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (16384 + 512) * 4);
  return (e1 == hipSuccess && e2 == hipSuccess && e3 == hipSuccess && e4 == hipSuccess) ? 0 : -1;
}
