// ntt_arith.h -- butterfly arithmetic shared by the NTT kernels (ntt.hip:
// one limb per workgroup; ntt2.hip: two-pass N = 2^15).  Device code only.
#pragma once
#include "common.h"

namespace {

// The limb is addressed through a buffer descriptor built from wave-uniform
// values: every access is a lane offset plus an immediate/SGPR offset, so no
// per-element VGPR addresses stay live (hipcc otherwise spills them), and the
// descriptor's range check confines the kernel to its limb.
__device__ __forceinline__ void buf_ld2(__amdgpu_buffer_rsrc_t r, u64& x, u64& y, int voff, int soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  x = ((u64)v[1] << 32) | v[0];
  y = ((u64)v[3] << 32) | v[2];
}
// timing switch: the cache-policy bits of the one-pass kernels' output
// stores (2 = non-temporal); 0 in the product
#ifndef NTT_ST_AUX
#define NTT_ST_AUX 0
#endif
__device__ __forceinline__ void buf_st2(__amdgpu_buffer_rsrc_t r, u64 x, u64 y, int voff, int soff) {
  __attribute__((ext_vector_type(4))) unsigned v = {(unsigned)x, (unsigned)(x >> 32), (unsigned)y,
                                                   (unsigned)(y >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, NTT_ST_AUX);
}
__device__ __forceinline__ u64 buf_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, u64 v, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), r,
                                        voff, soff, NTT_ST_AUX);
}

#define NTT_FENCE() __builtin_amdgcn_sched_barrier(0)
// An empty volatile asm that "redefines" a butterfly's two inputs: volatile
// asm statements stay in program order, so no butterfly can be hoisted above
// its predecessors by IR-level code motion (which sched_barrier cannot stop)
// -- this is what keeps the kernel at <= 128 VGPRs (1024 threads/CU).
#define PIN(x, y) asm volatile("" : "+v"(x), "+v"(y))

// ---------------------------------------------------------------------------
// arithmetic policies
// ---------------------------------------------------------------------------
#ifndef NTT_INT_DIET
#define NTT_INT_DIET 1
#endif
// 1: the forward (CT) butterfly's Shoup quotient drops the a0*s0 high word and
// its carries (floor(a*ws/2^64) under-estimated by at most 2, so t < 4q) and
// keeps values lazily in [0, 8q) instead of [0, 4q) (8q < 2^64 for q < 2^61)
#ifndef NTT_INT_CUT
#define NTT_INT_CUT 1
#endif
// 1: the inverse (GS) butterfly with the cut quotient too, values in [0, 4q)
#ifndef NTT_INV_CUT
#define NTT_INV_CUT 0
#endif
struct IntArith {
  typedef u64 T;
  typedef ulonglong2 W;
  u64 q, q2, q4, ninv, ninv_s, nq, wl, wl_s;
  __device__ IntArith(const ModConst& m)
      : q(m.q), q2(m.q << 1), q4(m.q << 2), ninv(m.ninv), ninv_s(m.ninv_s), nq(0 - m.q), wl(m.wl), wl_s(m.wl_s) {}
  __device__ __forceinline__ u64 smul(u64 a, u64 w, u64 ws) const {
    if constexpr (NTT_INT_CUT) return shoup_cut_nq(a, w, ws, nq);
    if constexpr (NTT_INT_DIET) return shoup_lazy_nq(a, w, ws, nq);
    return shoup_lazy(a, w, ws, q);
  }
  __device__ __forceinline__ W tw(__amdgpu_buffer_rsrc_t r, int vidx, int sidx) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vidx * 16, sidx * 16, 0);
    return make_ulonglong2(((u64)v[1] << 32) | v[0], ((u64)v[3] << 32) | v[2]);
  }
  __device__ __forceinline__ T from_u64(u64 x) const { return x; }
  // Harvey CT butterfly, values in [0, 4q) ([0, 8q) with the cut quotient)
  __device__ __forceinline__ void ct(T& X, T& Y, const W& w) const {
    if constexpr (NTT_INT_CUT) {
      const u64 x = X >= q4 ? X - q4 : X;
      const u64 t = smul(Y, w.x, w.y);
      X = x + t;
      Y = x - t + q4;
    } else {
      const u64 x = X >= q2 ? X - q2 : X;
      const u64 t = smul(Y, w.x, w.y);
      X = x + t;
      Y = x - t + q2;
    }
  }
  // Harvey GS butterfly, values in [0, 2q).  (The cut quotient of the forward
  // butterfly, with values in [0, 4q), spilled the inverse kernel in round 4:
  // 128 VGPRs + 172-196 B of scratch per lane at N = 2^15 -- against 120 VGPRs
  // here; NTT_INV_CUT retries it with a shorter twiddle prefetch ring.)
  // NTT_INV_CUT: values in [0, 4q): s = x + y < 8q reduced once into [0, 4q),
  // Y = cut Shoup of x - y + 4q < 8q (result in [0, 4q)), 8 instead of ~10
  // 32-bit multiplies and no 64-bit subtraction in the product
  __device__ __forceinline__ void gs(T& X, T& Y, const W& w, bool) const {
    const u64 x = X, y = Y;
    const u64 s = x + y;
    if constexpr (NTT_INV_CUT == 3) {  // cut quotient, the product in 64-bit form
      X = s >= q4 ? s - q4 : s;
      const u64 a = x - y + q4;
      const u32 a0 = (u32)a, a1 = (u32)(a >> 32), s0 = (u32)w.y, s1 = (u32)(w.y >> 32);
      const u64 m1 = (u64)a1 * s0;
      const u64 m2 = (u64)a0 * s1 + (u32)m1;
      const u64 qh = (u64)a1 * s1 + ((m1 >> 32) + (m2 >> 32));
      Y = a * w.x - qh * q;
    } else if constexpr (NTT_INV_CUT == 2) {  // the nq form of the full quotient: values stay in [0, 2q)
      X = s >= q2 ? s - q2 : s;
      Y = shoup_lazy_nq(x - y + q2, w.x, w.y, nq);
    } else if constexpr (NTT_INV_CUT) {
      X = s >= q4 ? s - q4 : s;
      Y = shoup_cut_nq(x - y + q4, w.x, w.y, nq);
    } else {
      X = s >= q2 ? s - q2 : s;
      Y = shoup_lazy(x - y + q2, w.x, w.y, q);
    }
  }
  // the last GS stage with N^-1 folded in (inputs in [0, 2q) / [0, 4q) with
  // NTT_INV_CUT, outputs in [0, 2q) / [0, 4q))
  __device__ __forceinline__ void gs_last(T& X, T& Y) const {
    const u64 x = X, y = Y;
    if constexpr (NTT_INV_CUT == 3) {
      X = shoup_lazy(x + y, ninv, ninv_s, q);
      Y = shoup_lazy(x - y + q4, wl, wl_s, q);
    } else if constexpr (NTT_INV_CUT == 2) {
      X = shoup_lazy_nq(x + y, ninv, ninv_s, nq);
      Y = shoup_lazy_nq(x - y + q2, wl, wl_s, nq);
    } else if constexpr (NTT_INV_CUT) {
      X = shoup_cut_nq(x + y, ninv, ninv_s, nq);
      Y = shoup_cut_nq(x - y + q4, wl, wl_s, nq);
    } else {
      X = shoup_lazy(x + y, ninv, ninv_s, q);
      Y = shoup_lazy(x - y + q2, wl, wl_s, q);
    }
  }
  __device__ __forceinline__ u64 final_inv_folded(T x) const {
    if constexpr (NTT_INV_CUT == 1) x = x >= q2 ? x - q2 : x;  // (3: gs_last ends in [0, 2q))
    return x >= q ? x - q : x;
  }
  __device__ __forceinline__ T reduce_round(T x) const { return x; }  // lazy range is invariant
  __device__ __forceinline__ u64 final_fwd(T x) const {
    if constexpr (NTT_INT_CUT) x = x >= q4 ? x - q4 : x;
    x = x >= q2 ? x - q2 : x;
    return x >= q ? x - q : x;
  }
  __device__ __forceinline__ u64 final_inv(T x) const {
    x = shoup_lazy(x, ninv, ninv_s, q);
    return x >= q ? x - q : x;
  }
};

struct F64Arith {
  typedef double T;
  typedef double W;
  double q, qinv, ninv, wl;
  __device__ F64Arith(const ModConst& m) : q(m.qd), qinv(m.qinv_d), ninv(m.ninv_d), wl(m.wl_d) {}
  __device__ __forceinline__ W tw(__amdgpu_buffer_rsrc_t r, int vidx, int sidx) const {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vidx * 8, sidx * 8, 0));
  }
  __device__ __forceinline__ T from_u64(u64 x) const { return (double)x; }
  // a*w mod q for exact integer doubles (|a| < 16q, |w| <= q/2, q < 2^46):
  // h + l == a*w exactly, k*q within 1.5q of h, so the result is exact and
  // |result| < 1.5q + ulp(h)/2 < 2q
  __device__ __forceinline__ double mulmod(double a, double w) const {
    const double h = a * w;
    const double l = __builtin_fma(a, w, -h);
    const double k = __builtin_rint(h * qinv);
    return __builtin_fma(-k, q, h) + l;
  }
  __device__ __forceinline__ double red(double x) const { return __builtin_fma(-__builtin_rint(x * qinv), q, x); }
  // CT: |x|, |y| stay below ~12q inside a round (reduced at round boundaries)
  __device__ __forceinline__ void ct(T& X, T& Y, const W& w) const {
    const double t = mulmod(Y, w);
    const double x = X;
    X = x + t;
    Y = x - t;
  }
  // GS: the sum is reduced every other stage
  __device__ __forceinline__ void gs(T& X, T& Y, const W& w, bool reduce_sum) const {
    const double x = X, y = Y;
    const double s = x + y;
    X = reduce_sum ? red(s) : s;
    Y = mulmod(x - y, w);
  }
  __device__ __forceinline__ T reduce_round(T x) const { return red(x); }
  __device__ __forceinline__ u64 to_u64(double x) const {
    x = red(x);
    x = x < 0 ? x + q : x;
    x = x >= q ? x - q : x;
    x = x < 0 ? x + q : x;
    return (u64)x;
  }
  __device__ __forceinline__ u64 final_fwd(T x) const { return to_u64(x); }
  __device__ __forceinline__ u64 final_inv(T x) const { return to_u64(mulmod(x, ninv)); }
  // the last GS stage with N^-1 folded in (|x|, |y| < 8q: |x +- y| < 16q)
  __device__ __forceinline__ void gs_last(T& X, T& Y) const {
    const double x = X, y = Y;
    X = mulmod(x + y, ninv);
    Y = mulmod(x - y, wl);
  }
  __device__ __forceinline__ u64 final_inv_folded(T x) const { return to_u64(x); }
};

template <class T>
__device__ __forceinline__ u64 to_bits(T x) {
  return __builtin_bit_cast(u64, x);
}
template <class T>
__device__ __forceinline__ T from_bits(u64 x) {
  return __builtin_bit_cast(T, x);
}

// wave-uniform pointer to row (c, l, b) of a LimbSet: the limb tables are
// indexed dynamically, so force the results into SGPRs so that every element
// address is SGPR base + lane offset
__device__ __forceinline__ u64* row_ptr(const LimbSet& s, int c, int l, int b) {
  const int pos = __builtin_amdgcn_readfirstlane(arg_byte(s.pos, l));
  const long long off = c * s.comp_stride + pos * s.limb_stride + b * s.batch_stride;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(off & 0xffffffffll));
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(off >> 32));
  return s.p + (long long)(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ void job_of(const NttIO& io, int job, int& c, int& l, int& b) {
  const LimbSet& d = io.dst;
  if (io.order == 2) {  // longest jobs first: a launch's last, partial round of workgroups holds the fast limbs
    b = job % d.nbatch;
    const int r = job / d.nbatch;
    c = r % d.ncomp;
    l = arg_byte(io.lord, r / d.ncomp);
  } else if (io.order == 1) {
    l = job % d.nlimb;
    const int r = job / d.nlimb;
    b = r % d.nbatch;
    c = r / d.nbatch;
  } else {
    b = job % d.nbatch;
    const int r = job / d.nbatch;
    l = r % d.nlimb;
    c = r / d.nlimb;
  }
}

}  // namespace
