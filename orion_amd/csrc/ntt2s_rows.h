// ntt2s_rows.h -- the radix-4 steps shared by the latency NTT kernels
// (ntt2s.hip) and the kernels that end in an inverse rows pass of their own
// output (kernels.hip: ks_mac's P limbs).  Device code only.
#pragma once
#include <type_traits>
#include "common.h"
#include "ntt_arith.h"

namespace {

// a twiddle table (t, bytes) as a buffer resource
__device__ __forceinline__ __amdgpu_buffer_rsrc_t twr_s(const void* t, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)t, 0, bytes, 0x00020000);
}

__device__ __forceinline__ int ins2(int j, int lo) {  // j with zero bits inserted at lo, lo + 1
  return ((j >> lo) << (lo + 2)) | (j & ((1 << lo) - 1));
}
template <class A>
__device__ __forceinline__ void ct4(const A& ar, typename A::T (&x)[4], const typename A::W& wa,
                                    const typename A::W& wb, const typename A::W& wc) {
  ar.ct(x[0], x[2], wa);  // upper stage: (e0, e2), (e1, e3)
  ar.ct(x[1], x[3], wa);
  ar.ct(x[0], x[1], wb);  // lower stage: (e0, e1), (e2, e3)
  ar.ct(x[2], x[3], wc);
}
template <class A>
__device__ __forceinline__ void gs4(const A& ar, typename A::T (&x)[4], const typename A::W& wa,
                                    const typename A::W& wb, const typename A::W& wc, bool red_lo, bool red_hi) {
  ar.gs(x[0], x[1], wa, red_lo);  // lower stage: (e0, e1), (e2, e3)
  ar.gs(x[2], x[3], wb, red_lo);
  ar.gs(x[0], x[2], wc, red_hi);  // upper stage: (e0, e2), (e1, e3)
  ar.gs(x[1], x[3], wc, red_hi);
}

// the forward rows pass (the second pass of the two-pass NTT, ntt2s.hip) of
// one 256-element row: x holds the intermediate's elements kk + 64 i on entry
// and the last step's elements 4 kk .. 4 kk + 3 (lazy range) on return; lr is
// the row's 256 words of LDS (one barrier per step but the last)
// (split in its twiddle loads and its steps, so a caller can issue more loads
// between the two: fwd_rows4_tw, fwd_rows4_run)
template <class A, int LOGN>
__device__ __forceinline__ void fwd_rows4_tw(int row, int kk, const A& ar, __amdgpu_buffer_rsrc_t tw,
                                             typename A::W (&wa)[4], typename A::W (&wb)[4], typename A::W (&wc)[4]) {
  constexpr int N = 1 << LOGN;
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int hb = 7 - 2 * st, g = kk >> (hb - 1);
    wa[st] = ar.tw(tw, (row << (7 - hb)) | g, N >> (hb + 1));
    wb[st] = ar.tw(tw, (row << (8 - hb)) | (2 * g), N >> hb);
    wc[st] = ar.tw(tw, (row << (8 - hb)) | (2 * g + 1), N >> hb);
  }
}
template <class A>
__device__ __forceinline__ void fwd_rows4_run(typename A::T (&x)[4], int kk, const A& ar, const typename A::W (&wa)[4],
                                              const typename A::W (&wb)[4], const typename A::W (&wc)[4], u64* lr) {
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int hb = 7 - 2 * st, lb = hb - 1;
    const int e0 = ins2(kk, lb), e1 = e0 + (1 << lb), e2 = e0 + (1 << hb), e3 = e2 + (1 << lb);
    if (st > 0) {
      x[0] = from_bits<typename A::T>(lr[e0]);
      x[1] = from_bits<typename A::T>(lr[e1]);
      x[2] = from_bits<typename A::T>(lr[e2]);
      x[3] = from_bits<typename A::T>(lr[e3]);
    }
    ct4(ar, x, wa[st], wb[st], wc[st]);
    if (st == 1)
      for (int i = 0; i < 4; ++i) x[i] = ar.reduce_round(x[i]);
    if (st < 3) {  // (a thread writes back only the words it read: one barrier per step)
      lr[e0] = to_bits(x[0]);
      lr[e1] = to_bits(x[1]);
      lr[e2] = to_bits(x[2]);
      lr[e3] = to_bits(x[3]);
      __syncthreads();
    }
  }
}
template <class A, int LOGN>
__device__ __forceinline__ void fwd_rows4_core(typename A::T (&x)[4], int row, int kk, const A& ar,
                                               __amdgpu_buffer_rsrc_t tw, u64* lr) {
  typename A::W wa[4], wb[4], wc[4];
  fwd_rows4_tw<A, LOGN>(row, kk, ar, tw, wa, wb, wc);
  fwd_rows4_run<A>(x, kk, ar, wa, wb, wc, lr);
}

// the inverse rows pass (the first pass of the two-pass INTT, ntt2s.hip) of
// one 256-element row: thread kk holds elements 4kk .. 4kk + 3 in x, lr is
// the row's 256 words of LDS (a thread writes back only the words it read, so
// one barrier per step, and none before the first), mid the row's
// intermediate (element kk + 64 i of the last step).  row: the row's index in
// the limb (the twiddles of its groups)
// (split like the forward: inv_rows4_tw, inv_rows4_run)
template <class A, int LOGN>
__device__ __forceinline__ void inv_rows4_tw(int row, int kk, const A& ar, __amdgpu_buffer_rsrc_t tw,
                                             typename A::W (&wa)[4], typename A::W (&wb)[4], typename A::W (&wc)[4]) {
  constexpr int N = 1 << LOGN;
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int lb = 2 * st, g = kk >> lb;
    wa[st] = ar.tw(tw, (row << (7 - lb)) | (2 * g), N >> (lb + 1));
    wb[st] = ar.tw(tw, (row << (7 - lb)) | (2 * g + 1), N >> (lb + 1));
    wc[st] = ar.tw(tw, (row << (6 - lb)) | g, N >> (lb + 2));
  }
}
template <class A>
__device__ __forceinline__ void inv_rows4_run(typename A::T (&x)[4], int kk, const A& ar, const typename A::W (&wa)[4],
                                              const typename A::W (&wb)[4], const typename A::W (&wc)[4], u64* lr,
                                              u64* mid, bool store = true) {
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int lb = 2 * st, hb = lb + 1;
    const int e0 = ins2(kk, lb), e1 = e0 + (1 << lb), e2 = e0 + (1 << hb), e3 = e2 + (1 << lb);
    if (st > 0) {
      x[0] = from_bits<typename A::T>(lr[e0]);
      x[1] = from_bits<typename A::T>(lr[e1]);
      x[2] = from_bits<typename A::T>(lr[e2]);
      x[3] = from_bits<typename A::T>(lr[e3]);
    }
    gs4(ar, x, wa[st], wb[st], wc[st], false, true);
    if (st < 3) {
      lr[e0] = to_bits(x[0]);
      lr[e1] = to_bits(x[1]);
      lr[e2] = to_bits(x[2]);
      lr[e3] = to_bits(x[3]);
      __syncthreads();
    }
  }
  if (store) {  // (store = false: a thread group that only keeps the barriers)
#pragma unroll
    for (int i = 0; i < 4; ++i) mid[kk + 64 * i] = to_bits(ar.reduce_round(x[i]));
  }
}
template <class A, int LOGN>
__device__ __forceinline__ void inv_rows4_core(typename A::T (&x)[4], int row, int kk, const A& ar,
                                               __amdgpu_buffer_rsrc_t tw, u64* lr, u64* mid, bool store = true) {
  typename A::W wa[4], wb[4], wc[4];
  inv_rows4_tw<A, LOGN>(row, kk, ar, tw, wa, wb, wc);
  inv_rows4_run<A>(x, kk, ar, wa, wb, wc, lr, mid, store);
}
// a twiddle word kept as two u64 (the float64 path's double in .x), so that
// twiddles of either arithmetic can be fetched early into one register array
__device__ __forceinline__ ulonglong2 w_raw(double w) { return make_ulonglong2(__builtin_bit_cast(u64, w), 0); }
__device__ __forceinline__ ulonglong2 w_raw(ulonglong2 w) { return w; }
template <class A>
__device__ __forceinline__ typename A::W w_of(ulonglong2 r) {
  if constexpr (std::is_same_v<typename A::W, double>) return __builtin_bit_cast(double, r.x);
  else return r;
}

}  // namespace
