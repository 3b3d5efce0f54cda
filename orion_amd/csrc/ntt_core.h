// ntt_core.h -- the one-limb-per-workgroup NTT building blocks of ntt.hip:
// LDS exchanges, the radix-32 round networks with their twiddle schedule and
// sources, and round reductions.  Device code only.
#pragma once
#include "common.h"

#include "ntt_arith.h"

// timing-only ablation builds (tools/build_ablation.py + tools/ab.sh); 0 in the product:
// bit 0 skips the butterfly rounds, bit 1 skips the LDS exchanges
#ifndef NTT_ABLATE
#define NTT_ABLATE 0
#endif
// timing switch: NTT_LAZY skips the forward round
// reductions for small float64 moduli
#ifndef NTT_LAZY
#define NTT_LAZY 1
#endif
// timing switch: 1 = the forward kernel stores its last round directly (each
// thread's 32 consecutive outputs as 16-B stores) instead of exchanging back
// to the strided layout first
#ifndef NTT_FWD_DIRECT
#define NTT_FWD_DIRECT 0
#endif
// timing switch: 1 = the inverse kernel loads coalesced (element t + 1024 k)
// and exchanges to the consecutive layout, instead of 16-B strided loads
#ifndef NTT_INV_COAL
#define NTT_INV_COAL 0
#endif
// scheduling windows: a sched_barrier after every NTT_FENCE_FWD (forward) /
// NTT_FENCE_INV (inverse) butterflies bounds the live registers to <= 128
#ifndef NTT_FENCE_FWD
#define NTT_FENCE_FWD 4
#endif
#ifndef NTT_FENCE_INV
#define NTT_FENCE_INV 2
#endif
// 1: the inverse's last stage multiplies by N^-1 (X) and w1 N^-1 (Y) instead
// of a separate N^-1 pass over every output (ntt.hip final_inv_folded)
#ifndef NTT_INV_FOLD
#define NTT_INV_FOLD 1
#endif
// 1: no float64 reductions between inverse rounds: a round of GS stages maps
// inputs below 8q to outputs below 3q (the sums are reduced every other stage,
// mulmod outputs are below 1.5q + ulp), so the bound holds round to round
#ifndef NTT_INV_NORED
#define NTT_INV_NORED 1
#endif
// 1: butterflies scheduled in pairs (see run_stage)
#ifndef NTT_PAIR
#define NTT_PAIR 0
#endif

namespace {

template <int LOGN>
struct NttGeom {
  static constexpr int N = 1 << LOGN;
  static constexpr int T = N / 32;  // threads
};

// LDS word of element e is pad(e) = e + (e >> 5).  With e = T | (k << B) (disjoint
// fields: T = thread part, k = slot) this splits into a per-thread base and a
// compile-time per-slot offset, so every ds_read/ds_write is base VGPR + immediate.
template <int B>
__device__ __forceinline__ int lds_base(int t) {
  const int T = ((t >> B) << (B + 5)) | (t & ((1 << B) - 1));
  return T + (T >> 5);
}
template <int B>
__host__ __device__ constexpr int lds_off(int k) {
  return (k << B) + ((k << B) >> 5);
}

// Redistribute a[] from window BOLD to window BNEW through LDS, one 32-bit
// half at a time (the whole limb does not fit in 160 KiB of LDS as u64).
// The halves live in two u32 arrays so the exchange needs no VGPRs beyond the
// data's own 64.
template <class T, int BOLD, int BNEW>
__device__ __forceinline__ void exchange(T (&a)[32], u32* lds, int t) {
  if (NTT_ABLATE & 2) return;
  u32 lo[32], hi[32];
  u32* const wr = lds + lds_base<BOLD>(t);
  u32* const rd = lds + lds_base<BNEW>(t);
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const u64 b = to_bits(a[k]);
    lo[k] = (u32)b;
    hi[k] = (u32)(b >> 32);
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
  for (int k = 0; k < 32; ++k) a[k] = from_bits<T>(((u64)hi[k] << 32) | lo[k]);
}

template <class T, int LOGN, int BOLD, int BNEW>
__device__ __forceinline__ void xchg(T (&a)[32], u32* lds, int t) {
  exchange<T, BOLD, BNEW>(a, lds, t);
}

// Twiddle schedule of one round: its stages in execution order, each with
// 2^(4-dk) distinct twiddles (dk = stage bit - window base B).  Twiddles are
// software-prefetched TW_PF groups ahead through a compile-time ring, so the
// L2 latency of a per-thread twiddle load is hidden behind earlier butterflies.
#ifndef TW_PF
#define TW_PF 4
#endif
template <int B, int DFIRST, int DLAST>
struct RoundPlan {
  static constexpr int DIR = DLAST >= DFIRST ? 1 : -1;
  static constexpr int nstage = (DLAST - DFIRST) * DIR + 1;
  static constexpr int d_of(int s) { return DFIRST + s * DIR; }
  static constexpr int g_of(int s) { return 1 << (4 - (d_of(s) - B)); }
  static constexpr int first(int s) { return s == 0 ? 0 : first(s - 1) + g_of(s - 1); }
  static constexpr int total() { return first(nstage - 1) + g_of(nstage - 1); }
  static constexpr int stage_of(int i, int s = 0) { return i < first(s) + g_of(s) ? s : stage_of(i, s + 1); }
};

// Twiddle sources: get(v, s) returns twiddle v + s (v per lane, s compile-time).
// TwVmem reads the limb's table in global memory (the one-pass kernels).
template <class A>
struct TwVmem {
  A ar;
  __amdgpu_buffer_rsrc_t w;
  __device__ __forceinline__ typename A::W get(int v, int s) const { return ar.tw(w, v, s); }
};

template <class A, int LOGN, int B, class Plan, int I, class TS>
__device__ __forceinline__ typename A::W tw_load(const TS& ts, int thigh) {
  constexpr int s = Plan::stage_of(I);
  constexpr int d = Plan::d_of(s), dk = d - B, khi = I - Plan::first(s);
  constexpr int m = (1 << LOGN) >> (d + 1);
  return ts.get(thigh << (4 - dk), m + khi);
}

template <class A, int LOGN, int B, class Plan, int I, class TS>
__device__ __forceinline__ void tw_prefetch(typename A::W (&ring)[TW_PF], const TS& ts, int thigh) {
  if constexpr (I < Plan::total()) ring[I % TW_PF] = tw_load<A, LOGN, B, Plan, I>(ts, thigh);
}

// One stage's 16 butterflies.  Twiddle of the butterfly group i = e >> (d+1)
// of stage d is w[m + i], m = N >> (d+1); with e = T | (k << B) that is
// m + ((t>>B) << (4-dk) | khi).
template <class A, int LOGN, int B, class Plan, int S, bool FWD, class TS>
__device__ __forceinline__ void run_stage(typename A::T (&a)[32], typename A::W (&ring)[TW_PF], const A& ar,
                                          const TS& ts, int thigh) {
  constexpr int d = Plan::d_of(S), dk = d - B;
  typename A::W W, Wp;
#pragma unroll
  for (int pr = 0; pr < 16; ++pr) {
    const int khi = pr >> dk, klo = pr & ((1 << dk) - 1);
    if (klo == 0) {
      const int i = Plan::first(S) + khi;
      W = ring[i % TW_PF];
      // refill the slot just consumed with the twiddle TW_PF groups ahead
      switch (i) {
#define TWC(J) case J: tw_prefetch<A, LOGN, B, Plan, J + TW_PF>(ring, ts, thigh); break;
        TWC(0) TWC(1) TWC(2) TWC(3) TWC(4) TWC(5) TWC(6) TWC(7) TWC(8) TWC(9) TWC(10) TWC(11) TWC(12)
        TWC(13) TWC(14) TWC(15) TWC(16) TWC(17) TWC(18) TWC(19) TWC(20) TWC(21) TWC(22) TWC(23) TWC(24)
        TWC(25) TWC(26) TWC(27) TWC(28) TWC(29) TWC(30) TWC(31)
#undef TWC
        default: break;
      }
    }
    const int k0 = (khi << (dk + 1)) | klo;
    const int k1 = k0 | (1 << dk);
    if constexpr (NTT_PAIR) {
      // two butterflies per scheduling region: the pins sit in front of the
      // pair, so the scheduler can interleave the two independent chains
      // (one butterfly is a dependent chain of 8 FP64 or ~30 integer ops)
      if ((pr & 1) == 0) {
        Wp = W;
        continue;
      }
      const int pe = pr - 1, ke = ((pe >> dk) << (dk + 1)) | (pe & ((1 << dk) - 1)), ke1 = ke | (1 << dk);
      PIN(a[ke], a[ke1]);
      PIN(a[k0], a[k1]);
      if constexpr (FWD) {
        ar.ct(a[ke], a[ke1], Wp);
        ar.ct(a[k0], a[k1], W);
        if ((pr & (NTT_FENCE_FWD - 1)) == NTT_FENCE_FWD - 1) NTT_FENCE();
      } else {
        ar.gs(a[ke], a[ke1], Wp, (S & 1) == 1);
        ar.gs(a[k0], a[k1], W, (S & 1) == 1);
        if ((pr & (NTT_FENCE_INV - 1)) == NTT_FENCE_INV - 1 || NTT_FENCE_INV < 2) NTT_FENCE();
      }
      continue;
    }
    PIN(a[k0], a[k1]);
    if constexpr (FWD) {
      ar.ct(a[k0], a[k1], W);
      if ((pr & (NTT_FENCE_FWD - 1)) == NTT_FENCE_FWD - 1) NTT_FENCE();
    } else {
      if constexpr (NTT_INV_FOLD && d == LOGN - 1)
        ar.gs_last(a[k0], a[k1]);
      else
        ar.gs(a[k0], a[k1], W, (S & 1) == 1);
      if ((pr & (NTT_FENCE_INV - 1)) == NTT_FENCE_INV - 1) NTT_FENCE();
    }
  }
}

template <class A, int LOGN, int B, class Plan, bool FWD, int S, class TS>
__device__ __forceinline__ void run_stages(typename A::T (&a)[32], typename A::W (&ring)[TW_PF], const A& ar,
                                           const TS& ts, int thigh) {
  if constexpr (S < Plan::nstage) {
    run_stage<A, LOGN, B, Plan, S, FWD, TS>(a, ring, ar, ts, thigh);
    run_stages<A, LOGN, B, Plan, FWD, S + 1, TS>(a, ring, ar, ts, thigh);
  }
}

// one round with twiddles from source ts
template <class A, int LOGN, int B, int DFIRST, int DLAST, bool FWD, class TS>
__device__ __forceinline__ void do_round_ts(typename A::T (&a)[32], const A& ar, const TS& ts, int t) {
  if (NTT_ABLATE & 1) return;
  typedef RoundPlan<B, DFIRST, DLAST> Plan;
  const int thigh = t >> B;
  typename A::W ring[TW_PF];
  tw_prefetch<A, LOGN, B, Plan, 0>(ring, ts, thigh);
  tw_prefetch<A, LOGN, B, Plan, 1>(ring, ts, thigh);
  tw_prefetch<A, LOGN, B, Plan, 2>(ring, ts, thigh);
  tw_prefetch<A, LOGN, B, Plan, 3>(ring, ts, thigh);
  run_stages<A, LOGN, B, Plan, FWD, 0>(a, ring, ar, ts, thigh);
}

template <class A, int LOGN, int B, int DFIRST, int DLAST, bool FWD>
__device__ __forceinline__ void do_round(typename A::T (&a)[32], const A& ar, __amdgpu_buffer_rsrc_t w, int t) {
  do_round_ts<A, LOGN, B, DFIRST, DLAST, FWD>(a, ar, TwVmem<A>{ar, w}, t);
}

// Forward CT stages for bits DHI..DLO (all inside the window starting at B).
template <class A, int LOGN, int B, int DHI, int DLO>
__device__ __forceinline__ void fwd_round(typename A::T (&a)[32], const A& ar, __amdgpu_buffer_rsrc_t w, int t) {
  do_round<A, LOGN, B, DHI, DLO, true>(a, ar, w, t);
}

// Inverse GS stages for bits DLO..DHI.
template <class A, int LOGN, int B, int DLO, int DHI>
__device__ __forceinline__ void inv_round(typename A::T (&a)[32], const A& ar, __amdgpu_buffer_rsrc_t w, int t) {
  do_round<A, LOGN, B, DLO, DHI, false>(a, ar, w, t);
}

template <class A>
__device__ __forceinline__ void reduce_all(typename A::T (&a)[32], const A& ar) {
#pragma unroll
  for (int k = 0; k < 32; ++k) a[k] = ar.reduce_round(a[k]);
}

}  // namespace
