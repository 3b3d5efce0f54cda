// ntt.hip -- batched negacyclic NTT / INTT over 64-bit primes for gfx950.
//
// Restates the Lattigo v6 ring NTT reached from every op in
// /root/reference/orion/backend/lattigo/evaluator.go:
// forward = Cooley-Tukey, natural order in, bit-reversed out, twiddle for the
// butterfly group i of the stage with m groups = psi^bitrev(m+i); inverse =
// Gentleman-Sande with psi^-1 and a final N^-1.  Outputs are fully reduced,
// so they are bit-identical to any exact NTT with the same psi.
//
// MI355X design (one limb per workgroup, register resident):
//   * N/32 threads per workgroup, 32 u64 per thread held in VGPRs (64 VGPRs);
//     N = 2^15 -> 1024 threads, the whole 256 KiB limb is on one CU and is
//     read from / written to HBM exactly once (16*N algorithmic bytes).
//   * 5 radix-2 stages per "round" run entirely in registers (a radix-32
//     butterfly network); between rounds the limb is re-distributed through
//     LDS in two 32-bit halves (N*4 B + padding = 132 KiB for N = 2^15), with
//     a one-word-per-32 pad that makes every exchange bank-conflict free.
//     The last (forward) / first (inverse) round is the one whose thread
//     holds 32 consecutive elements, accessed with 16-byte loads/stores.
//   * Two arithmetic paths, chosen per limb (block-uniform):
//       - integer (q >= 2^46): Harvey lazy butterflies with Shoup twiddles,
//         values in [0, 4q);
//       - float64 (q < 2^46, i.e. the 40-bit Q primes): values are signed
//         integers held exactly in doubles, a*w mod q = fma residuals
//         (h = a*w, l = fma(a, w, -h), k = rint(h/q), r = fma(-k, q, h) + l).
//         On gfx950 one FP64 op issues at the rate of one 32-bit integer
//         multiply piece (tools/ubench/valu_rates.hip), and the float path
//         needs ~9 of them per butterfly instead of ~30 integer instructions.
#include "common.h"
#include <stdlib.h>
#include <string.h>

#include "ntt_core.h"

namespace {

// Round windows: LOGN=15 -> bits [10,15), [5,10), [0,5); LOGN=14 -> [9,14),[4,9),[0,5)
// (last round only bits 3..0); LOGN=13 -> [8,13),[3,8),[0,5) (bits 2..0).
// Thread t loads / stores element t + (k << B0) (k < 32): fully coalesced.
// ConjugateInvariant fold (CI): b_e = a_e - W a_{N-e}, b_0 = a_0 (the ring
// element's degree-2N expansion reduced mod X^N - W, W = psi^N; oracle_ntt).
// Thread t's element e = t + k S (S = N/32) pairs with N - e = (S - t) + (31 - k) S,
// held at the same offsets of the mirrored thread, so the partner is one more
// coalesced (descending) load of the same limb, served by L2.
// 1: the subtract-and-scale epilogue loads its operand one group of 8 rows ahead
#ifndef NTT_EPI_PF
#define NTT_EPI_PF 1
#endif

__device__ __forceinline__ u64 ci_fold(u64 x, u64 y, const ModConst& mc) {
  return sub_mod(x, shoup_mul(y, mc.ciw, mc.ciw_s, mc.q), mc.q);
}

// NTT_PRO_BEXT, one-pass kernel: rows 4G .. 4G+3 of the thread's 32 formed
// by the exact basis extension, the next group's source loads in flight.  The
// groups recurse on a template index so that every a[] index is a constant
// (a loop over groups that is not unrolled would index a[] dynamically and put
// the whole limb in scratch); fenced so that no group's loads are hoisted
// ahead (the limb's 64 VGPRs leave no room for them)
template <int G, class A, int B0>
__device__ __forceinline__ void bext_rows(typename A::T (&a)[32], const u64 (&xa)[4], const u64 (&xb)[4], const A& ar,
                                          const BasisExtTable* __restrict__ T, int ti, int ns,
                                          __amdgpu_buffer_rsrc_t r0, __amdgpu_buffer_rsrc_t r1,
                                          int t) {
  if constexpr (G < 8) {
    u64 na[4], nb[4];
    if constexpr (G < 7) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        na[k] = buf_ld(r0, t * 8, ((4 * (G + 1) + k) << B0) * 8);
        nb[k] = ns > 1 ? buf_ld(r1, t * 8, ((4 * (G + 1) + k) << B0) * 8) : 0;
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      u64 x[2] = {xa[k], xb[k]}, y[2];
      const u64 v = bext_prep<2>(T, x, y);
      a[4 * G + k] = ar.from_u64(bext_target_sel<2>(T->tgt + ti, ns, y, v));
    }
    NTT_FENCE();
    if constexpr (G < 7) bext_rows<G + 1, A, B0>(a, na, nb, ar, T, ti, ns, r0, r1, t);
  }
}

template <class A, int LOGN, int PRO, int EPI, bool CI>
__device__ __forceinline__ void ntt_fwd_body(const NttIO& io, int c, int l, int b, const ModConst& mc, const A& ar,
                                             __amdgpu_buffer_rsrc_t w, u32* lds, const DeviceTables* __restrict__ tb) {
  constexpr int N = 1 << LOGN, B0 = LOGN - 5, B1 = LOGN - 10, S = NttGeom<LOGN>::T;
  // an opaque copy of the thread index per job: keeps the persistent job loop
  // from hoisting every thread-derived address out of the loop (LICM), whose
  // live ranges would then span the whole body and spill
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  typename A::T a[32];
  if constexpr (PRO == NTT_PRO_LOAD) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row_ptr(io.src, c, l, b), 0, N * 8, 0x00020000);
    if constexpr (CI) {
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        const u64 x = buf_ld(rs, t * 8, (k << B0) * 8);
        u64 y = buf_ld(rs, (S - t) * 8, ((31 - k) << B0) * 8);  // e = 0: offset N, outside the descriptor
        if (k == 0) y = t == 0 ? 0 : y;
        a[k] = ar.from_u64(ci_fold(x, y, mc));
      }
    } else {
#pragma unroll
      for (int k = 0; k < 32; ++k) a[k] = ar.from_u64(buf_ld(rs, t * 8, (k << B0) * 8));
    }
  } else if constexpr (PRO == NTT_PRO_BEXT) {
    // the exact basis extension of (at most 2) source limbs to this limb, in
    // registers (the value basis_ext_kernel would have stored)
    static_assert(!CI, "no fused basis extension on the ConjugateInvariant ring");
    const int tk = arg_byte(io.bx_tab, l), ti = arg_byte(io.bx_t, l), s0 = arg_byte(io.bx_s0, tk);
    const BasisExtTable* __restrict__ T = io.bx + tk;
    const int ns = T->ns;
    const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(row_ptr(io.src, c, s0, b), 0, N * 8, 0x00020000);
    const __amdgpu_buffer_rsrc_t r1 =
        __builtin_amdgcn_make_buffer_rsrc(row_ptr(io.src, c, s0 + (ns > 1 ? 1 : 0), b), 0, N * 8, 0x00020000);
    u64 xa[4], xb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      xa[k] = buf_ld(r0, t * 8, (k << B0) * 8);
      xb[k] = ns > 1 ? buf_ld(r1, t * 8, (k << B0) * 8) : 0;
    }
    bext_rows<0, A, B0>(a, xa, xb, ar, T, ti, ns, r0, r1, t);
  } else {  // NTT_PRO_RESCALE (DivRoundByLastModulusNTT), fused with the NTT of every other limb
    const u64* sp = row_ptr(io.src, c, 0, b);
    const u64 qL = tb->mc[io.modL].q, h = qL >> 1;
    const u64 hm = barrett128(0, h, mc);
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const u64 x = sub_mod(barrett128(0, add_mod(sp[t + (k << B0)], h, qL), mc), hm, mc.q);
      if constexpr (CI) {
        u64 y = sub_mod(barrett128(0, add_mod(sp[(N - t - (k << B0)) & (N - 1)], h, qL), mc), hm, mc.q);
        if (k == 0) y = t == 0 ? 0 : y;
        a[k] = ar.from_u64(ci_fold(x, y, mc));
      } else {
        a[k] = ar.from_u64(x);
      }
    }
  }
  // CT growth is additive (|t| < 2q per stage): from [0, q) the values stay
  // below 31 q over all 15 stages, exact in float64 for q < 2^41, so the
  // round-boundary reductions are only needed for larger float64 moduli
  const bool lazy = NTT_LAZY && mc.bar_k <= 41;
  fwd_round<A, LOGN, B0, LOGN - 1, B0>(a, ar, w, t);
  if (!lazy) reduce_all<A>(a, ar);
  xchg<typename A::T, LOGN, B0, B1>(a, lds, t);
  fwd_round<A, LOGN, B1, B0 - 1, B1>(a, ar, w, t);
  if (!lazy) reduce_all<A>(a, ar);
  xchg<typename A::T, LOGN, B1, 0>(a, lds, t);
  fwd_round<A, LOGN, 0, B1 - 1, 0>(a, ar, w, t);
  u64 r[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) r[k] = ar.final_fwd(a[k]);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(row_ptr(io.dst, c, l, b), 0, N * 8, 0x00020000);
  static_assert(!NTT_FWD_DIRECT || !epi_aut(EPI), "no automorphism epilogue in the direct-store build");
  if constexpr (NTT_FWD_DIRECT) {  // thread t holds outputs 32 t .. 32 t + 31
    if constexpr (EPI == NTT_EPI_STORE) {
#pragma unroll
      for (int k = 0; k < 32; k += 2) {
        buf_st2(rd, r[k], r[k + 1], t * 256, k * 8);
        if ((k & 7) == 6) NTT_FENCE();
      }
    } else {
      const __amdgpu_buffer_rsrc_t rx =
          __builtin_amdgcn_make_buffer_rsrc(row_ptr(io.ex, c, l, b), 0, N * 8, 0x00020000);
      const u64 s = io.s[l], ss = io.ss[l];
#pragma unroll
      for (int k = 0; k < 32; k += 2) {
        u64 x, y;
        buf_ld2(rx, x, y, t * 256, k * 8);
        buf_st2(rd, shoup_mul(sub_mod(x, r[k], mc.q), s, ss, mc.q), shoup_mul(sub_mod(y, r[k + 1], mc.q), s, ss, mc.q),
                t * 256, k * 8);
        if ((k & 7) == 6) NTT_FENCE();
      }
    }
    return;
  }
  xchg<u64, LOGN, 0, B0>(r, lds, t);
  if constexpr (EPI == NTT_EPI_STORE) {
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      buf_st(rd, r[k], t * 8, (k << B0) * 8);
      if ((k & 3) == 3) NTT_FENCE();
    }
  } else if constexpr (epi_aut(EPI)) {
    // dst[aut[e]] = (ex[e] - y[e]) * s_l (+ dst[aut[e]] for _ACC): the
    // rotation's NTT-domain automorphism folded into the ModDown's store (groups
    // of 8 rows: the ex words and the scatter indices of a group loaded before
    // it is stored)
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(row_ptr(io.ex, c, l, b), 0, N * 8, 0x00020000);
    const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)io.aut, 0, N * 4, 0x00020000);
    const u64 s = io.s[l], ss = io.ss[l];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u64 xv[8];
      u32 ix[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        xv[k] = buf_ld(rx, t * 8, ((8 * g + k) << B0) * 8);
        ix[k] = __builtin_amdgcn_raw_buffer_load_b32(ri, t * 4, ((8 * g + k) << B0) * 4, 0);
      }
      NTT_FENCE();
      if constexpr (EPI == NTT_EPI_SUBSCALE_AUT_ACC) {
        u64 ov[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) ov[k] = buf_ld(rd, (int)ix[k] * 8, 0);
        NTT_FENCE();
#pragma unroll
        for (int k = 0; k < 8; ++k)
          buf_st(rd, add_mod(ov[k], shoup_mul(sub_mod(xv[k], r[8 * g + k], mc.q), s, ss, mc.q), mc.q), (int)ix[k] * 8, 0);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) buf_st(rd, shoup_mul(sub_mod(xv[k], r[8 * g + k], mc.q), s, ss, mc.q), (int)ix[k] * 8, 0);
      }
      NTT_FENCE();
    }
  } else {  // NTT_EPI_SUBSCALE: dst = (ex - y) * s_l  (ModDown / rescale tail)
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(row_ptr(io.ex, c, l, b), 0, N * 8, 0x00020000);
    const u64 s = io.s[l], ss = io.ss[l];
    if constexpr (NTT_EPI_PF) {
      // ex in groups of 8 rows, the next group's loads issued before the
      // current group is consumed: one load latency per job instead of four
      u64 xa[8], xb[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) xa[k] = buf_ld(rx, t * 8, (k << B0) * 8);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (g < 3) {
#pragma unroll
          for (int k = 0; k < 8; ++k) xb[k] = buf_ld(rx, t * 8, ((8 * (g + 1) + k) << B0) * 8);
        }
        NTT_FENCE();
#pragma unroll
        for (int k = 0; k < 8; ++k)
          buf_st(rd, shoup_mul(sub_mod(xa[k], r[8 * g + k], mc.q), s, ss, mc.q), t * 8, ((8 * g + k) << B0) * 8);
        NTT_FENCE();
#pragma unroll
        for (int k = 0; k < 8; ++k) xa[k] = xb[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        const u64 x = buf_ld(rx, t * 8, (k << B0) * 8);
        buf_st(rd, shoup_mul(sub_mod(x, r[k], mc.q), s, ss, mc.q), t * 8, (k << B0) * 8);
        if ((k & 7) == 7) NTT_FENCE();
      }
    }
  }
}

template <class A, int LOGN, bool CI>
__device__ __forceinline__ void ntt_inv_body(const NttIO& io, int c, int l, int b, const ModConst& mc, const A& ar,
                                             __amdgpu_buffer_rsrc_t w, u32* lds) {
  constexpr int N = 1 << LOGN, B0 = LOGN - 5, B1 = LOGN - 10;
  // an opaque copy of the thread index per job: keeps the persistent job loop
  // from hoisting every thread-derived address out of the loop (LICM), whose
  // live ranges would then span the whole body and spill
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row_ptr(io.src, c, l, b), 0, N * 8, 0x00020000);
  typename A::T a[32];
  if constexpr (NTT_INV_COAL) {
    u64 x[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = buf_ld(rs, t * 8, (k << B0) * 8);
    xchg<u64, LOGN, B0, 0>(x, lds, t);
#pragma unroll
    for (int k = 0; k < 32; ++k) a[k] = ar.from_u64(x[k]);
  } else {
#pragma unroll
    for (int k = 0; k < 32; k += 2) {
      u64 x, y;
      buf_ld2(rs, x, y, t * 256, k * 8);
      a[k] = ar.from_u64(x);
      a[k + 1] = ar.from_u64(y);
    }
  }
  inv_round<A, LOGN, 0, 0, B1 - 1>(a, ar, w, t);
  if (!NTT_INV_NORED) reduce_all<A>(a, ar);
  xchg<typename A::T, LOGN, 0, B1>(a, lds, t);
  inv_round<A, LOGN, B1, B1, B0 - 1>(a, ar, w, t);
  if (!NTT_INV_NORED) reduce_all<A>(a, ar);
  xchg<typename A::T, LOGN, B1, B0>(a, lds, t);
  inv_round<A, LOGN, B0, B0, LOGN - 1>(a, ar, w, t);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(row_ptr(io.dst, c, l, b), 0, N * 8, 0x00020000);
  if constexpr (CI) {
    // ConjugateInvariant unfold: a_e = b_e + W b_{N-e} with b already scaled by
    // (2N)^-1 (ninv), a_0 = 2 b_0.  The partner of row k of thread t is row
    // 31 - k of thread S - t (t = 0: row 32 - k of thread 0), so each half of
    // the rows is finished against the other half staged in LDS as u64
    // (16 S words = 4N bytes, inside the exchange buffer): rows 16..31 against
    // rows 0..15, then rows 0..15 against rows 16..31.
    constexpr int S = NttGeom<LOGN>::T;
    u64* const l64 = reinterpret_cast<u64*>(lds);
    u64 r[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) r[k] = NTT_INV_FOLD ? ar.final_inv_folded(a[k]) : ar.final_inv(a[k]);
#pragma unroll
    for (int k = 0; k < 16; ++k) l64[k * S + t] = r[k];
    __syncthreads();
#pragma unroll
    for (int k = 16; k < 32; ++k) {
      u64 y = l64[(32 - k) * S - t];  // k = 16, t = 0: e = N/2 pairs with itself
      if (k == 16) y = t == 0 ? r[16] : y;
      buf_st(rd, add_mod(r[k], shoup_mul(y, mc.ciw, mc.ciw_s, mc.q), mc.q), t * 8, (k << B0) * 8);
      if ((k & 3) == 3) NTT_FENCE();
    }
    __syncthreads();
#pragma unroll
    for (int k = 16; k < 32; ++k) l64[(k - 16) * S + t] = r[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const u64 y = l64[(16 - k) * S - t];  // k = 0, t = 0: e = 0, no partner
      u64 v = add_mod(r[k], shoup_mul(y, mc.ciw, mc.ciw_s, mc.q), mc.q);
      if (k == 0) v = t == 0 ? add_mod(r[0], r[0], mc.q) : v;
      buf_st(rd, v, t * 8, (k << B0) * 8);
      if ((k & 3) == 3) NTT_FENCE();
    }
    __syncthreads();  // the next job of a persistent workgroup writes LDS in its first exchange
    return;
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    buf_st(rd, NTT_INV_FOLD ? ar.final_inv_folded(a[k]) : ar.final_inv(a[k]), t * 8, (k << B0) * 8);
    if ((k & 3) == 3) NTT_FENCE();
  }
}


// Persistent: a grid of at most one workgroup per CU walks the launch's jobs
// (job w + k G in round k, or G - 1 - w in odd rounds with NTT_SNAKE; in io.order), so a CU goes from one limb's
// stores straight to the next limb's loads: no workgroup retire/dispatch
// bubble between limbs, and the stores drain while the next limb loads and
// computes.  LDS needs no extra barrier between jobs: every exchange ends
// with one.
// The subtract-and-scale epilogue variants keep one job per workgroup: as a
// loop their extra live values spill (36-41 VGPRs at N = 2^15).
// Desynchronise the CUs of a persistent launch: half of each XCD's
// workgroups (blockIdx bit 3; workgroups go round-robin over the 8 XCDs)
// start late, so their memory phases fall into the other half's compute
// phases instead of all 256 CUs contending for HBM at once.
__device__ __forceinline__ void ntt_stagger(const NttIO& io) {
  if (io.stagger > 0 && (blockIdx.x & 8))
    for (int i = 0; i < io.stagger; ++i) __builtin_amdgcn_s_sleep(127);
}

// 1: the subtract-and-scale (ModDown / rescale tail) variants are persistent
// too (they no longer spill: 1 VGPR, outside the job loop)
#ifndef NTT_PERSIST_ALL
#define NTT_PERSIST_ALL 1
#endif
// 1: a persistent workgroup's jobs run in snake order -- job w of every even
// round, job G - 1 - w of every odd one (G workgroups).  With the integer-path
// (slower) limbs dispatched first, the workgroups that took the fast float64
// jobs of a round take the first jobs of the next: a 384-job launch (1.5
// rounds, one third integer-path) ends after one float64 job more on the
// float64 workgroups instead of one more after an integer job
#ifndef NTT_SNAKE
#define NTT_SNAKE 1
#endif
__device__ __forceinline__ int snake_job(int r, int w, int G) {
  return r * G + ((NTT_SNAKE && (r & 1)) ? G - 1 - w : w);
}

template <int EPI>
struct FwdPersist {
  static constexpr bool value = EPI == NTT_EPI_STORE || NTT_PERSIST_ALL;
};

template <int LOGN, int PRO, int EPI, bool CI>
__device__ __forceinline__ void ntt_fwd_job(const NttIO& io, int job, const DeviceTables* __restrict__ tb, u32* lds) {
  constexpr int N = 1 << LOGN;
  int c, l, b;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if (mc.f64) {
    const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)tb->fwd_d[mod], 0, N * 8, 0x00020000);
    ntt_fwd_body<F64Arith, LOGN, PRO, EPI, CI>(io, c, l, b, mc, F64Arith(mc), w, lds, tb);
  } else {
    const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)tb->fwd[mod], 0, N * 16, 0x00020000);
    ntt_fwd_body<IntArith, LOGN, PRO, EPI, CI>(io, c, l, b, mc, IntArith(mc), w, lds, tb);
  }
}

template <int LOGN, int PRO, int EPI, bool CI>
__global__ void __launch_bounds__(NttGeom<LOGN>::T) ntt_fwd_kernel(NttIO io, const DeviceTables* __restrict__ tb) {
  extern __shared__ u32 lds[];
  if constexpr (FwdPersist<EPI>::value) {
    ntt_stagger(io);
    const int nj = io.njob > 0 ? io.njob : io.jobs;
#pragma nounroll
    for (int r = 0; r * (int)gridDim.x < nj; ++r) {
      const int job = snake_job(r, blockIdx.x, gridDim.x);
      if (job < nj) ntt_fwd_job<LOGN, PRO, EPI, CI>(io, job, tb, lds);
    }
  } else {
    ntt_fwd_job<LOGN, PRO, EPI, CI>(io, blockIdx.x, tb, lds);
  }
}

template <int LOGN, bool CI>
__global__ void __launch_bounds__(NttGeom<LOGN>::T) ntt_inv_kernel(NttIO io, const DeviceTables* __restrict__ tb) {
  constexpr int N = 1 << LOGN;
  extern __shared__ u32 lds[];
  ntt_stagger(io);
  const int nj = io.njob > 0 ? io.njob : io.jobs;
#pragma nounroll
  for (int r = 0; r * (int)gridDim.x < nj; ++r) {
    const int job = snake_job(r, blockIdx.x, gridDim.x);
    if (job >= nj) continue;
    int c, l, b;
    job_of(io, job, c, l, b);
    const int mod = arg_byte(io.dst.mod, l);
    const ModConst mc = tb->mc[mod];
    if (mc.f64) {
      const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)tb->inv_d[mod], 0, N * 8, 0x00020000);
      ntt_inv_body<F64Arith, LOGN, CI>(io, c, l, b, mc, F64Arith(mc), w, lds);
    } else {
      const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)tb->inv[mod], 0, N * 16, 0x00020000);
      ntt_inv_body<IntArith, LOGN, CI>(io, c, l, b, mc, IntArith(mc), w, lds);
    }
  }
}

template <int LOGN, int PRO, int EPI, bool CI>
void set_lds_attr() {
  hipFuncSetAttribute((const void*)ntt_fwd_kernel<LOGN, PRO, EPI, CI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      ((1 << LOGN) + (1 << LOGN) / 32) * 4);
}

// workgroups of a persistent launch (0: one workgroup per job); set by orion_ntt_init
int g_ntt_grid = 0;

template <int LOGN, bool CI>
int launch_ntt_ring(const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st) {
  constexpr int N = 1 << LOGN;
  const int total = io.dst.ncomp * io.dst.nlimb * io.dst.nbatch;
  if (total == 0) return 0;
  if (io.jobs != total || io.njob < 0 || io.njob > total || io.job0 != 0) return -1;
  const int jobs = io.njob > 0 ? io.njob : total;  // njob: the first njob jobs only (a split launch)
  const size_t lds = (size_t)(N + N / 32) * sizeof(u32);
  const int gmax = io.grid > 0 ? io.grid : g_ntt_grid;
  const dim3 g(gmax > 0 && jobs > gmax ? gmax : jobs), blk(NttGeom<LOGN>::T);
  if (inverse) {
    if (io.pro != NTT_PRO_LOAD || io.epi != NTT_EPI_STORE) return -1;
    hipLaunchKernelGGL((ntt_inv_kernel<LOGN, CI>), g, blk, lds, st, io, tb);
    return 0;
  }
#define FWD(P, E)                                                                                     \
  if (io.pro == P && io.epi == E) {                                                                   \
    hipLaunchKernelGGL((ntt_fwd_kernel<LOGN, P, E, CI>), FwdPersist<E>::value ? g : dim3(jobs), blk, lds, st, io, tb); \
    return 0;                                                                                         \
  }
  FWD(NTT_PRO_LOAD, NTT_EPI_STORE)
  FWD(NTT_PRO_LOAD, NTT_EPI_SUBSCALE)
  if constexpr (!CI) {
    if (epi_aut(io.epi) && !io.aut) return -1;
    FWD(NTT_PRO_LOAD, NTT_EPI_SUBSCALE_AUT)
    FWD(NTT_PRO_LOAD, NTT_EPI_SUBSCALE_AUT_ACC)
  }
  FWD(NTT_PRO_RESCALE, NTT_EPI_SUBSCALE)
  if constexpr (!CI) {
    FWD(NTT_PRO_BEXT, NTT_EPI_STORE)
    FWD(NTT_PRO_BEXT, NTT_EPI_SUBSCALE)
  }
#undef FWD
  return -1;
}

// NTT_ONLY15 (register-usage experiments only, never shipped): instantiate
// the N = 2^15 Standard-ring kernels alone, so one compile takes seconds
template <int LOGN>
int launch_ntt(const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st) {
#ifdef NTT_ONLY15
  return io.ci ? -1 : launch_ntt_ring<LOGN, false>(io, tb, inverse, st);
#else
  return io.ci ? launch_ntt_ring<LOGN, true>(io, tb, inverse, st) : launch_ntt_ring<LOGN, false>(io, tb, inverse, st);
#endif
}

template <int LOGN, bool CI>
void init_lds_ring() {
  set_lds_attr<LOGN, NTT_PRO_LOAD, NTT_EPI_STORE, CI>();
  set_lds_attr<LOGN, NTT_PRO_LOAD, NTT_EPI_SUBSCALE, CI>();
  set_lds_attr<LOGN, NTT_PRO_RESCALE, NTT_EPI_SUBSCALE, CI>();
  if constexpr (!CI) set_lds_attr<LOGN, NTT_PRO_LOAD, NTT_EPI_SUBSCALE_AUT, CI>();
  if constexpr (!CI) set_lds_attr<LOGN, NTT_PRO_LOAD, NTT_EPI_SUBSCALE_AUT_ACC, CI>();
  if constexpr (!CI) {
    set_lds_attr<LOGN, NTT_PRO_BEXT, NTT_EPI_STORE, CI>();
    set_lds_attr<LOGN, NTT_PRO_BEXT, NTT_EPI_SUBSCALE, CI>();
  }
  hipFuncSetAttribute((const void*)ntt_inv_kernel<LOGN, CI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      ((1 << LOGN) + (1 << LOGN) / 32) * 4);
}
template <int LOGN>
void init_lds() {
  init_lds_ring<LOGN, false>();
#ifndef NTT_ONLY15
  init_lds_ring<LOGN, true>();
#endif
}

}  // namespace

// host entry: NTT (inverse=false) or INTT with the fused prologue / epilogue of io
int orion_launch_ntt_io(int logN, const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st) {
  switch (logN) {
#ifndef NTT_ONLY15
    case 13: return launch_ntt<13>(io, tb, inverse, st);
    case 14: return launch_ntt<14>(io, tb, inverse, st);
#endif
    case 15: return launch_ntt<15>(io, tb, inverse, st);
    default: return -1;
  }
}

// in-place NTT / INTT of every limb in s
int orion_launch_ntt(int logN, const LimbSet& s, const DeviceTables* tb, bool inverse, hipStream_t st) {
  NttIO io;
  memset(&io, 0, sizeof(io));
  io.dst = io.src = s;
  io.jobs = s.ncomp * s.nlimb * s.nbatch;
  return orion_launch_ntt_io(logN, io, tb, inverse, st);
}

// allow >64 KiB dynamic LDS for the N = 2^14, 2^15 kernels; size the
// persistent grid: ORION_NTT_PERSIST workgroups per CU (0 = one per job)
int orion_ntt_init() {
#ifndef NTT_ONLY15
  init_lds<13>();
  init_lds<14>();
#endif
  init_lds<15>();
  const char* e = getenv("ORION_NTT_PERSIST");
  const int per_cu = e ? atoi(e) : 1;
  int dev = 0, ncu = 0;
  if (per_cu > 0 && hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
    g_ntt_grid = per_cu * ncu;
  else
    g_ntt_grid = 0;
  if (getenv("ORION_NTT_GRID")) g_ntt_grid = atoi(getenv("ORION_NTT_GRID"));  // timing switch: workgroups
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
