// ntt2s.hip -- latency-oriented two-pass NTT / INTT for launches of few
// limb-transforms (one image: the batch-1 forward pass, small decompositions)
// at N = 2^15 and 2^16.
//
// The same transform and the same pass split as ntt2.hip (Lattigo v6 ring
// convention, e = col + 256 * row; cols pass = the stages on the row bits,
// rows pass = the stages on bits 7..0), but each thread owns ONE butterfly of
// every stage instead of a 16-point sub-transform: the tile sits in LDS and
// every stage is one LDS read, one butterfly, one LDS write and one barrier.
// ntt2.hip's thread runs 32 butterflies back to back per pass, which a launch
// of a few limbs (under one wave per SIMD) cannot hide; here the per-thread
// chain is R or 8 butterflies and a launch has 16x the threads.  Large
// launches keep ntt2.hip / ntt.hip (more LDS traffic and barriers per
// butterfly here).  Outputs are fully reduced, so they are bit-identical to
// the other kernels'.
#include <type_traits>

#include "common.h"
#include "ntt_arith.h"
#include "ntt2s_rows.h"

namespace {

// columns per cols-pass workgroup at N = 2^15, rows per rows-pass workgroup:
// a launch of J jobs runs J 256/CW (J 2^R/RW) workgroups, and with a few jobs
// (one image) the time is that of the CUs holding the most workgroups
#ifndef NTT2S_CW15
#define NTT2S_CW15 8
#endif
#ifndef NTT2S_RW
#define NTT2S_RW 4
#endif
// timing-only ablation (tools/build_ablation.py; 0 in the product): bit 0 =
// no inverse columns butterflies, bit 1 = no basis-extension / rescale
// prologue arithmetic in ntt2s_ifwd_cols_p, bit 2 = no forward columns butterflies
#ifndef NTT2S_ABLATE
#define NTT2S_ABLATE 0
#endif
// 1: ntt2s_ifwd_cols_p fetches its forward twiddles before the INTT half
#ifndef NTT2S_FWD_PREFETCH
#define NTT2S_FWD_PREFETCH 0
#endif
template <int LOGN>
struct S2 {
  static constexpr int R = LOGN - 8;            // row bits: the cols pass transforms 2^R-point columns
  static constexpr int CW = LOGN == 15 ? NTT2S_CW15 : 4;  // columns per cols-pass workgroup
  static constexpr int H = 1 << (R - 1);         // butterflies per column per stage
  static constexpr int CT = CW * H;              // cols-pass threads (512)
  static constexpr int CTILES = 256 / CW;        // cols-pass workgroups per limb
  static constexpr int RW = NTT2S_RW;           // rows per rows-pass workgroup
  static constexpr int RT = RW * 128;            // rows-pass threads (512)
  static constexpr int RTILES = (1 << R) / RW;   // rows-pass workgroups per limb
  static constexpr int CT4 = CW << (R - 2);      // radix-4 cols-pass threads (256)
  static constexpr int RT4 = RW * 64;            // radix-4 rows-pass threads (256)
};


// lower index of butterfly k of a stage on bit `bit` (pairs lo, lo + 2^bit)
[[maybe_unused]] __device__ __forceinline__ int lo_of(int k, int bit) { return ((k >> bit) << (bit + 1)) | (k & ((1 << bit) - 1)); }

__device__ __forceinline__ u64* mid_row_s(const NttIO& io, int job, int c, int l, int b) {
  if (io.mid_compact) {
    const unsigned r = __builtin_amdgcn_readfirstlane((unsigned)(job - io.job0));
    return io.mid.p + (long long)r * io.mid.batch_stride;
  }
  return row_ptr(io.mid, c, l, b);
}

// forward prologue: element e of job (c, l, b)
template <class A, int PRO>
__device__ __forceinline__ typename A::T fwd_load(const NttIO& io, int c, int l, int b, int e, const ModConst& mc,
                                                  const A& ar, const DeviceTables* __restrict__ tb) {
  if constexpr (PRO == NTT_PRO_LOAD) {
    return ar.from_u64(row_ptr(io.src, c, l, b)[e]);
  } else if constexpr (PRO == NTT_PRO_BEXT) {
    const int k = arg_byte(io.bx_tab, l), ti = arg_byte(io.bx_t, l), s0 = arg_byte(io.bx_s0, k);
    const BasisExtTable* __restrict__ T = io.bx + k;
    const int ns = T->ns;
    u64 x[2] = {row_ptr(io.src, c, s0, b)[e], ns > 1 ? row_ptr(io.src, c, s0 + 1, b)[e] : 0}, y[2];
    const u64 v = bext_prep<2>(T, x, y);
    return ar.from_u64(bext_target_sel<2>(T->tgt + ti, ns, y, v));
  } else {  // NTT_PRO_RESCALE
    const u64 qL = tb->mc[io.modL].q, h = qL >> 1;
    const u64 hm = barrett128(0, h, mc);
    const u64 x = row_ptr(io.src, c, 0, b)[e];
    return ar.from_u64(sub_mod(barrett128(0, add_mod(x, h, qL), mc), hm, mc.q));
  }
}

// ---------------------------------------------------------------------------
// forward cols pass: thread (cl, k) owns butterfly k of column cl in each of
// the R stages d = LOGN-1 .. 8 (row bit rb = d - 8); twiddle of row group
// i = lo >> (rb + 1) = k >> rb is w[(N >> (d+1)) + i]
// ---------------------------------------------------------------------------
template <class A, int LOGN>
__device__ __forceinline__ void s_fwd_cols_core(const NttIO& io, int job, int c, int l, int b, int tile,
                                                typename A::T x, typename A::T y, const A& ar,
                                                __amdgpu_buffer_rsrc_t tw, u64* lds) {
  constexpr int N = 1 << LOGN, R = S2<LOGN>::R, CW = S2<LOGN>::CW;
  const int t = threadIdx.x, cl = t % CW, k = t / CW, col = tile * CW + cl;
  typename A::W w[R];
#pragma unroll
  for (int s = 0; s < R; ++s) {
    const int rb = R - 1 - s;
    w[s] = ar.tw(tw, k >> rb, N >> (rb + 9));
  }
#pragma unroll
  for (int s = 0; s < R; ++s) {
    const int rb = R - 1 - s, lo = lo_of(k, rb);
    if (s > 0) {
      x = from_bits<typename A::T>(lds[lo * CW + cl]);
      y = from_bits<typename A::T>(lds[(lo + (1 << rb)) * CW + cl]);
    }
    ar.ct(x, y, w[s]);
    if (s == 3) x = ar.reduce_round(x), y = ar.reduce_round(y);  // float64: |x| stays below 16q
    if (s < R - 1) {
      lds[lo * CW + cl] = to_bits(x);
      lds[(lo + (1 << rb)) * CW + cl] = to_bits(y);
      __syncthreads();
    }
  }
  x = ar.reduce_round(x), y = ar.reduce_round(y);
  u64* mid = mid_row_s(io, job, c, l, b);
  const int lo = 2 * k;  // the last stage's pair: rows 2k, 2k + 1
  mid[col + (lo << 8)] = to_bits(x);
  mid[col + ((lo + 1) << 8)] = to_bits(y);
}
template <class A, int LOGN, int PRO>
__device__ __forceinline__ void s_fwd_cols(const NttIO& io, int job, int c, int l, int b, int tile, const ModConst& mc,
                                           const A& ar, __amdgpu_buffer_rsrc_t tw, u64* lds,
                                           const DeviceTables* __restrict__ tb) {
  constexpr int CW = S2<LOGN>::CW, H = S2<LOGN>::H;
  const int t = threadIdx.x, cl = t % CW, k = t / CW, col = tile * CW + cl;
  const typename A::T x = fwd_load<A, PRO>(io, c, l, b, col + (k << 8), mc, ar, tb);
  const typename A::T y = fwd_load<A, PRO>(io, c, l, b, col + ((k + H) << 8), mc, ar, tb);
  s_fwd_cols_core<A, LOGN>(io, job, c, l, b, tile, x, y, ar, tw, lds);
}

// forward rows pass: thread (rr, kk) owns butterfly kk of row rr in each of
// the stages d = 7 .. 0; twiddle w[(N >> (d+1)) + ((row << (7-d)) | (kk >> d))]
template <class A, int LOGN, int EPI>
__device__ __forceinline__ void s_fwd_rows(const NttIO& io, int job, int c, int l, int b, int tile, const ModConst& mc,
                                           const A& ar, __amdgpu_buffer_rsrc_t tw, u64* lds) {
  constexpr int N = 1 << LOGN;
  const int t = threadIdx.x, rr = t >> 7, kk = t & 127, row = tile * S2<LOGN>::RW + rr;
  typename A::W w[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int d = 7 - s;
    w[s] = ar.tw(tw, (row << (7 - d)) | (kk >> d), N >> (d + 1));
  }
  const u64* mid = mid_row_s(io, job, c, l, b) + (row << 8);
  typename A::T x = from_bits<typename A::T>(mid[kk]);
  typename A::T y = from_bits<typename A::T>(mid[kk + 128]);
  u64* lr = lds + rr * 256;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int d = 7 - s, lo = lo_of(kk, d);
    if (s > 0) {
      x = from_bits<typename A::T>(lr[lo]);
      y = from_bits<typename A::T>(lr[lo + (1 << d)]);
    }
    ar.ct(x, y, w[s]);
    if (s == 3) x = ar.reduce_round(x), y = ar.reduce_round(y);
    if (s < 7) {
      lr[lo] = to_bits(x);
      lr[lo + (1 << d)] = to_bits(y);
      __syncthreads();
    }
  }
  // the last stage's pair: columns 2kk, 2kk + 1
  u64* dst = row_ptr(io.dst, c, l, b) + (row << 8) + 2 * kk;
  const u64 ox = ar.final_fwd(x), oy = ar.final_fwd(y);
  if constexpr (EPI == NTT_EPI_STORE) {
    *(ulonglong2*)dst = make_ulonglong2(ox, oy);
  } else {  // NTT_EPI_SUBSCALE: dst = (ex - y) * s_l
    const ulonglong2 e = *(const ulonglong2*)(row_ptr(io.ex, c, l, b) + (row << 8) + 2 * kk);
    const u64 s = io.s[l], ss = io.ss[l];
    *(ulonglong2*)dst = make_ulonglong2(shoup_mul(sub_mod(e.x, ox, mc.q), s, ss, mc.q),
                                        shoup_mul(sub_mod(e.y, oy, mc.q), s, ss, mc.q));
  }
}

// inverse rows pass (first): stages d = 0 .. 7, GS; the sum reduced every other stage
template <class A, int LOGN>
__device__ __forceinline__ void s_inv_rows(const NttIO& io, int job, int c, int l, int b, int tile, const A& ar,
                                           __amdgpu_buffer_rsrc_t tw, u64* lds) {
  constexpr int N = 1 << LOGN;
  const int t = threadIdx.x, rr = t >> 7, kk = t & 127, row = tile * S2<LOGN>::RW + rr;
  typename A::W w[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) w[s] = ar.tw(tw, (row << (7 - s)) | (kk >> s), N >> (s + 1));
  const ulonglong2 v = *(const ulonglong2*)(row_ptr(io.src, c, l, b) + (row << 8) + 2 * kk);
  typename A::T x = ar.from_u64(v.x), y = ar.from_u64(v.y);
  u64* lr = lds + rr * 256;
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    const int lo = lo_of(kk, d);
    if (d > 0) {
      x = from_bits<typename A::T>(lr[lo]);
      y = from_bits<typename A::T>(lr[lo + (1 << d)]);
    }
    ar.gs(x, y, w[d], (d & 1) == 1);
    if (d < 7) {
      lr[lo] = to_bits(x);
      lr[lo + (1 << d)] = to_bits(y);
      __syncthreads();
    }
  }
  x = ar.reduce_round(x), y = ar.reduce_round(y);
  u64* mid = mid_row_s(io, job, c, l, b) + (row << 8);
  mid[kk] = to_bits(x);  // the last stage's pair: columns kk, kk + 128
  mid[kk + 128] = to_bits(y);
}

// inverse cols pass (second): stages d = 8 .. LOGN-1 (row bit rb = d - 8), times N^-1
template <class A, int LOGN>
__device__ __forceinline__ void s_inv_cols(const NttIO& io, int job, int c, int l, int b, int tile, const A& ar,
                                           __amdgpu_buffer_rsrc_t tw, u64* lds) {
  constexpr int N = 1 << LOGN, R = S2<LOGN>::R, CW = S2<LOGN>::CW, H = S2<LOGN>::H;
  const int t = threadIdx.x, cl = t % CW, k = t / CW, col = tile * CW + cl;
  typename A::W w[R];
#pragma unroll
  for (int rb = 0; rb < R; ++rb) w[rb] = ar.tw(tw, k >> rb, N >> (rb + 9));
  const u64* mid = mid_row_s(io, job, c, l, b);
  typename A::T x = from_bits<typename A::T>(mid[col + ((2 * k) << 8)]);
  typename A::T y = from_bits<typename A::T>(mid[col + ((2 * k + 1) << 8)]);
#pragma unroll
  for (int rb = 0; rb < R; ++rb) {
    const int lo = lo_of(k, rb);
    if (rb > 0) {
      x = from_bits<typename A::T>(lds[lo * CW + cl]);
      y = from_bits<typename A::T>(lds[(lo + (1 << rb)) * CW + cl]);
    }
    ar.gs(x, y, w[rb], (rb & 1) == 1);
    if (rb < R - 1) {
      lds[lo * CW + cl] = to_bits(x);
      lds[(lo + (1 << rb)) * CW + cl] = to_bits(y);
      __syncthreads();
    }
  }
  u64* dst = row_ptr(io.dst, c, l, b);  // the last stage's pair: rows k, k + H
  dst[col + (k << 8)] = ar.final_inv(x);
  dst[col + ((k + H) << 8)] = ar.final_inv(y);
}

// the inverse's columns pass over one column tile of up to two source limbs
// (interleaved, one LDS region each), kept in registers: thread (cl, k) ends
// with rows k and k + H of column col of every source -- exactly the pair its
// forward columns pass starts from, so the two passes meet without an exchange
template <class A0, class A1, int LOGN, bool TWO>
__device__ __forceinline__ void s_inv_cols_src(const u64* m0, const u64* m1, const A0& a0, const A1& a1,
                                               __amdgpu_buffer_rsrc_t tw0, __amdgpu_buffer_rsrc_t tw1, u64* lds,
                                               u64 (&xa)[2], u64 (&xb)[2]) {
  constexpr int N = 1 << LOGN, R = S2<LOGN>::R, CW = S2<LOGN>::CW;
  const int t = threadIdx.x, cl = t % CW, k = t / CW, col = blockIdx.x % S2<LOGN>::CTILES * CW + cl;
  typename A0::W w0[R];
  typename A1::W w1[R];
#pragma unroll
  for (int rb = 0; rb < R; ++rb) {
    w0[rb] = a0.tw(tw0, k >> rb, N >> (rb + 9));
    if (TWO) w1[rb] = a1.tw(tw1, k >> rb, N >> (rb + 9));
  }
  typename A0::T x0 = from_bits<typename A0::T>(m0[col + ((2 * k) << 8)]);
  typename A0::T y0 = from_bits<typename A0::T>(m0[col + ((2 * k + 1) << 8)]);
  typename A1::T x1{}, y1{};
  if (TWO) {
    x1 = from_bits<typename A1::T>(m1[col + ((2 * k) << 8)]);
    y1 = from_bits<typename A1::T>(m1[col + ((2 * k + 1) << 8)]);
  }
  u64* const l0 = lds;
  u64* const l1 = lds + (CW << R);
#pragma unroll
  for (int rb = 0; rb < R; ++rb) {
    const int lo = lo_of(k, rb), hi = lo + (1 << rb);
    if (rb > 0) {
      x0 = from_bits<typename A0::T>(l0[lo * CW + cl]);
      y0 = from_bits<typename A0::T>(l0[hi * CW + cl]);
      if (TWO) {
        x1 = from_bits<typename A1::T>(l1[lo * CW + cl]);
        y1 = from_bits<typename A1::T>(l1[hi * CW + cl]);
      }
    }
    a0.gs(x0, y0, w0[rb], (rb & 1) == 1);
    if (TWO) a1.gs(x1, y1, w1[rb], (rb & 1) == 1);
    if (rb < R - 1) {
      l0[lo * CW + cl] = to_bits(x0);
      l0[hi * CW + cl] = to_bits(y0);
      if (TWO) {
        l1[lo * CW + cl] = to_bits(x1);
        l1[hi * CW + cl] = to_bits(y1);
      }
      __syncthreads();
    }
  }
  xa[0] = a0.final_inv(x0), xb[0] = a0.final_inv(y0);
  if (TWO) xa[1] = a1.final_inv(x1), xb[1] = a1.final_inv(y1);
}

template <class A0, int LOGN>
__device__ __forceinline__ void s_inv_cols_src2(const u64* m0, const u64* m1, const A0& a0, int mod1, bool two,
                                                const DeviceTables* __restrict__ tb, __amdgpu_buffer_rsrc_t tw0,
                                                u64* lds, u64 (&xa)[2], u64 (&xb)[2]) {
  if (!two) {
    s_inv_cols_src<A0, A0, LOGN, false>(m0, m0, a0, a0, tw0, tw0, lds, xa, xb);
    return;
  }
  const ModConst& mc1 = tb->mc[mod1];
  if (mc1.f64)
    s_inv_cols_src<A0, F64Arith, LOGN, true>(m0, m1, a0, F64Arith(mc1), tw0, twr_s(tb->inv_d[mod1], 8 << LOGN), lds,
                                             xa, xb);
  else
    s_inv_cols_src<A0, IntArith, LOGN, true>(m0, m1, a0, IntArith(mc1), tw0, twr_s(tb->inv[mod1], 16 << LOGN), lds,
                                             xa, xb);
}

// ---------------------------------------------------------------------------
// radix-4 form (NTT2S_R4): a thread owns 4 elements and runs two stages per
// LDS exchange (two butterflies per stage), so a pass has half the barriers
// and exchanges of the one-butterfly form with half the threads.  Step on
// bits (b, b - 1) (forward) or (b, b + 1) (inverse) over elements
//   e0 = j with two zero bits inserted at those positions, e1 = e0 + 2^lo_bit,
//   e2 = e0 + 2^hi_bit, e3 = e2 + 2^lo_bit.
// An odd stage count ends (forward) or ends (inverse) with one radix-2 stage.
// A forward columns pass starts on, and an inverse columns pass ends on, the
// set {j, j + 2^(R-2), j + 2^(R-1), j + 3 2^(R-2)} -- so ntt2s_ifwd_cols needs
// no exchange between its inverse and forward halves.
// ---------------------------------------------------------------------------
// forward columns pass, radix 4: thread (cl, j), j < 2^(R-2)
// the twiddles of thread row j's forward columns stages (wa/wb/wc per radix-4
// step, wl for an odd last stage)
template <class A, int LOGN>
__device__ __forceinline__ void s_fwd_cols4_tw(const A& ar, __amdgpu_buffer_rsrc_t tw, int j,
                                               typename A::W (&wa)[S2<LOGN>::R / 2],
                                               typename A::W (&wb)[S2<LOGN>::R / 2],
                                               typename A::W (&wc)[S2<LOGN>::R / 2], typename A::W (&wl)[2]) {
  constexpr int N = 1 << LOGN, R = S2<LOGN>::R, NS = R / 2;
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int hb = R - 1 - 2 * st, g = j >> (hb - 1);
    wa[st] = ar.tw(tw, g, N >> (hb + 9));
    wb[st] = ar.tw(tw, 2 * g, N >> (hb + 8));
    wc[st] = ar.tw(tw, 2 * g + 1, N >> (hb + 8));
  }
  if (R & 1) wl[0] = ar.tw(tw, 2 * j, N >> 9), wl[1] = ar.tw(tw, 2 * j + 1, N >> 9);
}
template <class A, int LOGN>
__device__ __forceinline__ void s_fwd_cols4_run(const NttIO& io, int job, int c, int l, int b, int tile,
                                                typename A::T (&x)[4], const A& ar,
                                                const typename A::W (&wa)[S2<LOGN>::R / 2],
                                                const typename A::W (&wb)[S2<LOGN>::R / 2],
                                                const typename A::W (&wc)[S2<LOGN>::R / 2],
                                                const typename A::W (&wl)[2], u64* lds, int t) {
  constexpr int R = S2<LOGN>::R, CW = S2<LOGN>::CW, NS = R / 2;
  const int cl = t % CW, j = t / CW, col = tile * CW + cl;
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int hb = R - 1 - 2 * st, lb = hb - 1;
    const int e0 = ins2(j, lb), e1 = e0 + (1 << lb), e2 = e0 + (1 << hb), e3 = e2 + (1 << lb);
    if (st > 0) {
      x[0] = from_bits<typename A::T>(lds[e0 * CW + cl]);
      x[1] = from_bits<typename A::T>(lds[e1 * CW + cl]);
      x[2] = from_bits<typename A::T>(lds[e2 * CW + cl]);
      x[3] = from_bits<typename A::T>(lds[e3 * CW + cl]);
    }
    if (!(NTT2S_ABLATE & 4)) ct4(ar, x, wa[st], wb[st], wc[st]);
    if (st == 1)  // after 4 stages (float64: |x| stays below 16q)
      for (int i = 0; i < 4; ++i) x[i] = ar.reduce_round(x[i]);
    if (st < NS - 1 || (R & 1)) {
      lds[e0 * CW + cl] = to_bits(x[0]);
      lds[e1 * CW + cl] = to_bits(x[1]);
      lds[e2 * CW + cl] = to_bits(x[2]);
      lds[e3 * CW + cl] = to_bits(x[3]);
      __syncthreads();
    }
  }
  if (R & 1) {  // the last stage (bit 0): pairs (4j, 4j + 1), (4j + 2, 4j + 3)
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = from_bits<typename A::T>(lds[(4 * j + i) * CW + cl]);
    if (!(NTT2S_ABLATE & 4)) ar.ct(x[0], x[1], wl[0]);
    if (!(NTT2S_ABLATE & 4)) ar.ct(x[2], x[3], wl[1]);
  }
  u64* mid = mid_row_s(io, job, c, l, b);
#pragma unroll
  for (int i = 0; i < 4; ++i) mid[col + ((4 * j + i) << 8)] = to_bits(ar.reduce_round(x[i]));
}
template <class A, int LOGN>
__device__ __forceinline__ void s_fwd_cols4_core(const NttIO& io, int job, int c, int l, int b, int tile,
                                                 typename A::T (&x)[4], const A& ar, __amdgpu_buffer_rsrc_t tw,
                                                 u64* lds, int t) {
  constexpr int NS = S2<LOGN>::R / 2;
  typename A::W wa[NS], wb[NS], wc[NS], wl[2];
  s_fwd_cols4_tw<A, LOGN>(ar, tw, t / S2<LOGN>::CW, wa, wb, wc, wl);
  s_fwd_cols4_run<A, LOGN>(io, job, c, l, b, tile, x, ar, wa, wb, wc, wl, lds, t);
}
template <class A, int LOGN, int PRO>
__device__ __forceinline__ void s_fwd_cols4(const NttIO& io, int job, int c, int l, int b, int tile,
                                            const ModConst& mc, const A& ar, __amdgpu_buffer_rsrc_t tw, u64* lds,
                                            const DeviceTables* __restrict__ tb) {
  constexpr int R = S2<LOGN>::R, CW = S2<LOGN>::CW, Q = 1 << (R - 2);
  const int t = threadIdx.x, cl = t % CW, j = t / CW, col = tile * CW + cl;
  typename A::T x[4];
  if constexpr (PRO == NTT_PRO_BEXT) {
    // the extension's constants once per thread, through the scalar cache (bext2_load)
    const int k = arg_byte(io.bx_tab, l), ti = arg_byte(io.bx_t, l), s0 = arg_byte(io.bx_s0, k);
    const Bext2 bc = bext2_load(io.bx + k, ti);
    const u64* p0 = row_ptr(io.src, c, s0, b);
    const u64* p1 = row_ptr(io.src, c, s0 + (bc.ns > 1 ? 1 : 0), b);
    u64 x0[4], x1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x0[i] = p0[col + ((j + i * Q) << 8)];
      x1[i] = bc.ns > 1 ? p1[col + ((j + i * Q) << 8)] : 0;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = ar.from_u64(bext2_apply(bc, x0[i], x1[i]));
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = fwd_load<A, PRO>(io, c, l, b, col + ((j + i * Q) << 8), mc, ar, tb);
  }
  s_fwd_cols4_core<A, LOGN>(io, job, c, l, b, tile, x, ar, tw, lds, (int)threadIdx.x);
}

// forward rows pass, radix 4: thread (rr, kk), kk < 64
template <class A, int LOGN, int EPI>
__device__ __forceinline__ void s_fwd_rows4(const NttIO& io, int job, int c, int l, int b, int tile, const ModConst& mc,
                                            const A& ar, __amdgpu_buffer_rsrc_t tw, u64* lds) {
  const int t = threadIdx.x, rr = t >> 6, kk = t & 63, row = tile * S2<LOGN>::RW + rr;
  const u64* mid = mid_row_s(io, job, c, l, b) + (row << 8);
  typename A::T x[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = from_bits<typename A::T>(mid[kk + 64 * i]);
  typename A::W wa[4], wb[4], wc[4];
  fwd_rows4_tw<A, LOGN>(row, kk, ar, tw, wa, wb, wc);
  // the epilogue's operands are loaded before the steps, so their latency
  // overlaps them: ex, the scatter index and (_ACC) the words at aut[e] (aut
  // is a permutation: no other thread of the launch writes them)
  [[maybe_unused]] ulonglong2 e01, e23;
  [[maybe_unused]] uint4 ix;
  [[maybe_unused]] u64 dv[4];
  if constexpr (EPI != NTT_EPI_STORE) {
    const u64* ex = row_ptr(io.ex, c, l, b) + (row << 8) + 4 * kk;
    e01 = *(const ulonglong2*)ex, e23 = *(const ulonglong2*)(ex + 2);
  }
  u64* const d = row_ptr(io.dst, c, l, b);
  if constexpr (epi_aut(EPI)) {
    ix = *(const uint4*)(io.aut + (row << 8) + 4 * kk);
    if constexpr (EPI == NTT_EPI_SUBSCALE_AUT_ACC) dv[0] = d[ix.x], dv[1] = d[ix.y], dv[2] = d[ix.z], dv[3] = d[ix.w];
  }
  fwd_rows4_run<A>(x, kk, ar, wa, wb, wc, lds + rr * 256);
  // the last step's elements: columns 4kk .. 4kk + 3
  u64* dst = d + (row << 8) + 4 * kk;
  u64 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = ar.final_fwd(x[i]);
  if constexpr (EPI != NTT_EPI_STORE) {  // dst = (ex - y) * s_l
    const u64 ev[4] = {e01.x, e01.y, e23.x, e23.y};
    const u64 s = io.s[l], ss = io.ss[l];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = shoup_mul(sub_mod(ev[i], o[i], mc.q), s, ss, mc.q);
  }
  if constexpr (epi_aut(EPI)) {  // element e to position aut[e] (added to the word there for _ACC)
    if constexpr (EPI == NTT_EPI_SUBSCALE_AUT_ACC) {
      o[0] = add_mod(o[0], dv[0], mc.q);
      o[1] = add_mod(o[1], dv[1], mc.q);
      o[2] = add_mod(o[2], dv[2], mc.q);
      o[3] = add_mod(o[3], dv[3], mc.q);
    }
    d[ix.x] = o[0];
    d[ix.y] = o[1];
    d[ix.z] = o[2];
    d[ix.w] = o[3];
    return;
  }
  *(ulonglong2*)dst = make_ulonglong2(o[0], o[1]);
  *(ulonglong2*)(dst + 2) = make_ulonglong2(o[2], o[3]);
}

// inverse rows pass, radix 4 (first): steps on bits (0, 1) .. (6, 7)
// (inv_rows4_core, ntt2s_rows.h)
template <class A, int LOGN>
__device__ __forceinline__ void s_inv_rows4(const NttIO& io, int job, int c, int l, int b, int tile, const A& ar,
                                            __amdgpu_buffer_rsrc_t tw, u64* lds) {
  const int t = threadIdx.x, rr = t >> 6, kk = t & 63, row = tile * S2<LOGN>::RW + rr;
  const u64* src = row_ptr(io.src, c, l, b) + (row << 8) + 4 * kk;
  const ulonglong2 v01 = *(const ulonglong2*)src, v23 = *(const ulonglong2*)(src + 2);
  typename A::T x[4] = {ar.from_u64(v01.x), ar.from_u64(v01.y), ar.from_u64(v23.x), ar.from_u64(v23.y)};
  inv_rows4_core<A, LOGN>(x, row, kk, ar, tw, lds + rr * 256, mid_row_s(io, job, c, l, b) + (row << 8));
}

// inverse columns pass, radix 4 (second), up to two source limbs interleaved
// (ntt2s_ifwd_cols) or one (ntt2s_inv_cols); ends on the forward's first set
template <class A0, class A1, int LOGN, bool TWO>
__device__ __forceinline__ void s_inv_cols4_src(const u64* m0, const u64* m1, const A0& a0, const A1& a1,
                                                __amdgpu_buffer_rsrc_t tw0, __amdgpu_buffer_rsrc_t tw1, u64* lds,
                                                typename A0::T (&x)[4], typename A1::T (&y)[4], int t, int tile) {
  constexpr int N = 1 << LOGN, R = S2<LOGN>::R, CW = S2<LOGN>::CW, NS = R / 2, Q = 1 << (R - 2);
  const int cl = t % CW, j = t / CW, col = tile * CW + cl;
  typename A0::W wa0[NS], wb0[NS], wc0[NS], wl0;
  typename A1::W wa1[NS], wb1[NS], wc1[NS], wl1;
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int lb = 2 * st, g = j >> lb;
    wa0[st] = a0.tw(tw0, 2 * g, N >> (lb + 9));
    wb0[st] = a0.tw(tw0, 2 * g + 1, N >> (lb + 9));
    wc0[st] = a0.tw(tw0, g, N >> (lb + 10));
    if (TWO) {
      wa1[st] = a1.tw(tw1, 2 * g, N >> (lb + 9));
      wb1[st] = a1.tw(tw1, 2 * g + 1, N >> (lb + 9));
      wc1[st] = a1.tw(tw1, g, N >> (lb + 10));
    }
  }
  if (R & 1) {  // the last stage (bit R - 1): one twiddle
    wl0 = a0.tw(tw0, 0, N >> (R + 8));
    if (TWO) wl1 = a1.tw(tw1, 0, N >> (R + 8));
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    x[i] = from_bits<typename A0::T>(m0[col + ((4 * j + i) << 8)]);
    if (TWO) y[i] = from_bits<typename A1::T>(m1[col + ((4 * j + i) << 8)]);
  }
  u64* const l0 = lds;
  u64* const l1 = lds + (CW << R);
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int lb = 2 * st, hb = lb + 1;
    const int e0 = ins2(j, lb), e1 = e0 + (1 << lb), e2 = e0 + (1 << hb), e3 = e2 + (1 << lb);
    const int e[4] = {e0, e1, e2, e3};
    if (st > 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[i] = from_bits<typename A0::T>(l0[e[i] * CW + cl]);
        if (TWO) y[i] = from_bits<typename A1::T>(l1[e[i] * CW + cl]);
      }
    }
    if (!(NTT2S_ABLATE & 1)) {
      gs4(a0, x, wa0[st], wb0[st], wc0[st], false, true);
      if (TWO) gs4(a1, y, wa1[st], wb1[st], wc1[st], false, true);
    }
    if (st < NS - 1 || (R & 1)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        l0[e[i] * CW + cl] = to_bits(x[i]);
        if (TWO) l1[e[i] * CW + cl] = to_bits(y[i]);
      }
      __syncthreads();
    }
  }
  if (R & 1) {  // bit R - 1: pairs (j, j + 2Q), (j + Q, j + 3Q); the sum is not reduced (stage R - 1 even)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[i] = from_bits<typename A0::T>(l0[(j + i * Q) * CW + cl]);
      if (TWO) y[i] = from_bits<typename A1::T>(l1[(j + i * Q) * CW + cl]);
    }
    if (!(NTT2S_ABLATE & 1)) a0.gs(x[0], x[2], wl0, ((R - 1) & 1) == 1);
    if (!(NTT2S_ABLATE & 1)) a0.gs(x[1], x[3], wl0, ((R - 1) & 1) == 1);
    if (TWO && !(NTT2S_ABLATE & 1)) {
      a1.gs(y[0], y[2], wl1, ((R - 1) & 1) == 1);
      a1.gs(y[1], y[3], wl1, ((R - 1) & 1) == 1);
    }
  }
}

// the radix-4 inverse columns pass of the sources, to canonical residues:
// v[s][i] = element i of the thread's set, source s
template <class A0, int LOGN>
__device__ __forceinline__ void s_inv_cols4_src2(const u64* m0, const u64* m1, const A0& a0, int mod1, bool two,
                                                 const DeviceTables* __restrict__ tb, __amdgpu_buffer_rsrc_t tw0,
                                                 u64* lds, u64 (&v)[2][4], int t, int tile) {
  typename A0::T x[4];
  if (!two) {
    typename A0::T y[4];
    s_inv_cols4_src<A0, A0, LOGN, false>(m0, m0, a0, a0, tw0, tw0, lds, x, y, t, tile);
  } else {
    const ModConst& mc1 = tb->mc[mod1];
    if (mc1.f64) {
      const F64Arith a1(mc1);
      double y[4];
      s_inv_cols4_src<A0, F64Arith, LOGN, true>(m0, m1, a0, a1, tw0, twr_s(tb->inv_d[mod1], 8 << LOGN), lds, x, y, t,
                                                  tile);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[1][i] = a1.final_inv(y[i]);
    } else {
      const IntArith a1(mc1);
      u64 y[4];
      s_inv_cols4_src<A0, IntArith, LOGN, true>(m0, m1, a0, a1, tw0, twr_s(tb->inv[mod1], 16 << LOGN), lds, x, y, t,
                                                  tile);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[1][i] = a1.final_inv(y[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) v[0][i] = a0.final_inv(x[i]);
}

// forward columns pass of a launch whose sources skipped the inverse's columns
// pass (NttIO.ifuse): each workgroup (target job, column tile) finishes the
// sources' INTT on its tile, forms the prologue (the basis extension, or the
// rescale prep) from registers, and runs the forward columns stages -- the
// INTT output never goes to HBM and its second launch disappears
template <int LOGN, int PRO>
__global__ void __launch_bounds__(NTT2S_R4 ? S2<LOGN>::CT4 : S2<LOGN>::CT)
    ntt2s_ifwd_cols(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[2 * (S2<LOGN>::CW << S2<LOGN>::R)];
  const int job = io.job0 + blockIdx.x / S2<LOGN>::CTILES, tile = blockIdx.x % S2<LOGN>::CTILES;
  int c, l, b;
  job_of(io, job, c, l, b);
  // the sources: limbs sl0 (, sl0 + 1) of src, inverse intermediate in imid
  int sl0 = 0, ns = 1, ti = 0;
  const BasisExtTable* __restrict__ T = nullptr;
  if constexpr (PRO == NTT_PRO_BEXT) {
    const int kt = arg_byte(io.bx_tab, l);
    ti = arg_byte(io.bx_t, l);
    sl0 = arg_byte(io.bx_s0, kt);
    T = io.bx + kt;
    ns = T->ns;
  }
  [[maybe_unused]] Bext2 bc;  // the extension's constants, before the INTT half (bext2_load)
  if constexpr (PRO == NTT_PRO_BEXT) bc = bext2_load(T, ti);
  const int m0 = arg_byte(io.src.mod, sl0), m1 = ns > 1 ? arg_byte(io.src.mod, sl0 + 1) : m0;
  const u64* p0 = row_ptr(io.imid, c, sl0, b);
  const u64* p1 = ns > 1 ? row_ptr(io.imid, c, sl0 + 1, b) : p0;
  const ModConst& mc0 = tb->mc[m0];
  constexpr int NE = NTT2S_R4 ? 4 : 2;  // elements per thread
  u64 v[2][NE];
  if constexpr (NTT2S_R4) {
    if (mc0.f64)
      s_inv_cols4_src2<F64Arith, LOGN>(p0, p1, F64Arith(mc0), m1, ns > 1, tb, twr_s(tb->inv_d[m0], 8 << LOGN), lds, v,
                                       (int)threadIdx.x, tile);
    else
      s_inv_cols4_src2<IntArith, LOGN>(p0, p1, IntArith(mc0), m1, ns > 1, tb, twr_s(tb->inv[m0], 16 << LOGN), lds, v,
                                       (int)threadIdx.x, tile);
  } else {
    u64 xa[2] = {0, 0}, xb[2] = {0, 0};
    if (mc0.f64)
      s_inv_cols_src2<F64Arith, LOGN>(p0, p1, F64Arith(mc0), m1, ns > 1, tb, twr_s(tb->inv_d[m0], 8 << LOGN), lds, xa,
                                      xb);
    else
      s_inv_cols_src2<IntArith, LOGN>(p0, p1, IntArith(mc0), m1, ns > 1, tb, twr_s(tb->inv[m0], 16 << LOGN), lds, xa,
                                      xb);
    v[0][0] = xa[0], v[1][0] = xa[1], v[0][1] = xb[0], v[1][1] = xb[1];
  }
  __syncthreads();  // the forward stages reuse the LDS
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  u64 o[NE];
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    if constexpr (PRO == NTT_PRO_BEXT) {
      o[i] = bext2_apply(bc, v[0][i], ns > 1 ? v[1][i] : 0);
    } else {  // NTT_PRO_RESCALE: ((x + h) mod q_L) mod q_l - (h mod q_l)
      const u64 qL = tb->mc[io.modL].q, h = qL >> 1;
      const u64 hm = barrett128(0, h, mc);
      o[i] = sub_mod(barrett128(0, add_mod(v[0][i], h, qL), mc), hm, mc.q);
    }
  }
  auto fwd = [&](const auto& ar, __amdgpu_buffer_rsrc_t tw) {
    using A = std::decay_t<decltype(ar)>;
    if constexpr (NTT2S_R4) {
      typename A::T x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = ar.from_u64(o[i]);
      s_fwd_cols4_core<A, LOGN>(io, job, c, l, b, tile, x, ar, tw, lds, (int)threadIdx.x);
    } else {
      s_fwd_cols_core<A, LOGN>(io, job, c, l, b, tile, ar.from_u64(o[0]), ar.from_u64(o[1]), ar, tw, lds);
    }
  };
  if (mc.f64)
    fwd(F64Arith(mc), twr_s(tb->fwd_d[mod], 8 << LOGN));
  else
    fwd(IntArith(mc), twr_s(tb->fwd[mod], 16 << LOGN));
}

// the same with the sources' INTT columns shared by a segment of G targets
// (NttIO.tgroup = G > 1, radix-4; targets that read the same source limbs): a
// workgroup of G groups of 256 threads per (row, segment, column tile) runs
// the sources' INTT columns once -- source s on group s, concurrently -- then
// every group forms its own target's prologue from the shared values and runs
// that target's forward columns stages.  The arithmetic is ntt2s_ifwd_cols's
// (bit-identical); the columns work that kernel redoes for every target is
// done once per segment, on as many threads per workgroup as targets.
template <int LOGN>
__device__ __forceinline__ void idle_inv_cols4_barriers() {  // the barriers of s_inv_cols4_src
  constexpr int R = S2<LOGN>::R, NS = R / 2;
#pragma unroll
  for (int k = 0; k < NS - 1 + (R & 1); ++k) __syncthreads();
}
template <int LOGN, int PRO, int G>
__global__ void __launch_bounds__(G * S2<LOGN>::CT4) ntt2s_ifwd_cols_p(NttIO io, const DeviceTables* __restrict__ tb) {
  static_assert(NTT2S_R4 || LOGN < 0, "radix-4 only");
  constexpr int CT = S2<LOGN>::CT4, REG = S2<LOGN>::CW << S2<LOGN>::R;  // LDS words per group
  __shared__ u64 lds[G * REG + 2 * 4 * CT];
  u64* const sb = lds + G * REG;  // the sources' INTT values, [source][element][thread]
  // BEXT: the sources' y_i (in sb) and float-quotient terms, formed once per
  // source in phase 1 instead of once per target in phase 2
  [[maybe_unused]] __shared__ double sf[PRO == NTT_PRO_BEXT ? 2 * 4 * CT : 1];
  const int grp = threadIdx.x / CT, t = threadIdx.x % CT;  // (group-uniform, so wave-uniform)
  const int tile = blockIdx.x % S2<LOGN>::CTILES, q = blockIdx.x / S2<LOGN>::CTILES;
  const int seg = q % io.ntg, row = q / io.ntg;
  const int b = row % io.dst.nbatch, c = row / io.dst.nbatch;
  // surplus groups of a short segment redo its last target (identical stores)
  const int l = arg_byte(io.tg_l0, seg) + min(grp, arg_byte(io.tg_n, seg) - 1);
  int sl0 = 0, ns = 1, ti = 0;
  const BasisExtTable* __restrict__ T = nullptr;
  if constexpr (PRO == NTT_PRO_BEXT) {
    const int kt = arg_byte(io.bx_tab, l);
    ti = arg_byte(io.bx_t, l);
    sl0 = arg_byte(io.bx_s0, kt);
    T = io.bx + kt;
    ns = T->ns;
  }
  // the extension's constants, in SGPRs before the INTT half (bext2_load)
  [[maybe_unused]] Bext2 bc;
  if constexpr (PRO == NTT_PRO_BEXT) bc = bext2_load(T, ti);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  // NTT2S_FWD_PREFETCH: the forward stages' twiddles are fetched before the
  // INTT half, so their latency overlaps it (timing switch)
  constexpr int NS = S2<LOGN>::R / 2;
  [[maybe_unused]] ulonglong2 pw[3 * NS + 2];
  if constexpr (NTT2S_FWD_PREFETCH) {
    auto pre = [&](const auto& ar, __amdgpu_buffer_rsrc_t tw) {
      using A = std::decay_t<decltype(ar)>;
      typename A::W wa[NS], wb[NS], wc[NS], wl[2];
      s_fwd_cols4_tw<A, LOGN>(ar, tw, t / S2<LOGN>::CW, wa, wb, wc, wl);
#pragma unroll
      for (int k = 0; k < NS; ++k) pw[k] = w_raw(wa[k]), pw[NS + k] = w_raw(wb[k]), pw[2 * NS + k] = w_raw(wc[k]);
      if (S2<LOGN>::R & 1) pw[3 * NS] = w_raw(wl[0]), pw[3 * NS + 1] = w_raw(wl[1]);
    };
    if (mc.f64)
      pre(F64Arith(mc), twr_s(tb->fwd_d[mod], 8 << LOGN));
    else
      pre(IntArith(mc), twr_s(tb->fwd[mod], 16 << LOGN));
  }
  // phase 1: group s < ns finishes source s's INTT columns on this tile
  if (grp < ns) {
    const int ms = arg_byte(io.src.mod, sl0 + grp);
    const u64* p = row_ptr(io.imid, c, sl0 + grp, b);
    const ModConst& mcs = tb->mc[ms];
    auto inv = [&](const auto& ar, __amdgpu_buffer_rsrc_t tw) {
      using A = std::decay_t<decltype(ar)>;
      typename A::T x[4], y[4];
      s_inv_cols4_src<A, A, LOGN, false>(p, p, ar, ar, tw, tw, lds + grp * REG, x, y, t, tile);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        u64 xv = ar.final_inv(x[i]);
        if constexpr (PRO == NTT_PRO_BEXT && !(NTT2S_ABLATE & 2)) {
          if (!bc.centered) {  // (grp wave-uniform: constant table indices on each branch)
            double f;
            xv = __builtin_amdgcn_readfirstlane(grp) == 0 ? bext2_src(bc, 0, xv, f) : bext2_src(bc, 1, xv, f);
            sf[(grp * 4 + i) * CT + t] = f;
          }
        }
        sb[(grp * 4 + i) * CT + t] = xv;
      }
    };
    if (mcs.f64)
      inv(F64Arith(mcs), twr_s(tb->inv_d[ms], 8 << LOGN));
    else
      inv(IntArith(mcs), twr_s(tb->inv[ms], 16 << LOGN));
  } else {
    idle_inv_cols4_barriers<LOGN>();
  }
  __syncthreads();  // sb complete; the group regions are free for the forward stages
  u64 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u64 v0 = sb[i * CT + t];
    if constexpr (NTT2S_ABLATE & 2) {
      o[i] = v0 + (ns > 1 ? sb[(4 + i) * CT + t] : 0);
    } else if constexpr (PRO == NTT_PRO_BEXT) {
      const u64 y1 = ns > 1 ? sb[(4 + i) * CT + t] : 0;
      const double f0 = bc.centered ? 0.0 : sf[i * CT + t];
      const double f1 = (bc.centered || ns < 2) ? 0.0 : sf[(4 + i) * CT + t];
      o[i] = bext2_tgt(bc, v0, y1, bext2_v(bc, v0, f0, f1));
    } else {  // NTT_PRO_RESCALE
      const u64 qL = tb->mc[io.modL].q, h = qL >> 1;
      const u64 hm = barrett128(0, h, mc);
      o[i] = sub_mod(barrett128(0, add_mod(v0, h, qL), mc), hm, mc.q);
    }
  }
  auto fwd = [&](const auto& ar, __amdgpu_buffer_rsrc_t tw) {
    using A = std::decay_t<decltype(ar)>;
    typename A::T x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = ar.from_u64(o[i]);
    if constexpr (NTT2S_FWD_PREFETCH) {
      typename A::W wa[NS], wb[NS], wc[NS], wl[2];
#pragma unroll
      for (int k = 0; k < NS; ++k)
        wa[k] = w_of<A>(pw[k]), wb[k] = w_of<A>(pw[NS + k]), wc[k] = w_of<A>(pw[2 * NS + k]);
      wl[0] = w_of<A>(pw[3 * NS]), wl[1] = w_of<A>(pw[3 * NS + 1]);
      s_fwd_cols4_run<A, LOGN>(io, 0, c, l, b, tile, x, ar, wa, wb, wc, wl, lds + grp * REG, t);
    } else {
      s_fwd_cols4_core<A, LOGN>(io, 0, c, l, b, tile, x, ar, tw, lds + grp * REG, t);
    }
  };
  if (mc.f64)
    fwd(F64Arith(mc), twr_s(tb->fwd_d[mod], 8 << LOGN));
  else
    fwd(IntArith(mc), twr_s(tb->fwd[mod], 16 << LOGN));
}

// ---------------------------------------------------------------------------
// kernels: blockIdx.x = job * tiles + tile
// ---------------------------------------------------------------------------
template <int LOGN, int PRO>
__global__ void __launch_bounds__(NTT2S_R4 ? S2<LOGN>::CT4 : S2<LOGN>::CT)
    ntt2s_fwd_cols(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[S2<LOGN>::CW << S2<LOGN>::R];
  const int job = io.job0 + blockIdx.x / S2<LOGN>::CTILES, tile = blockIdx.x % S2<LOGN>::CTILES;
  int c, l, b;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if constexpr (NTT2S_R4) {
    if (mc.f64)
      s_fwd_cols4<F64Arith, LOGN, PRO>(io, job, c, l, b, tile, mc, F64Arith(mc), twr_s(tb->fwd_d[mod], 8 << LOGN), lds,
                                       tb);
    else
      s_fwd_cols4<IntArith, LOGN, PRO>(io, job, c, l, b, tile, mc, IntArith(mc), twr_s(tb->fwd[mod], 16 << LOGN), lds,
                                       tb);
  } else if (mc.f64)
    s_fwd_cols<F64Arith, LOGN, PRO>(io, job, c, l, b, tile, mc, F64Arith(mc), twr_s(tb->fwd_d[mod], 8 << LOGN), lds, tb);
  else
    s_fwd_cols<IntArith, LOGN, PRO>(io, job, c, l, b, tile, mc, IntArith(mc), twr_s(tb->fwd[mod], 16 << LOGN), lds, tb);
}

template <int LOGN, int EPI>
__global__ void __launch_bounds__(NTT2S_R4 ? S2<LOGN>::RT4 : S2<LOGN>::RT)
    ntt2s_fwd_rows(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[S2<LOGN>::RW * 256];
  const int job = io.job0 + blockIdx.x / S2<LOGN>::RTILES, tile = blockIdx.x % S2<LOGN>::RTILES;
  int c, l, b;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  static_assert(NTT2S_R4 || !epi_aut(EPI), "the automorphism epilogue is radix-4 only");
  if constexpr (NTT2S_R4) {
    if (mc.f64)
      s_fwd_rows4<F64Arith, LOGN, EPI>(io, job, c, l, b, tile, mc, F64Arith(mc), twr_s(tb->fwd_d[mod], 8 << LOGN), lds);
    else
      s_fwd_rows4<IntArith, LOGN, EPI>(io, job, c, l, b, tile, mc, IntArith(mc), twr_s(tb->fwd[mod], 16 << LOGN), lds);
  } else if (mc.f64)
    s_fwd_rows<F64Arith, LOGN, EPI>(io, job, c, l, b, tile, mc, F64Arith(mc), twr_s(tb->fwd_d[mod], 8 << LOGN), lds);
  else
    s_fwd_rows<IntArith, LOGN, EPI>(io, job, c, l, b, tile, mc, IntArith(mc), twr_s(tb->fwd[mod], 16 << LOGN), lds);
}

template <int LOGN>
__global__ void __launch_bounds__(NTT2S_R4 ? S2<LOGN>::RT4 : S2<LOGN>::RT)
    ntt2s_inv_rows(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[S2<LOGN>::RW * 256];
  const int job = io.job0 + blockIdx.x / S2<LOGN>::RTILES, tile = blockIdx.x % S2<LOGN>::RTILES;
  int c, l, b;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if constexpr (NTT2S_R4) {
    if (mc.f64)
      s_inv_rows4<F64Arith, LOGN>(io, job, c, l, b, tile, F64Arith(mc), twr_s(tb->inv_d[mod], 8 << LOGN), lds);
    else
      s_inv_rows4<IntArith, LOGN>(io, job, c, l, b, tile, IntArith(mc), twr_s(tb->inv[mod], 16 << LOGN), lds);
  } else if (mc.f64)
    s_inv_rows<F64Arith, LOGN>(io, job, c, l, b, tile, F64Arith(mc), twr_s(tb->inv_d[mod], 8 << LOGN), lds);
  else
    s_inv_rows<IntArith, LOGN>(io, job, c, l, b, tile, IntArith(mc), twr_s(tb->inv[mod], 16 << LOGN), lds);
}

template <int LOGN>
__global__ void __launch_bounds__(NTT2S_R4 ? S2<LOGN>::CT4 : S2<LOGN>::CT)
    ntt2s_inv_cols(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[S2<LOGN>::CW << S2<LOGN>::R];
  const int job = io.job0 + blockIdx.x / S2<LOGN>::CTILES, tile = blockIdx.x % S2<LOGN>::CTILES;
  int c, l, b;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if constexpr (NTT2S_R4) {
    auto inv = [&](const auto& ar, __amdgpu_buffer_rsrc_t tw) {
      using A = std::decay_t<decltype(ar)>;
      constexpr int CW = S2<LOGN>::CW, Q = 1 << (S2<LOGN>::R - 2);
      const int t = threadIdx.x, cl = t % CW, j = t / CW, col = tile * CW + cl;
      typename A::T x[4], y[4];
      const u64* m = mid_row_s(io, job, c, l, b);
      s_inv_cols4_src<A, A, LOGN, false>(m, m, ar, ar, tw, tw, lds, x, y, t, tile);
      u64* dst = row_ptr(io.dst, c, l, b);
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[col + ((j + i * Q) << 8)] = ar.final_inv(x[i]);
    };
    if (mc.f64)
      inv(F64Arith(mc), twr_s(tb->inv_d[mod], 8 << LOGN));
    else
      inv(IntArith(mc), twr_s(tb->inv[mod], 16 << LOGN));
  } else if (mc.f64)
    s_inv_cols<F64Arith, LOGN>(io, job, c, l, b, tile, F64Arith(mc), twr_s(tb->inv_d[mod], 8 << LOGN), lds);
  else
    s_inv_cols<IntArith, LOGN>(io, job, c, l, b, tile, IntArith(mc), twr_s(tb->inv[mod], 16 << LOGN), lds);
}

template <int LOGN>
int launch2s(const NttIO& io, const DeviceTables* tb, bool inverse, bool rows_only, hipStream_t st) {
  const int total = io.dst.ncomp * io.dst.nlimb * io.dst.nbatch;
  if (total == 0) return 0;
  if (io.jobs != total || io.ci) return -1;
  const int jobs = io.njob ? io.njob : total;
  if (io.job0 < 0 || io.job0 + jobs > total) return -1;
  if (io.mid_compact && io.mid.batch_stride < (1 << LOGN)) return -1;
  const dim3 ga(jobs * S2<LOGN>::CTILES), ba(NTT2S_R4 ? S2<LOGN>::CT4 : S2<LOGN>::CT), gb(jobs * S2<LOGN>::RTILES),
      bb(NTT2S_R4 ? S2<LOGN>::RT4 : S2<LOGN>::RT);
  if (inverse) {
    if (io.pro != NTT_PRO_LOAD || io.epi != NTT_EPI_STORE) return -1;
    hipLaunchKernelGGL(ntt2s_inv_rows<LOGN>, gb, bb, 0, st, io, tb);
    // rows_only: the columns pass is left to the forward launch that consumes
    // this INTT (NttIO.ifuse; the intermediate stays in io.mid)
    if (!rows_only) hipLaunchKernelGGL(ntt2s_inv_cols<LOGN>, ga, ba, 0, st, io, tb);
    return 0;
  }
  if (io.ifuse && io.tgroup > 1) {
    if (io.mid_compact || !io.imid.p || io.job0 != 0 || jobs != total || io.ntg < 1) return -1;
    const dim3 gg(io.dst.ncomp * io.dst.nbatch * io.ntg * S2<LOGN>::CTILES);
    if constexpr (NTT2S_R4) {
      const bool bx = io.pro == NTT_PRO_BEXT;
      if (!bx && io.pro != NTT_PRO_RESCALE) return -1;
      if (io.tgroup == 2) {
        const dim3 bg(2 * S2<LOGN>::CT4);
        if (bx)
          hipLaunchKernelGGL((ntt2s_ifwd_cols_p<LOGN, NTT_PRO_BEXT, 2>), gg, bg, 0, st, io, tb);
        else
          hipLaunchKernelGGL((ntt2s_ifwd_cols_p<LOGN, NTT_PRO_RESCALE, 2>), gg, bg, 0, st, io, tb);
      } else if (io.tgroup == 4) {
        const dim3 bg(4 * S2<LOGN>::CT4);
        if (bx)
          hipLaunchKernelGGL((ntt2s_ifwd_cols_p<LOGN, NTT_PRO_BEXT, 4>), gg, bg, 0, st, io, tb);
        else
          hipLaunchKernelGGL((ntt2s_ifwd_cols_p<LOGN, NTT_PRO_RESCALE, 4>), gg, bg, 0, st, io, tb);
      } else {
        return -1;
      }
    } else {
      return -1;
    }
  } else if (io.ifuse) {
    if (io.mid_compact || !io.imid.p) return -1;
    if (io.pro == NTT_PRO_BEXT)
      hipLaunchKernelGGL((ntt2s_ifwd_cols<LOGN, NTT_PRO_BEXT>), ga, ba, 0, st, io, tb);
    else if (io.pro == NTT_PRO_RESCALE)
      hipLaunchKernelGGL((ntt2s_ifwd_cols<LOGN, NTT_PRO_RESCALE>), ga, ba, 0, st, io, tb);
    else
      return -1;
  } else if (io.pro == NTT_PRO_LOAD)
    hipLaunchKernelGGL((ntt2s_fwd_cols<LOGN, NTT_PRO_LOAD>), ga, ba, 0, st, io, tb);
  else if (io.pro == NTT_PRO_BEXT)
    hipLaunchKernelGGL((ntt2s_fwd_cols<LOGN, NTT_PRO_BEXT>), ga, ba, 0, st, io, tb);
  else if (io.pro == NTT_PRO_RESCALE)
    hipLaunchKernelGGL((ntt2s_fwd_cols<LOGN, NTT_PRO_RESCALE>), ga, ba, 0, st, io, tb);
  else
    return -1;
  if (io.cols_only) {  // the rows pass runs in the consumer
    if (io.epi != NTT_EPI_STORE) return -1;
    return 0;
  }
  if (io.epi == NTT_EPI_STORE)
    hipLaunchKernelGGL((ntt2s_fwd_rows<LOGN, NTT_EPI_STORE>), gb, bb, 0, st, io, tb);
  else if (io.epi == NTT_EPI_SUBSCALE)
    hipLaunchKernelGGL((ntt2s_fwd_rows<LOGN, NTT_EPI_SUBSCALE>), gb, bb, 0, st, io, tb);
  else if (io.epi == NTT_EPI_SUBSCALE_AUT && NTT2S_R4 && io.aut)
    hipLaunchKernelGGL((ntt2s_fwd_rows<LOGN, NTT2S_R4 ? NTT_EPI_SUBSCALE_AUT : NTT_EPI_SUBSCALE>), gb, bb, 0, st, io, tb);
  else if (io.epi == NTT_EPI_SUBSCALE_AUT_ACC && NTT2S_R4 && io.aut)
    hipLaunchKernelGGL((ntt2s_fwd_rows<LOGN, NTT2S_R4 ? NTT_EPI_SUBSCALE_AUT_ACC : NTT_EPI_SUBSCALE>), gb, bb, 0, st, io, tb);
  else
    return -1;
  return 0;
}

}  // namespace

// host entry: two launches on stream st (same contract as orion_launch_ntt2);
// inverse with rows_only: the rows pass alone (its columns pass then runs
// inside the forward launch that reads this INTT, NttIO.ifuse)
int orion_launch_ntt2s(int logN, const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st,
                       bool rows_only) {
  if (rows_only && (!inverse || io.mid_compact)) return -1;
  switch (logN) {
    case 15: return launch2s<15>(io, tb, inverse, rows_only, st);
    case 16: return launch2s<16>(io, tb, inverse, rows_only, st);
    default: return -1;
  }
}
