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
#include "common.h"
#include "ntt_arith.h"

namespace {

template <int LOGN>
struct S2 {
  static constexpr int R = LOGN - 8;            // row bits: the cols pass transforms 2^R-point columns
  static constexpr int CW = LOGN == 15 ? 8 : 4;  // columns per cols-pass workgroup
  static constexpr int H = 1 << (R - 1);         // butterflies per column per stage
  static constexpr int CT = CW * H;              // cols-pass threads (512)
  static constexpr int CTILES = 256 / CW;        // cols-pass workgroups per limb
  static constexpr int RW = 4;                   // rows per rows-pass workgroup
  static constexpr int RT = RW * 128;            // rows-pass threads (512)
  static constexpr int RTILES = (1 << R) / RW;   // rows-pass workgroups per limb
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t twr_s(const void* t, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)t, 0, bytes, 0x00020000);
}

// lower index of butterfly k of a stage on bit `bit` (pairs lo, lo + 2^bit)
__device__ __forceinline__ int lo_of(int k, int bit) { return ((k >> bit) << (bit + 1)) | (k & ((1 << bit) - 1)); }

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
    const u64 v = bext_prep<2>(T, tb, x, y);
    return ar.from_u64(bext_target_sel<2>(T, ti, ns, mc.q, y, v));
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
template <class A, int LOGN, int PRO>
__device__ __forceinline__ void s_fwd_cols(const NttIO& io, int job, int c, int l, int b, int tile, const ModConst& mc,
                                           const A& ar, __amdgpu_buffer_rsrc_t tw, u64* lds,
                                           const DeviceTables* __restrict__ tb) {
  constexpr int N = 1 << LOGN, R = S2<LOGN>::R, CW = S2<LOGN>::CW, H = S2<LOGN>::H;
  const int t = threadIdx.x, cl = t % CW, k = t / CW, col = tile * CW + cl;
  typename A::W w[R];
#pragma unroll
  for (int s = 0; s < R; ++s) {
    const int rb = R - 1 - s;
    w[s] = ar.tw(tw, k >> rb, N >> (rb + 9));
  }
  typename A::T x = fwd_load<A, PRO>(io, c, l, b, col + (k << 8), mc, ar, tb);
  typename A::T y = fwd_load<A, PRO>(io, c, l, b, col + ((k + H) << 8), mc, ar, tb);
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

// ---------------------------------------------------------------------------
// kernels: blockIdx.x = job * tiles + tile
// ---------------------------------------------------------------------------
template <int LOGN, int PRO>
__global__ void __launch_bounds__(S2<LOGN>::CT) ntt2s_fwd_cols(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[S2<LOGN>::CW << S2<LOGN>::R];
  const int job = io.job0 + blockIdx.x / S2<LOGN>::CTILES, tile = blockIdx.x % S2<LOGN>::CTILES;
  int c, l, b;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if (mc.f64)
    s_fwd_cols<F64Arith, LOGN, PRO>(io, job, c, l, b, tile, mc, F64Arith(mc), twr_s(tb->fwd_d[mod], 8 << LOGN), lds, tb);
  else
    s_fwd_cols<IntArith, LOGN, PRO>(io, job, c, l, b, tile, mc, IntArith(mc), twr_s(tb->fwd[mod], 16 << LOGN), lds, tb);
}

template <int LOGN, int EPI>
__global__ void __launch_bounds__(S2<LOGN>::RT) ntt2s_fwd_rows(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[S2<LOGN>::RW * 256];
  const int job = io.job0 + blockIdx.x / S2<LOGN>::RTILES, tile = blockIdx.x % S2<LOGN>::RTILES;
  int c, l, b;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if (mc.f64)
    s_fwd_rows<F64Arith, LOGN, EPI>(io, job, c, l, b, tile, mc, F64Arith(mc), twr_s(tb->fwd_d[mod], 8 << LOGN), lds);
  else
    s_fwd_rows<IntArith, LOGN, EPI>(io, job, c, l, b, tile, mc, IntArith(mc), twr_s(tb->fwd[mod], 16 << LOGN), lds);
}

template <int LOGN>
__global__ void __launch_bounds__(S2<LOGN>::RT) ntt2s_inv_rows(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[S2<LOGN>::RW * 256];
  const int job = io.job0 + blockIdx.x / S2<LOGN>::RTILES, tile = blockIdx.x % S2<LOGN>::RTILES;
  int c, l, b;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if (mc.f64)
    s_inv_rows<F64Arith, LOGN>(io, job, c, l, b, tile, F64Arith(mc), twr_s(tb->inv_d[mod], 8 << LOGN), lds);
  else
    s_inv_rows<IntArith, LOGN>(io, job, c, l, b, tile, IntArith(mc), twr_s(tb->inv[mod], 16 << LOGN), lds);
}

template <int LOGN>
__global__ void __launch_bounds__(S2<LOGN>::CT) ntt2s_inv_cols(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[S2<LOGN>::CW << S2<LOGN>::R];
  const int job = io.job0 + blockIdx.x / S2<LOGN>::CTILES, tile = blockIdx.x % S2<LOGN>::CTILES;
  int c, l, b;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if (mc.f64)
    s_inv_cols<F64Arith, LOGN>(io, job, c, l, b, tile, F64Arith(mc), twr_s(tb->inv_d[mod], 8 << LOGN), lds);
  else
    s_inv_cols<IntArith, LOGN>(io, job, c, l, b, tile, IntArith(mc), twr_s(tb->inv[mod], 16 << LOGN), lds);
}

template <int LOGN>
int launch2s(const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st) {
  const int total = io.dst.ncomp * io.dst.nlimb * io.dst.nbatch;
  if (total == 0) return 0;
  if (io.jobs != total || io.ci) return -1;
  const int jobs = io.njob ? io.njob : total;
  if (io.job0 < 0 || io.job0 + jobs > total) return -1;
  if (io.mid_compact && io.mid.batch_stride < (1 << LOGN)) return -1;
  const dim3 ga(jobs * S2<LOGN>::CTILES), ba(S2<LOGN>::CT), gb(jobs * S2<LOGN>::RTILES), bb(S2<LOGN>::RT);
  if (inverse) {
    if (io.pro != NTT_PRO_LOAD || io.epi != NTT_EPI_STORE) return -1;
    hipLaunchKernelGGL(ntt2s_inv_rows<LOGN>, gb, bb, 0, st, io, tb);
    hipLaunchKernelGGL(ntt2s_inv_cols<LOGN>, ga, ba, 0, st, io, tb);
    return 0;
  }
  if (io.pro == NTT_PRO_LOAD)
    hipLaunchKernelGGL((ntt2s_fwd_cols<LOGN, NTT_PRO_LOAD>), ga, ba, 0, st, io, tb);
  else if (io.pro == NTT_PRO_BEXT)
    hipLaunchKernelGGL((ntt2s_fwd_cols<LOGN, NTT_PRO_BEXT>), ga, ba, 0, st, io, tb);
  else if (io.pro == NTT_PRO_RESCALE)
    hipLaunchKernelGGL((ntt2s_fwd_cols<LOGN, NTT_PRO_RESCALE>), ga, ba, 0, st, io, tb);
  else
    return -1;
  if (io.epi == NTT_EPI_STORE)
    hipLaunchKernelGGL((ntt2s_fwd_rows<LOGN, NTT_EPI_STORE>), gb, bb, 0, st, io, tb);
  else if (io.epi == NTT_EPI_SUBSCALE)
    hipLaunchKernelGGL((ntt2s_fwd_rows<LOGN, NTT_EPI_SUBSCALE>), gb, bb, 0, st, io, tb);
  else
    return -1;
  return 0;
}

}  // namespace

// host entry: two launches on stream st (same contract as orion_launch_ntt2)
int orion_launch_ntt2s(int logN, const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st) {
  switch (logN) {
    case 15: return launch2s<15>(io, tb, inverse, st);
    case 16: return launch2s<16>(io, tb, inverse, st);
    default: return -1;
  }
}
