// ntt2.hip -- two-pass negacyclic NTT / INTT for N = 2^15 and 2^16 on gfx950
// (the only NTT for N = 2^16, whose 512 KiB limb cannot live in one CU).
//
// The same transform as ntt.hip (Lattigo v6 ring convention, SURVEY.md App.
// A.3: forward Cooley-Tukey, natural order in, bit-reversed out, twiddle of the
// butterfly group i of stage d = w[(N >> (d+1)) + i]; inverse Gentleman-Sande
// with psi^-1 and a final N^-1), split by element bits, e = col + 256 * row:
//   cols pass: the stages on bits LOGN-1..8 -- 256 independent 2^R-point
//              transforms down the columns (R = LOGN - 8 = 7 or 8); 16 columns
//              per workgroup of 16 * 2^(R-4) threads;
//   rows pass: the stages on bits 7..0 -- 2^R independent 256-point transforms
//              along contiguous rows; 16 rows per 256-thread workgroup.
// Every thread holds 16 elements (32 VGPRs) and a workgroup 18 / 34 KiB of
// LDS, so a CU keeps several workgroups in flight and overlaps their loads,
// butterflies and stores -- the one-limb-per-CU kernel of ntt.hip (256 KiB of
// registers, 132 KiB of LDS per limb) cannot.  The price is a second pass over
// the limb: the first pass writes the raw butterfly values (lazy u64 or
// float64 bits) and the second re-reads them while they are still resident in
// the 256 MiB Infinity Cache.
//
// Twiddles of the cols pass depend only on the row bits of the butterfly
// group, identical for every column: they are wave-uniform scalar loads.
#include "common.h"
#include "ntt_arith.h"

namespace {

// timing-only ablation (tools/build_ablation.py; 0 in the product): bit 0 =
// the forward rows pass's per-lane (second-phase) twiddles replaced by one
// loaded twiddle, bit 1 = the same for the inverse rows pass's first phase
#ifndef NTT2_TW_ABLATE
#define NTT2_TW_ABLATE 0
#endif
constexpr int A_STRIDE = 18;   // cols pass LDS: [2^R rows][18] u64, conflict-free both ways
constexpr int B_STRIDE = 272;  // rows pass LDS: [16 rows][256 + 16 pad] u64
__device__ __forceinline__ int b_lds(int rr, int col) { return rr * B_STRIDE + col + (col >> 4); }

// twiddle tables through a buffer descriptor: w[vidx + sidx], vidx per lane,
// sidx wave-uniform (an SGPR / immediate offset)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t twr(const void* t, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)t, 0, bytes, 0x00020000);
}

// intermediate row of job (c, l, b): dst's geometry, or a compact scratch row
__device__ __forceinline__ u64* mid_row(const NttIO& io, int job, int c, int l, int b) {
  if (io.mid_compact) {
    const unsigned r = __builtin_amdgcn_readfirstlane((unsigned)(job - io.job0));
    return io.mid.p + (long long)r * io.mid.batch_stride;
  }
  return row_ptr(io.mid, c, l, b);
}

template <class A>
__device__ __forceinline__ void reduce16(typename A::T (&a)[16], const A& ar) {
#pragma unroll
  for (int k = 0; k < 16; ++k) a[k] = ar.reduce_round(a[k]);
}

// ---------------------------------------------------------------------------
// forward, cols pass (R = LOGN - 8 row bits; RG = 2^(R-4) row groups;
// J = 2^(R-4) rows per phase-2 group, G = 16 / J groups):
//   phase 1: thread (cl = t & 15, rg = t >> 4) holds rows r = rg + RG i,
//            i = r bits R-4..R-1: stages d = LOGN-1 .. LOGN-4 (wave-uniform twiddles)
//   phase 2: rows r = J (rg + RG g) + j, j = r bits 0..R-5, slot j + J g:
//            stages d = LOGN-5 .. 8
// ---------------------------------------------------------------------------
template <class A, int LOGN, int PRO>
__device__ __forceinline__ void fwd_cols(const NttIO& io, int job, int c, int l, int b, int tile, const ModConst& mc,
                                         const A& ar, __amdgpu_buffer_rsrc_t tw, u64* lds, bool lazy,
                                         const DeviceTables* __restrict__ tb) {
  constexpr int R = LOGN - 8, RG = 1 << (R - 4), J = 1 << (R - 4), G = 16 / J;
  const int t = threadIdx.x, cl = t & 15, rg = t >> 4;
  const int col = tile * 16 + cl;
  typename A::T a[16];
  if constexpr (PRO == NTT_PRO_LOAD) {
    const u64* src = row_ptr(io.src, c, l, b);
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = ar.from_u64(src[col + ((rg + RG * i) << 8)]);
  } else if constexpr (PRO == NTT_PRO_BEXT) {
    // the exact basis extension of (at most 2) source limbs to this limb, in
    // registers: the value basis_ext_kernel would have stored
    const int k = arg_byte(io.bx_tab, l), ti = arg_byte(io.bx_t, l), s0 = arg_byte(io.bx_s0, k);
    const BasisExtTable* __restrict__ T = io.bx + k;
    const int ns = T->ns;
    const u64* sp0 = row_ptr(io.src, c, s0, b);
    const u64* sp1 = row_ptr(io.src, c, s0 + (ns > 1 ? 1 : 0), b);
    u64 x0[16], x1[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      x0[i] = sp0[col + ((rg + RG * i) << 8)];
      x1[i] = ns > 1 ? sp1[col + ((rg + RG * i) << 8)] : 0;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      u64 x[2] = {x0[i], x1[i]}, y[2];
      const u64 v = bext_prep<2>(T, x, y);
      a[i] = ar.from_u64(bext_target_sel<2>(T->tgt + ti, ns, y, v));
    }
  } else {  // NTT_PRO_RESCALE (DivRoundByLastModulusNTT prep of every other limb)
    const u64* src = row_ptr(io.src, c, 0, b);
    const u64 qL = tb->mc[io.modL].q, h = qL >> 1;
    const u64 hm = barrett128(0, h, mc);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const u64 x = src[col + ((rg + RG * i) << 8)];
      a[i] = ar.from_u64(sub_mod(barrett128(0, add_mod(x, h, qL), mc), hm, mc.q));
    }
  }
#pragma unroll
  for (int k = 3; k >= 0; --k) {  // d = LOGN-4+k: r bit R-4+k = i bit k; group = i >> (k+1)
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (!((i >> k) & 1)) ar.ct(a[i], a[i | (1 << k)], ar.tw(tw, 0, (1 << (3 - k)) + (i >> (k + 1))));
  }
  if (!lazy) reduce16<A>(a, ar);
#pragma unroll
  for (int i = 0; i < 16; ++i) lds[(rg + RG * i) * A_STRIDE + cl] = to_bits(a[i]);
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < J; ++j) a[j + J * g] = from_bits<typename A::T>(lds[(J * (rg + RG * g) + j) * A_STRIDE + cl]);
#pragma unroll
  for (int bb = R - 5; bb >= 0; --bb) {  // d = 8 + bb: r bit bb = j bit bb; group = r >> (bb+1)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < J; ++j)
        if (!((j >> bb) & 1)) {
          const int r = J * (rg + RG * g) + j;
          ar.ct(a[j + J * g], a[(j | (1 << bb)) + J * g], ar.tw(tw, (1 << (R - 1 - bb)) + (r >> (bb + 1)), 0));
        }
  }
  if (!lazy) reduce16<A>(a, ar);
  u64* mid = mid_row(io, job, c, l, b);
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < J; ++j) mid[col + ((J * (rg + RG * g) + j) << 8)] = to_bits(a[j + J * g]);
}

// ---------------------------------------------------------------------------
// forward, rows pass: stages d = 7..4 (phase 1: thread (rr, jc) holds columns
// jc + 16 i) then d = 3..0 (phase 2: columns 16 ig + j, ig = t & 15)
// ---------------------------------------------------------------------------
template <class A, int LOGN, int EPI>
__device__ __forceinline__ void fwd_rows(const NttIO& io, int job, int c, int l, int b, int tile, const ModConst& mc,
                                         const A& ar, __amdgpu_buffer_rsrc_t tw, u64* lds, bool lazy) {
  const int t = threadIdx.x, rr = t >> 4, jc = t & 15;
  const int row = tile * 16 + rr;
  typename A::T a[16];
  const u64* mid = mid_row(io, job, c, l, b) + (row << 8);
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = from_bits<typename A::T>(mid[jc + 16 * i]);
#pragma unroll
  for (int k = 3; k >= 0; --k) {  // d = 4 + k: col bit d = i bit k
    const int d = 4 + k;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (!((i >> k) & 1))
        ar.ct(a[i], a[i | (1 << k)], ar.tw(tw, (1 << (LOGN - 1 - d)) + ((row << (7 - d)) | (i >> (k + 1))), 0));
  }
  if (!lazy) reduce16<A>(a, ar);
#pragma unroll
  for (int i = 0; i < 16; ++i) lds[b_lds(rr, jc + 16 * i)] = to_bits(a[i]);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = from_bits<typename A::T>(lds[b_lds(rr, 16 * jc + j)]);
  [[maybe_unused]] const typename A::W w_abl = ar.tw(tw, (1 << (LOGN - 4)) + (row << 4), 0);
#pragma unroll
  for (int d = 3; d >= 0; --d) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (!((j >> d) & 1))
        ar.ct(a[j], a[j | (1 << d)],
              (NTT2_TW_ABLATE & 1) ? w_abl
                                   : ar.tw(tw, (1 << (LOGN - 1 - d)) + ((row << (7 - d)) | ((16 * jc + j) >> (d + 1))), 0));
  }
  u64* dst = row_ptr(io.dst, c, l, b) + (row << 8) + 16 * jc;
  if constexpr (EPI == NTT_EPI_STORE) {
#pragma unroll
    for (int j = 0; j < 16; j += 2)
      *(ulonglong2*)(dst + j) = make_ulonglong2(ar.final_fwd(a[j]), ar.final_fwd(a[j + 1]));
  } else if constexpr (epi_aut(EPI)) {
    // (ex - y) * s_l stored at position aut[e] of the limb (added to the word
    // there for _ACC): the rotation's NTT-domain automorphism in the ModDown's
    // store, as in the one-pass and latency kernels
    const u64* ex = row_ptr(io.ex, c, l, b) + (row << 8) + 16 * jc;
    const u32* ai = io.aut + (row << 8) + 16 * jc;
    u64* const d = row_ptr(io.dst, c, l, b);
    const u64 s = io.s[l], ss = io.ss[l];
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
      const uint4 ix = *(const uint4*)(ai + j);
      const ulonglong2 e01 = *(const ulonglong2*)(ex + j), e23 = *(const ulonglong2*)(ex + j + 2);
      u64 o0 = shoup_mul(sub_mod(e01.x, ar.final_fwd(a[j]), mc.q), s, ss, mc.q);
      u64 o1 = shoup_mul(sub_mod(e01.y, ar.final_fwd(a[j + 1]), mc.q), s, ss, mc.q);
      u64 o2 = shoup_mul(sub_mod(e23.x, ar.final_fwd(a[j + 2]), mc.q), s, ss, mc.q);
      u64 o3 = shoup_mul(sub_mod(e23.y, ar.final_fwd(a[j + 3]), mc.q), s, ss, mc.q);
      if constexpr (EPI == NTT_EPI_SUBSCALE_AUT_ACC) {
        o0 = add_mod(o0, d[ix.x], mc.q);
        o1 = add_mod(o1, d[ix.y], mc.q);
        o2 = add_mod(o2, d[ix.z], mc.q);
        o3 = add_mod(o3, d[ix.w], mc.q);
      }
      d[ix.x] = o0;
      d[ix.y] = o1;
      d[ix.z] = o2;
      d[ix.w] = o3;
    }
  } else {  // NTT_EPI_SUBSCALE: dst = (ex - y) * s_l
    const u64* ex = row_ptr(io.ex, c, l, b) + (row << 8) + 16 * jc;
    const u64 s = io.s[l], ss = io.ss[l];
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      const ulonglong2 x = *(const ulonglong2*)(ex + j);
      *(ulonglong2*)(dst + j) = make_ulonglong2(shoup_mul(sub_mod(x.x, ar.final_fwd(a[j]), mc.q), s, ss, mc.q),
                                                shoup_mul(sub_mod(x.y, ar.final_fwd(a[j + 1]), mc.q), s, ss, mc.q));
    }
  }
}

// ---------------------------------------------------------------------------
// inverse, rows pass (first): stages d = 0..3 on columns 16 ig + j, then
// d = 4..7 on columns jc + 16 i; the sum of a float64 GS butterfly is reduced
// every other stage and every phase ends with a full reduction
// ---------------------------------------------------------------------------
template <class A, int LOGN>
__device__ __forceinline__ void inv_rows(const NttIO& io, int job, int c, int l, int b, int tile, const A& ar,
                                         __amdgpu_buffer_rsrc_t tw, u64* lds) {
  const int t = threadIdx.x, rr = t >> 4, jc = t & 15;
  const int row = tile * 16 + rr;
  typename A::T a[16];
  const u64* src = row_ptr(io.src, c, l, b) + (row << 8) + 16 * jc;
#pragma unroll
  for (int j = 0; j < 16; j += 2) {
    const ulonglong2 x = *(const ulonglong2*)(src + j);
    a[j] = ar.from_u64(x.x);
    a[j + 1] = ar.from_u64(x.y);
  }
  [[maybe_unused]] const typename A::W w_abl = ar.tw(tw, (1 << (LOGN - 4)) + (row << 4), 0);
#pragma unroll
  for (int d = 0; d < 4; ++d) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (!((j >> d) & 1))
        ar.gs(a[j], a[j | (1 << d)],
              (NTT2_TW_ABLATE & 2) ? w_abl
                                   : ar.tw(tw, (1 << (LOGN - 1 - d)) + ((row << (7 - d)) | ((16 * jc + j) >> (d + 1))), 0),
              (d & 1) == 1);
  }
  reduce16<A>(a, ar);
#pragma unroll
  for (int j = 0; j < 16; ++j) lds[b_lds(rr, 16 * jc + j)] = to_bits(a[j]);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = from_bits<typename A::T>(lds[b_lds(rr, jc + 16 * i)]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // d = 4 + k
    const int d = 4 + k;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (!((i >> k) & 1))
        ar.gs(a[i], a[i | (1 << k)], ar.tw(tw, (1 << (LOGN - 1 - d)) + ((row << (7 - d)) | (i >> (k + 1))), 0),
              (k & 1) == 1);
  }
  reduce16<A>(a, ar);
  u64* mid = mid_row(io, job, c, l, b) + (row << 8);
#pragma unroll
  for (int i = 0; i < 16; ++i) mid[jc + 16 * i] = to_bits(a[i]);
}

// inverse, cols pass (second): stages d = 8..LOGN-5 (rows J (rg + RG g) + j),
// then d = LOGN-4..LOGN-1 (rows rg + RG i, wave-uniform twiddles), times N^-1
template <class A, int LOGN>
__device__ __forceinline__ void inv_cols(const NttIO& io, int job, int c, int l, int b, int tile, const A& ar,
                                         __amdgpu_buffer_rsrc_t tw, u64* lds) {
  constexpr int R = LOGN - 8, RG = 1 << (R - 4), J = 1 << (R - 4), G = 16 / J;
  const int t = threadIdx.x, cl = t & 15, rg = t >> 4;
  const int col = tile * 16 + cl;
  typename A::T a[16];
  const u64* mid = mid_row(io, job, c, l, b);
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < J; ++j) a[j + J * g] = from_bits<typename A::T>(mid[col + ((J * (rg + RG * g) + j) << 8)]);
#pragma unroll
  for (int bb = 0; bb <= R - 5; ++bb) {  // d = 8 + bb
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < J; ++j)
        if (!((j >> bb) & 1)) {
          const int r = J * (rg + RG * g) + j;
          ar.gs(a[j + J * g], a[(j | (1 << bb)) + J * g], ar.tw(tw, (1 << (R - 1 - bb)) + (r >> (bb + 1)), 0),
                (bb & 1) == 1);
        }
  }
  reduce16<A>(a, ar);
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < J; ++j) lds[(J * (rg + RG * g) + j) * A_STRIDE + cl] = to_bits(a[j + J * g]);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = from_bits<typename A::T>(lds[(rg + RG * i) * A_STRIDE + cl]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // d = LOGN-4+k
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (!((i >> k) & 1)) ar.gs(a[i], a[i | (1 << k)], ar.tw(tw, 0, (1 << (3 - k)) + (i >> (k + 1))), (k & 1) == 1);
  }
  u64* dst = row_ptr(io.dst, c, l, b);
#pragma unroll
  for (int i = 0; i < 16; ++i) dst[col + ((rg + RG * i) << 8)] = ar.final_inv(a[i]);
}

// ---------------------------------------------------------------------------
// kernels: blockIdx.x = job * tiles + tile (the tiles of one limb are adjacent);
// cols pass: 16 tiles of 16 columns, 16 * 2^(LOGN-12) threads; rows pass:
// 2^(LOGN-12) tiles of 16 rows, 256 threads
// ---------------------------------------------------------------------------
template <int LOGN>
struct N2 {
  static constexpr int R = LOGN - 8, ATHREADS = 16 << (R - 4), BTILES = 1 << (R - 4);
};

#ifndef NTT2_COLS_WAVES
#define NTT2_COLS_WAVES 0  // minimum waves per SIMD for the forward columns pass (0: the compiler's choice)
#endif
template <int LOGN, int PRO>
__global__ void __launch_bounds__(N2<LOGN>::ATHREADS) __attribute__((amdgpu_waves_per_eu(NTT2_COLS_WAVES > 0 ? NTT2_COLS_WAVES : 1)))
ntt2_fwd_cols(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[(1 << N2<LOGN>::R) * A_STRIDE];
  int c, l, b;
  const int job = io.job0 + (blockIdx.x >> 4);
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  const bool lazy = mc.bar_k <= 41;
  if (mc.f64)
    fwd_cols<F64Arith, LOGN, PRO>(io, job, c, l, b, blockIdx.x & 15, mc, F64Arith(mc), twr(tb->fwd_d[mod], (8 << LOGN)),
                                  lds, lazy, tb);
  else
    fwd_cols<IntArith, LOGN, PRO>(io, job, c, l, b, blockIdx.x & 15, mc, IntArith(mc), twr(tb->fwd[mod], (16 << LOGN)),
                                  lds, true, tb);
}

template <int LOGN, int EPI>
__global__ void __launch_bounds__(256) ntt2_fwd_rows(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[16 * B_STRIDE];
  constexpr int T = N2<LOGN>::BTILES;
  int c, l, b;
  const int job = io.job0 + blockIdx.x / T;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if (mc.f64)
    fwd_rows<F64Arith, LOGN, EPI>(io, job, c, l, b, blockIdx.x % T, mc, F64Arith(mc), twr(tb->fwd_d[mod], (8 << LOGN)),
                                  lds, mc.bar_k <= 41);
  else
    fwd_rows<IntArith, LOGN, EPI>(io, job, c, l, b, blockIdx.x % T, mc, IntArith(mc), twr(tb->fwd[mod], (16 << LOGN)),
                                  lds, true);
}

template <int LOGN>
__global__ void __launch_bounds__(256) ntt2_inv_rows(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[16 * B_STRIDE];
  constexpr int T = N2<LOGN>::BTILES;
  int c, l, b;
  const int job = io.job0 + blockIdx.x / T;
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if (mc.f64)
    inv_rows<F64Arith, LOGN>(io, job, c, l, b, blockIdx.x % T, F64Arith(mc), twr(tb->inv_d[mod], (8 << LOGN)), lds);
  else
    inv_rows<IntArith, LOGN>(io, job, c, l, b, blockIdx.x % T, IntArith(mc), twr(tb->inv[mod], (16 << LOGN)), lds);
}

template <int LOGN>
__global__ void __launch_bounds__(N2<LOGN>::ATHREADS) ntt2_inv_cols(NttIO io, const DeviceTables* __restrict__ tb) {
  __shared__ u64 lds[(1 << N2<LOGN>::R) * A_STRIDE];
  int c, l, b;
  const int job = io.job0 + (blockIdx.x >> 4);
  job_of(io, job, c, l, b);
  const int mod = arg_byte(io.dst.mod, l);
  const ModConst mc = tb->mc[mod];
  if (mc.f64)
    inv_cols<F64Arith, LOGN>(io, job, c, l, b, blockIdx.x & 15, F64Arith(mc), twr(tb->inv_d[mod], (8 << LOGN)), lds);
  else
    inv_cols<IntArith, LOGN>(io, job, c, l, b, blockIdx.x & 15, IntArith(mc), twr(tb->inv[mod], (16 << LOGN)), lds);
}

template <int LOGN>
int launch2(const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st) {
  const int total = io.dst.ncomp * io.dst.nlimb * io.dst.nbatch;
  if (total == 0) return 0;
  if (io.jobs != total) return -1;
  const int jobs = io.njob ? io.njob : total;
  if (io.job0 < 0 || io.job0 + jobs > total) return -1;
  if (io.mid_compact && io.mid.batch_stride < (1 << LOGN)) return -1;
  const dim3 ga(jobs * 16), ba(N2<LOGN>::ATHREADS), gb(jobs * N2<LOGN>::BTILES), bb(256);
  if (inverse) {
    if (io.pro != NTT_PRO_LOAD || io.epi != NTT_EPI_STORE) return -1;
    hipLaunchKernelGGL(ntt2_inv_rows<LOGN>, gb, bb, 0, st, io, tb);
    hipLaunchKernelGGL(ntt2_inv_cols<LOGN>, ga, ba, 0, st, io, tb);
    return 0;
  }
  if (io.pro == NTT_PRO_LOAD)
    hipLaunchKernelGGL((ntt2_fwd_cols<LOGN, NTT_PRO_LOAD>), ga, ba, 0, st, io, tb);
  else if (io.pro == NTT_PRO_BEXT && !io.ci)
    hipLaunchKernelGGL((ntt2_fwd_cols<LOGN, NTT_PRO_BEXT>), ga, ba, 0, st, io, tb);
  else if (io.pro == NTT_PRO_RESCALE)
    hipLaunchKernelGGL((ntt2_fwd_cols<LOGN, NTT_PRO_RESCALE>), ga, ba, 0, st, io, tb);
  else
    return -1;
  if (io.epi == NTT_EPI_STORE)
    hipLaunchKernelGGL((ntt2_fwd_rows<LOGN, NTT_EPI_STORE>), gb, bb, 0, st, io, tb);
  else if (io.epi == NTT_EPI_SUBSCALE)
    hipLaunchKernelGGL((ntt2_fwd_rows<LOGN, NTT_EPI_SUBSCALE>), gb, bb, 0, st, io, tb);
  else if (io.epi == NTT_EPI_SUBSCALE_AUT && io.aut)
    hipLaunchKernelGGL((ntt2_fwd_rows<LOGN, NTT_EPI_SUBSCALE_AUT>), gb, bb, 0, st, io, tb);
  else if (io.epi == NTT_EPI_SUBSCALE_AUT_ACC && io.aut)
    hipLaunchKernelGGL((ntt2_fwd_rows<LOGN, NTT_EPI_SUBSCALE_AUT_ACC>), gb, bb, 0, st, io, tb);
  else
    return -1;
  return 0;
}

}  // namespace

// host entry: two launches on stream st; io.mid must have dst's geometry and
// must not alias io.ex (the epilogue reads ex after the first pass wrote mid)
int orion_launch_ntt2(int logN, const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st) {
  switch (logN) {
    case 15: return launch2<15>(io, tb, inverse, st);
    case 16: return launch2<16>(io, tb, inverse, st);
    default: return -1;
  }
}
