// kernels.hip -- coefficient-wise, rescale, basis-extension, key-switch MAC
// and automorphism kernels for the gfx950 RNS-CKKS backend.
//
// Every kernel here is HBM-bound integer work (no MFMA).  Grid shape: x covers
// the N coefficients of one limb (2 coefficients per thread, 16-B accesses),
// y covers the (comp, limb, image) rows.  Operands that are shared by the
// whole batch (plaintexts, LT diagonals, evaluation keys) are passed with
// batch_stride = 0 and are read once per row from L2.
#include <type_traits>

#include "common.h"
#include "ntt2s_rows.h"

// timing-only ablation of lt_bsgs (0 in the product): bit 0 skips the giant
// inner products of moduli below 2^48, bit 1 skips the baby gadget products,
// bit 2 the giant products of the integer-path (>= 2^48) moduli, bit 3 their
// baby gadget products, bit 4 replaces the giants' diagonal loads by values
// formed in registers
#ifndef LT_ABLATE
#define LT_ABLATE 0
#endif
// 1: ks_mac reduces once per output on moduli below 2^52 instead of once per
// chunk of 4 digits.  Off: the accumulators live across the digit loop (84 ->
// 102 VGPRs, 5 -> 4 waves per SIMD) and the LoLA bench measured ks_mac 1.31
// -> 1.48 ms per step with it (profiles/r03n_ab.txt); LoLA's decompositions
// have at most 3 digits, so there is one chunk anyway
#ifndef KS_MAC_ACC
#define KS_MAC_ACC 0
#endif
// ks_mac: digits per load chunk (4 -> 2: 84 -> 62 VGPRs, 5 -> 8 waves per
// SIMD; ks_mac 104.3 -> 96.6 us per launch, profiles/r03z_ks_mac_chunk_ab.txt)
#ifndef KS_CH
#define KS_CH 2
#endif
// 1: lt_giant accumulates all giants unreduced on moduli below 2^52
#ifndef LT_GIANT_ACC
#define LT_GIANT_ACC 1
#endif
#ifndef LT_INT_ACC8
#define LT_INT_ACC8 1
#endif
#ifndef LT_WAVES8
#define LT_WAVES8 4  // lt_bsgs_kernel8: minimum waves per SIMD (VGPR budget 512 / this)
#endif
// 1: lt_bsgs's 48..60-bit limbs multiply 30-bit pieces (split30 diagonals)
#ifndef LT_INT30
#define LT_INT30 1
#endif
// images per lt_giant thread
#ifndef LT_GIANT_IB
#define LT_GIANT_IB 4
#endif
#ifndef LT_GIANT_B1
#define LT_GIANT_B1 1  // 1: one-image launches take lt_giant_kernel<1, ...>
#endif
#ifndef LT_GIANT_CH
#define LT_GIANT_CH 0  // lt_giant digits per load chunk (0: 2 at IB >= 4, else 4)
#endif
// 1: lt_bsgs runs every register slot of every giant without branches: the
// plan points the slots a giant does not use at a zero diagonal, so their
// products add zero (0: one uniform branch per slot)
#ifndef LT_DENSE
#define LT_DENSE 1
#endif
// 1: lt_bsgs cuts the baby rotations into 30-bit pieces once, before the
// integer giant loop (0: per giant)
#ifndef LT_PRESPLIT
#define LT_PRESPLIT 1
#endif

namespace {

// the workgroup size of every kernel in this file (launch_bounds and launches:
// 256).  As a constant, not blockDim.x: HIP reads blockDim.x from the
// dispatch's implicit arguments (the remainder for a partial last block) with
// a 16-bit vector load and waits for it before any address is formed
constexpr int kBlk = 256;

// p[i] through a global-address-space pointer: for a pointer read from device
// memory (a plan's diagonal table) the compiler cannot infer the address
// space and emits a flat load, whose completion is only trackable with
// vmcnt(0) lgkmcnt(0) -- every product would wait for all loads in flight
__device__ __forceinline__ u64 gld(const u64* p, long long i) {
  return ((const __attribute__((address_space(1))) u64*)p)[i];
}

__device__ __forceinline__ long long row_off(const LimbSet& s, int c, int l, int b) {
  return c * s.comp_stride + arg_byte(s.pos, l) * s.limb_stride + b * s.batch_stride;
}

enum EwOp : int {
  EW_ADD = 0,      // o = a + b
  EW_SUB = 1,      // o = a - b
  EW_MUL = 2,      // o = a * b
  EW_MULADD = 3,   // o = o + a * b
  EW_NEG = 4,      // o = -a
  EW_SCALE = 5,    // o = a * s_l            (Shoup scalar per limb)
  EW_ADDC = 6,     // o = a + s_l            (constant per limb)
  EW_SUBSCALE = 7, // o = (a - b) * s_l
  EW_COPY = 8,     // o = a
  EW_ADDSCALE = 9, // o = o + a * s_l
  EW_SPLIT24 = 10, // o = split24(a) on limbs below 2^48, split30(a) on limbs up to 2^60 (LT_INT30), else a
                   // (lt_bsgs's split-MAC operand forms)
};

struct Scalars {
  u64 s[ORION_MAXLIMB];
  u64 ss[ORION_MAXLIMB];
};

template <int OP>
__global__ void __launch_bounds__(256) ew_kernel(LimbSet o, LimbSet a, LimbSet b, Scalars sc,
                                                 const DeviceTables* __restrict__ tb, int N) {
  const int row = blockIdx.y;
  const int bi = row % o.nbatch;
  const int r = row / o.nbatch;
  const int l = r % o.nlimb;
  const int c = r / o.nlimb;
  const int n = (blockIdx.x * kBlk + threadIdx.x) * 2;
  if (n >= N) return;
  const ModConst mc = tb->mc[arg_byte(o.mod, l)];
  const u64 q = mc.q;
  ulonglong2* po = (ulonglong2*)(o.p + row_off(o, c, l, bi) + n);
  const ulonglong2 x = *(const ulonglong2*)(a.p + row_off(a, c, l, bi) + n);
  ulonglong2 y = make_ulonglong2(0, 0), z;
  if (OP == EW_ADD || OP == EW_SUB || OP == EW_MUL || OP == EW_MULADD || OP == EW_SUBSCALE)
    y = *(const ulonglong2*)(b.p + row_off(b, c, l, bi) + n);
  switch (OP) {
    case EW_ADD: z.x = add_mod(x.x, y.x, q); z.y = add_mod(x.y, y.y, q); break;
    case EW_SUB: z.x = sub_mod(x.x, y.x, q); z.y = sub_mod(x.y, y.y, q); break;
    case EW_MUL: z.x = mul_mod(x.x, y.x, mc); z.y = mul_mod(x.y, y.y, mc); break;
    case EW_MULADD: {
      const ulonglong2 w = *po;
      z.x = add_mod(w.x, mul_mod(x.x, y.x, mc), q);
      z.y = add_mod(w.y, mul_mod(x.y, y.y, mc), q);
      break;
    }
    case EW_NEG: z.x = x.x ? q - x.x : 0; z.y = x.y ? q - x.y : 0; break;
    case EW_SCALE: z.x = shoup_mul(x.x, sc.s[l], sc.ss[l], q); z.y = shoup_mul(x.y, sc.s[l], sc.ss[l], q); break;
    case EW_ADDC: z.x = add_mod(x.x, sc.s[l], q); z.y = add_mod(x.y, sc.s[l], q); break;
    case EW_SUBSCALE:
      z.x = shoup_mul(sub_mod(x.x, y.x, q), sc.s[l], sc.ss[l], q);
      z.y = shoup_mul(sub_mod(x.y, y.y, q), sc.s[l], sc.ss[l], q);
      break;
    case EW_COPY: z = x; break;
    case EW_SPLIT24:
      z = mc.bar_k <= 48                 ? make_ulonglong2(split24(x.x), split24(x.y))
          : (LT_INT30 && mc.bar_k <= 60) ? make_ulonglong2(split30(x.x), split30(x.y))
                                         : x;
      break;
    case EW_ADDSCALE: {
      const ulonglong2 w = *po;
      z.x = add_mod(w.x, shoup_mul(x.x, sc.s[l], sc.ss[l], q), q);
      z.y = add_mod(w.y, shoup_mul(x.y, sc.s[l], sc.ss[l], q), q);
      break;
    }
  }
  *po = z;
}

// ct x ct tensor: d0 = a0 b0, d1 = a0 b1 + a1 b0, d2 = a1 b1  (a, b: 2 comps; d: 3 comps)
__global__ void __launch_bounds__(256) tensor_kernel(LimbSet d, LimbSet a, LimbSet b,
                                                     const DeviceTables* __restrict__ tb, int N) {
  const int row = blockIdx.y;
  const int bi = row % d.nbatch;
  const int l = row / d.nbatch;
  const int n = (blockIdx.x * kBlk + threadIdx.x) * 2;
  if (n >= N) return;
  const ModConst mc = tb->mc[arg_byte(d.mod, l)];
  const u64 q = mc.q;
  const ulonglong2 a0 = *(const ulonglong2*)(a.p + row_off(a, 0, l, bi) + n);
  const ulonglong2 a1 = *(const ulonglong2*)(a.p + row_off(a, 1, l, bi) + n);
  const ulonglong2 b0 = *(const ulonglong2*)(b.p + row_off(b, 0, l, bi) + n);
  const ulonglong2 b1 = *(const ulonglong2*)(b.p + row_off(b, 1, l, bi) + n);
  ulonglong2 d0, d1, d2;
  d0.x = mul_mod(a0.x, b0.x, mc); d0.y = mul_mod(a0.y, b0.y, mc);
  d1.x = add_mod(mul_mod(a0.x, b1.x, mc), mul_mod(a1.x, b0.x, mc), q);
  d1.y = add_mod(mul_mod(a0.y, b1.y, mc), mul_mod(a1.y, b0.y, mc), q);
  d2.x = mul_mod(a1.x, b1.x, mc); d2.y = mul_mod(a1.y, b1.y, mc);
  *(ulonglong2*)(d.p + row_off(d, 0, l, bi) + n) = d0;
  *(ulonglong2*)(d.p + row_off(d, 1, l, bi) + n) = d1;
  *(ulonglong2*)(d.p + row_off(d, 2, l, bi) + n) = d2;
}

// Exact basis extension (Lattigo ModUpExact restated; the
// source-side math is bext_prep in common.h, the target side bext_target_sel).
// in: ns source limbs (coefficient domain), out: nt target limbs.  Two
// coefficients per thread (16-B accesses).
template <int MS>
__global__ void __launch_bounds__(256) basis_ext_kernel(LimbSet out, LimbSet in, const BasisExtTable* __restrict__ T,
                                                        int N, int tchunk) {
  const int row = blockIdx.y;  // (comp, image)
  const int bi = row % out.nbatch;
  const int c = row / out.nbatch;
  const int n = (blockIdx.x * kBlk + threadIdx.x) * 2;
  if (n >= N) return;
  const int ns = T->ns, nt = T->nt;
  u64 x0[MS], x1[MS], y0[MS], y1[MS];
#pragma unroll
  for (int i = 0; i < MS; ++i) {
    if (i >= ns) break;
    const ulonglong2 v = *(const ulonglong2*)(in.p + row_off(in, c, i, bi) + n);
    x0[i] = v.x;
    x1[i] = v.y;
  }
  const u64 v0 = bext_prep<MS>(T, x0, y0), v1 = bext_prep<MS>(T, x1, y1);
  const int tend = min(nt, (int)(blockIdx.z + 1) * tchunk);
  for (int t = blockIdx.z * tchunk; t < tend; ++t) {
    u64 o0, o1;
    bext_target2<MS>(T->tgt + t, ns, y0, v0, y1, v1, o0, o1);
    *(ulonglong2*)(out.p + row_off(out, c, t, bi) + n) = make_ulonglong2(o0, o1);
  }
}

// ModUp of every digit of a decomposition in one launch (small launches:
// one image at N = 2^13..2^15 gives a per-digit basis_ext only 16..64
// workgroups).  Row = (comp c, digit i, image); blockIdx.z = a chunk of the
// nqp QP positions.  Digit i's own positions [iK, iK + ns) are not written
// (consumers read the own limbs from the NTT-domain input, and the NTT that
// follows covers only the target positions).
// D: comps c*beta + i, limb j at position j; Ts[i] = digit i's table.
template <int MS>
__global__ void __launch_bounds__(256) modup_all_kernel(LimbSet D, LimbSet in, const BasisExtTable* __restrict__ Ts,
                                                        int beta, int K, int nqp, int N, int tchunk) {
  const int row = blockIdx.y;
  const int bi = row % D.nbatch;
  const int r = row / D.nbatch;
  const int i = r % beta;
  const int c = r / beta;
  const int n = (blockIdx.x * kBlk + threadIdx.x) * 2;
  if (n >= N) return;
  const BasisExtTable* __restrict__ T = Ts + i;
  const int ns = T->ns, lo = i * K;
  u64 x0[MS], x1[MS], y0[MS], y1[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= ns) break;
    const ulonglong2 v = *(const ulonglong2*)(in.p + row_off(in, c, lo + s, bi) + n);
    x0[s] = v.x;
    x1[s] = v.y;
  }
  const u64 v0 = bext_prep<MS>(T, x0, y0), v1 = bext_prep<MS>(T, x1, y1);
  // D's positions are the identity (checked at launch): limb j of the row is
  // limb_stride past limb j - 1, so the loop carries one pointer and one
  // target record instead of re-deriving both from (j, pos[j], dst_mod[t])
  // own limbs [lo, lo + ns) are not written: every consumer reads them from
  // the NTT-domain input of the decomposition; positions below them are
  // targets 0.., positions above them targets lo..
  const int j0 = blockIdx.z * tchunk, jend = min(nqp, j0 + tchunk);
  u64* const dst = D.p + row_off(D, c * beta + i, 0, bi) + n;
  auto targets = [&](int ja, int jb, int toff) {
    u64* op = dst + (long long)ja * D.limb_stride;
    const BextTarget* __restrict__ R = T->tgt + (ja - toff);
    for (int j = ja; j < jb; ++j, ++R, op += D.limb_stride) {
      u64 o0, o1;
      bext_target2<MS>(R, ns, y0, v0, y1, v1, o0, o1);
      *(ulonglong2*)op = make_ulonglong2(o0, o1);
    }
  };
  targets(j0, min(jend, lo), 0);
  targets(max(j0, lo + ns), jend, ns);
}

// Gadget-product MAC over G groups (one evaluation key per group):
//   out_g,c[j] = add0_g[j]*(c == 0) + sum_i D_g,i[j] * key_g[i][c][mod_j]   (c = 0, 1)
// D: comps = digits, limbs = QP positions; group g's digits start at
// D.p + g*d_gstride (d_gstride = 0: one decomposition shared by every group,
// the hoisted baby steps of a BSGS transform).  If own.p is set, digit i's
// own Q limbs (l / K == i) are read from `own` (the NTT-domain input of the
// decomposition, group stride own_gstride) instead of D, so the decomposition
// never copies them.  out comps 0/1 of group g at out.p + g*out_gstride.
// key layout [digit][2][klvl+1+K][N] (common.h key_pos).
template <bool ROWS, bool FR = false, bool PRE = false>
__device__ __forceinline__ void ks_mac_body(LimbSet& out, LimbSet& D, LimbSet& own, MacGroups& G, int beta,
                                            const DeviceTables* __restrict__ tb, int N, u64* lds) {
  const int row = blockIdx.y;
  const int bi = row % out.nbatch;
  const int r = row / out.nbatch;
  const int l = r % out.nlimb;
  const int g = r / out.nlimb;
  const int n = (blockIdx.x * kBlk + threadIdx.x) * 2;
  if (n >= N) return;
  const int m = arg_byte(out.mod, l);
  const ModConst mc = tb->mc[m];
  const u64 q = mc.q;
  const u64* key = G.key[g];
  const u64* dp = D.p + g * G.d_gstride;
  const int owndigit = (own.p && l < own.nlimb) ? l / G.K : -1;
  u64* op = out.p + g * G.out_gstride;
  ulonglong2 r0 = make_ulonglong2(0, 0), r1 = make_ulonglong2(0, 0);
  if (G.add_nq > 0) {
    if (l < G.add_nq) {
      const long long ao = g * G.add_gstride + row_off(out, 0, l, bi) + n;
      const u64 s = G.add_s[l], ss = G.add_ss[l];
      const ulonglong2 a = *(const ulonglong2*)(G.add0 + ao);
      r0 = make_ulonglong2(shoup_mul(a.x, s, ss, q), shoup_mul(a.y, s, ss, q));
      if (G.add1) {
        const ulonglong2 b = *(const ulonglong2*)(G.add1 + ao);
        r1 = make_ulonglong2(shoup_mul(b.x, s, ss, q), shoup_mul(b.y, s, ss, q));
      }
    }
  } else if (G.add0) {
    r0 = *(const ulonglong2*)(G.add0 + g * G.add_gstride + row_off(out, 0, l, bi) + n);
  }
  const int kl = G.klvl[g];
  const long long kstride = (long long)(kl + 1 + G.K) * N;
  const u64* kp = key + (long long)key_pos(m, G.L, kl) * N + n;
  // FR: the decomposition's forward NTT stopped after its columns pass; rows
  // 2 bx and 2 bx + 1 of every non-own digit's row set go through the
  // forward rows pass here, 4 rows at a time (groups past the last row keep
  // the barriers on their own LDS row), into fr = [digit][2 rows][256]
  [[maybe_unused]] const u64* fr = nullptr;
  // FR with at most 4 digits (the batch-1 key switches): the key words and the
  // own digit's words are loaded before the rows pass, so their latency
  // overlaps it instead of following it
  // (PRE: an instantiation of its own, so the other launches keep their registers)
  constexpr bool pre = FR && PRE;
  [[maybe_unused]] ulonglong2 pkb[4], pka[4], pown = make_ulonglong2(0, 0);
  if constexpr (pre) {
    {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u < beta) {
          pkb[u] = *(const ulonglong2*)(kp + (2 * u + 0) * kstride);
          pka[u] = *(const ulonglong2*)(kp + (2 * u + 1) * kstride);
        }
      }
      if (owndigit >= 0) pown = *(const ulonglong2*)(own.p + g * G.own_gstride + row_off(own, 0, l, bi) + n);
    }
  }
  // ... and a P limb's inverse-rows twiddles (the ROWS epilogue below), raw
  [[maybe_unused]] ulonglong2 itw[12];
  if constexpr (pre && ROWS) {
    if (l >= G.rows_from) {  // (block-uniform)
      const int t = threadIdx.x, rr = t >> 6, kk = t & 63, row = 2 * blockIdx.x + (rr & 1);
      auto tws = [&](const auto& ar, __amdgpu_buffer_rsrc_t tw) {
        using A = std::decay_t<decltype(ar)>;
        typename A::W wa[4], wb[4], wc[4];
        if (G.logN == 15)
          inv_rows4_tw<A, 15>(row, kk, ar, tw, wa, wb, wc);
        else
          inv_rows4_tw<A, 16>(row, kk, ar, tw, wa, wb, wc);
#pragma unroll
        for (int st = 0; st < 4; ++st) itw[st] = w_raw(wa[st]), itw[4 + st] = w_raw(wb[st]), itw[8 + st] = w_raw(wc[st]);
      };
      if (mc.f64)
        tws(F64Arith(mc), twr_s(tb->inv_d[m], 8 * N));
      else
        tws(IntArith(mc), twr_s(tb->inv[m], 16 * N));
    }
  }
  if constexpr (FR) {
    u64* const frw = lds + 4 * 256;
    const int t = threadIdx.x, rr = t >> 6, kk = t & 63;
    for (int q0 = 0; q0 < 2 * beta; q0 += 4) {  // (uniform)
      if (q0 > 0) __syncthreads();  // the previous round's exchange reads done
      const int q = q0 + rr, i = q >> 1, rw = 2 * blockIdx.x + (q & 1);
      const bool live = q < 2 * beta && i != owndigit;
      const u64* const src = dp + row_off(D, live ? i : 0, l, bi) + ((long long)rw << 8);
      auto rows = [&](const auto& ar, __amdgpu_buffer_rsrc_t tw) {
        using A = std::decay_t<decltype(ar)>;
        typename A::T x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = from_bits<typename A::T>(live ? src[kk + 64 * k] : 0);
        if (G.logN == 15)
          fwd_rows4_core<A, 15>(x, rw, kk, ar, tw, lds + rr * 256);
        else
          fwd_rows4_core<A, 16>(x, rw, kk, ar, tw, lds + rr * 256);
        if (live) {
#pragma unroll
          for (int k = 0; k < 4; ++k) frw[q * 256 + 4 * kk + k] = ar.final_fwd(x[k]);
        }
      };
      if (mc.f64)
        rows(F64Arith(mc), twr_s(tb->fwd_d[m], 8 * N));
      else
        rows(IntArith(mc), twr_s(tb->fwd[m], 16 * N));
    }
    __syncthreads();  // fr complete
    fr = frw;
  }
  // moduli below 2^52 (block-uniform): the digits' products are reduced once
  // at the end (mac_reduce_small takes up to 128), not once per chunk of 4
  const bool small = KS_MAC_ACC && mc.bar_k <= 52 && beta <= 120;
  MacAcc s0x, s0y, s1x, s1y;
  mac_zero(s0x), mac_zero(s0y), mac_zero(s1x), mac_zero(s1y);
  if constexpr (pre) {
    {  // the preloaded words, in chunks of 2 digits as below
      const int lt = 2 * (int)threadIdx.x;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u < beta) {
          const ulonglong2 d = u == owndigit ? pown
                                             : make_ulonglong2(fr[(2 * u + (lt >> 8)) * 256 + (lt & 255)],
                                                               fr[(2 * u + (lt >> 8)) * 256 + (lt & 255) + 1]);
          mac_add(s0x, d.x, pkb[u].x);
          mac_add(s0y, d.y, pkb[u].y);
          mac_add(s1x, d.x, pka[u].x);
          mac_add(s1y, d.y, pka[u].y);
        }
        if ((u & 1) && u - 1 < beta) {
          r0.x = add_mod(r0.x, mac_reduce(s0x, mc), q);
          r0.y = add_mod(r0.y, mac_reduce(s0y, mc), q);
          r1.x = add_mod(r1.x, mac_reduce(s1x, mc), q);
          r1.y = add_mod(r1.y, mac_reduce(s1y, mc), q);
          mac_zero(s0x), mac_zero(s0y), mac_zero(s1x), mac_zero(s1y);
        }
      }
    }
  }
  for (int i0 = 0; i0 < (pre ? 0 : beta); i0 += KS_CH) {  // chunks of KS_CH digits: 3 KS_CH loads in flight
    ulonglong2 d[KS_CH], kb[KS_CH], ka[KS_CH];
#pragma unroll
    for (int u = 0; u < KS_CH; ++u) {
      const int i = i0 + u;
      if (i < beta) {
        if (i == owndigit) {
          d[u] = *(const ulonglong2*)(own.p + g * G.own_gstride + row_off(own, 0, l, bi) + n);
        } else if constexpr (FR) {  // this thread's 2 coefficients: local 2t, 2t + 1 of the block's 2 rows
          const int lt = 2 * (int)threadIdx.x;
          d[u] = make_ulonglong2(fr[(2 * i + (lt >> 8)) * 256 + (lt & 255)], fr[(2 * i + (lt >> 8)) * 256 + (lt & 255) + 1]);
        } else {
          d[u] = *(const ulonglong2*)(dp + row_off(D, i, l, bi) + n);
        }
        kb[u] = *(const ulonglong2*)(kp + (2 * i + 0) * kstride);
        ka[u] = *(const ulonglong2*)(kp + (2 * i + 1) * kstride);
      }
    }
#pragma unroll
    for (int u = 0; u < KS_CH; ++u) {
      if (i0 + u < beta) {
        mac_add(s0x, d[u].x, kb[u].x);
        mac_add(s0y, d[u].y, kb[u].y);
        mac_add(s1x, d[u].x, ka[u].x);
        mac_add(s1y, d[u].y, ka[u].y);
      }
    }
    if (!small) {
      r0.x = add_mod(r0.x, mac_reduce(s0x, mc), q);
      r0.y = add_mod(r0.y, mac_reduce(s0y, mc), q);
      r1.x = add_mod(r1.x, mac_reduce(s1x, mc), q);
      r1.y = add_mod(r1.y, mac_reduce(s1y, mc), q);
      mac_zero(s0x), mac_zero(s0y), mac_zero(s1x), mac_zero(s1y);
    }
  }
  if (small) {
    r0.x = add_mod(r0.x, mac_reduce_small(s0x, mc), q);
    r0.y = add_mod(r0.y, mac_reduce_small(s0y, mc), q);
    r1.x = add_mod(r1.x, mac_reduce_small(s1x, mc), q);
    r1.y = add_mod(r1.y, mac_reduce_small(s1y, mc), q);
  }
  if constexpr (ROWS) {
    if (l >= G.rows_from) {  // (block-uniform) a P limb: the ModDown INTT's rows pass, here
      // the block's 512 coefficients are rows 2 bx and 2 bx + 1 of both
      // components: staged in LDS as 4 rows (comp-major), then thread
      // (rr, kk) runs the radix-4 inverse rows steps on elements 4 kk .. 4 kk + 3
      const int t = threadIdx.x, lrw = (2 * t) >> 8, col = (2 * t) & 255;
      lds[lrw * 256 + col] = r0.x, lds[lrw * 256 + col + 1] = r0.y;
      lds[(2 + lrw) * 256 + col] = r1.x, lds[(2 + lrw) * 256 + col + 1] = r1.y;
      __syncthreads();
      const int rr = t >> 6, kk = t & 63, row = 2 * blockIdx.x + (rr & 1);
      u64* const lr = lds + rr * 256;
      u64* const mid = op + row_off(out, rr >> 1, l, bi) + (row << 8);
      auto rows = [&](const auto& ar, __amdgpu_buffer_rsrc_t tw) {
        using A = std::decay_t<decltype(ar)>;
        typename A::T x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = ar.from_u64(lr[4 * kk + i]);
        if constexpr (pre) {  // the twiddles fetched at the start
          typename A::W wa[4], wb[4], wc[4];
#pragma unroll
          for (int st = 0; st < 4; ++st)
            wa[st] = w_of<A>(itw[st]), wb[st] = w_of<A>(itw[4 + st]), wc[st] = w_of<A>(itw[8 + st]);
          inv_rows4_run<A>(x, kk, ar, wa, wb, wc, lr, mid);
        } else if (G.logN == 15) {
          inv_rows4_core<A, 15>(x, row, kk, ar, tw, lr, mid);
        } else {
          inv_rows4_core<A, 16>(x, row, kk, ar, tw, lr, mid);
        }
      };
      if (mc.f64)
        rows(F64Arith(mc), twr_s(tb->inv_d[m], 8 * N));
      else
        rows(IntArith(mc), twr_s(tb->inv[m], 16 * N));
      return;
    }
  }
  *(ulonglong2*)(op + row_off(out, 0, l, bi) + n) = r0;
  *(ulonglong2*)(op + row_off(out, 1, l, bi) + n) = r1;
}
__global__ void __launch_bounds__(256) ks_mac_kernel(LimbSet out, LimbSet D, LimbSet own, MacGroups G, int beta,
                                                     const DeviceTables* __restrict__ tb, int N) {
  ks_mac_body<false>(out, D, own, G, beta, tb, N, nullptr);
}
// the same, the P limbs' results through the INTT's rows pass (MacGroups.rows_from)
__global__ void __launch_bounds__(256) ks_mac_rows_kernel(LimbSet out, LimbSet D, LimbSet own, MacGroups G, int beta,
                                                          const DeviceTables* __restrict__ tb, int N) {
  __shared__ u64 lds[4 * 256];
  ks_mac_body<true>(out, D, own, G, beta, tb, N, lds);
}
// the same, and before the products the decomposition's forward rows pass
// (MacGroups.fwd_rows; dynamic LDS: (4 + 2 beta) rows of 256 words)
template <bool PRE>
__global__ void __launch_bounds__(256) ks_mac_full_kernel(LimbSet out, LimbSet D, LimbSet own, MacGroups G, int beta,
                                                          const DeviceTables* __restrict__ tb, int N) {
  extern __shared__ u64 lds_dyn[];
  ks_mac_body<true, true, PRE>(out, D, own, G, beta, tb, N, lds_dyn);
}

// NTT-domain automorphism: o[j] = a[idx[j]]  (optionally o += a[idx[j]])
__global__ void __launch_bounds__(256) automorph_kernel(LimbSet o, LimbSet a, const u32* __restrict__ idx,
                                                        const DeviceTables* __restrict__ tb, int N, int accumulate) {
  const int row = blockIdx.y;
  const int bi = row % o.nbatch;
  const int r = row / o.nbatch;
  const int l = r % o.nlimb;
  const int c = r / o.nlimb;
  const int n = (blockIdx.x * kBlk + threadIdx.x) * 2;
  if (n >= N) return;
  const u64 q = tb->mc[arg_byte(o.mod, l)].q;
  const u64* src = a.p + row_off(a, c, l, bi);
  u64* dst = o.p + row_off(o, c, l, bi) + n;
  const uint2 ix = *(const uint2*)(idx + n);
  ulonglong2 z = make_ulonglong2(src[ix.x], src[ix.y]);
  if (accumulate) {
    const ulonglong2 w = *(const ulonglong2*)dst;
    z.x = add_mod(z.x, w.x, q);
    z.y = add_mod(z.y, w.y, q);
  }
  *(ulonglong2*)dst = z;
}

// One gadget product of a hoisted key switch, read at the automorphism index j:
//   (sum_i D_i[j] * key[i][0][m][j],  sum_i D_i[j] * key[i][1][m][j])   mod q
// D_i rows at dp + i*dstride; digit `owndigit` comes from ownp instead.
// Digits go in chunks of 4: all 12 loads of a chunk are issued before the
// first product, so their latencies overlap.
// key: made for level klvl (limb of modulus m at key_pos(m, L, klvl), K P limbs)
__device__ __forceinline__ void gadget_at(const u64* __restrict__ dp, long long dstride, const u64* ownp,
                                          int owndigit, const u64* __restrict__ key, int beta, int L, int K, int klvl,
                                          int m, int N, int j, const ModConst& mc, u64& r0, u64& r1) {
  r0 = r1 = 0;
  const long long kstride = (long long)(klvl + 1 + K) * N;
  const u64* kp = key + (long long)key_pos(m, L, klvl) * N + j;
  for (int i0 = 0; i0 < beta; i0 += 4) {
    u64 d[4], k0[4], k1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u;
      if (i < beta) {
        d[u] = i == owndigit ? ownp[j] : dp[i * dstride + j];
        k0[u] = kp[(2 * i + 0) * kstride];
        k1[u] = kp[(2 * i + 1) * kstride];
      }
    }
    MacAcc a0, a1;
    mac_zero(a0), mac_zero(a1);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i0 + u < beta) {
        mac_add(a0, d[u], k0[u]);
        mac_add(a1, d[u], k1[u]);
      }
    }
    r0 = add_mod(r0, mac_reduce(a0, mc), mc.q);
    r1 = add_mod(r1, mac_reduce(a1, mc), mc.q);
  }
}

__device__ __forceinline__ void mac_add1(MacAcc& a, u64 x) {
  a.lo += x;
  a.c += (a.lo < x);
}

// XCD-aware block order for the grids (images, coefficient blocks, limbs) of
// lt_bsgs / lt_giant: workgroups go round-robin to the 8 XCDs by linear id,
// so with the image index fastest every XCD would see every coefficient block
// and fill its own L2 with all of the blocks' shared words (diagonals, keys).
// Here linear id L runs on XCD L % 8 over coefficient blocks = XCD (mod 8),
// images fastest: each block's shared words are read into one XCD's L2 only.
// (x, y, z) = (image, coefficient block, limb); needs gridDim.y % 8 == 0.
__device__ __forceinline__ void lt_xcd_decode(int& x, int& y, int& z) {
  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const unsigned xcd = lin & 7, k = lin >> 3, cpx = gy >> 3;
  x = (int)(k % gx);
  const unsigned rest = k / gx;
  y = (int)((rest % cpx) * 8 + xcd);
  z = (int)(rest / cpx);
}

// Hoisted BSGS linear transform, baby steps and giant inner products fused
// (lintrans MultiplyByDiagMatrixBSGS):
//   rot_s  = sigma_s( gadget(D, key_s) + (P * ct0, 0) )   s != 0   (QP, hoisted key switch)
//   rot_0  = (P * ct0, P * ct1) on Q, 0 on P
//   t_g[c] = sum_{s in babies(g)} pt_{g,s} * rot_s[c]
// The NTT-domain automorphism maps every aligned block of 2^k coefficients
// onto an aligned block, so the gathers of one wave stay inside one 512-B
// segment of each source row.  Each thread builds all baby rotations of its
// coefficient in registers and loops over the giants: the rotations never
// touch HBM, and every diagonal (shared by the batch; the image index is the
// fastest grid dimension) is read from L2.
template <int MB>
__device__ __forceinline__ void lt_bsgs_body(LimbSet& t0, LimbSet& t1, const LimbSet& D, const LimbSet& ct,
                                             const LtBabies& Bb, const LtPlan* __restrict__ P, int g0, int g1,
                                             int accumulate, const LimbSet& ptl, const DeviceTables* __restrict__ tb,
                                             int N, int z0) {
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (Bb.xcd) lt_xcd_decode(bx, by, bz);
  const int bi = bx;
  const int n = by * kBlk + threadIdx.x;
  const int l = z0 + bz;
  if (n >= N) return;
  const int m = arg_byte(t0.mod, l);
  const ModConst mc = tb->mc[m];
  const bool isq = l <= Bb.level;
  const long long ro = row_off(t0, 0, l, bi) + n;
  const long long po = (long long)arg_byte(ptl.pos, l) * ptl.limb_stride + n;
  const u64* c0p = ct.p + row_off(ct, 0, isq ? l : 0, bi);
  const u64* c1p = ct.p + row_off(ct, 1, isq ? l : 0, bi);
  const u64* dp = D.p + row_off(D, 0, l, bi);
  const int owndigit = isq ? l / Bb.K : -1;
  const u64 pq = Bb.pq[l], pqs = Bb.pqs[l];
  u64 x0[MB], x1[MB];
  int jx[MB];
#pragma unroll
  for (int s = 0; s < MB; ++s) jx[s] = (s < Bb.nb && Bb.key[s]) ? (int)Bb.idx[s][n] : n;
#pragma unroll
  for (int s = 0; s < MB; ++s) {
    x0[s] = x1[s] = 0;
    if (s < Bb.nb) {
      if (Bb.key[s] && !(LT_ABLATE & 2) && !((LT_ABLATE & 8) && mc.bar_k > 48)) {
        const int j = jx[s];
        u64 r0, r1;
        // (a split30 copy of the keys with carry-free MacW products measured
        // 1848 -> 1947 us per lt_bsgs_kernel8 launch just for being compiled in,
        // and no faster when used: profiles/r04h_lt_gadget_w_ab.txt)
        gadget_at(dp, D.comp_stride, c1p, owndigit, Bb.key[s], Bb.beta, Bb.L, Bb.K, Bb.klvl[s], m, N, j, mc, r0, r1);
        if (isq) r0 = add_mod(r0, shoup_mul(c0p[j], pq, pqs, mc.q), mc.q);
        x0[s] = r0;
        x1[s] = r1;
      } else if (isq) {
        x0[s] = shoup_mul(c0p[n], pq, pqs, mc.q);
        x1[s] = shoup_mul(c1p[n], pq, pqs, mc.q);
      }
    }
  }
  const bool small = mc.bar_k <= 48;  // block-uniform
  if (small) {
    // < 2^48 moduli: float64 split products (MacD), one reduction per giant;
    // the baby rotations as 24-bit pieces in doubles
    double xb0[MB], xa0[MB], xb1[MB], xa1[MB];
#pragma unroll
    for (int s = 0; s < MB; ++s) {
      xb0[s] = (double)(u32)(x0[s] & 0xffffffull), xa0[s] = (double)(u32)(x0[s] >> 24);
      xb1[s] = (double)(u32)(x1[s] & 0xffffffull), xa1[s] = (double)(u32)(x1[s] >> 24);
    }
    // the giant loop instantiated with and without accumulation (uniform)
    auto giants = [&](auto acc_tag) {
      constexpr bool ACC = decltype(acc_tag)::value;
      for (int g = g0; g < g1; ++g) {
        const unsigned long long mask = P->mask[g] >> Bb.s0;
        u64 r0 = 0, r1 = 0;
        if (ACC) {
          r0 = t0.p[(long long)(g - g0) * t0.comp_stride + ro];
          r1 = t1.p[(long long)(g - g0) * t1.comp_stride + ro];
        }
        u64 pv[MB];
#pragma unroll
        for (int s = 0; s < MB; ++s) pv[s] = (LT_DENSE || ((mask >> s) & 1ull)) ? ((LT_ABLATE & 16) ? (u64)(po + 977 * s + g) : gld(P->pt[g][Bb.s0 + s], po)) : 0;
        MacD a0, a1;
        macd_zero(a0), macd_zero(a1);
#pragma unroll
        for (int s = 0; s < MB; ++s) {
          if ((LT_DENSE || ((mask >> s) & 1ull)) && !(LT_ABLATE & 1)) {
            // the plan's diagonal copies are stored split (EW_SPLIT24): pieces in the two dwords
            // (signed conversions of the dwords: converting (u32)(pv >> 32) went
            // through the u64 conversion and left an add of 0.0 * 2^32 behind)
            u32 w[2];
            __builtin_memcpy(w, &pv[s], 8);
            const double pb = (double)(int)w[0], pa = (double)(int)w[1];  // pieces < 2^24
            macd_add(a0, xb0[s], xa0[s], pb, pa);
            macd_add(a1, xb1[s], xa1[s], pb, pa);
          }
        }
        const u64 v0 = macd_reduce(a0, mc), v1 = macd_reduce(a1, mc);
        r0 = ACC ? add_mod(r0, v0, mc.q) : v0;
        r1 = ACC ? add_mod(r1, v1, mc.q) : v1;
        t0.p[(long long)(g - g0) * t0.comp_stride + ro] = r0;
        t1.p[(long long)(g - g0) * t1.comp_stride + ro] = r1;
      }
    };
    if (accumulate) giants(std::true_type{});
    else giants(std::false_type{});
    return;
  }
  if (LT_INT30 && mc.bar_k <= 60) {
    // 48..60-bit moduli: 30-bit piece products accumulated without carries
    // (MacW, one v_mad_u64_u32 each), one reduction per 8 babies; the plan's
    // diagonal copies are stored split30, and the baby rotations are cut into
    // their pieces once here (the split30 word takes the same two VGPRs), not
    // per giant
    if (LT_PRESPLIT) {
#pragma unroll
      for (int s = 0; s < MB; ++s) x0[s] = split30(x0[s]), x1[s] = split30(x1[s]);
    }
    for (int g = g0; g < g1; ++g) {
      const unsigned long long mask = P->mask[g] >> Bb.s0;
      u64 r0 = 0, r1 = 0;
      if (accumulate) {
        r0 = t0.p[(long long)(g - g0) * t0.comp_stride + ro];
        r1 = t1.p[(long long)(g - g0) * t1.comp_stride + ro];
      }
      u64 pv[MB];
#pragma unroll
      for (int s = 0; s < MB; ++s) pv[s] = (LT_DENSE || ((mask >> s) & 1ull)) ? ((LT_ABLATE & 16) ? (u64)(po + 977 * s + g) : gld(P->pt[g][Bb.s0 + s], po)) : 0;
      MacW a0, a1;
      macw_zero(a0), macw_zero(a1);
#pragma unroll
      for (int s = 0; s < MB; ++s) {
        if ((LT_DENSE || ((mask >> s) & 1ull)) && !(LT_ABLATE & 4)) {
          const u32 yb = (u32)pv[s], ya = (u32)(pv[s] >> 32);
          if (LT_PRESPLIT) {
            macw_add(a0, (u32)x0[s], (u32)(x0[s] >> 32), yb, ya);
            macw_add(a1, (u32)x1[s], (u32)(x1[s] >> 32), yb, ya);
          } else {
            macw_add(a0, (u32)x0[s] & 0x3fffffffu, (u32)(x0[s] >> 30), yb, ya);
            macw_add(a1, (u32)x1[s] & 0x3fffffffu, (u32)(x1[s] >> 30), yb, ya);
          }
        }
        if ((s & 7) == 7) {
          r0 = add_mod(r0, macw_reduce8(a0, mc), mc.q);
          r1 = add_mod(r1, macw_reduce8(a1, mc), mc.q);
          macw_zero(a0), macw_zero(a1);
        }
      }
      t0.p[(long long)(g - g0) * t0.comp_stride + ro] = r0;
      t1.p[(long long)(g - g0) * t1.comp_stride + ro] = r1;
    }
    return;
  }
  // moduli of at most 60 bits: 8 products per reduction (mac_reduce8)
  const bool acc8 = LT_INT_ACC8 && mc.bar_k <= 60;
  for (int g = g0; g < g1; ++g) {
    const unsigned long long mask = P->mask[g] >> Bb.s0;
    u64 r0 = 0, r1 = 0;
    if (accumulate) {
      r0 = t0.p[(long long)(g - g0) * t0.comp_stride + ro];
      r1 = t1.p[(long long)(g - g0) * t1.comp_stride + ro];
    }
    // issue every diagonal load of this giant before the first product so
    // their latencies overlap (the branches are wave-uniform)
    u64 pv[MB];
#pragma unroll
    for (int s = 0; s < MB; ++s) pv[s] = (LT_DENSE || ((mask >> s) & 1ull)) ? ((LT_ABLATE & 16) ? (u64)(po + 977 * s + g) : gld(P->pt[g][Bb.s0 + s], po)) : 0;
    MacAcc a0, a1;
    mac_zero(a0), mac_zero(a1);
#pragma unroll
    for (int s = 0; s < MB; ++s) {
      if ((LT_DENSE || ((mask >> s) & 1ull)) && !(LT_ABLATE & 4)) {
        mac_add(a0, pv[s], x0[s]);
        mac_add(a1, pv[s], x1[s]);
      }
      if (acc8 ? (s & 7) == 7 : (s & 3) == 3) {  // (acc8 is block-uniform)
        r0 = add_mod(r0, acc8 ? mac_reduce8(a0, mc) : mac_reduce(a0, mc), mc.q);
        r1 = add_mod(r1, acc8 ? mac_reduce8(a1, mc) : mac_reduce(a1, mc), mc.q);
        mac_zero(a0), mac_zero(a1);
      }
    }
    t0.p[(long long)(g - g0) * t0.comp_stride + ro] = r0;
    t1.p[(long long)(g - g0) * t1.comp_stride + ro] = r1;
  }
}

// MB = 8 at 4 waves per SIMD (<= 128 VGPRs); MB = 16 holds twice the babies
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LT_WAVES8)))
lt_bsgs_kernel8(LimbSet t0, LimbSet t1, LimbSet D, LimbSet ct, LtBabies Bb, const LtPlan* __restrict__ P, int g0,
                int g1, int accumulate, LimbSet ptl, const DeviceTables* __restrict__ tb, int N, int z0) {
  lt_bsgs_body<8>(t0, t1, D, ct, Bb, P, g0, g1, accumulate, ptl, tb, N, z0);
}
__global__ void __launch_bounds__(256)
lt_bsgs_kernel16(LimbSet t0, LimbSet t1, LimbSet D, LimbSet ct, LtBabies Bb, const LtPlan* __restrict__ P, int g0,
                 int g1, int accumulate, LimbSet ptl, const DeviceTables* __restrict__ tb, int N, int z0) {
  lt_bsgs_body<16>(t0, t1, D, ct, Bb, P, g0, g1, accumulate, ptl, tb, N, z0);
}

// Giant steps of a hoisted BSGS transform, key switches and accumulation fused:
//   acc[c] = sum_g sigma_g( gadget(D_g, key_g)[c] + (c == 0) * t0_g ) + z[c]
// D_g: decomposition of ModDown(t1_g) (digit i of group g at D.p + g*d_gstride
// + i*D.comp_stride; its own Q limbs read from `own`, the ModDown output);
// z = the zero giant's (t0, t1), added without automorphism.
// Each thread takes one coefficient of IB images: the automorphism index, the
// key words and every pointer step are shared by the IB images, so the key
// reads from L2 and the scalar address work per product drop IB-fold.
#ifndef LT_GIANT_WAVES
#define LT_GIANT_WAVES 0  // timing switch: minimum waves per SIMD for lt_giant (0: the compiler's choice)
#endif
template <int IB, bool ROWS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LT_GIANT_WAVES > 0 ? LT_GIANT_WAVES : 1)))
lt_giant_kernel(LimbSet acc, LimbSet D, LimbSet own, LimbSet t0, LimbSet z,
                                                       LtGiants G, const DeviceTables* __restrict__ tb, int N) {
  constexpr int CH = LT_GIANT_CH > 0 ? LT_GIANT_CH : (IB >= 4 ? 2 : 4);  // digits per load chunk
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (G.xcd) lt_xcd_decode(bx, by, bz);
  const int b0 = bx * IB;
  const int n = by * kBlk + threadIdx.x;
  const int l = bz;
  if (n >= N) return;
  const int nb = acc.nbatch - b0 < IB ? acc.nbatch - b0 : IB;  // uniform
  const int m = arg_byte(acc.mod, l);
  const ModConst mc = tb->mc[m];
  const bool isq = l <= G.level;
  const int owndigit = isq ? l / G.K : -1;
  const long long dro = row_off(D, 0, l, b0), oro = row_off(own, 0, isq ? l : 0, b0), tro = row_off(t0, 0, l, b0);
  const long long dbs = D.batch_stride, obs = own.batch_stride, tbs = t0.batch_stride;
  u64 r0[IB], r1[IB];
#pragma unroll
  for (int b = 0; b < IB; ++b) r0[b] = r1[b] = 0;
  // the giant loop, instantiated for the two reduction schemes
  auto giants = [&](auto small_tag) {
    constexpr bool SMALL = decltype(small_tag)::value;
    MacAcc a0[IB], a1[IB];
    if (SMALL) {
#pragma unroll
      for (int b = 0; b < IB; ++b) mac_zero(a0[b]), mac_zero(a1[b]);
    }
    int cnt = 0;
    int jn = G.ng > 0 ? (int)G.idx[0][n] : 0;
    for (int g = 0; g < G.ng; ++g) {
      const int j = jn;
      if (g + 1 < G.ng) jn = G.idx[g + 1][n];  // prefetch the next giant's index
      const int klvl = G.klvl[g];
      const long long kstride = (long long)(klvl + 1 + G.K) * N;
      const u64* kp = G.key[g] + (long long)key_pos(m, G.L, klvl) * N + j;
      const u64* dp = D.p + g * G.d_gstride + dro + j;
      const u64* op = own.p + g * G.own_gstride + oro + j;
      for (int i0 = 0; i0 < G.beta; i0 += CH) {
        u64 d[CH][IB], k0[CH], k1[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int i = i0 + u;
          if (i < G.beta) {
            k0[u] = kp[(2 * i + 0) * kstride];
            k1[u] = kp[(2 * i + 1) * kstride];
            const u64* src = i == owndigit ? op : dp + i * D.comp_stride;
            const long long bs = i == owndigit ? obs : dbs;
#pragma unroll
            for (int b = 0; b < IB; ++b)
              if (b < nb) d[u][b] = src[b * bs];
          }
        }
        if (SMALL) {
#pragma unroll
          for (int u = 0; u < CH; ++u)
            if (i0 + u < G.beta) {
#pragma unroll
              for (int b = 0; b < IB; ++b)
                if (b < nb) mac_add(a0[b], d[u][b], k0[u]), mac_add(a1[b], d[u][b], k1[u]);
            }
        } else {
#pragma unroll
          for (int b = 0; b < IB; ++b) {
            if (b >= nb) break;
            MacAcc c0, c1;
            mac_zero(c0), mac_zero(c1);
#pragma unroll
            for (int u = 0; u < CH; ++u)
              if (i0 + u < G.beta) mac_add(c0, d[u][b], k0[u]), mac_add(c1, d[u][b], k1[u]);
            r0[b] = add_mod(r0[b], mac_reduce(c0, mc), mc.q);
            r1[b] = add_mod(r1[b], mac_reduce(c1, mc), mc.q);
          }
        }
      }
      const u64* tp = t0.p + g * G.t0_gstride + tro + j;
#pragma unroll
      for (int b = 0; b < IB; ++b)
        if (b < nb) {
          const u64 t = tp[b * tbs];
          if (SMALL) mac_add1(a0[b], t);
          else r0[b] = add_mod(r0[b], t, mc.q);
        }
      if (SMALL) {
        cnt += G.beta + 1;
        if (cnt + G.beta + 1 > 120) {
#pragma unroll
          for (int b = 0; b < IB; ++b) {
            r0[b] = add_mod(r0[b], mac_reduce_small(a0[b], mc), mc.q);
            r1[b] = add_mod(r1[b], mac_reduce_small(a1[b], mc), mc.q);
            mac_zero(a0[b]), mac_zero(a1[b]);
          }
          cnt = 0;
        }
      }
    }
    if (SMALL) {
#pragma unroll
      for (int b = 0; b < IB; ++b) {
        r0[b] = add_mod(r0[b], mac_reduce_small(a0[b], mc), mc.q);
        r1[b] = add_mod(r1[b], mac_reduce_small(a1[b], mc), mc.q);
      }
    }
  };
  // moduli below 2^52: every giant's products and its t0 term go into one
  // unreduced accumulator per image, reduced once per <= 120 products instead
  // of once per giant (the Barrett reduction is ~40 VALU ops per component)
  if (LT_GIANT_ACC && mc.bar_k <= 52) giants(std::true_type{});  // block-uniform
  else giants(std::false_type{});
#pragma unroll
  for (int b = 0; b < IB; ++b) {
    if (b >= nb) break;
    u64 x0 = r0[b], x1 = r1[b];
    if (G.has_zero) {
      x0 = add_mod(x0, z.p[row_off(z, 0, l, b0 + b) + n], mc.q);
      x1 = add_mod(x1, z.p[row_off(z, 1, l, b0 + b) + n], mc.q);
    }
    r0[b] = x0, r1[b] = x1;
  }
  if constexpr (ROWS) {
    if (l >= G.rows_from) {  // (block-uniform) a P limb: the final ModDown INTT's rows pass, here
      // the block's 256 coefficients are row `by` of the limb, for 2 nb
      // (image, component) rows q = 2 b + c: staged in LDS, then 4 rows at a
      // time, thread (rr, kk) runs the radix-4 inverse rows steps on elements
      // 4 kk .. 4 kk + 3 of row q0 + rr and stores the INTT's intermediate in
      // place of the row.  A group past the last row works on a spare LDS row
      // of its own and stores nothing, so every thread keeps the barriers.
      constexpr int NR = 2 * IB > 4 ? 2 * IB : 4;
      __shared__ u64 lds[NR * 256];
      const int t = threadIdx.x;
#pragma unroll
      for (int b = 0; b < IB; ++b)
        if (b < nb) lds[(2 * b) * 256 + t] = r0[b], lds[(2 * b + 1) * 256 + t] = r1[b];
      __syncthreads();
      const int rr = t >> 6, kk = t & 63;
      for (int q0 = 0; q0 < 2 * nb; q0 += 4) {  // (uniform)
        const int q = q0 + rr;
        const bool live = q < 2 * nb;
        u64* const lr = lds + q * 256;
        u64* const mid = acc.p + row_off(acc, q & 1, l, b0 + (live ? q >> 1 : 0)) + (by << 8);
        auto rows = [&](const auto& ar, __amdgpu_buffer_rsrc_t tw) {
          using A = std::decay_t<decltype(ar)>;
          typename A::T x[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) x[i] = ar.from_u64(lr[4 * kk + i]);
          if (G.logN == 15)
            inv_rows4_core<A, 15>(x, by, kk, ar, tw, lr, mid, live);
          else
            inv_rows4_core<A, 16>(x, by, kk, ar, tw, lr, mid, live);
        };
        if (mc.f64)
          rows(F64Arith(mc), twr_s(tb->inv_d[m], 8 * N));
        else
          rows(IntArith(mc), twr_s(tb->inv[m], 16 * N));
      }
      return;
    }
  }
#pragma unroll
  for (int b = 0; b < IB; ++b) {
    if (b >= nb) break;
    acc.p[row_off(acc, 0, l, b0 + b) + n] = r0[b];
    acc.p[row_off(acc, 1, l, b0 + b) + n] = r1[b];
  }
}

inline dim3 ew_grid(int N, int rows) { return dim3((N / 2 + 255) / 256, rows); }
// split the targets of a small basis extension over blockIdx.z until the
// launch has ~2048 workgroups (8 per CU); the per-coefficient prologue is
// recomputed per chunk, which costs ns multiplies against nt/chunk targets
inline unsigned target_chunks(dim3 g, int nt) {
  const long long wg = (long long)g.x * g.y;
  long long z = (2048 + wg - 1) / wg;
  if (z > nt / 4) z = nt / 4;  // keep >= 4 targets per chunk
  return z < 1 ? 1u : (unsigned)z;
}

}  // namespace

// ------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------
int orion_launch_ew(int op, const LimbSet& o, const LimbSet& a, const LimbSet& b, const u64* s, const u64* ss,
                    const DeviceTables* tb, int N, hipStream_t st) {
  Scalars sc;
  for (int l = 0; l < o.nlimb; ++l) {
    sc.s[l] = s ? s[l] : 0;
    sc.ss[l] = ss ? ss[l] : 0;
  }
  const int rows = o.ncomp * o.nlimb * o.nbatch;
  if (rows == 0) return 0;
  dim3 g = ew_grid(N, rows), blk(256);
  switch (op) {
#define CASE(OPC) \
  case OPC: hipLaunchKernelGGL(ew_kernel<OPC>, g, blk, 0, st, o, a, b, sc, tb, N); break;
    CASE(EW_ADD) CASE(EW_SUB) CASE(EW_MUL) CASE(EW_MULADD) CASE(EW_NEG) CASE(EW_SCALE) CASE(EW_ADDC)
    CASE(EW_SUBSCALE) CASE(EW_COPY) CASE(EW_ADDSCALE) CASE(EW_SPLIT24)
#undef CASE
    default: return -1;
  }
  return 0;
}

int orion_launch_tensor(const LimbSet& d, const LimbSet& a, const LimbSet& b, const DeviceTables* tb, int N,
                        hipStream_t st) {
  const int rows = d.nlimb * d.nbatch;
  hipLaunchKernelGGL(tensor_kernel, ew_grid(N, rows), dim3(256), 0, st, d, a, b, tb, N);
  return 0;
}


int orion_launch_basis_ext(const LimbSet& out, const LimbSet& in, const BasisExtTable* T, const DeviceTables* tb,
                           int N, hipStream_t st) {
  const int rows = out.ncomp * out.nbatch;
  dim3 g = ew_grid(N, rows);
  const int nt = out.nlimb;
  g.z = target_chunks(g, nt);
  const int tc = (nt + g.z - 1) / g.z;
  // the kernel's source arrays sized for in.nlimb (= the table's ns)
  if (in.nlimb <= 2)
    hipLaunchKernelGGL(basis_ext_kernel<2>, g, dim3(256), 0, st, out, in, T, N, tc);
  else if (in.nlimb <= 4)
    hipLaunchKernelGGL(basis_ext_kernel<4>, g, dim3(256), 0, st, out, in, T, N, tc);
  else if (in.nlimb <= ORION_MAXSRC)
    hipLaunchKernelGGL(basis_ext_kernel<ORION_MAXSRC>, g, dim3(256), 0, st, out, in, T, N, tc);
  else
    return -1;
  return 0;
}

int orion_launch_modup_all(const LimbSet& D, const LimbSet& in, const BasisExtTable* Ts, int beta, int K,
                           int nqp, const DeviceTables* tb, int N, hipStream_t st) {
  if (beta < 1 || nqp > ORION_MAXLIMB || D.ncomp != in.ncomp * beta) return -1;
  for (int j = 0; j < nqp; ++j)
    if (D.pos[j] != j) return -1;  // the kernel walks the limbs with one pointer
  const int rows = D.ncomp * D.nbatch;
  dim3 g = ew_grid(N, rows);
  g.z = target_chunks(g, nqp);
  const int tc = (nqp + g.z - 1) / g.z;
  if (K <= 2)  // every digit has at most K sources
    hipLaunchKernelGGL(modup_all_kernel<2>, g, dim3(256), 0, st, D, in, Ts, beta, K, nqp, N, tc);
  else if (K <= 4)
    hipLaunchKernelGGL(modup_all_kernel<4>, g, dim3(256), 0, st, D, in, Ts, beta, K, nqp, N, tc);
  else if (K <= ORION_MAXSRC)
    hipLaunchKernelGGL(modup_all_kernel<ORION_MAXSRC>, g, dim3(256), 0, st, D, in, Ts, beta, K, nqp, N, tc);
  else
    return -1;
  return 0;
}

int orion_launch_ks_mac(const LimbSet& out, const LimbSet& D, const LimbSet& own, const MacGroups& G, int ngroup,
                        int beta, const DeviceTables* tb, int N, hipStream_t st) {
  const int rows = ngroup * out.nlimb * out.nbatch;
  if (rows == 0) return 0;
  if (ngroup > ORION_MAXGROUP) return -1;
  if (G.rows_from > 0) {
    if ((G.logN != 15 && G.logN != 16) || N != (1 << G.logN) || ngroup != 1) return -1;
    if (G.fwd_rows) {
      if (beta > 16 || G.d_gstride) return -1;
      // (4 + 2 beta) x 2 KiB of LDS: up to 72 KiB at beta = 16, past the
      // 64 KiB a launch gets without the attribute (set once, for the largest)
      static const bool lds_attr = hipFuncSetAttribute((const void*)ks_mac_full_kernel<false>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (4 + 2 * 16) * 256 * 8) == hipSuccess;
      if (!lds_attr) return -1;
      const size_t lds = (size_t)(4 + 2 * beta) * 256 * 8;
      if (beta <= 4)  // the key words loaded before the rows pass (12 KiB of LDS at most)
        hipLaunchKernelGGL(ks_mac_full_kernel<true>, ew_grid(N, rows), dim3(256), lds, st, out, D, own, G, beta, tb, N);
      else
        hipLaunchKernelGGL(ks_mac_full_kernel<false>, ew_grid(N, rows), dim3(256), lds, st, out, D, own, G, beta, tb, N);
      return 0;
    }
    hipLaunchKernelGGL(ks_mac_rows_kernel, ew_grid(N, rows), dim3(256), 0, st, out, D, own, G, beta, tb, N);
    return 0;
  }
  hipLaunchKernelGGL(ks_mac_kernel, ew_grid(N, rows), dim3(256), 0, st, out, D, own, G, beta, tb, N);
  return 0;
}

int orion_launch_lt_bsgs(const LimbSet& t0, const LimbSet& t1, const LimbSet& D, const LimbSet& ct,
                         const LtBabies& Bb, const LtPlan* plan, int g0, int g1, int accumulate, const LimbSet& ptl,
                         const DeviceTables* tb, int N, hipStream_t st) {
  if (Bb.nb < 1 || Bb.nb > LT_MAXB || g1 <= g0) return -1;
  auto launch = [&](int z0, int nz) {
    if (nz <= 0) return;
    dim3 g(t0.nbatch, (N + 255) / 256, nz);
    if (Bb.nb <= 8)
      hipLaunchKernelGGL(lt_bsgs_kernel8, g, dim3(256), 0, st, t0, t1, D, ct, Bb, plan, g0, g1, accumulate, ptl, tb,
                         N, z0);
    else
      hipLaunchKernelGGL(lt_bsgs_kernel16, g, dim3(256), 0, st, t0, t1, D, ct, Bb, plan, g0, g1, accumulate, ptl, tb,
                         N, z0);
  };
  // ORION_LT_SPLIT=1 (timing diagnostics): three launches, limb 0, the middle
  // Q limbs and the last Bb.K (P) limbs, so a kernel trace times each class
  static const bool split = getenv("ORION_LT_SPLIT") && atoi(getenv("ORION_LT_SPLIT")) == 1;
  if (split && t0.nlimb > Bb.K + 1) {
    launch(0, 1);
    launch(1, t0.nlimb - 1 - Bb.K);
    launch(t0.nlimb - Bb.K, Bb.K);
  } else {
    launch(0, t0.nlimb);
  }
  return 0;
}

int orion_launch_lt_giant(const LimbSet& acc, const LimbSet& D, const LimbSet& own, const LimbSet& t0,
                          const LimbSet& z, const LtGiants& G, const DeviceTables* tb, int N, hipStream_t st) {
  if (G.ng > ORION_MAXGROUP) return -1;
  if (G.rows_from > 0 && ((G.logN != 15 && G.logN != 16) || N != (1 << G.logN))) return -1;
  // one image (batch 1): the one-image instantiation, whose registers are a
  // quarter of IB = 4's (more waves per SIMD, more loads in flight per CU)
  const bool one = acc.nbatch == 1 && LT_GIANT_B1;
  if (one) {
    const dim3 g(1, (N + 255) / 256, acc.nlimb);
    if (G.rows_from > 0)
      hipLaunchKernelGGL((lt_giant_kernel<1, true>), g, dim3(256), 0, st, acc, D, own, t0, z, G, tb, N);
    else
      hipLaunchKernelGGL((lt_giant_kernel<1, false>), g, dim3(256), 0, st, acc, D, own, t0, z, G, tb, N);
    return 0;
  }
  constexpr int IB = LT_GIANT_IB;
  dim3 g((acc.nbatch + IB - 1) / IB, (N + 255) / 256, acc.nlimb);
  if (G.rows_from > 0) {
    hipLaunchKernelGGL((lt_giant_kernel<IB, true>), g, dim3(256), 0, st, acc, D, own, t0, z, G, tb, N);
    return 0;
  }
  hipLaunchKernelGGL((lt_giant_kernel<IB, false>), g, dim3(256), 0, st, acc, D, own, t0, z, G, tb, N);
  return 0;
}

int orion_launch_automorph(const LimbSet& o, const LimbSet& a, const u32* idx, const DeviceTables* tb, int N,
                           int accumulate, hipStream_t st) {
  const int rows = o.ncomp * o.nlimb * o.nbatch;
  hipLaunchKernelGGL(automorph_kernel, ew_grid(N, rows), dim3(256), 0, st, o, a, idx, tb, N, accumulate);
  return 0;
}
