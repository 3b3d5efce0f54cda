// common.h -- shared types and 64-bit modular arithmetic for the MI355X
// (gfx950) RNS-CKKS backend.  Device and host.
//
// Layout conventions:
//   * a residue polynomial limb is N u64 words, NTT domain unless stated,
//     fully reduced in [0, q) at every kernel boundary;
//   * a ciphertext batch is [comp][limb][batch][N]: one limb-plane per
//     (comp, limb) holds the B independent images contiguously, so kernels
//     index (comp, limb, image) -> one workgroup (NTT) or one grid row;
//   * QP moduli index space = [q_0 .. q_{L-1}, p_0 .. p_{K-1}].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint64_t u64;
typedef uint32_t u32;

#define ORION_MAXMOD 80   // max |Q| + |P|
#ifndef ORION_MAXLIMB
#define ORION_MAXLIMB 64  // max limbs touched by one kernel launch (QP at one level)
#endif

// ---------------------------------------------------------------------------
// per-modulus constants (device-resident table, indexed by QP modulus index)
// ---------------------------------------------------------------------------
struct ModConst {
  u64 q;        // modulus
  u64 bar_mu;   // floor(2^(2k) / q), k = bitlen(q)   (Barrett)
  int bar_k;    // bitlen(q)
  int f64;      // 1: NTT in float64 arithmetic (q < 2^ORION_F64_BITS)
  u64 bar_mu2;  // floor(2^(2k+2) / q)                    (Barrett for x < 4 q^2)
  u64 bar_mu8;  // floor(2^(2k+8) / q), k <= 52           (Barrett for x < 256 q^2)
  u64 bar_mu3;  // floor(2^(2k+3) / q), k <= 60           (Barrett for x < 8 q^2)
  u64 ninv, ninv_s;  // N^-1 and its Shoup companion
  double qd, qinv_d, ninv_d;  // float64 path: q, 1/q, centered N^-1
  // ConjugateInvariant ring (scheme.go:49-52, NthRoot 4N): W = psi^N (a square
  // root of -1 mod q) and its Shoup companion.  The forward NTT folds its input
  // b_e = a_e - W a_{N-e} (the expansion reduced mod X^N - W), the inverse
  // unfolds a_e = (b_e + W b_{N-e}) / 2, with the 1/2 folded into ninv = (2N)^-1.
  // Zero in a Standard ring.
  u64 ciw, ciw_s;
  // the inverse NTT's last stage with N^-1 folded in (ntt.hip NTT_INV_FOLD):
  // X = (x + y) N^-1, Y = (x - y) w1 N^-1, w1 = the stage's twiddle (inv[1])
  u64 wl, wl_s;
  double wl_d;  // centered
};
#define ORION_F64_BITS 46

struct DeviceTables {
  ModConst mc[ORION_MAXMOD];
  // twiddles, interleaved {w, floor(w*2^64/q)} : fwd[m][k] = psi^bitrev(k), inv = psi^-bitrev(k)
  const ulonglong2* fwd[ORION_MAXMOD];
  const ulonglong2* inv[ORION_MAXMOD];
  // float64 path: centered twiddles (|w| <= q/2) as doubles, same indexing
  const double* fwd_d[ORION_MAXMOD];
  const double* inv_d[ORION_MAXMOD];
};

// ---------------------------------------------------------------------------
// a batch of limbs: element (c, l, b, n) at p[c*comp_stride + pos[l]*limb_stride + b*batch_stride + n]
// ---------------------------------------------------------------------------
struct LimbSet {
  u64* p;
  long long comp_stride, limb_stride, batch_stride;
  int ncomp, nlimb, nbatch;
  int pad;
  unsigned char mod[ORION_MAXLIMB];  // QP modulus index of limb l
  unsigned char pos[ORION_MAXLIMB];  // limb l lives at p + pos[l]*limb_stride
};

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
// byte i (wave-uniform) of a small table in the kernel arguments, read as its
// aligned dword: scalar loads are dword-granular, so a byte load at a dynamic
// index would be a vector load followed by vmcnt(0) -- and vector memory
// operations retire in order, so that wait also drains every load and store
// still in flight (a persistent kernel decodes its next job while the
// previous job's stores drain)
__device__ __forceinline__ int arg_byte(const unsigned char* a, int i) {
  i = __builtin_amdgcn_readfirstlane(i);
  const unsigned w = reinterpret_cast<const unsigned*>(a)[i >> 2];
  return (int)((w >> ((i & 3) * 8)) & 0xff);
}
#endif

// ---------------------------------------------------------------------------
// modular arithmetic (q < 2^62)
// ---------------------------------------------------------------------------
__host__ __device__ static inline u64 mulhi64(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (u64)(((unsigned __int128)a * b) >> 64);
#endif
}

__host__ __device__ static inline u64 add_mod(u64 a, u64 b, u64 q) {
  u64 c = a + b;
  return c >= q ? c - q : c;
}
__host__ __device__ static inline u64 sub_mod(u64 a, u64 b, u64 q) {
  return a >= b ? a - b : a + q - b;
}
// Shoup: a*w mod q in [0, 2q), ws = floor(w*2^64/q), any a < 2^64
__host__ __device__ static inline u64 shoup_lazy(u64 a, u64 w, u64 ws, u64 q) {
  return a * w - mulhi64(a, ws) * q;
}
__host__ __device__ static inline u64 shoup_mul(u64 a, u64 w, u64 ws, u64 q) {
  u64 r = shoup_lazy(a, w, ws, q);
  return r >= q ? r - q : r;
}
// Shoup's a*w mod q in [0, 2q) from 32-bit pieces, the quotient product added
// as qh * (2^64 - q): t = a*w + qh*nq (mod 2^64) needs no 64-bit subtraction
// (and no carry-chain hazards); 4 v_mad_u64_u32 + 4 v_mul_lo_u32 + 1 v_mul_hi_u32
__device__ __forceinline__ u64 shoup_lazy_nq(u64 a, u64 w, u64 ws, u64 nq) {
  const u32 a0 = (u32)a, a1 = (u32)(a >> 32), s0 = (u32)ws, s1 = (u32)(ws >> 32);
  const u64 m1 = (u64)a1 * s0 + __umulhi(a0, s0);
  const u64 m2 = (u64)a0 * s1 + (u32)m1;
  const u64 qh = (u64)a1 * s1 + ((m1 >> 32) + (m2 >> 32));  // floor(a * ws / 2^64)
  const u32 h0 = (u32)qh, h1 = (u32)(qh >> 32), w0 = (u32)w, w1 = (u32)(w >> 32);
  const u32 n0 = (u32)nq, n1 = (u32)(nq >> 32);
  const u64 lo = (u64)h0 * n0 + (u64)a0 * w0;
  const u32 hi = (u32)(lo >> 32) + a0 * w1 + a1 * w0 + h0 * n1 + h1 * n0;
  return ((u64)hi << 32) | (u32)lo;
}

// the same with the quotient cut: the high word of a0*s0 and the low carries
// are dropped, so qh <= floor(a*ws/2^64) <= qh + 2 and the result is in
// [0, 4q) (ntt_arith.h NTT_INT_CUT): 4 v_mad_u64_u32 + 4 v_mul_lo_u32
__device__ __forceinline__ u64 shoup_cut_nq(u64 a, u64 w, u64 ws, u64 nq) {
  const u32 a0 = (u32)a, a1 = (u32)(a >> 32), s0 = (u32)ws, s1 = (u32)(ws >> 32);
  const u64 m1 = (u64)a1 * s0;
  const u64 m2 = (u64)a0 * s1 + (u32)m1;
  const u64 qh = (u64)a1 * s1 + ((m1 >> 32) + (m2 >> 32));
  const u32 h0 = (u32)qh, h1 = (u32)(qh >> 32), w0 = (u32)w, w1 = (u32)(w >> 32);
  const u32 n0 = (u32)nq, n1 = (u32)(nq >> 32);
  const u64 lo = (u64)h0 * n0 + (u64)a0 * w0;
  const u32 hi = (u32)(lo >> 32) + a0 * w1 + a1 * w0 + h0 * n1 + h1 * n0;
  return ((u64)hi << 32) | (u32)lo;
}

// Barrett reduction of the 128-bit value hi:lo < q^2 (q < 2^62)
__host__ __device__ static inline u64 barrett128(u64 hi, u64 lo, const ModConst& m) {
  const int k = m.bar_k;
  // t1 = x >> (k-1)  (< 2^(k+1))
  u64 t1 = (lo >> (k - 1)) | (hi << (65 - k));
  // t2 = (t1 * mu) >> (k+1)
  u64 ph = mulhi64(t1, m.bar_mu), pl = t1 * m.bar_mu;
  u64 t2 = (pl >> (k + 1)) | (ph << (63 - k));
  u64 r = lo - t2 * m.q;
  if (r >= m.q) r -= m.q;
  if (r >= m.q) r -= m.q;
  return r;
}
__host__ __device__ static inline u64 mul_mod(u64 a, u64 b, const ModConst& m) {
  return barrett128(mulhi64(a, b), a * b, m);
}
// 128-bit accumulator helpers
struct Acc128 {
  u64 hi, lo;
};
__host__ __device__ static inline void mac128(Acc128& a, u64 x, u64 y) {
  const u64 l = x * y, h = mulhi64(x, y);
  const u64 nl = a.lo + l;
  a.hi += h + (nl < l);
  a.lo = nl;
}

// ---------------------------------------------------------------------------
// host-side tables for basis extension (ModUp / ModDown), device-resident
//   y_i  = x_i * qhatinv[i] mod s_i
//   v    = (u64) sum_i (double)y_i / (double)s_i    (Lattigo reconstructRNS:
//          correctly rounded divisions summed in source order, truncated)
//   out_t = sum_i y_i * qhat_t[t][i] - v * S_t[t]   mod t
// centered (a gadget digit of one prime, Lattigo DecomposeAndSplit's
// decompLvl == -1 branch): v = (x >= s >> 1), i.e. x - s is extended
// ---------------------------------------------------------------------------
#define ORION_MAXSRC 8
#define ORION_MAXBABY 64  // baby steps fused into one BSGS giant-step MAC launch
// the constants of one target t, in one record so that a kernel reads them
// from a single wave-uniform base (s_load_dwordx* at fixed offsets).  The
// target sum sum_i y_i qh_i + v nS (then mod t) is formed in one of four ways,
// chosen per target on the host from the moduli's sizes (BasisExtTable.ns >=
// 3 for the last two):
//   BEXT_LAZY:   Shoup products, the running sum kept in [0, 2t)
//   BEXT_NARROW: sources and t below 2^32 and (sum s_i + ns) t < 2^63: the whole
//                sum in one u64 of 32x32-bit products, one float64 reduction
//   BEXT_WT:     sources below 2^32, t wide: qh cut into 30-bit pieces on the
//                host, three carry-free u64 columns of 32x32-bit products, one
//                Barrett reduction of the 128-bit sum (x < 4 t^2)
//   BEXT_NT:     t below 2^31, sources wide: y cut into 30-bit pieces, three
//                carry-free columns, folded to 128 bits and reduced in float64
enum { BEXT_LAZY = 0, BEXT_NARROW = 1, BEXT_WT = 2, BEXT_NT = 3 };
struct BextTarget {
  u64 q;                // t
  double tinv, tinv32;  // RN(1 / t) and 2^32 times it (BEXT_NARROW, BEXT_NT)
  double qd;            // (double)t
  int mode, k;          // k = bitlen(t) (BEXT_WT's Barrett)
  u64 mu2;              // floor(2^(2k+2) / t) (BEXT_WT)
  u64 c64;              // 2^64 mod t (BEXT_NT)
  u64 nS, nSs;          // (t - S mod t) mod t (v * nS = Lattigo's vtimesqmodp[v]) and its Shoup companion
  u64 vS[3];            // v nS mod t for v = 0, 1, 2 (BEXT_LAZY with at most 2 sources: selected, not multiplied)
  u32 n0, n1, n2;       // nS in 30-bit pieces (BEXT_WT)
  u32 pad;
  u64 qh[ORION_MAXSRC];  // (S/s_i) mod t
  u64 qhs[ORION_MAXSRC]; // its Shoup companion
  u32 h0[ORION_MAXSRC], h1[ORION_MAXSRC], h2[ORION_MAXSRC];  // qh in 30-bit pieces (BEXT_WT)
};
struct BasisExtTable {
  int ns, nt;
  int centered;
  int pad0;
  u64 chalf;  // s_0 >> 1 (centered tables)
  int src_mod[ORION_MAXSRC];
  int dst_mod[ORION_MAXLIMB];
  u64 sq[ORION_MAXSRC];  // s_i
  u64 qhatinv[ORION_MAXSRC], qhatinv_s[ORION_MAXSRC];
  double qinv_f[ORION_MAXSRC];  // RN(1 / (double)s_i)
  double qf[ORION_MAXSRC];      // (double)s_i (rounded, as Lattigo's float64(Q[i]))
  BextTarget tgt[ORION_MAXLIMB];
};

// ---------------------------------------------------------------------------
// grouped launches (one launch for many independent key switches / rotations)
// ---------------------------------------------------------------------------
#define ORION_MAXGROUP 64
// An evaluation key made for level klvl holds the digits 0..ceil((klvl+1)/K)-1
// over the limbs [q_0 .. q_klvl, p_0 .. p_{K-1}] ([digit][2][klvl+1+K][N]); a
// full-chain key has klvl = L - 1.  QP modulus m sits at limb key_pos(m).
__host__ __device__ static inline int key_pos(int m, int L, int klvl) { return m < L ? m : klvl + 1 + (m - L); }

struct MacGroups {  // ks_mac_kernel: group g uses key[g], made for level klvl[g]
  const u64* key[ORION_MAXGROUP];
  int klvl[ORION_MAXGROUP];
  int L;            // Q moduli of the chain (P modulus index L + k)
  long long out_gstride, d_gstride, add_gstride, own_gstride;
  const u64* add0;  // optional comp-0 addend, layout of out comp 0 (stride add_gstride per group)
  int K;            // digit width (own limbs of digit i: l / K == i)
  // add_nq > 0: scaled Q addends instead -- out limb l < add_nq gets
  // add{0,1}[l] * add_s[l] (the caller passes P mod q_l, so the ModDown that
  // follows yields keyswitch + add exactly), limbs l >= add_nq (P) get 0
  int add_nq;
  const u64* add1;
  u64 add_s[ORION_MAXLIMB], add_ss[ORION_MAXLIMB];
  // rows_from > 0 (ks_mac_rows_kernel, N = 2^logN, logN 15 or 16): out limbs
  // l >= rows_from (the P limbs, read only by the ModDown's INTT) are stored
  // after the INTT's radix-4 rows pass, as its intermediate (ntt2s_rows.h)
  int rows_from, logN;
  // fwd_rows (with rows_from, one group): the decomposition's target rows of
  // D hold its forward NTT's columns-pass intermediate; the gadget product
  // runs their forward rows pass itself, in LDS, before the products
  int fwd_rows;
};

// BSGS linear transform plan (device-resident, one per LinTrans): giants in
// evaluation order, baby slots in the order of LinTrans::babies
#define LT_MAXB 16   // baby rotations held in registers by one lt_bsgs launch
#define LT_MAXG 64   // giants per plan
#define LT_MAXSLOT 64
struct LtPlan {
  unsigned long long mask[LT_MAXG];      // bit s: giant g uses baby slot s
  const u64* pt[LT_MAXG][LT_MAXSLOT];    // diagonal (QP plaintext) of (giant, slot), or null
};
struct LtBabies {  // the baby steps of register slots [s0, s0 + nb) of one lt_bsgs launch
  const u64* key[LT_MAXB];  // Galois key of the slot (null: the zero baby)
  const u32* idx[LT_MAXB];  // its NTT-domain automorphism index
  int klvl[LT_MAXB];        // level the key was made for
  int nb, s0, beta, K, level, L;
  u64 pq[ORION_MAXLIMB], pqs[ORION_MAXLIMB];  // P mod q_l and Shoup companion (0 on the P limbs)
  int xcd;  // 1: XCD-aware block order (lt_xcd_decode)
};
struct LtGiants {  // the nonzero giant steps of one lt_giant launch
  const u64* key[ORION_MAXGROUP];
  const u32* idx[ORION_MAXGROUP];
  int klvl[ORION_MAXGROUP];
  int ng, beta, K, level, L, has_zero;
  long long d_gstride, own_gstride, t0_gstride;
  int xcd;  // 1: XCD-aware block order (lt_xcd_decode)
  // rows_from > 0 (lt_giant_kernel<IB, true>, N = 2^logN, logN 15 or 16): acc
  // limbs l >= rows_from (the P limbs, read only by the final ModDown's INTT)
  // are stored after the INTT's radix-4 rows pass (ntt2s_rows.h)
  int rows_from, logN;
};

// ---------------------------------------------------------------------------
// split multiply-accumulate: up to 4 products x*y of operands < 2^61 summed in
// three 64-bit partial sums, 4 v_mad_u64_u32 + 3 adds per product:
//   lo (+ carries c) = sum x0*y0,  mid = sum x0*y1 + x1*y0,  hi = sum x1*y1
// (x1, y1 < 2^29: mid < 8 * 2^61 = 2^64).  mac_reduce folds the parts into a
// 128-bit value < 4 q^2 and Barrett-reduces it to [0, q).
// ---------------------------------------------------------------------------
struct MacAcc {
  u64 lo, mid, hi;
  u32 c;
};
__device__ __forceinline__ void mac_zero(MacAcc& a) {
  a.lo = a.mid = a.hi = 0;
  a.c = 0;
}
__device__ __forceinline__ void mac_add(MacAcc& a, u64 x, u64 y) {
  const u32 x0 = (u32)x, x1 = (u32)(x >> 32), y0 = (u32)y, y1 = (u32)(y >> 32);
  const u64 p = (u64)x0 * y0;
  a.lo += p;
  a.c += (a.lo < p);
  a.mid += (u64)x0 * y1;
  a.mid += (u64)x1 * y0;
  a.hi += (u64)x1 * y1;
}
// Barrett reduction of hi:lo = x < 4 q^2 (bitlen(q) = k <= 61) with
// mu2 = floor(2^(2k+2)/q): t1 = x >> (k-1) < 2^(k+3), q_est = (t1*mu2) >> (k+3)
// is low by at most 2, so two conditional subtractions finish it.
__device__ __forceinline__ u64 barrett_4q2(u64 hi, u64 lo, const ModConst& m) {
  const int k = m.bar_k;
  const u64 t1 = (lo >> (k - 1)) | (hi << (65 - k));
  const u64 ph = mulhi64(t1, m.bar_mu2), pl = t1 * m.bar_mu2;
  const u64 t2 = (k < 61 ? pl >> (k + 3) : 0) | (ph << (61 - k));
  u64 r = lo - t2 * m.q;
  r = r >= m.q ? r - m.q : r;
  return r >= m.q ? r - m.q : r;
}
// Barrett reduction of hi:lo = x < 256 q^2 for moduli of k <= 52 bits
// (t1 = x >> (k-1) < 2^(k+9) fits 64 bits; q_est low by at most 2)
__device__ __forceinline__ u64 barrett_256q2(u64 hi, u64 lo, const ModConst& m) {
  const int k = m.bar_k;
  const u64 t1 = (lo >> (k - 1)) | (hi << (65 - k));
  const u64 ph = mulhi64(t1, m.bar_mu8), pl = t1 * m.bar_mu8;
  const u64 t2 = (pl >> (k + 9)) | (ph << (55 - k));
  u64 r = lo - t2 * m.q;
  r = r >= m.q ? r - m.q : r;
  return r >= m.q ? r - m.q : r;
}
// Barrett reduction of hi:lo = x < 8 q^2 for moduli of k <= 60 bits
// (t1 = x >> (k-1) < 2^(k+4) <= 2^64, mu3 < 2^(k+4); q_est low by at most 2)
__device__ __forceinline__ u64 barrett_8q2(u64 hi, u64 lo, const ModConst& m) {
  const int k = m.bar_k;
  const u64 t1 = (lo >> (k - 1)) | (hi << (65 - k));
  const u64 ph = mulhi64(t1, m.bar_mu3), pl = t1 * m.bar_mu3;
  const u64 t2 = (k < 60 ? pl >> (k + 4) : 0) | (ph << (60 - k));
  u64 r = lo - t2 * m.q;
  r = r >= m.q ? r - m.q : r;
  return r >= m.q ? r - m.q : r;
}
// a MacAcc of up to 8 products of operands below 2^60 (x1, y1 < 2^28 keep
// the 16 mid terms below 2^64), reduced once (x < 8 q^2)
__device__ __forceinline__ u64 mac_reduce8(const MacAcc& a, const ModConst& m) {
  const u64 ml = a.mid << 32;
  const u64 L = a.lo + ml;
  const u64 H = a.hi + (a.mid >> 32) + a.c + (L < ml);
  return barrett_8q2(H, L, m);
}
// a MacAcc of up to 128 products of operands < 2^52, reduced once (x < 128 q^2;
// x1, y1 < 2^20 keep mid and hi far below 2^64)
__device__ __forceinline__ u64 mac_reduce_small(const MacAcc& a, const ModConst& m) {
  const u64 ml = a.mid << 32;
  const u64 L = a.lo + ml;
  const u64 H = a.hi + (a.mid >> 32) + a.c + (L < ml);
  return barrett_256q2(H, L, m);
}
__device__ __forceinline__ u64 mac_reduce(const MacAcc& a, const ModConst& m) {
  const u64 ml = a.mid << 32;
  const u64 L = a.lo + ml;
  const u64 H = a.hi + (a.mid >> 32) + a.c + (L < ml);
  return barrett_4q2(H, L, m);
}

// ---------------------------------------------------------------------------
// exact basis extension of one coefficient (Lattigo ModUpExact restated;
// SURVEY App. A.5): sources x_i (i < ns, coefficient domain) -> target t.
// The float64 quotient is Lattigo reconstructRNS's: vi += float64(y_i) /
// float64(s_i) in source order.  Each correctly rounded division is formed
// as q0 = RN(y * RN(1/s)), r = y - q0 s (exact by FMA), RN(q0 + r RN(1/s))
// (Markstein: with RN(1/s) and q0 within an ulp of y/s this is RN(y/s) in
// round-to-nearest; checked on 4e8 adversarial pairs against IEEE division,
// and the GPU parity tests compare with the oracle's plain division).
// y[] and v are shared by every target.
// ---------------------------------------------------------------------------
template <int MS = ORION_MAXSRC>  // MS >= ns: the register arrays' size
__device__ __forceinline__ u64 bext_prep(const BasisExtTable* __restrict__ T, const u64* x, u64* y) {
  if (T->centered) {  // one source, qhatinv = 1 (wave-uniform)
    y[0] = x[0];
    return x[0] >= T->chalf ? 1 : 0;
  }
  double vf = 0.0;
  const int ns = T->ns;
#pragma unroll
  for (int i = 0; i < MS; ++i) {
    if (i >= ns) break;
    y[i] = shoup_mul(x[i], T->qhatinv[i], T->qhatinv_s[i], T->sq[i]);
    const double yd = (double)y[i], rc = T->qinv_f[i];
    const double q0 = __dmul_rn(yd, rc);
    const double r = __builtin_fma(-q0, T->qf[i], yd);
    vf = __dadd_rn(vf, __builtin_fma(r, rc, q0));
  }
  return (u64)vf;
}
// the target side of the exact basis extension: sum_i y_i (S/s_i mod t) -
// v S mod t (basis_ext_kernel, modup_all_kernel and the NTT prologue
// NTT_PRO_BEXT).  The per-target constants are wave-uniform (SGPR); the
// correction -v S is one more term of the sum, v times nS = -S mod t (v <= ns
// is small), except on the lazy path with at most 2 sources, where it is one
// of 3 precomputed values
__device__ __forceinline__ u64 bext_narrow_red(u64 acc, const BextTarget* __restrict__ R) {
  // acc mod t for t < 2^32, any acc < 2^64, in float64: k = rint(acc / t)
  // from the two words (|acc/t - k| <= 1/2 + 2^-18), then acc - k t exactly as
  // fma(-k, t, hi 2^32) + lo (every intermediate an integer below 2^53), in
  // [-t/2 - 1, t/2 + 1], and one correction into [0, t).  (The high word goes
  // through an opaque register: converting (u32)(acc >> 32) directly left an
  // add of 0.0 * 2^32 behind.)
  u32 hw = (u32)(acc >> 32);
  asm volatile("" : "+v"(hw));
  const double ah = (double)hw, al = (double)(u32)acc;
  const double k = __builtin_rint(__builtin_fma(ah, R->tinv32, al * R->tinv));
  double r = __builtin_fma(-k, R->qd, ah * 0x1p32) + al;
  r = r < 0.0 ? r + R->qd : r;
  return (u64)(u32)r;
}
// hi 2^60 + mid 2^30 + lo as a 128-bit H:L
__device__ __forceinline__ void bext_fold(u64 lo, u64 mid, u64 hi, u64& H, u64& L) {
  const u64 ml = mid << 30, hl = hi << 60;
  const u64 L1 = lo + ml;
  L = L1 + hl;
  H = (mid >> 34) + (hi >> 4) + (L1 < ml) + (L < hl);
}
// BEXT_WT: y_i < 2^32, qh_i = h2 2^60 + h1 2^30 + h0 (host pieces)
template <int MS>
__device__ __forceinline__ u64 bext_wt(const BextTarget* __restrict__ R, int ns, const u64* y, u64 v) {
  const u32 vv = (u32)v;
  u64 lo = (u64)vv * R->n0, mid = (u64)vv * R->n1, hi = (u64)vv * R->n2;
#pragma unroll
  for (int i = 0; i < MS; ++i) {
    if (i >= ns) break;
    u32 yy = (u32)y[i];
    asm volatile("" : "+v"(yy));  // (kept in the target loop, as in bext_nt)
    lo += (u64)yy * R->h0[i];
    mid += (u64)yy * R->h1[i];
    hi += (u64)yy * R->h2[i];
  }
  u64 H, L;
  bext_fold(lo, mid, hi, H, L);
  // Barrett of x < 4 t^2 (barrett_4q2 with the record's constants)
  const int k = R->k;
  const u64 q = R->q;
  const u64 t1 = (L >> (k - 1)) | (H << (65 - k));
  const u64 ph = mulhi64(t1, R->mu2), pl = t1 * R->mu2;
  const u64 t2 = (k < 61 ? pl >> (k + 3) : 0) | (ph << (61 - k));
  u64 r = L - t2 * q;
  r = r >= q ? r - q : r;
  return r >= q ? r - q : r;
}
// BEXT_NT: t < 2^31, y_i = y2 2^60 + y1 2^30 + y0 cut here
template <int MS>
__device__ __forceinline__ u64 bext_nt(const BextTarget* __restrict__ R, int ns, const u64* y, u64 v) {
  u64 lo = (u64)(u32)v * (u32)R->nS, mid = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < MS; ++i) {
    if (i >= ns) break;
    const u32 h = (u32)R->qh[i];
    // the pieces are cut per target: hoisted out of the target loop they hold
    // 3 x ns VGPRs per coefficient, and the kernels dropped to 2 waves per SIMD
    u64 yy = y[i];
    asm volatile("" : "+v"(yy));
    lo += (u64)((u32)yy & 0x3fffffffu) * h;
    mid += (u64)((u32)(yy >> 30) & 0x3fffffffu) * h;
    hi += (u64)(u32)(yy >> 60) * h;
  }
  u64 H, L;
  bext_fold(lo, mid, hi, H, L);
  // x = H 2^64 + L, H < 2^32: (H (2^64 mod t) + (L mod t)) < 2^63, reduced again
  return bext_narrow_red(H * R->c64 + bext_narrow_red(L, R), R);
}
template <int MS>
__device__ __forceinline__ u64 bext_target_sel(const BextTarget* __restrict__ R, int ns, const u64* y, u64 v) {
  const int mode = R->mode;  // wave-uniform
  if (mode == BEXT_NARROW) {  // sources and target < 2^32 (ResNet's 30-bit chains)
    // the whole sum in one u64: one 32x32 -> 64 multiply-add per term
    u64 acc = (u64)(u32)v * (u32)R->nS;
#pragma unroll
    for (int i = 0; i < MS; ++i) {
      if (i >= ns) break;
      acc += (u64)(u32)y[i] * (u32)R->qh[i];
    }
    return bext_narrow_red(acc, R);
  }
  if constexpr (MS > 2) {
    if (mode == BEXT_WT) return bext_wt<MS>(R, ns, y, v);
    if (mode == BEXT_NT) return bext_nt<MS>(R, ns, y, v);
  }
  // lazy: each Shoup product is in [0, 2q) and the running sum is kept in
  // [0, 2q) by one conditional subtraction (4q < 2^63 for q < 2^61)
  const u64 q = R->q, q2 = q << 1, nq = 0 - q;
  u64 acc;
  if constexpr (MS <= 2) {
    acc = R->vS[0];
    acc = v == 1 ? R->vS[1] : acc;
    acc = v == 2 ? R->vS[2] : acc;
  } else {
    acc = shoup_lazy_nq((u32)v, R->nS, R->nSs, nq);  // (v <= ns: the high words fold away)
  }
#pragma unroll
  for (int i = 0; i < MS; ++i) {
    if (i >= ns) break;
    acc += shoup_lazy_nq(y[i], R->qh[i], R->qhs[i], nq);
    acc = acc >= q2 ? acc - q2 : acc;
  }
  return acc >= q ? acc - q : acc;
}
// the same for two coefficients at once (basis_ext_kernel, modup_all_kernel):
// one pass over the target's constants and one branch for both
template <int MS>
__device__ __forceinline__ void bext_target2(const BextTarget* __restrict__ R, int ns, const u64* y0, u64 v0,
                                             const u64* y1, u64 v1, u64& o0, u64& o1) {
  const int mode = R->mode;
  if (mode == BEXT_NARROW) {
    const u32 s = (u32)R->nS;
    u64 a0 = (u64)(u32)v0 * s, a1 = (u64)(u32)v1 * s;
#pragma unroll
    for (int i = 0; i < MS; ++i) {
      if (i >= ns) break;
      const u32 h = (u32)R->qh[i];
      a0 += (u64)(u32)y0[i] * h;
      a1 += (u64)(u32)y1[i] * h;
    }
    o0 = bext_narrow_red(a0, R);
    o1 = bext_narrow_red(a1, R);
    return;
  }
  if constexpr (MS > 2) {
    if (mode == BEXT_WT) {
      o0 = bext_wt<MS>(R, ns, y0, v0);
      o1 = bext_wt<MS>(R, ns, y1, v1);
      return;
    }
    if (mode == BEXT_NT) {
      o0 = bext_nt<MS>(R, ns, y0, v0);
      o1 = bext_nt<MS>(R, ns, y1, v1);
      return;
    }
  }
  const u64 q = R->q, q2 = q << 1, nq = 0 - q;
  u64 a0, a1;
  if constexpr (MS <= 2) {
    const u64 s1 = R->vS[1], s2 = R->vS[2];
    a0 = v0 == 1 ? s1 : v0 == 2 ? s2 : R->vS[0];
    a1 = v1 == 1 ? s1 : v1 == 2 ? s2 : R->vS[0];
  } else {
    a0 = shoup_lazy_nq((u32)v0, R->nS, R->nSs, nq);
    a1 = shoup_lazy_nq((u32)v1, R->nS, R->nSs, nq);
  }
#pragma unroll
  for (int i = 0; i < MS; ++i) {
    if (i >= ns) break;
    const u64 h = R->qh[i], hs = R->qhs[i];
    a0 += shoup_lazy_nq(y0[i], h, hs, nq);
    a1 += shoup_lazy_nq(y1[i], h, hs, nq);
    a0 = a0 >= q2 ? a0 - q2 : a0;
    a1 = a1 >= q2 ? a1 - q2 : a1;
  }
  o0 = a0 >= q ? a0 - q : a0;
  o1 = a1 >= q ? a1 - q : a1;
}
// A load through the constant address space: with a wave-uniform address it
// is a scalar (SMEM) load into SGPRs, issued where it is written
template <class T>
__device__ __forceinline__ T cload(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
}
// The constants of an extension of at most 2 sources to one target, for a
// kernel that forms several coefficients late in its run (the fused INTT
// columns + forward kernel, ntt2s_ifwd_cols_p): loaded once, at the start,
// through the scalar cache -- read where bext_prep / bext_target_sel read
// them, the table fields were a chain of dependent vector loads per
// coefficient after the INTT half.  bext2_apply is their arithmetic, bit for
// bit (bext_prep<2> then bext_target_sel<2>: the centered, BEXT_NARROW and
// BEXT_LAZY cases).
struct Bext2 {
  u64 chalf, sq[2], qhi[2], qhis[2];
  double qinv_f[2], qf[2];
  u64 q, vS0, vS1, vS2, qh[2], qhs[2], nS;
  double tinv, tinv32, qd;
  int centered, ns, mode;
};
__device__ __forceinline__ Bext2 bext2_load(const BasisExtTable* T, int ti) {  // T, ti wave-uniform
  Bext2 c;
  c.centered = cload(&T->centered);
  c.ns = cload(&T->ns);
  c.chalf = cload(&T->chalf);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    c.sq[i] = cload(&T->sq[i]);
    c.qhi[i] = cload(&T->qhatinv[i]);
    c.qhis[i] = cload(&T->qhatinv_s[i]);
    c.qinv_f[i] = cload(&T->qinv_f[i]);
    c.qf[i] = cload(&T->qf[i]);
  }
  const BextTarget* R = T->tgt + ti;
  c.mode = cload(&R->mode);
  c.q = cload(&R->q);
  c.vS0 = cload(&R->vS[0]);
  c.vS1 = cload(&R->vS[1]);
  c.vS2 = cload(&R->vS[2]);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    c.qh[i] = cload(&R->qh[i]);
    c.qhs[i] = cload(&R->qhs[i]);
  }
  c.nS = cload(&R->nS);
  c.tinv = cload(&R->tinv);
  c.tinv32 = cload(&R->tinv32);
  c.qd = cload(&R->qd);
  return c;
}
// source side, source i (not centered): y_i = x_i qhatinv_i mod s_i and its
// term of the float quotient
__device__ __forceinline__ u64 bext2_src(const Bext2& c, int i, u64 x, double& f) {
  const u64 y = shoup_mul(x, c.qhi[i], c.qhis[i], c.sq[i]);
  const double yd = (double)y, rc = c.qinv_f[i];
  const double q0 = __dmul_rn(yd, rc);
  const double r = __builtin_fma(-q0, c.qf[i], yd);
  f = __builtin_fma(r, rc, q0);
  return y;
}
// v from the sources' float terms (summed in source order) or the centered test
__device__ __forceinline__ u64 bext2_v(const Bext2& c, u64 y0, double f0, double f1) {
  if (c.centered) return y0 >= c.chalf ? 1 : 0;
  double vf = __dadd_rn(0.0, f0);
  if (c.ns > 1) vf = __dadd_rn(vf, f1);
  return (u64)vf;
}
// target side: sum_i y_i (S/s_i mod t) - v S mod t
__device__ __forceinline__ u64 bext2_tgt(const Bext2& c, u64 y0, u64 y1, u64 v) {
  const u64 y[2] = {y0, y1};
  if (c.mode == BEXT_NARROW) {  // bext_target_sel's narrow sum and bext_narrow_red
    u64 acc = (u64)(u32)v * (u32)c.nS;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i >= c.ns) break;
      acc += (u64)(u32)y[i] * (u32)c.qh[i];
    }
    u32 hw = (u32)(acc >> 32);
    asm volatile("" : "+v"(hw));
    const double ah = (double)hw, al = (double)(u32)acc;
    const double k = __builtin_rint(__builtin_fma(ah, c.tinv32, al * c.tinv));
    double r = __builtin_fma(-k, c.qd, ah * 0x1p32) + al;
    r = r < 0.0 ? r + c.qd : r;
    return (u64)(u32)r;
  }
  const u64 q = c.q, q2 = q << 1, nq = 0 - q;
  // v in {0, 1, 2} selects vS_v, by masks: as selects between the fields the
  // compiler made one load from a selected address, which put the struct in scratch
  const u64 m1 = 0 - (u64)(v == 1), m2 = 0 - (u64)(v == 2);
  u64 acc = (c.vS0 & ~(m1 | m2)) | (c.vS1 & m1) | (c.vS2 & m2);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (i >= c.ns) break;
    acc += shoup_lazy_nq(y[i], c.qh[i], c.qhs[i], nq);
    acc = acc >= q2 ? acc - q2 : acc;
  }
  return acc >= q ? acc - q : acc;
}
__device__ __forceinline__ u64 bext2_apply(const Bext2& c, u64 x0, u64 x1) {
  if (c.centered) return bext2_tgt(c, x0, 0, bext2_v(c, x0, 0.0, 0.0));
  double f0 = 0.0, f1 = 0.0;
  const u64 y0 = bext2_src(c, 0, x0, f0);
  const u64 y1 = c.ns > 1 ? bext2_src(c, 1, x1, f1) : 0;
  return bext2_tgt(c, y0, y1, bext2_v(c, y0, f0, f1));
}
// ---------------------------------------------------------------------------
// NTT launch descriptor: transform + fused producer (prologue) / consumer
// (epilogue).  Job j = (c, l, b) over dst's (ncomp, nlimb, nbatch); the limb's
// modulus is dst.mod[l].
//   prologue NTT_PRO_LOAD:    load row (c, l, b) of src (src == dst: in place)
//            NTT_PRO_RESCALE: ((x + h) mod q_L) mod q_l - (h mod q_l), x = row (c, 0, b) of src
//            NTT_PRO_BEXT:    the exact basis extension of the sources to dst limb l,
//                             formed in registers (ModUp of a gadget digit, or
//                             ModDown's extension of the P limbs): table bx + bx_tab[l],
//                             target bx_t[l], sources = src rows (c, bx_s0[table] + i, b),
//                             coefficient domain -- bit-identical to basis_ext_kernel
//   epilogue NTT_EPI_STORE:   store to row (c, l, b) of dst
//            NTT_EPI_SUBSCALE (forward only): dst = (ex - y) * s_l, ex row (c, l, b)
//            NTT_EPI_SUBSCALE_AUT: the same, element e stored at position aut[e]
//            NTT_EPI_SUBSCALE_AUT_ACC: ... added to the word at aut[e]
// ---------------------------------------------------------------------------
enum { NTT_PRO_LOAD = 0, NTT_PRO_RESCALE = 2, NTT_PRO_BEXT = 3 };
// NTT_EPI_SUBSCALE_AUT: the subtract-and-scale epilogue storing element e at
// position aut[e] -- the NTT-domain automorphism of a rotation (its scatter
// index, the gather index of the inverse Galois element) applied in the
// ModDown's store instead of by a separate automorph launch
// NTT_EPI_SUBSCALE_AUT_ACC: the same, added to the word already at aut[e] (a
// rotation whose result is added to its own input, x += sigma_g(x))
enum { NTT_EPI_STORE = 0, NTT_EPI_SUBSCALE = 1, NTT_EPI_SUBSCALE_AUT = 2, NTT_EPI_SUBSCALE_AUT_ACC = 3 };
__host__ __device__ constexpr bool epi_aut(int epi) { return epi == NTT_EPI_SUBSCALE_AUT || epi == NTT_EPI_SUBSCALE_AUT_ACC; }
// 1: the latency kernels (ntt2s.hip) run in radix-4 form
#ifndef NTT2S_R4
#define NTT2S_R4 1
#endif
struct NttIO {
  LimbSet dst, src, ex;
  LimbSet mid;  // two-pass N = 2^15 kernels: intermediate between the passes (dst's geometry)
  int modL;
  int order;    // job decode: 0 = image fastest, 1 = limb fastest (mixes moduli inside a dispatch wave),
                // 2 = image fastest, then component, limbs in the order lord[] (slow integer-path limbs first)
  int jobs;     // ncomp * nlimb * nbatch of dst
  int pro, epi;
  int stagger;  // persistent kernels: s_sleep(127) iterations before the first job of every other CU (timing switch)
  int ci;       // ConjugateInvariant ring: the forward folds its input, the inverse unfolds its output (ModConst::ciw)
  // two-pass kernels, chunked: this launch covers jobs [job0, job0 + njob) and
  // mid is a compact scratch of njob rows (row = job - job0), reused by every
  // chunk so the intermediate can stay in the Infinity Cache
  int job0, njob, mid_compact;
  int grid;  // one-pass persistent launch: workgroups (0 = one per CU), e.g. a CU-masked co-split share
  u64 s[ORION_MAXLIMB], ss[ORION_MAXLIMB];
  unsigned char lord[ORION_MAXLIMB];  // order 2: dispatch order of dst's limbs
  // NTT_PRO_BEXT: the basis-extension tables, and per dst limb its table and
  // target index, per table its first source limb in src
  const BasisExtTable* bx;
  unsigned char bx_tab[ORION_MAXLIMB], bx_t[ORION_MAXLIMB], bx_s0[ORION_MAXLIMB];
  // ifuse (ntt2s.hip, forward launches with the BEXT / RESCALE prologue): the
  // source limbs of src have been through the inverse's rows pass only, whose
  // intermediate sits in imid (src's geometry); the forward columns pass runs
  // their inverse columns pass itself, in registers and LDS
  int ifuse;
  LimbSet imid;
  // ifuse, radix-4, tgroup = G > 1 (ntt2s_ifwd_cols_p): a workgroup of G x 256
  // threads per (component, image) row, target segment and column tile; the
  // ntg segments (consecutive target limbs that read the same source limbs)
  // start at limb tg_l0[k] and hold tg_n[k] <= G targets
  int tgroup, ntg;
  unsigned char tg_l0[ORION_MAXLIMB], tg_n[ORION_MAXLIMB];
  // forward latency launch (ntt2s): the columns pass alone -- the rows pass
  // runs in the consumer (the key switch's gadget product, MacGroups.fwd_rows)
  int cols_only;
  const u32* aut;  // NTT_EPI_SUBSCALE_AUT: the scatter index (N entries)
};

// ---------------------------------------------------------------------------
// operands of moduli below 2^48 split at bit 24 and kept as (lo 24 bits | hi
// part << 32) (lt_bsgs's diagonal copies); the partial sums of split products
// are folded by macs_reduce.
// ---------------------------------------------------------------------------
__device__ __forceinline__ u64 split24(u64 x) { return (x & 0xffffffull) | ((x >> 24) << 32); }
// operands of 48..60-bit moduli split at bit 30, kept as (lo 30 bits | hi 30
// bits << 32) (lt_bsgs's diagonal copies): the four 30 x 30-bit piece products
// accumulate without carries -- 8 products keep lo and hi below 2^63 and the
// 16 mid terms below 2^64 -- one v_mad_u64_u32 each
__device__ __forceinline__ u64 split30(u64 x) { return (x & 0x3fffffffull) | ((x >> 30) << 32); }
struct MacW {
  u64 lo, mid, hi;
};
__device__ __forceinline__ void macw_zero(MacW& a) { a.lo = a.mid = a.hi = 0; }
// x = xa 2^30 + xb, y = ya 2^30 + yb
__device__ __forceinline__ void macw_add(MacW& a, u32 xb, u32 xa, u32 yb, u32 ya) {
  a.lo += (u64)xb * yb;
  a.mid += (u64)xb * ya;
  a.mid += (u64)xa * yb;
  a.hi += (u64)xa * ya;
}
// up to 8 products of operands below q <= 2^60: x = hi 2^60 + mid 2^30 + lo
// < 8 q^2, folded into 128 bits and Barrett-reduced
__device__ __forceinline__ u64 macw_reduce8(const MacW& a, const ModConst& m) {
  const u64 ml = a.mid << 30, hl = a.hi << 60;
  const u64 L1 = a.lo + ml;
  const u64 L = L1 + hl;
  const u64 H = (a.mid >> 34) + (a.hi >> 4) + (L1 < ml) + (L < hl);
  return barrett_8q2(H, L, m);
}
struct MacS {
  u64 lo, mid, hi;
};
// x = hi 2^48 + mid 2^24 + lo  (< 128 q^2)  ->  x mod q
__device__ __forceinline__ u64 macs_reduce(const MacS& a, const ModConst& m) {
  const u64 L1 = a.lo + (a.mid << 24);
  const u64 L2 = L1 + (a.hi << 48);
  const u64 H = (a.mid >> 40) + (a.hi >> 16) + (L1 < a.lo) + (L2 < L1);
  return barrett_256q2(H, L2, m);
}

// ---------------------------------------------------------------------------
// the same split products in float64 (moduli below 2^48): the 24-bit pieces
// convert to doubles exactly, each piece product is below 2^48 and the sums
// of up to 16 operand pairs stay below 2^53, so every FMA is exact.  FP64 FMA
// issues at full rate, the 32-bit integer multiplies at quarter rate.
// ---------------------------------------------------------------------------
struct MacD {
  double lo, mid, hi;
};
__device__ __forceinline__ void macd_zero(MacD& a) { a.lo = a.mid = a.hi = 0.0; }
// x = xa 2^24 + xb, y = ya 2^24 + yb
__device__ __forceinline__ void macd_add(MacD& a, double xb, double xa, double yb, double ya) {
  a.lo = __builtin_fma(xb, yb, a.lo);
  a.mid = __builtin_fma(xa, yb, a.mid);
  a.mid = __builtin_fma(xb, ya, a.mid);
  a.hi = __builtin_fma(xa, ya, a.hi);
}
// exact integer double in [0, 2^53) -> u64
__device__ __forceinline__ u64 d53_to_u64(double d) {
  const double h = __builtin_floor(d * 0x1p-32);
  const double l = __builtin_fma(-h, 0x1p32, d);
  return ((u64)(u32)h << 32) | (u32)l;
}
#ifndef LT_F64_RED
#define LT_F64_RED 1
#endif
// a representative of x mod q for an exact integer double x (below 2^53, or a
// reduced value times a power of two as below): x - rint(x RN(1/q)) q.  The
// estimate x RN(1/q) is within (x/q) 2^-51 of x/q, so the exact remainder is
// below q (1/2 + (x/q) 2^-51) in magnitude -- a small integer the FMA forms
// without rounding
__device__ __forceinline__ double f64_rem(double x, double q, double qi) {
  return __builtin_fma(-__builtin_rint(x * qi), q, x);
}
__device__ __forceinline__ u64 macd_reduce(const MacD& a, const ModConst& m) {
  if (LT_F64_RED) {
    // x = hi 2^48 + mid 2^24 + lo reduced in float64: each piece (< 2^53) to
    // |r| < 2.5 q, the two high ones scaled by their power of two (exact) and
    // reduced again (r 2^48 / q < 2^50: the estimate is within 1/2 of the
    // real quotient, |r| < q), the three summed exactly (< 2^51), reduced to
    // |s| <= q/2 + 1 and brought to [0, q)
    const double q = m.qd, qi = m.qinv_d;
    const double rl = f64_rem(a.lo, q, qi);
    const double rm = f64_rem(f64_rem(a.mid, q, qi) * 0x1p24, q, qi);
    const double rh = f64_rem(f64_rem(a.hi, q, qi) * 0x1p48, q, qi);
    double s = f64_rem((rl + rm) + rh, q, qi);
    s = s < 0.0 ? s + q : s;
    return d53_to_u64(s);
  }
  MacS s;
  s.lo = d53_to_u64(a.lo);
  s.mid = d53_to_u64(a.mid);
  s.hi = d53_to_u64(a.hi);
  return macs_reduce(s, m);
}

// ---------------------------------------------------------------------------
// encryption sampler (encoder.hip): ChaCha20 key, encryption index, and the
// cumulative table of the discrete Gaussian (sigma 3.2, |e| <= BOUND):
// e = -BOUND + #{t : x >= cdt[t]} for a uniform 64-bit x
// ---------------------------------------------------------------------------
#define ORION_GAUSS_BOUND 19
#define ORION_ENC_DOMAIN 0x454e0000u  // 'EN': nonce word 2 of encryption streams
struct EncSampler {
  u32 key[8];
  u32 enc;
  u32 pad;
  u64 cdt[2 * ORION_GAUSS_BOUND];
};
