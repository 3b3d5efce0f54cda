// kernels.hip -- coefficient-wise, rescale, basis-extension, key-switch MAC
// and automorphism kernels for the gfx950 RNS-CKKS backend.
//
// Every kernel here is HBM-bound integer work (no MFMA).  Grid shape: x covers
// the N coefficients of one limb (2 coefficients per thread, 16-B accesses),
// y covers the (comp, limb, image) rows.  Operands that are shared by the
// whole batch (plaintexts, LT diagonals, evaluation keys) are passed with
// batch_stride = 0 and are read once per row from L2.
#include "common.h"

namespace {

__device__ __forceinline__ long long row_off(const LimbSet& s, int c, int l, int b) {
  return c * s.comp_stride + s.pos[l] * s.limb_stride + b * s.batch_stride;
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
  const int n = (blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (n >= N) return;
  const ModConst mc = tb->mc[o.mod[l]];
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
  const int n = (blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (n >= N) return;
  const ModConst mc = tb->mc[d.mod[l]];
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

// rescale step 1 (DivRoundByLastModulusNTT): from the INTT'ed last limb x_L
// (coefficient domain, rows of src = images), t_i = ((x_L + h) mod q_L) mod q_i - (h mod q_i)
__global__ void __launch_bounds__(256) rescale_prep_kernel(LimbSet dst, const u64* __restrict__ src,
                                                           long long src_comp_stride, long long src_batch_stride,
                                                           int modL, const DeviceTables* __restrict__ tb, int N) {
  const int row = blockIdx.y;
  const int bi = row % dst.nbatch;
  const int r = row / dst.nbatch;
  const int l = r % dst.nlimb;
  const int c = r / dst.nlimb;
  const int n = (blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (n >= N) return;
  const u64 qL = tb->mc[modL].q;
  const u64 h = qL >> 1;
  const ModConst mc = tb->mc[dst.mod[l]];
  const u64 hm = barrett128(0, h, mc);
  const ulonglong2 x = *(const ulonglong2*)(src + c * src_comp_stride + bi * src_batch_stride + n);
  ulonglong2 z;
  z.x = sub_mod(barrett128(0, add_mod(x.x, h, qL), mc), hm, mc.q);
  z.y = sub_mod(barrett128(0, add_mod(x.y, h, qL), mc), hm, mc.q);
  *(ulonglong2*)(dst.p + row_off(dst, c, l, bi) + n) = z;
}

// Exact basis extension (Lattigo ModUpExact restated).
// in: ns source limbs (coefficient domain), out: nt target limbs.
// The float64 quotient is accumulated in source order with explicit
// round-to-nearest multiply and add (no FMA contraction) so that it matches
// the CPU restatement bit for bit.
__global__ void __launch_bounds__(256) basis_ext_kernel(LimbSet out, LimbSet in, const BasisExtTable* __restrict__ T,
                                                        const DeviceTables* __restrict__ tb, int N) {
  const int row = blockIdx.y;  // (comp, image)
  const int bi = row % out.nbatch;
  const int c = row / out.nbatch;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int ns = T->ns, nt = T->nt;
  u64 y[ORION_MAXSRC];
  double vf = 0.0;
  for (int i = 0; i < ns; ++i) {
    const u64 si = tb->mc[T->src_mod[i]].q;
    u64 x = in.p[row_off(in, c, i, bi) + n];
    y[i] = shoup_mul(x, T->qhatinv[i], T->qhatinv_s[i], si);
    vf = __dadd_rn(vf, __dmul_rn((double)y[i], T->qinv_f[i]));
  }
  const u64 v = (u64)vf;
  // out_t = sum_i y_i * (S/s_i mod t) - v*S  (mod t); y_i < s_i may exceed t, the
  // Shoup product accepts any 64-bit multiplicand and returns [0, 2t)
  for (int t = 0; t < nt; ++t) {
    const u64 q = tb->mc[T->dst_mod[t]].q;
    u64 acc = T->vS_t[t][v];
    for (int i = 0; i < ns; ++i) {
      u64 r = shoup_lazy(y[i], T->qhat_t[t][i], T->qhat_ts[t][i], q);
      r = r >= q ? r - q : r;
      acc = add_mod(acc, r, q);
    }
    out.p[row_off(out, c, t, bi) + n] = acc;
  }
}

// Gadget-product MAC: out_c[j] = sum_i D_i[j] * key[i][c][mod_j]  (c = 0, 1)
// D: comps = digits, limbs = QP positions.  key layout [dnum][2][L+K][N].
__global__ void __launch_bounds__(256) ks_mac_kernel(LimbSet out, LimbSet D, const u64* __restrict__ key,
                                                     int beta, int nmod_key, const DeviceTables* __restrict__ tb,
                                                     int N, int accumulate) {
  const int row = blockIdx.y;
  const int bi = row % out.nbatch;
  const int l = row / out.nbatch;
  const int n = (blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (n >= N) return;
  const int m = out.mod[l];
  const ModConst mc = tb->mc[m];
  const u64 q = mc.q;
  ulonglong2 r0 = make_ulonglong2(0, 0), r1 = make_ulonglong2(0, 0);
  if (accumulate) {
    r0 = *(const ulonglong2*)(out.p + row_off(out, 0, l, bi) + n);
    r1 = *(const ulonglong2*)(out.p + row_off(out, 1, l, bi) + n);
  }
  // d, key < q: each product < q^2; sum 4 of them in 128 bits, reduce once
  Acc128 s0x = {0, 0}, s0y = {0, 0}, s1x = {0, 0}, s1y = {0, 0};
  for (int i = 0; i < beta; ++i) {
    const ulonglong2 d = *(const ulonglong2*)(D.p + row_off(D, i, l, bi) + n);
    const u64* kb = key + ((long long)(i * 2 + 0) * nmod_key + m) * N + n;
    const u64* ka = key + ((long long)(i * 2 + 1) * nmod_key + m) * N + n;
    const ulonglong2 b = *(const ulonglong2*)kb;
    const ulonglong2 a = *(const ulonglong2*)ka;
    mac128(s0x, d.x, b.x);
    mac128(s0y, d.y, b.y);
    mac128(s1x, d.x, a.x);
    mac128(s1y, d.y, a.y);
    if ((i & 3) == 3 || i == beta - 1) {
      r0.x = add_mod(r0.x, barrett128_4(s0x.hi, s0x.lo, mc), q);
      r0.y = add_mod(r0.y, barrett128_4(s0y.hi, s0y.lo, mc), q);
      r1.x = add_mod(r1.x, barrett128_4(s1x.hi, s1x.lo, mc), q);
      r1.y = add_mod(r1.y, barrett128_4(s1y.hi, s1y.lo, mc), q);
      s0x = s0y = s1x = s1y = Acc128{0, 0};
    }
  }
  *(ulonglong2*)(out.p + row_off(out, 0, l, bi) + n) = r0;
  *(ulonglong2*)(out.p + row_off(out, 1, l, bi) + n) = r1;
}

// NTT-domain automorphism: o[j] = a[idx[j]]  (optionally o += a[idx[j]])
__global__ void __launch_bounds__(256) automorph_kernel(LimbSet o, LimbSet a, const u32* __restrict__ idx,
                                                        const DeviceTables* __restrict__ tb, int N, int accumulate) {
  const int row = blockIdx.y;
  const int bi = row % o.nbatch;
  const int r = row / o.nbatch;
  const int l = r % o.nlimb;
  const int c = r / o.nlimb;
  const int n = (blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (n >= N) return;
  const u64 q = tb->mc[o.mod[l]].q;
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

// BSGS giant-step MAC (lintrans MultiplyByDiagMatrixBSGS inner loop, fused):
//   t[c][l][b] = sum_i pt_i[l] * rot_i[c][l][b]   for c = 0, 1
// rot_i share t's layout; pt_i is one limb plane per QP position (pt_pos[l]).
// Grid: x = image (fastest, so the blocks that reuse a pt chunk run together),
// y = coefficient chunk, z = limb.  Products are summed in 128 bits and
// reduced once per 4 terms.
struct LtMacArgs {
  const u64* rot[ORION_MAXBABY];
  const u64* pt[ORION_MAXBABY];
};
__global__ void __launch_bounds__(256) lt_mac_kernel(LimbSet t, LtMacArgs A, int m, const unsigned char* __restrict__ pt_pos_unused,
                                                     LimbSet ptl, const DeviceTables* __restrict__ tb, int N) {
  const int bi = blockIdx.x;
  const int n = (blockIdx.y * blockDim.x + threadIdx.x) * 2;
  const int l = blockIdx.z;
  if (n >= N) return;
  const ModConst mc = tb->mc[t.mod[l]];
  const long long ro0 = row_off(t, 0, l, bi) + n, ro1 = row_off(t, 1, l, bi) + n;
  const long long po = (long long)ptl.pos[l] * ptl.limb_stride + n;
  Acc128 a0x = {0, 0}, a0y = {0, 0}, a1x = {0, 0}, a1y = {0, 0};
  u64 r0x = 0, r0y = 0, r1x = 0, r1y = 0;
  for (int i = 0; i < m; ++i) {
    const ulonglong2 p = *(const ulonglong2*)(A.pt[i] + po);
    const ulonglong2 x0 = *(const ulonglong2*)(A.rot[i] + ro0);
    const ulonglong2 x1 = *(const ulonglong2*)(A.rot[i] + ro1);
    mac128(a0x, p.x, x0.x);
    mac128(a0y, p.y, x0.y);
    mac128(a1x, p.x, x1.x);
    mac128(a1y, p.y, x1.y);
    if ((i & 3) == 3 || i == m - 1) {
      r0x = add_mod(r0x, barrett128_4(a0x.hi, a0x.lo, mc), mc.q);
      r0y = add_mod(r0y, barrett128_4(a0y.hi, a0y.lo, mc), mc.q);
      r1x = add_mod(r1x, barrett128_4(a1x.hi, a1x.lo, mc), mc.q);
      r1y = add_mod(r1y, barrett128_4(a1y.hi, a1y.lo, mc), mc.q);
      a0x = a0y = a1x = a1y = Acc128{0, 0};
    }
  }
  *(ulonglong2*)(t.p + ro0) = make_ulonglong2(r0x, r0y);
  *(ulonglong2*)(t.p + ro1) = make_ulonglong2(r1x, r1y);
}

inline dim3 ew_grid(int N, int rows) { return dim3((N / 2 + 255) / 256, rows); }

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
    CASE(EW_SUBSCALE) CASE(EW_COPY) CASE(EW_ADDSCALE)
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

int orion_launch_rescale_prep(const LimbSet& dst, const u64* src, long long src_comp_stride,
                              long long src_batch_stride, int modL, const DeviceTables* tb, int N, hipStream_t st) {
  const int rows = dst.ncomp * dst.nlimb * dst.nbatch;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(rescale_prep_kernel, ew_grid(N, rows), dim3(256), 0, st, dst, src, src_comp_stride,
                     src_batch_stride, modL, tb, N);
  return 0;
}

int orion_launch_basis_ext(const LimbSet& out, const LimbSet& in, const BasisExtTable* T, const DeviceTables* tb,
                           int N, hipStream_t st) {
  const int rows = out.ncomp * out.nbatch;
  hipLaunchKernelGGL(basis_ext_kernel, dim3((N + 255) / 256, rows), dim3(256), 0, st, out, in, T, tb, N);
  return 0;
}

int orion_launch_ks_mac(const LimbSet& out, const LimbSet& D, const u64* key, int beta, int nmod_key,
                        const DeviceTables* tb, int N, int accumulate, hipStream_t st) {
  const int rows = out.nlimb * out.nbatch;
  hipLaunchKernelGGL(ks_mac_kernel, ew_grid(N, rows), dim3(256), 0, st, out, D, key, beta, nmod_key, tb, N,
                     accumulate);
  return 0;
}

int orion_launch_lt_mac(const LimbSet& t, const u64* const* rot, const u64* const* pt, int m, const LimbSet& ptl,
                        const DeviceTables* tb, int N, hipStream_t st) {
  if (m < 1 || m > ORION_MAXBABY) return -1;
  LtMacArgs A;
  for (int i = 0; i < m; ++i) {
    A.rot[i] = rot[i];
    A.pt[i] = pt[i];
  }
  dim3 g(t.nbatch, (N / 2 + 255) / 256, t.nlimb);
  hipLaunchKernelGGL(lt_mac_kernel, g, dim3(256), 0, st, t, A, m, (const unsigned char*)nullptr, ptl, tb, N);
  return 0;
}

int orion_launch_automorph(const LimbSet& o, const LimbSet& a, const u32* idx, const DeviceTables* tb, int N,
                           int accumulate, hipStream_t st) {
  const int rows = o.ncomp * o.nlimb * o.nbatch;
  hipLaunchKernelGGL(automorph_kernel, ew_grid(N, rows), dim3(256), 0, st, o, a, idx, tb, N, accumulate);
  return 0;
}
