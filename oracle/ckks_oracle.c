/*
 * ckks_oracle.c -- CPU restatement of Lattigo-v6 RNS-CKKS arithmetic used by
 * Orion's backend (TEST INFRASTRUCTURE: parity oracle + CPU baseline only).
 * See ckks_oracle.h for the scope statement and reference citations.
 * "parity unpinned" w.r.t. Lattigo itself: no golden vectors exist upstream.
 *
 * Built with -O2 -ffp-contract=off so that the float64 quotient inside the
 * exact basis extension and the encoder FFT round exactly as written.
 */
#include "ckks_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;

#define MAXMOD 80

struct oracle_ctx {
  int logN, N, L, K;
  /* ConjugateInvariant ring (scheme.go:49-52): degree N, NthRoot 4N.  Its
   * NTT is the first half of the degree-2N negacyclic NTT of the element's
   * expansion p (p_j = a_j, p_N = 0, p_{2N-j} = -a_j): a fold
   * b_e = a_e - W a_{N-e} (W = psi^N, the 2N NTT's first-stage twiddle),
   * then the 2N NTT's remaining stages on the first half (twiddles
   * fw[m + i] = fw_2N[2m + i]).  The inverse unfolds with
   * a_e = (b_e + W b_{N-e}) / 2. */
  int ci;
  u64 ciw[MAXMOD], ciws[MAXMOD], inv2[MAXMOD];
  u64 mod[MAXMOD];
  u64 psi[MAXMOD];
  u64 *fw[MAXMOD];  /* fw[bitrev(j)] = psi^j            */
  u64 *fws[MAXMOD]; /* Shoup companions floor(w 2^64/q)  */
  u64 *iw[MAXMOD];  /* iw[bitrev(j)] = psi^-j           */
  u64 *iws[MAXMOD];
  u64 ninv[MAXMOD], ninvs[MAXMOD];
};

/* ------------------------------------------------------------------ */
/* modular helpers                                                     */
/* ------------------------------------------------------------------ */
static inline u64 mulmod(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }
static inline u64 addmod(u64 a, u64 b, u64 q) { u64 c = a + b; return c >= q ? c - q : c; }
static inline u64 submod(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }
static u64 powmod(u64 b, u64 e, u64 q) {
  u64 r = 1 % q;
  b %= q;
  while (e) {
    if (e & 1) r = mulmod(r, b, q);
    b = mulmod(b, b, q);
    e >>= 1;
  }
  return r;
}
static u64 invmod(u64 a, u64 q) { return powmod(a % q, q - 2, q); }
static inline u64 shoup(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }
/* Shoup product, result in [0, 2q) for any a < 2^64 */
static inline u64 mul_shoup_lazy(u64 a, u64 w, u64 ws, u64 q) {
  u64 hi = (u64)(((u128)a * ws) >> 64);
  return a * w - hi * q;
}

static u64 bitrev(u64 x, int bits) {
  u64 r = 0;
  for (int i = 0; i < bits; i++) {
    r = (r << 1) | (x & 1);
    x >>= 1;
  }
  return r;
}

/* ------------------------------------------------------------------ */
/* primes (Lattigo GenModuli / NTTFriendlyPrimesGenerator) */
/* ------------------------------------------------------------------ */
static int is_prime_u64(u64 n) {
  if (n < 2) return 0;
  static const u64 small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  for (int i = 0; i < 12; i++) {
    if (n % small[i] == 0) return n == small[i];
  }
  u64 d = n - 1;
  int s = 0;
  while ((d & 1) == 0) {
    d >>= 1;
    s++;
  }
  for (int i = 0; i < 12; i++) {
    u64 x = powmod(small[i], d, n);
    if (x == 1 || x == n - 1) continue;
    int comp = 1;
    for (int r = 1; r < s; r++) {
      x = mulmod(x, x, n);
      if (x == n - 1) {
        comp = 0;
        break;
      }
    }
    if (comp) return 0;
  }
  return 1;
}

typedef struct {
  double size;
  u64 nthroot, next, prev;
  int check_next, check_prev;
} primegen;

static void pg_init(primegen *g, int bitlen, u64 nthroot) {
  g->size = (double)bitlen;
  g->nthroot = nthroot;
  g->next = ((u64)1 << bitlen) + 1;
  g->prev = ((u64)1 << bitlen) + 1;
  g->check_next = g->check_prev = 1;
}

static u64 pg_next_downstream(primegen *g) {
  for (;;) {
    if (g->prev < g->nthroot) return 0;
    g->prev -= g->nthroot;
    if (g->size - log2((double)g->prev) >= 0.5) return 0;
    if (is_prime_u64(g->prev)) return g->prev;
  }
}

static u64 pg_next_alternating(primegen *g) {
  for (;;) {
    if (!(g->check_next || g->check_prev)) return 0;
    if (g->check_next) {
      if (g->next > UINT64_MAX - g->nthroot || log2((double)g->next) - g->size >= 0.5) {
        g->check_next = 0;
      } else {
        g->next += g->nthroot;
        if (is_prime_u64(g->next)) return g->next;
      }
    }
    if (g->check_prev) {
      if (g->prev < g->nthroot || g->size - log2((double)g->prev) >= 0.5) {
        g->check_prev = 0;
      } else {
        g->prev -= g->nthroot;
        if (is_prime_u64(g->prev)) return g->prev;
      }
    }
  }
}

int oracle_gen_moduli(int logN, const int *logQ, int lenQ, const int *logP, int lenP,
                      u64 *out) {
  /* Standard ring: NthRoot = 2N.  Primes of each distinct bit size are drawn
   * in one stream and handed out first to Q (in order), then to P. */
  u64 nthroot = (u64)2 << logN;
  int sizes[MAXMOD], counts[MAXMOD], nsz = 0;
  for (int i = 0; i < lenQ + lenP; i++) {
    int b = i < lenQ ? logQ[i] : logP[i - lenQ];
    int k;
    for (k = 0; k < nsz; k++)
      if (sizes[k] == b) break;
    if (k == nsz) {
      sizes[nsz] = b;
      counts[nsz++] = 0;
    }
    counts[k]++;
  }
  u64 pool[MAXMOD][MAXMOD];
  int used[MAXMOD] = {0};
  for (int k = 0; k < nsz; k++) {
    primegen g;
    pg_init(&g, sizes[k], nthroot);
    for (int c = 0; c < counts[k]; c++) {
      u64 p = sizes[k] == 61 ? pg_next_downstream(&g) : pg_next_alternating(&g);
      if (!p) return -1;
      pool[k][c] = p;
    }
  }
  for (int i = 0; i < lenQ + lenP; i++) {
    int b = i < lenQ ? logQ[i] : logP[i - lenQ];
    int k;
    for (k = 0; k < nsz; k++)
      if (sizes[k] == b) break;
    out[i] = pool[k][used[k]++];
  }
  return 0;
}

/* smallest primitive root, candidates 3, 4, 5, ... (Lattigo PrimitiveRoot:
 * g starts at 2 and is incremented before the first test) */
u64 oracle_primitive_root(u64 q) {
  u64 factors[64];
  int nf = 0;
  u64 m = q - 1;
  for (u64 f = 2; f * f <= m; f += (f == 2 ? 1 : 2)) {
    if (m % f == 0) {
      factors[nf++] = f;
      while (m % f == 0) m /= f;
    }
  }
  if (m > 1) factors[nf++] = m;
  for (u64 g = 3;; g++) {
    int ok = 1;
    for (int i = 0; i < nf; i++) {
      if (powmod(g, (q - 1) / factors[i], q) == 1) {
        ok = 0;
        break;
      }
    }
    if (ok) return g;
  }
}

/* ------------------------------------------------------------------ */
/* context                                                             */
/* ------------------------------------------------------------------ */
oracle_ctx *oracle_new_ring(int logN, const u64 *moduli, int L, int K, int ci) {
  if (L + K > MAXMOD) return NULL;
  oracle_ctx *c = (oracle_ctx *)calloc(1, sizeof(oracle_ctx));
  c->logN = logN;
  c->N = 1 << logN;
  c->L = L;
  c->K = K;
  c->ci = ci ? 1 : 0;
  const int N = c->N, logM = logN + c->ci, M = 1 << logM; /* M: degree of the negacyclic NTT */
  u64 *tf = (u64 *)malloc(sizeof(u64) * M), *ti = (u64 *)malloc(sizeof(u64) * M);
  for (int m = 0; m < L + K; m++) {
    u64 q = moduli[m];
    c->mod[m] = q;
    u64 g = oracle_primitive_root(q);
    u64 psi = powmod(g, (q - 1) / (2 * (u64)M), q); /* primitive 2M-th root (2N, or 4N for CI) */
    u64 psii = invmod(psi, q);
    c->psi[m] = psi;
    c->fw[m] = (u64 *)malloc(sizeof(u64) * N);
    c->fws[m] = (u64 *)malloc(sizeof(u64) * N);
    c->iw[m] = (u64 *)malloc(sizeof(u64) * N);
    c->iws[m] = (u64 *)malloc(sizeof(u64) * N);
    u64 a = 1, b = 1;
    for (int j = 0; j < M; j++) {
      u64 r = bitrev(j, logM);
      tf[r] = a;
      ti[r] = b;
      a = mulmod(a, psi, q);
      b = mulmod(b, psii, q);
    }
    for (int k = 0; k < N; k++) {
      /* CI: the N-point stage with m groups uses the 2N table's entry 2m + i */
      int mm = 1;
      while (2 * mm <= k) mm <<= 1;
      const int src = c->ci ? (k ? k + mm : 0) : k;
      c->fw[m][k] = tf[src];
      c->fws[m][k] = shoup(tf[src], q);
      c->iw[m][k] = ti[src];
      c->iws[m][k] = shoup(ti[src], q);
    }
    c->ninv[m] = invmod((u64)N, q);
    c->ninvs[m] = shoup(c->ninv[m], q);
    if (c->ci) {
      c->ciw[m] = tf[1]; /* psi^N */
      c->ciws[m] = shoup(tf[1], q);
      c->inv2[m] = (q + 1) / 2;
    }
  }
  free(tf);
  free(ti);
  return c;
}
oracle_ctx *oracle_new(int logN, const u64 *moduli, int L, int K) { return oracle_new_ring(logN, moduli, L, K, 0); }
int oracle_is_ci(const oracle_ctx *c) { return c->ci; }

void oracle_free(oracle_ctx *c) {
  if (!c) return;
  for (int m = 0; m < c->L + c->K; m++) {
    free(c->fw[m]);
    free(c->fws[m]);
    free(c->iw[m]);
    free(c->iws[m]);
  }
  free(c);
}

int oracle_N(const oracle_ctx *c) { return c->N; }
u64 oracle_psi(const oracle_ctx *c, int m) { return c->psi[m]; }

/* ------------------------------------------------------------------ */
/* NTT (Cooley-Tukey, natural -> bit-reversed; Harvey lazy butterflies) */
/* ------------------------------------------------------------------ */
void oracle_ntt(const oracle_ctx *c, int mi, u64 *a) {
  const int N = c->N;
  const u64 q = c->mod[mi], q2 = 2 * q;
  const u64 *w = c->fw[mi], *ws = c->fws[mi];
  if (c->ci) { /* fold: b_e = a_e - W a_{N-e}, b_0 = a_0 */
    u64 *b = (u64 *)malloc(sizeof(u64) * N);
    b[0] = a[0];
    for (int e = 1; e < N; e++) b[e] = submod(a[e], mulmod(a[N - e], c->ciw[mi], q), q);
    memcpy(a, b, sizeof(u64) * N);
    free(b);
  }
  int t = N;
  for (int m = 1; m < N; m <<= 1) {
    t >>= 1;
    for (int i = 0; i < m; i++) {
      const u64 W = w[m + i], Ws = ws[m + i];
      u64 *x = a + 2 * i * t, *y = x + t;
      for (int j = 0; j < t; j++) {
        u64 X = x[j];
        if (X >= q2) X -= q2;
        u64 T = mul_shoup_lazy(y[j], W, Ws, q);
        x[j] = X + T;
        y[j] = X - T + q2;
      }
    }
  }
  for (int j = 0; j < N; j++) {
    u64 X = a[j];
    if (X >= q2) X -= q2;
    if (X >= q) X -= q;
    a[j] = X;
  }
}

void oracle_intt(const oracle_ctx *c, int mi, u64 *a) {
  const int N = c->N;
  const u64 q = c->mod[mi], q2 = 2 * q;
  const u64 *w = c->iw[mi], *ws = c->iws[mi];
  int t = 1;
  for (int m = N >> 1; m >= 1; m >>= 1) {
    for (int i = 0; i < m; i++) {
      const u64 W = w[m + i], Ws = ws[m + i];
      u64 *x = a + 2 * i * t, *y = x + t;
      for (int j = 0; j < t; j++) {
        u64 U = x[j], V = y[j];
        u64 S = U + V;
        if (S >= q2) S -= q2;
        x[j] = S;
        y[j] = mul_shoup_lazy(U - V + q2, W, Ws, q);
      }
    }
    t <<= 1;
  }
  for (int j = 0; j < N; j++) {
    u64 X = mul_shoup_lazy(a[j], c->ninv[mi], c->ninvs[mi], q);
    if (X >= q) X -= q;
    a[j] = X;
  }
  if (c->ci) { /* unfold: a_e = (b_e + W b_{N-e}) / 2, a_0 = b_0 */
    u64 *b = (u64 *)malloc(sizeof(u64) * N);
    memcpy(b, a, sizeof(u64) * N);
    for (int e = 1; e < N; e++)
      a[e] = mulmod(addmod(b[e], mulmod(b[N - e], c->ciw[mi], q), q), c->inv2[mi], q);
    free(b);
  }
}

/* ------------------------------------------------------------------ */
/* exact basis extension (Lattigo ModUpExact restated, App. A.5)        */
/*   y_i = x_i * (S/s_i)^-1 mod s_i                                     */
/*   v   = (u64) sum_i (double)y_i / (double)s_i   (source order)       */
/*   out_t = sum_i y_i * (S/s_i mod t) - v * (S mod t)   mod t          */
/* The quotient is Lattigo v6's reconstructRNS (ring/basis_extension.go */
/* [U], lattigo/v6 v6.2.0 per orion/backend/lattigo/go.mod:5):          */
/* `vi += float64(y_i) / float64(Q[i])`, a correctly rounded division   */
/* accumulated in source order, then truncated by uint64(vi).  It is    */
/* not always floor(x / S): near an integer the rounding decides, and   */
/* a reciprocal multiply (y_i * (1/s_i)) can truncate to another v      */
/* (tests/golden/kat_ckks.json "bext_quotient" holds such coefficients).*/
/* centered (DecomposeAndSplit's single-prime digit, decompLvl == -1):  */
/*   x >= s >> 1 is extended as x - s (v = 1), else as x (v = 0).       */
/* ------------------------------------------------------------------ */
static void basis_extend_impl(const oracle_ctx *c, const u64 *x, const int *src, int ns,
                              u64 *out, const int *dst, int nt, int centered) {
  const int N = c->N;
  u64 qhatinv[MAXMOD];
  double qf[MAXMOD];
  u64 qhat_t[MAXMOD][MAXMOD]; /* [t][i] */
  u64 S_t[MAXMOD];
  for (int i = 0; i < ns; i++) {
    u64 si = c->mod[src[i]];
    u64 prod = 1;
    for (int k = 0; k < ns; k++)
      if (k != i) prod = mulmod(prod, c->mod[src[k]] % si, si);
    qhatinv[i] = invmod(prod, si);
    qf[i] = (double)si;
  }
  for (int t = 0; t < nt; t++) {
    u64 tm = c->mod[dst[t]];
    u64 S = 1;
    for (int k = 0; k < ns; k++) S = mulmod(S, c->mod[src[k]] % tm, tm);
    S_t[t] = S;
    for (int i = 0; i < ns; i++) {
      u64 p = 1;
      for (int k = 0; k < ns; k++)
        if (k != i) p = mulmod(p, c->mod[src[k]] % tm, tm);
      qhat_t[t][i] = p;
    }
  }
  u64 y[MAXMOD];
  const u64 half0 = c->mod[src[0]] >> 1;
  for (int n = 0; n < N; n++) {
    u64 v;
    if (centered && ns == 1) {
      y[0] = x[n] % c->mod[src[0]];
      v = y[0] >= half0 ? 1 : 0;
    } else {
      double vf = 0.0;
      for (int i = 0; i < ns; i++) {
        u64 si = c->mod[src[i]];
        y[i] = mulmod(x[(size_t)i * N + n] % si, qhatinv[i], si);
        volatile double quo = (double)y[i] / qf[i];
        vf = vf + quo;
      }
      v = (u64)vf;
    }
    for (int t = 0; t < nt; t++) {
      u64 tm = c->mod[dst[t]];
      u128 acc = 0;
      for (int i = 0; i < ns; i++) acc += (u128)y[i] * qhat_t[t][i];
      u64 r = (u64)(acc % tm);
      u64 vs = mulmod(v % tm, S_t[t], tm);
      out[(size_t)t * N + n] = submod(r, vs, tm);
    }
  }
}

void oracle_basis_extend(const oracle_ctx *c, const u64 *x, const int *src, int ns,
                         u64 *out, const int *dst, int nt) {
  basis_extend_impl(c, x, src, ns, out, dst, nt, 0);
}

/* ModUp of one gadget digit (Lattigo Decomposer.DecomposeAndSplit [U]): a */
/* single-prime digit is extended from its centered representative, a     */
/* wider one by ModUpExact                                                  */
void oracle_modup_digit(const oracle_ctx *c, const u64 *x, const int *src, int ns,
                        u64 *out, const int *dst, int nt) {
  basis_extend_impl(c, x, src, ns, out, dst, nt, 1);
}

/* ------------------------------------------------------------------ */
/* rescale: round(x / q_l)  (DivRoundByLastModulusNTT, App. A.4)        */
/* ------------------------------------------------------------------ */
void oracle_rescale(const oracle_ctx *c, int level, int ncomp, const u64 *ct, u64 *out) {
  const int N = c->N;
  const u64 ql = c->mod[level];
  const u64 half = ql >> 1;
  u64 *last = (u64 *)malloc(sizeof(u64) * N);
  u64 *t = (u64 *)malloc(sizeof(u64) * N);
  for (int comp = 0; comp < ncomp; comp++) {
    const u64 *in = ct + (size_t)comp * (level + 1) * N;
    u64 *o = out + (size_t)comp * level * N;
    memcpy(last, in + (size_t)level * N, sizeof(u64) * N);
    oracle_intt(c, level, last);
    for (int n = 0; n < N; n++) last[n] = addmod(last[n], half, ql);
    for (int i = 0; i < level; i++) {
      u64 qi = c->mod[i];
      u64 hmod = half % qi;
      for (int n = 0; n < N; n++) t[n] = submod(last[n] % qi, hmod, qi);
      oracle_ntt(c, i, t);
      u64 qlinv = invmod(ql % qi, qi);
      for (int n = 0; n < N; n++) o[(size_t)i * N + n] = mulmod(submod(in[(size_t)i * N + n], t[n], qi), qlinv, qi);
    }
  }
  free(last);
  free(t);
}

/* ------------------------------------------------------------------ */
/* ModDown QP -> Q: (x_Q - ext_{P->Q}(x_P)) * P^-1                      */
/* ------------------------------------------------------------------ */
void oracle_moddown(const oracle_ctx *c, int level, const u64 *x, u64 *out) {
  const int N = c->N, L = c->L, K = c->K;
  int src[MAXMOD], dst[MAXMOD];
  u64 *xp = (u64 *)malloc(sizeof(u64) * N * K);
  u64 *ext = (u64 *)malloc(sizeof(u64) * N * (level + 1));
  memcpy(xp, x + (size_t)(level + 1) * N, sizeof(u64) * N * K);
  for (int k = 0; k < K; k++) {
    src[k] = L + k;
    oracle_intt(c, L + k, xp + (size_t)k * N);
  }
  for (int j = 0; j <= level; j++) dst[j] = j;
  oracle_basis_extend(c, xp, src, K, ext, dst, level + 1);
  for (int j = 0; j <= level; j++) {
    u64 qj = c->mod[j];
    oracle_ntt(c, j, ext + (size_t)j * N);
    u64 P = 1;
    for (int k = 0; k < K; k++) P = mulmod(P, c->mod[L + k] % qj, qj);
    u64 pinv = invmod(P, qj);
    for (int n = 0; n < N; n++)
      out[(size_t)j * N + n] = mulmod(submod(x[(size_t)j * N + n], ext[(size_t)j * N + n], qj), pinv, qj);
  }
  free(xp);
  free(ext);
}

/* ------------------------------------------------------------------ */
/* gadget product (hybrid key switching, App. A.5)                      */
/* digit i covers Q limbs [i*K, min((i+1)*K, level+1))                  */
/* ------------------------------------------------------------------ */
void oracle_gadget_product_lazy(const oracle_ctx *c, int level, const u64 *cx,
                                const u64 *evk, u64 *out0, u64 *out1) {
  const int N = c->N, L = c->L, K = c->K;
  const int nqp = level + 1 + K;
  const int dnum_full = (L + K - 1) / K;
  const int beta = (level + 1 + K - 1) / K;
  (void)dnum_full;
  u64 *cinv = (u64 *)malloc(sizeof(u64) * N * (level + 1));
  u64 *d = (u64 *)malloc(sizeof(u64) * N * nqp);
  memcpy(cinv, cx, sizeof(u64) * N * (level + 1));
  for (int j = 0; j <= level; j++) oracle_intt(c, j, cinv + (size_t)j * N);
  memset(out0, 0, sizeof(u64) * N * nqp);
  memset(out1, 0, sizeof(u64) * N * nqp);
  for (int i = 0; i < beta; i++) {
    int lo = i * K, hi = (i + 1) * K;
    if (hi > level + 1) hi = level + 1;
    int src[MAXMOD], dst[MAXMOD], pos[MAXMOD], nt = 0;
    for (int j = lo; j < hi; j++) src[j - lo] = j;
    for (int j = 0; j < nqp; j++) {
      int mi = j <= level ? j : L + (j - level - 1);
      if (j >= lo && j < hi) continue;
      dst[nt] = mi;
      pos[nt++] = j;
    }
    u64 *ext = (u64 *)malloc(sizeof(u64) * N * (nt ? nt : 1));
    oracle_modup_digit(c, cinv + (size_t)lo * N, src, hi - lo, ext, dst, nt);
    for (int t = 0; t < nt; t++) {
      oracle_ntt(c, dst[t], ext + (size_t)t * N);
      memcpy(d + (size_t)pos[t] * N, ext + (size_t)t * N, sizeof(u64) * N);
    }
    for (int j = lo; j < hi; j++) memcpy(d + (size_t)j * N, cx + (size_t)j * N, sizeof(u64) * N);
    free(ext);
    /* MAC with key digit i: key limb index for QP position j */
    const u64 *b = evk + (size_t)i * 2 * (L + K) * N;
    const u64 *a = b + (size_t)(L + K) * N;
    for (int j = 0; j < nqp; j++) {
      int mi = j <= level ? j : L + (j - level - 1);
      u64 q = c->mod[mi];
      const u64 *bj = b + (size_t)mi * N, *aj = a + (size_t)mi * N, *dj = d + (size_t)j * N;
      u64 *o0 = out0 + (size_t)j * N, *o1 = out1 + (size_t)j * N;
      for (int n = 0; n < N; n++) {
        o0[n] = addmod(o0[n], mulmod(dj[n], bj[n], q), q);
        o1[n] = addmod(o1[n], mulmod(dj[n], aj[n], q), q);
      }
    }
  }
  free(cinv);
  free(d);
}

void oracle_keyswitch(const oracle_ctx *c, int level, const u64 *cx, const u64 *evk,
                      u64 *out0, u64 *out1) {
  const int N = c->N, K = c->K;
  size_t sz = sizeof(u64) * N * (level + 1 + K);
  u64 *t0 = (u64 *)malloc(sz), *t1 = (u64 *)malloc(sz);
  oracle_gadget_product_lazy(c, level, cx, evk, t0, t1);
  oracle_moddown(c, level, t0, out0);
  oracle_moddown(c, level, t1, out1);
  free(t0);
  free(t1);
}

/* ------------------------------------------------------------------ */
/* automorphisms                                                         */
/* ------------------------------------------------------------------ */
uint64_t oracle_galois_element(const oracle_ctx *c, int k) {
  u64 M = (2 * (u64)c->N) << c->ci; /* NthRoot: 2N, or 4N for the CI ring */
  u64 e = (u64)((int64_t)k) & (M - 1);
  return powmod(5, e, M);
}

/* index over the degree-M NTT (M = 2N for CI); the CI ring keeps its first
 * half, which every 5^k (= 1 mod 4) maps onto itself */
static void automorphism_index(const oracle_ctx *c, u64 g, uint32_t *idx) {
  const int N = c->N, logM = c->logN + c->ci;
  const u64 mask = (2 * (u64)N << c->ci) - 1;
  for (int j = 0; j < N; j++) {
    u64 t1 = 2 * bitrev(j, logM) + 1;
    u64 t2 = (((g * t1) & mask) - 1) >> 1;
    idx[j] = (uint32_t)bitrev(t2, logM);
  }
}

void oracle_automorphism_ntt(const oracle_ctx *c, u64 g, const u64 *in, u64 *out, int nl) {
  const int N = c->N;
  uint32_t *idx = (uint32_t *)malloc(sizeof(uint32_t) * N);
  automorphism_index(c, g, idx);
  for (int l = 0; l < nl; l++)
    for (int j = 0; j < N; j++) out[(size_t)l * N + j] = in[(size_t)l * N + idx[j]];
  free(idx);
}

/* ------------------------------------------------------------------ */
/* ciphertext ops                                                        */
/* ------------------------------------------------------------------ */
void oracle_mul_coeffs(const oracle_ctx *c, const int *mods, int nl, const u64 *a,
                       const u64 *b, u64 *out) {
  const int N = c->N;
  for (int l = 0; l < nl; l++) {
    u64 q = c->mod[mods[l]];
    for (int n = 0; n < N; n++) out[(size_t)l * N + n] = mulmod(a[(size_t)l * N + n], b[(size_t)l * N + n], q);
  }
}

void oracle_mul_relin(const oracle_ctx *c, int level, const u64 *a, const u64 *b,
                      const u64 *rlk, u64 *out) {
  const int N = c->N;
  const size_t P = (size_t)(level + 1) * N;
  u64 *d2 = (u64 *)malloc(sizeof(u64) * P);
  u64 *k0 = (u64 *)malloc(sizeof(u64) * P), *k1 = (u64 *)malloc(sizeof(u64) * P);
  const u64 *a0 = a, *a1 = a + P, *b0 = b, *b1 = b + P;
  for (int j = 0; j <= level; j++) {
    u64 q = c->mod[j];
    for (int n = 0; n < N; n++) {
      size_t x = (size_t)j * N + n;
      out[x] = mulmod(a0[x], b0[x], q);
      out[P + x] = addmod(mulmod(a0[x], b1[x], q), mulmod(a1[x], b0[x], q), q);
      d2[x] = mulmod(a1[x], b1[x], q);
    }
  }
  oracle_keyswitch(c, level, d2, rlk, k0, k1);
  for (int j = 0; j <= level; j++) {
    u64 q = c->mod[j];
    for (int n = 0; n < N; n++) {
      size_t x = (size_t)j * N + n;
      out[x] = addmod(out[x], k0[x], q);
      out[P + x] = addmod(out[P + x], k1[x], q);
    }
  }
  free(d2);
  free(k0);
  free(k1);
}

void oracle_rotate(const oracle_ctx *c, int level, const u64 *ct, u64 g, const u64 *gk,
                   u64 *out) {
  const int N = c->N;
  const size_t P = (size_t)(level + 1) * N;
  u64 *k = (u64 *)malloc(sizeof(u64) * 2 * P);
  oracle_keyswitch(c, level, ct + P, gk, k, k + P);
  for (int j = 0; j <= level; j++) {
    u64 q = c->mod[j];
    for (int n = 0; n < N; n++) {
      size_t x = (size_t)j * N + n;
      k[x] = addmod(k[x], ct[x], q);
    }
  }
  oracle_automorphism_ntt(c, g, k, out, level + 1);
  oracle_automorphism_ntt(c, g, k + P, out + P, level + 1);
  free(k);
}

/* ------------------------------------------------------------------ */
/* BSGS linear transform (lintrans MultiplyByDiagMatrixBSGS restated)   */
/* ------------------------------------------------------------------ */
static void bsgs_split(int rot, int slots, int N1, int *giant, int *baby) {
  rot &= (slots - 1);
  *giant = ((rot / N1) * N1) & (slots - 1);
  *baby = rot & (N1 - 1);
}

int oracle_find_best_bsgs_n1(const int *diag_idx, int nd, int slots, int logMaxRatio) {
  double maxRatio = (double)(1 << logMaxRatio);
  for (int N1 = 1; N1 < slots; N1 <<= 1) {
    /* count distinct giant / baby indices */
    int *g = (int *)malloc(sizeof(int) * nd), *b = (int *)malloc(sizeof(int) * nd);
    int ng = 0, nb = 0;
    for (int d = 0; d < nd; d++) {
      int gi, bi, k;
      bsgs_split(diag_idx[d], slots, N1, &gi, &bi);
      for (k = 0; k < ng; k++)
        if (g[k] == gi) break;
      if (k == ng) g[ng++] = gi;
      for (k = 0; k < nb; k++)
        if (b[k] == bi) break;
      if (k == nb) b[nb++] = bi;
    }
    free(g);
    free(b);
    double r = (double)(nb - 1) / (double)(ng - 1);
    if (r == maxRatio) return N1;
    if (r > maxRatio) return N1 / 2;
  }
  return 1;
}

static const u64 *find_key(u64 g, int ngk, const u64 *gels, const u64 *const *gks) {
  for (int i = 0; i < ngk; i++)
    if (gels[i] == g) return gks[i];
  return NULL;
}

static int cmp_int(const void *a, const void *b) { return (*(const int *)a > *(const int *)b) - (*(const int *)a < *(const int *)b); }

void oracle_lt_bsgs(const oracle_ctx *c, int level, const u64 *ct, int nd, const int *diag_idx,
                    const u64 *const *pts, int N1, int ngk, const u64 *gels,
                    const u64 *const *gks, u64 *out) {
  const int N = c->N, L = c->L, K = c->K, slots = c->ci ? N : N / 2;
  const int nq = level + 1, nqp = nq + K;
  const size_t PQ = (size_t)nq * N, PQP = (size_t)nqp * N;
  int mods[MAXMOD];
  for (int j = 0; j < nqp; j++) mods[j] = j < nq ? j : L + (j - nq);

  /* giant/baby decomposition */
  int *gi = (int *)malloc(sizeof(int) * nd), *bi = (int *)malloc(sizeof(int) * nd);
  int *giants = (int *)malloc(sizeof(int) * nd), *babies = (int *)malloc(sizeof(int) * nd);
  int ng = 0, nb = 0;
  for (int d = 0; d < nd; d++) {
    int k;
    bsgs_split(diag_idx[d], slots, N1, &gi[d], &bi[d]);
    for (k = 0; k < ng; k++)
      if (giants[k] == gi[d]) break;
    if (k == ng) giants[ng++] = gi[d];
    for (k = 0; k < nb; k++)
      if (babies[k] == bi[d]) break;
    if (k == nb) babies[nb++] = bi[d];
  }
  qsort(giants, ng, sizeof(int), cmp_int);

  /* hoisted baby-step rotations in QP: rot_i = phi_i((c0*P + u0, u1)) */
  u64 **rot0 = (u64 **)calloc(nb, sizeof(u64 *)), **rot1 = (u64 **)calloc(nb, sizeof(u64 *));
  u64 *u0 = (u64 *)malloc(sizeof(u64) * PQP), *u1 = (u64 *)malloc(sizeof(u64) * PQP);
  for (int b = 0; b < nb; b++) {
    rot0[b] = (u64 *)malloc(sizeof(u64) * PQP);
    rot1[b] = (u64 *)malloc(sizeof(u64) * PQP);
    if (babies[b] == 0) {
      /* (c0*P, c1*P) in Q, zero P part */
      for (int j = 0; j < nq; j++) {
        u64 q = c->mod[j], Pm = 1;
        for (int k = 0; k < K; k++) Pm = mulmod(Pm, c->mod[L + k] % q, q);
        for (int n = 0; n < N; n++) {
          rot0[b][(size_t)j * N + n] = mulmod(ct[(size_t)j * N + n], Pm, q);
          rot1[b][(size_t)j * N + n] = mulmod(ct[PQ + (size_t)j * N + n], Pm, q);
        }
      }
      memset(rot0[b] + PQ, 0, sizeof(u64) * K * N);
      memset(rot1[b] + PQ, 0, sizeof(u64) * K * N);
      continue;
    }
    u64 g = oracle_galois_element(c, babies[b]);
    const u64 *key = find_key(g, ngk, gels, gks);
    if (!key) abort();
    oracle_gadget_product_lazy(c, level, ct + PQ, key, u0, u1);
    for (int j = 0; j < nq; j++) {
      u64 q = c->mod[j], Pm = 1;
      for (int k = 0; k < K; k++) Pm = mulmod(Pm, c->mod[L + k] % q, q);
      for (int n = 0; n < N; n++)
        u0[(size_t)j * N + n] = addmod(u0[(size_t)j * N + n], mulmod(ct[(size_t)j * N + n], Pm, q), q);
    }
    oracle_automorphism_ntt(c, g, u0, rot0[b], nqp);
    oracle_automorphism_ntt(c, g, u1, rot1[b], nqp);
  }

  u64 *acc0 = (u64 *)calloc(PQP, sizeof(u64)), *acc1 = (u64 *)calloc(PQP, sizeof(u64));
  u64 *t0 = (u64 *)malloc(sizeof(u64) * PQP), *t1 = (u64 *)malloc(sizeof(u64) * PQP);
  u64 *t1q = (u64 *)malloc(sizeof(u64) * PQ);
  u64 *c0 = (u64 *)malloc(sizeof(u64) * PQP), *c1 = (u64 *)malloc(sizeof(u64) * PQP);
  u64 *r0 = (u64 *)malloc(sizeof(u64) * PQP), *r1 = (u64 *)malloc(sizeof(u64) * PQP);
  for (int G = 0; G < ng; G++) {
    int j = giants[G];
    memset(t0, 0, sizeof(u64) * PQP);
    memset(t1, 0, sizeof(u64) * PQP);
    for (int d = 0; d < nd; d++) {
      if (gi[d] != j) continue;
      int b;
      for (b = 0; b < nb; b++)
        if (babies[b] == bi[d]) break;
      for (int l = 0; l < nqp; l++) {
        u64 q = c->mod[mods[l]];
        for (int n = 0; n < N; n++) {
          size_t x = (size_t)l * N + n;
          t0[x] = addmod(t0[x], mulmod(pts[d][x], rot0[b][x], q), q);
          t1[x] = addmod(t1[x], mulmod(pts[d][x], rot1[b][x], q), q);
        }
      }
    }
    if (j != 0) {
      u64 g = oracle_galois_element(c, j);
      const u64 *key = find_key(g, ngk, gels, gks);
      if (!key) abort();
      oracle_moddown(c, level, t1, t1q);
      oracle_gadget_product_lazy(c, level, t1q, key, c0, c1);
      for (int l = 0; l < nqp; l++) {
        u64 q = c->mod[mods[l]];
        for (int n = 0; n < N; n++) {
          size_t x = (size_t)l * N + n;
          c0[x] = addmod(c0[x], t0[x], q);
        }
      }
      oracle_automorphism_ntt(c, g, c0, r0, nqp);
      oracle_automorphism_ntt(c, g, c1, r1, nqp);
    } else {
      memcpy(r0, t0, sizeof(u64) * PQP);
      memcpy(r1, t1, sizeof(u64) * PQP);
    }
    for (int l = 0; l < nqp; l++) {
      u64 q = c->mod[mods[l]];
      for (int n = 0; n < N; n++) {
        size_t x = (size_t)l * N + n;
        acc0[x] = addmod(acc0[x], r0[x], q);
        acc1[x] = addmod(acc1[x], r1[x], q);
      }
    }
  }
  oracle_moddown(c, level, acc0, out);
  oracle_moddown(c, level, acc1, out + PQ);

  for (int b = 0; b < nb; b++) {
    free(rot0[b]);
    free(rot1[b]);
  }
  free(rot0); free(rot1); free(u0); free(u1);
  free(acc0); free(acc1); free(t0); free(t1); free(t1q);
  free(c0); free(c1); free(r0); free(r1);
  free(gi); free(bi); free(giants); free(babies);
}

/* ------------------------------------------------------------------ */
/* encoder (Standard ring, n = N/2 slots; HEAAN/Lattigo special FFT)    */
/* ------------------------------------------------------------------ */
typedef struct {
  double re, im;
} cplx;

static void special_tables(int n, int M, int **rot, cplx **roots) {
  *rot = (int *)malloc(sizeof(int) * n);
  *roots = (cplx *)malloc(sizeof(cplx) * (M + 1));
  int r = 1;
  for (int i = 0; i < n; i++) {
    (*rot)[i] = r;
    r = (int)(((long)r * 5) % M);
  }
  for (int i = 0; i <= M; i++) {
    double ang = 2.0 * M_PI * (double)i / (double)M;
    (*roots)[i].re = cos(ang);
    (*roots)[i].im = sin(ang);
  }
}

static void bitrev_cplx(cplx *v, int n) {
  int logn = 0;
  while ((1 << logn) < n) logn++;
  for (int i = 0; i < n; i++) {
    int j = (int)bitrev(i, logn);
    if (i < j) {
      cplx t = v[i];
      v[i] = v[j];
      v[j] = t;
    }
  }
}

static inline cplx cmul(cplx a, cplx b) {
  cplx r;
  double ac = a.re * b.re, bd = a.im * b.im, ad = a.re * b.im, bc = a.im * b.re;
  r.re = ac - bd;
  r.im = ad + bc;
  return r;
}

static void special_ifft(cplx *v, int n, int M, const int *rot, const cplx *roots) {
  for (int len = n; len >= 2; len >>= 1) {
    int lenh = len >> 1, lenq = len << 2;
    for (int i = 0; i < n; i += len) {
      for (int j = 0; j < lenh; j++) {
        int idx = (lenq - (rot[j] % lenq)) * (M / lenq);
        cplx u, w;
        u.re = v[i + j].re + v[i + j + lenh].re;
        u.im = v[i + j].im + v[i + j + lenh].im;
        w.re = v[i + j].re - v[i + j + lenh].re;
        w.im = v[i + j].im - v[i + j + lenh].im;
        v[i + j] = u;
        v[i + j + lenh] = cmul(w, roots[idx]);
      }
    }
  }
  bitrev_cplx(v, n);
  double inv = 1.0 / (double)n;
  for (int i = 0; i < n; i++) {
    v[i].re *= inv;
    v[i].im *= inv;
  }
}

static void special_fft(cplx *v, int n, int M, const int *rot, const cplx *roots) {
  bitrev_cplx(v, n);
  for (int len = 2; len <= n; len <<= 1) {
    int lenh = len >> 1, lenq = len << 2;
    for (int i = 0; i < n; i += len) {
      for (int j = 0; j < lenh; j++) {
        int idx = (rot[j] % lenq) * (M / lenq);
        cplx u = v[i + j];
        cplx w = cmul(v[i + j + lenh], roots[idx]);
        v[i + j].re = u.re + w.re;
        v[i + j].im = u.im + w.im;
        v[i + j + lenh].re = u.re - w.re;
        v[i + j + lenh].im = u.im - w.im;
      }
    }
  }
}

/* Lattigo SingleFloat64ToFixedPointCRT restated: c = floor(|v|*scale + 0.5),
 * negative values map to q - (c mod q) (fully reduced here). */
static void to_crt(double v, double scale, const oracle_ctx *c, const int *mods, int nm,
                   u64 *out, size_t stride) {
  if (v == 0.0) {
    for (int m = 0; m < nm; m++) out[m * stride] = 0;
    return;
  }
  int neg = v < 0;
  double x = neg ? v * (-scale) : v * scale;
  if (!(x < 18446744073709551616.0)) {
    /* |v*scale| >= 2^64: Lattigo's big.Int path.  x is an integer
     * mant * 2^e (e > 11); reduce it exactly. */
    int ex;
    double fr = frexp(x, &ex);
    u64 mant = (u64)ldexp(fr, 53);
    for (int m = 0; m < nm; m++) {
      u64 q = c->mod[mods[m]];
      u64 r = mulmod(mant % q, powmod(2 % q, (u64)(ex - 53), q), q);
      out[m * stride] = neg ? (r ? q - r : 0) : r;
    }
    return;
  }
  u64 cval = (u64)(x + 0.5);
  for (int m = 0; m < nm; m++) {
    u64 q = c->mod[mods[m]];
    u64 r = cval % q;
    out[m * stride] = neg ? (r ? q - r : 0) : r;
  }
}

/* CI ring: n = N real slots, cyclotomic order 4N; the coefficients are the
 * real parts of the special iFFT (the imaginary parts are the expansion's
 * upper half, -a_{N-j}, which the CI ring does not store) */
void oracle_encode(const oracle_ctx *c, const double *values, int nvals, double scale,
                   const int *mods, int nm, u64 *out) {
  const int N = c->N, n = c->ci ? N : N / 2, M = 4 * n;
  int *rot;
  cplx *roots;
  special_tables(n, M, &rot, &roots);
  cplx *v = (cplx *)calloc(n, sizeof(cplx));
  for (int i = 0; i < nvals && i < n; i++) v[i].re = values[i];
  special_ifft(v, n, M, rot, roots);
  for (int i = 0; i < n; i++) {
    to_crt(v[i].re, scale, c, mods, nm, out + i, (size_t)N);
    if (!c->ci) to_crt(v[i].im, scale, c, mods, nm, out + i + n, (size_t)N);
  }
  for (int m = 0; m < nm; m++) oracle_ntt(c, mods[m], out + (size_t)m * N);
  free(v);
  free(rot);
  free(roots);
}

/* centered CRT reconstruction of one coefficient -> double (tests only) */
static double crt_centered_double(const oracle_ctx *c, int level, const u64 *res) {
  /* mixed-radix (Garner) digits, then evaluate in long double with the
   * centered correction x - Q when x > Q/2 (decided on the top digit). */
  int nl = level + 1;
  u64 d[MAXMOD];
  for (int i = 0; i < nl; i++) {
    u64 qi = c->mod[i];
    u64 x = res[i] % qi;
    for (int k = 0; k < i; k++) {
      u64 qk = c->mod[k] % qi;
      x = mulmod(submod(x, d[k] % qi, qi), invmod(qk, qi), qi);
    }
    d[i] = x;
  }
  /* value = d0 + d1 q0 + d2 q0 q1 + ...; compare with Q/2 via the mixed-radix
   * digits of Q-1 halved: x > Q/2  <=>  x >= ceil(Q/2).  Use long double for
   * the magnitude, exact sign decision through digit comparison. */
  /* half digits of (Q-1)/2 in mixed radix */
  u64 h[MAXMOD];
  {
    /* (Q-1) digits are (q_i - 1); divide by 2 from the top */
    u64 rem = 0;
    for (int i = nl - 1; i >= 0; i--) {
      u128 cur = (u128)rem * c->mod[i] + (c->mod[i] - 1);
      h[i] = (u64)(cur / 2);
      rem = (u64)(cur % 2);
    }
  }
  int greater = 0;
  for (int i = nl - 1; i >= 0; i--) {
    if (d[i] != h[i]) {
      greater = d[i] > h[i];
      break;
    }
  }
  long double val = 0.0L, base = 1.0L;
  if (!greater) {
    for (int i = 0; i < nl; i++) {
      val += (long double)d[i] * base;
      base *= (long double)c->mod[i];
    }
  } else {
    /* Q - x with mixed radix borrow arithmetic: digits of (Q-1-x) + 1 */
    u64 e[MAXMOD];
    for (int i = 0; i < nl; i++) e[i] = c->mod[i] - 1 - d[i];
    for (int i = 0; i < nl; i++) {
      if (e[i] + 1 < c->mod[i]) {
        e[i] += 1;
        break;
      }
      e[i] = 0;
    }
    for (int i = 0; i < nl; i++) {
      val += (long double)e[i] * base;
      base *= (long double)c->mod[i];
    }
    val = -val;
  }
  return (double)val;
}

void oracle_decode(const oracle_ctx *c, int level, const u64 *pt, double scale,
                   double *values) {
  const int N = c->N, n = c->ci ? N : N / 2, M = 4 * n, nl = level + 1;
  u64 *x = (u64 *)malloc(sizeof(u64) * N * nl);
  memcpy(x, pt, sizeof(u64) * N * nl);
  for (int j = 0; j < nl; j++) oracle_intt(c, j, x + (size_t)j * N);
  int *rot;
  cplx *roots;
  special_tables(n, M, &rot, &roots);
  cplx *v = (cplx *)calloc(n, sizeof(cplx));
  u64 res[MAXMOD];
  for (int i = 0; i < N; i++) {
    for (int j = 0; j < nl; j++) res[j] = x[(size_t)j * N + i];
    double f = crt_centered_double(c, level, res) / scale;
    if (c->ci) { /* slot input c_j = a_j - i a_{N-j} (c_0 = a_0) */
      v[i].re = f;
      if (i) v[N - i].im = -f;
    } else if (i < n) {
      v[i].re = f;
    } else {
      v[i - n].im = f;
    }
  }
  special_fft(v, n, M, rot, roots);
  for (int i = 0; i < n; i++) values[i] = v[i].re;
  free(x);
  free(v);
  free(rot);
  free(roots);
}

/* ------------------------------------------------------------------ */
/* test-only keygen / encryption (seeded SplitMix64)                    */
/* ------------------------------------------------------------------ */
static u64 sm64(u64 *s) {
  u64 z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static u64 uniform_mod(u64 *s, u64 q) {
  int bits = 64 - __builtin_clzll(q);
  u64 mask = bits == 64 ? ~0ull : (((u64)1 << bits) - 1);
  for (;;) {
    u64 r = sm64(s) & mask;
    if (r < q) return r;
  }
}
static int64_t gauss(u64 *s) {
  for (;;) {
    double u1 = ((double)(sm64(s) >> 11) + 1.0) / 9007199254740993.0;
    double u2 = (double)(sm64(s) >> 11) / 9007199254740992.0;
    double z = sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2) * 3.2;
    if (fabs(z) <= 19.2) return (int64_t)llround(z);
  }
}
static void small_to_ntt(const oracle_ctx *c, const int64_t *v, int m, u64 *out) {
  u64 q = c->mod[m];
  for (int n = 0; n < c->N; n++) out[n] = v[n] >= 0 ? (u64)v[n] % q : q - ((u64)(-v[n]) % q);
  oracle_ntt(c, m, out);
}

void oracle_gen_secret(const oracle_ctx *c, u64 seed, int h, u64 *sk) {
  const int N = c->N;
  u64 s = seed;
  int64_t *v = (int64_t *)calloc(N, sizeof(int64_t));
  int *perm = (int *)malloc(sizeof(int) * N);
  for (int i = 0; i < N; i++) perm[i] = i;
  if (h > N) h = N;
  for (int i = 0; i < h; i++) {
    int j = i + (int)(sm64(&s) % (u64)(N - i));
    int t = perm[i];
    perm[i] = perm[j];
    perm[j] = t;
    v[perm[i]] = (sm64(&s) & 1) ? 1 : -1;
  }
  for (int m = 0; m < c->L + c->K; m++) small_to_ntt(c, v, m, sk + (size_t)m * N);
  free(v);
  free(perm);
}

void oracle_gen_evk(const oracle_ctx *c, u64 seed, const u64 *s_in, const u64 *s_out, u64 *evk) {
  const int N = c->N, L = c->L, K = c->K, nm = L + K;
  const int dnum = (L + K - 1) / K;
  u64 s = seed;
  int64_t *e = (int64_t *)malloc(sizeof(int64_t) * N);
  u64 *et = (u64 *)malloc(sizeof(u64) * N);
  for (int i = 0; i < dnum; i++) {
    u64 *b = evk + (size_t)i * 2 * nm * N;
    u64 *a = b + (size_t)nm * N;
    for (int n = 0; n < N; n++) e[n] = gauss(&s);
    for (int m = 0; m < nm; m++) {
      u64 q = c->mod[m];
      small_to_ntt(c, e, m, et);
      u64 Pm = 1;
      for (int k = 0; k < K; k++) Pm = mulmod(Pm, c->mod[L + k] % q, q);
      int in_digit = m < L && m >= i * K && m < (i + 1) * K;
      for (int n = 0; n < N; n++) {
        size_t x = (size_t)m * N + n;
        a[x] = uniform_mod(&s, q);
        u64 v = submod(et[n], mulmod(a[x], s_out[x], q), q);
        if (in_digit) v = addmod(v, mulmod(Pm, s_in[x], q), q);
        b[x] = v;
      }
    }
  }
  free(e);
  free(et);
}

void oracle_encrypt_sk(const oracle_ctx *c, u64 seed, int level, const u64 *sk, const u64 *pt,
                       u64 *ct) {
  const int N = c->N;
  const size_t P = (size_t)(level + 1) * N;
  u64 s = seed;
  int64_t *e = (int64_t *)malloc(sizeof(int64_t) * N);
  u64 *et = (u64 *)malloc(sizeof(u64) * N);
  for (int n = 0; n < N; n++) e[n] = gauss(&s);
  for (int j = 0; j <= level; j++) {
    u64 q = c->mod[j];
    small_to_ntt(c, e, j, et);
    for (int n = 0; n < N; n++) {
      size_t x = (size_t)j * N + n;
      u64 a = uniform_mod(&s, q);
      ct[P + x] = a;
      ct[x] = addmod(submod(et[n], mulmod(a, sk[x], q), q), pt[x], q);
    }
  }
  free(e);
  free(et);
}

void oracle_decrypt(const oracle_ctx *c, int level, const u64 *sk, const u64 *ct, u64 *pt) {
  const int N = c->N;
  const size_t P = (size_t)(level + 1) * N;
  for (int j = 0; j <= level; j++) {
    u64 q = c->mod[j];
    for (int n = 0; n < N; n++) {
      size_t x = (size_t)j * N + n;
      pt[x] = addmod(ct[x], mulmod(ct[P + x], sk[x], q), q);
    }
  }
}

/* ------------------------------------------------------------------ */
/* public-key encryption sampler of the MI355X backend (encoder.hip),  */
/* restated: ChaCha20 (RFC 8439 §2.3) counter-mode stream per          */
/* (encryption index, image, component), uniform ternary u and a       */
/* cumulative-table discrete Gaussian (sigma 3.2, |e| <= 19).          */
/* ------------------------------------------------------------------ */
static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
#define QR(a, b, c, d)                          \
  do {                                          \
    a += b; d ^= a; d = rotl32(d, 16);          \
    c += d; b ^= c; b = rotl32(b, 12);          \
    a += b; d ^= a; d = rotl32(d, 8);           \
    c += d; b ^= c; b = rotl32(b, 7);           \
  } while (0)

void oracle_chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3],
                           uint32_t out[16]) {
  uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  for (int i = 0; i < 8; i++) st[4 + i] = key[i];
  st[12] = counter;
  for (int i = 0; i < 3; i++) st[13 + i] = nonce[i];
  uint32_t x[16];
  memcpy(x, st, sizeof(x));
  for (int r = 0; r < 10; r++) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + st[i];
}
#undef QR

void oracle_enc_key(u64 seed, uint32_t key[8]) {
  u64 z = seed ^ 0x6a09e667f3bcc909ull;
  for (int i = 0; i < 4; i++) {
    u64 t = (z += 0x9E3779B97F4A7C15ull);
    t = (t ^ (t >> 30)) * 0xBF58476D1CE4E5B9ull;
    t = (t ^ (t >> 27)) * 0x94D049BB133111EBull;
    t ^= t >> 31;
    key[2 * i] = (uint32_t)t;
    key[2 * i + 1] = (uint32_t)(t >> 32);
  }
}

#define GAUSS_BOUND 19
void oracle_gauss_cdt(double sigma, int bound, u64 *t) {
  double rho[2 * 64 + 1], sum = 0.0, acc = 0.0;
  for (int x = -bound; x <= bound; x++) {
    rho[x + bound] = exp(-(double)(x * x) / (2.0 * sigma * sigma));
    sum += rho[x + bound];
  }
  for (int i = 0; i < 2 * bound; i++) {
    acc += rho[i];
    double cv = ldexp(acc / sum, 64);
    t[i] = cv >= 18446744073709551616.0 ? ~0ull : (u64)cv;
  }
}

/* component comp (0 = u, 1 = e0, 2 = e1) of image `image` of encryption `enc` */
void oracle_enc_sample(int N, const uint32_t key[8], uint32_t enc, uint32_t image, int comp,
                       int64_t *out) {
  u64 cdt[2 * GAUSS_BOUND];
  oracle_gauss_cdt(3.2, GAUSS_BOUND, cdt);
  const uint32_t nonce[3] = {enc, image, 0x454e0000u | (uint32_t)comp};
  uint32_t w[16];
  for (int blk = 0; blk < N / 8; blk++) {
    oracle_chacha20_block(key, (uint32_t)blk, nonce, w);
    for (int k = 0; k < 8; k++) {
      u64 x = (u64)w[2 * k] | ((u64)w[2 * k + 1] << 32);
      int64_t v;
      if (comp == 0) {
        v = (int64_t)(((x >> 32) * 3) >> 32) - 1;
      } else {
        int cnt = 0;
        for (int t = 0; t < 2 * GAUSS_BOUND; t++) cnt += x >= cdt[t];
        v = cnt - GAUSS_BOUND;
      }
      out[blk * 8 + k] = v;
    }
  }
}

/* c0 = u pk0 + e0 + pt, c1 = u pk1 + e1 at `level` (pk: [2][L+K][N] NTT) */
void oracle_encrypt_pk(const oracle_ctx *c, const uint32_t key[8], uint32_t enc, uint32_t image,
                       int level, const u64 *pk, const u64 *pt, u64 *ct) {
  const int N = c->N, LK = c->L + c->K;
  const size_t P = (size_t)(level + 1) * N;
  int64_t *smp[3];
  u64 *t[3];
  for (int k = 0; k < 3; k++) {
    smp[k] = (int64_t *)malloc(sizeof(int64_t) * N);
    t[k] = (u64 *)malloc(sizeof(u64) * N);
    oracle_enc_sample(N, key, enc, image, k, smp[k]);
  }
  for (int j = 0; j <= level; j++) {
    u64 q = c->mod[j];
    for (int k = 0; k < 3; k++) small_to_ntt(c, smp[k], j, t[k]);
    for (int n = 0; n < N; n++) {
      size_t x = (size_t)j * N + n;
      u64 pk0 = pk[(size_t)j * N + n], pk1 = pk[(size_t)(LK + j) * N + n];
      ct[x] = addmod(addmod(mulmod(t[0][n], pk0, q), t[1][n], q), pt[x], q);
      ct[P + x] = addmod(mulmod(t[0][n], pk1, q), t[2][n], q);
    }
  }
  for (int k = 0; k < 3; k++) {
    free(smp[k]);
    free(t[k]);
  }
}

/* ------------------------------------------------------------------ */
/* polynomial evaluation of the HIP backend (backend.hip eval_poly,    */
/* reached from polyeval.go:63-84), restated: power basis T_{2s} by    */
/* squaring (Chebyshev: 2 T_s^2 - 1), recursion p = q T_s + r down to  */
/* linear leaves, every node accumulated at an exact nominal scale.    */
/* A ciphertext here is [2][level+1][N] with its level and scale.      */
/* ------------------------------------------------------------------ */
typedef struct {
  int level;
  long double scale;
  u64 *v;
} pct;

static pct pct_alloc(const oracle_ctx *c, int level, long double scale) {
  pct r = {level, scale, (u64 *)calloc((size_t)2 * (level + 1) * c->N, sizeof(u64))};
  return r;
}
/* first level+1 limbs of each component of a */
static u64 *pct_at(const oracle_ctx *c, const pct *a, int level) {
  const size_t L = (size_t)(level + 1) * c->N, A = (size_t)(a->level + 1) * c->N;
  u64 *o = (u64 *)malloc(sizeof(u64) * 2 * L);
  memcpy(o, a->v, sizeof(u64) * L);
  memcpy(o + L, a->v + A, sizeof(u64) * L);
  return o;
}
static void big_const_res(const oracle_ctx *c, long double v, int level, u64 *r) {
  int neg = v < 0;
  long double a = floorl((neg ? -v : v) + 0.5L);
  u64 m;
  int e = 0;
  if (a >= 9223372036854775808.0L) {
    int ex;
    long double fr = frexpl(a, &ex);
    m = (u64)ldexpl(fr, 64);
    e = ex - 64;
  } else {
    m = (u64)a;
  }
  for (int j = 0; j <= level; j++) {
    u64 q = c->mod[j];
    u64 x = mulmod(m % q, powmod(2 % q, (u64)e, q), q);
    r[j] = neg ? (x ? q - x : 0) : x;
  }
}
static void pct_rescale(const oracle_ctx *c, pct *a) {
  u64 *o = (u64 *)malloc(sizeof(u64) * 2 * (size_t)a->level * c->N);
  oracle_rescale(c, a->level, 2, a->v, o);
  free(a->v);
  a->v = o;
  a->scale /= (long double)c->mod[a->level];
  a->level -= 1;
}
static pct pct_mul_relin(const oracle_ctx *c, const pct *a, const pct *b, const u64 *rlk) {
  int lv = a->level < b->level ? a->level : b->level;
  u64 *x = pct_at(c, a, lv), *y = pct_at(c, b, lv);
  pct o = pct_alloc(c, lv, a->scale * b->scale);
  oracle_mul_relin(c, lv, x, y, rlk, o.v);
  free(x);
  free(y);
  return o;
}

typedef struct {
  const oracle_ctx *c;
  const pct *x;
  int cheb;
  pct pw[17];   /* pw[k] = T_{2^k}, k >= 1 */
  pct baby[256]; /* T_j, j < 2^logSplit not a power of two (v == NULL until computed) */
  const u64 *rlk;
} poly_run;

static int ceil_log2i(int j) {
  int k = 0;
  while ((1 << k) < j) k++;
  return k;
}
/* Lattigo bignum.OptimalSplit */
static int optimal_split(int logd) {
  int ls = logd >> 1;
  int a = (1 << ls) + (1 << (logd - ls)) + logd - ls - 3;
  int b = (1 << (ls + 1)) + (1 << (logd - ls - 1)) + logd - ls - 4;
  if (a > b) ls++;
  return ls;
}
/* T_j: x, a power from pw, or a baby step 2 T_a T_b - T_c (Chebyshev) / T_a T_b
 * with a = 2^k - 1, b = j + 1 - 2^k (Lattigo genPower), T_c scaled by
 * round(s_a s_b / s_c) before the rescale */
static const pct *poly_T(poly_run *R, int j) {
  const oracle_ctx *c = R->c;
  if (j == 1) return R->x;
  if ((j & (j - 1)) == 0) return &R->pw[ceil_log2i(j)];
  if (R->baby[j].v) return &R->baby[j];
  int k = ceil_log2i(j) - 1, a = (1 << k) - 1, b = j + 1 - (1 << k), cc = a > b ? a - b : b - a;
  const pct *A = poly_T(R, a), *B = poly_T(R, b);
  pct t = pct_mul_relin(c, A, B, R->rlk);
  if (R->cheb) {
    const size_t P = (size_t)(t.level + 1) * c->N;
    u64 kk[MAXMOD];
    for (size_t i = 0; i < 2 * P; i++) {
      int l = (int)((i % P) / c->N);
      t.v[i] = addmod(t.v[i], t.v[i], c->mod[l]);
    }
    if (cc == 0) {
      big_const_res(c, -t.scale, t.level, kk);
      for (int l = 0; l <= t.level; l++)
        for (int i = 0; i < c->N; i++) t.v[(size_t)l * c->N + i] = addmod(t.v[(size_t)l * c->N + i], kk[l], c->mod[l]);
    } else {
      const pct *C = poly_T(R, cc);
      u64 *cv = pct_at(c, C, t.level);
      big_const_res(c, -(t.scale / C->scale), t.level, kk);
      for (size_t i = 0; i < 2 * P; i++) {
        int l = (int)((i % P) / c->N);
        t.v[i] = addmod(t.v[i], mulmod(cv[i], kk[l], c->mod[l]), c->mod[l]);
      }
      free(cv);
    }
  }
  pct_rescale(c, &t);
  R->baby[j] = t;
  return &R->baby[j];
}

static int bitlen_i(int v) {
  int k = 0;
  while (v >> k) k++;
  return k;
}
/* leaf (Lattigo EvaluatePolynomialVectorFromPowerBasis): c_0 S + sum_j
 * round(c_j S / scale(T_j)) T_j, at the lowest level among lam and the T_j
 * used (MulThenAdd takes the lower level) */
static pct poly_leaf(poly_run *R, const long double *cf, int n, int lam, long double S) {
  const oracle_ctx *c = R->c;
  const int N = c->N, deg = n - 1;
  u64 k[MAXMOD];
  int lv = lam;
  for (int j = 1; j <= deg; j++)
    if (cf[j] != 0) {
      const pct *T = poly_T(R, j);
      if (T->level < lv) lv = T->level;
    }
  const size_t P = (size_t)(lv + 1) * N;
  pct o = pct_alloc(c, lv, S);
  for (int j = 1; j <= deg; j++) {
    if (cf[j] == 0) continue;
    const pct *T = poly_T(R, j);
    big_const_res(c, cf[j] * S / T->scale, lv, k);
    u64 *x = pct_at(c, T, lv);
    for (int comp = 0; comp < 2; comp++)
      for (int l = 0; l <= lv; l++)
        for (int i = 0; i < N; i++) {
          size_t at = comp * P + (size_t)l * N + i;
          o.v[at] = addmod(o.v[at], mulmod(x[at], k[l], c->mod[l]), c->mod[l]);
        }
    free(x);
  }
  if (cf[0] != 0) {
    big_const_res(c, cf[0] * S, lv, k);
    for (int l = 0; l <= lv; l++)
      for (int i = 0; i < N; i++) o.v[(size_t)l * N + i] = addmod(o.v[(size_t)l * N + i], k[l], c->mod[l]);
  }
  return o;
}

/* Lattigo v6 recursePS (he/polynomial.go) with the ckks simEvaluator's
 * UpdateLevelAndScale{Baby,Giant}Step: a node of degree < 2^logSplit is a
 * leaf unless it is a lead node (on the quotient chain from the top) with
 * maxdeg > 2^bitlen(maxdeg) - 2^(logSplit-1), which is re-split with
 * logSplit = OptimalSplit(bitlen(deg)); otherwise p = q X^m + r with m the
 * smallest power of two >= 2^logSplit and >= deg/2 + 1 (splitCoeffs; the
 * Chebyshev split uses T_{m+j} = 2 T_m T_j - T_{m-j}).  The q branch runs one
 * level up at S q_i / scale(X^m) (q_i = q_lam for a lead node, q_{lam+1}
 * otherwise), is rescaled and multiplied by X^m; the r branch runs at that
 * product's scale; a lead leaf is evaluated at S q_lam. */
static pct poly_ps(poly_run *R, const long double *cf, int n, int lead, int maxdeg, int logSplit, int lam,
                   long double S) {
  const oracle_ctx *c = R->c;
  const int N = c->N, deg = n - 1, cheb = R->cheb;
  if (deg < (1 << logSplit)) {
    if (lead && logSplit > 1 && maxdeg > (1 << bitlen_i(maxdeg)) - (1 << (logSplit - 1)))
      return poly_ps(R, cf, n, lead, maxdeg, optimal_split(bitlen_i(deg)), lam, S);
    return poly_leaf(R, cf, n, lam, lead ? S * (long double)c->mod[lam] : S);
  }
  int m = 1 << logSplit;
  while (m < (deg >> 1) + 1) m <<= 1;
  long double *q = (long double *)malloc(sizeof(long double) * (deg - m + 1));
  long double *r = (long double *)malloc(sizeof(long double) * m);
  for (int j = 0; j <= deg - m; j++) q[j] = cf[m + j];
  for (int j = 0; j < m; j++) r[j] = cf[j];
  if (cheb)
    for (int j = 1; j <= deg - m; j++) {
      q[j] = 2 * cf[m + j];
      r[m - j] -= cf[m + j];
    }
  const int rmax = maxdeg == deg ? m - 1 : maxdeg - (deg - m + 1);
  const pct *X = &R->pw[ceil_log2i(m)];
  const long double qi = (long double)c->mod[lead ? lam : lam + 1];
  pct qc = poly_ps(R, q, deg - m + 1, lead, maxdeg, logSplit, lam + 1, S * qi / X->scale);
  pct_rescale(c, &qc);
  pct o = pct_mul_relin(c, &qc, X, R->rlk);
  pct rc = poly_ps(R, r, m, 0, rmax, logSplit, lam, o.scale);
  const int lv = o.level < rc.level ? o.level : rc.level; /* Add takes the lower level */
  if (lv < o.level) {
    u64 *v = pct_at(c, &o, lv);
    free(o.v);
    o.v = v;
    o.level = lv;
  }
  u64 *y = pct_at(c, &rc, lv);
  const size_t P = (size_t)(lv + 1) * N;
  for (int comp = 0; comp < 2; comp++)
    for (int l = 0; l <= lv; l++)
      for (int i = 0; i < N; i++) {
        size_t at = comp * P + (size_t)l * N + i;
        o.v[at] = addmod(o.v[at], y[at], c->mod[l]);
      }
  free(y);
  free(qc.v);
  free(rc.v);
  free(q);
  free(r);
  return o;
}

/* ct: [2][level+1][N] at `level`, scale xscale; coeffs lowest degree first.
 * out: [2][out_level+1][N]; returns out_level (-1 if level < depth). */
int oracle_eval_poly(const oracle_ctx *c, int level, const u64 *ct, long double xscale, const double *coeffs,
                     int n, int cheb, long double target, const u64 *rlk, u64 *out, long double *out_scale) {
  long double *cf = (long double *)malloc(sizeof(long double) * (n > 0 ? n : 1));
  for (int i = 0; i < n; i++) cf[i] = (long double)coeffs[i];
  int r = oracle_eval_poly_ld(c, level, ct, xscale, cf, n, cheb, target, rlk, out, out_scale);
  free(cf);
  return r;
}

/* long double scales passed by address (80-bit values through ctypes) */
int oracle_eval_poly_ldp(const oracle_ctx *c, int level, const u64 *ct, const long double *xscale,
                         const double *coeffs, int n, int cheb, const long double *target, const u64 *rlk, u64 *out,
                         long double *out_scale) {
  return oracle_eval_poly(c, level, ct, *xscale, coeffs, n, cheb, *target, rlk, out, out_scale);
}

/* the same with long double coefficients (the bootstrapping cosine's) */
int oracle_eval_poly_ld(const oracle_ctx *c, int level, const u64 *ct, long double xscale, const long double *coeffs,
                        int n, int cheb, long double target, const u64 *rlk, u64 *out, long double *out_scale) {
  const int deg = n - 1;
  int depth = 0;
  while ((1 << depth) <= deg) depth++;
  if (level < depth || depth > 16) return -1;
  pct x = {level, xscale, (u64 *)ct};
  poly_run R;
  memset(&R, 0, sizeof(R));
  R.c = c;
  R.x = &x;
  R.rlk = rlk;
  R.cheb = cheb;
  long double *cf = (long double *)malloc(sizeof(long double) * n);
  for (int i = 0; i < n; i++) cf[i] = coeffs[i];
  u64 k[MAXMOD];
  for (int ks = 0; (2 << ks) <= deg; ks++) {
    const pct *a = ks == 0 ? &x : &R.pw[ks];
    pct t = pct_mul_relin(c, a, a, rlk);
    pct_rescale(c, &t);
    if (cheb) {
      const size_t P = (size_t)(t.level + 1) * c->N;
      for (size_t i = 0; i < 2 * P; i++) {
        int j = (int)((i % P) / c->N);
        t.v[i] = addmod(t.v[i], t.v[i], c->mod[j]);
      }
      big_const_res(c, -t.scale, t.level, k);
      for (int j = 0; j <= t.level; j++)
        for (int i = 0; i < c->N; i++)
          t.v[(size_t)j * c->N + i] = addmod(t.v[(size_t)j * c->N + i], k[j], c->mod[j]);
    }
    R.pw[ks + 1] = t;
  }
  pct o;
  if (deg == 0) {
    o = poly_leaf(&R, cf, n, level, target);
  } else {
    o = poly_ps(&R, cf, n, 1, deg, optimal_split(depth), level - depth + 1, target);
    pct_rescale(c, &o);
    o.scale = target;
  }
  memcpy(out, o.v, sizeof(u64) * 2 * (size_t)(o.level + 1) * c->N);
  *out_scale = o.scale;
  free(o.v);
  for (int i = 1; i < 17; i++) free(R.pw[i].v);
  for (int i = 0; i < 256; i++) free(R.baby[i].v);
  free(cf);
  return o.level;
}

/* ------------------------------------------------------------------ */
/* bootstrapping (bootstrapper.go:19-80 is the call site; Orion sets    */
/* LogN, LogP, Xs and LogSlots, bootstrapper.go:33-38, and every other  */
/* parameter is Lattigo v6's default bootstrapping.ParametersLiteral    */
/* [U], restated here from the parameters alone -- no constant, prime   */
/* or diagonal comes from the library under test; the shared inputs    */
/* are the keys and the input ciphertext):                               */
/*   CoeffsToSlots 4 x 56-bit levels, SlotsToCoeffs 3 x 39-bit levels,   */
/*   EvalMod 60-bit levels, K = 16, Mod1 degree 30, 3 double angles,     */
/*   Mod1InvDegree 0, LogMessageRatio 8, LogBSGSRatio 1 for the DFT      */
/*   matrices, an ephemeral secret of Hamming weight 32.                 */
/* Circuit:                                                              */
/*   x  = F * (level-0 residues), F = round(q0 / 2^(8 + logScale))       */
/*   x  = (x0, 0) + KS_{s -> s_eph}(x1) at level 0                       */
/*   t  = NTT(centred lift of INTT(x) to every Q limb), scale q0         */
/*   t  = (t0, 0) + KS_{s_eph -> s}(t1) at the top level                 */
/*   gap > 1: t = gap^-1 t, then t += sigma_g(t) for each trace element  */
/*   z  = the 4 CoeffsToSlots transforms, each followed by a rescale     */
/*   gap > 1: y = EvalMod(z + conj z)                                    */
/*   else:    y = i EvalMod(i (conj z - z)) + EvalMod(z + conj z)        */
/*   EvalMod(u) = cosine polynomial at target t0, then r double angles   */
/*        y <- rescale(2 y^2 - a^(2^(k+1)))                              */
/*   o  = the 3 SlotsToCoeffs transforms with rescales                   */
/*   out = gap * o (residual top level, scheme primes)                   */
/* ------------------------------------------------------------------ */
#define BTP_CTS 4
#define BTP_CTS_BITS 56
#define BTP_STC 3
#define BTP_STC_BITS 39
#define BTP_MOD_BITS 60
#define BTP_DEG 30
#define BTP_DEPTH 5 /* bits.Len64(BTP_DEG) */
#define BTP_R 3
#define BTP_K 16
#define BTP_LOGMSG 8
#define BTP_LOGBSGS 1
#define BTP_EPH_H 32
static const long double BTP_PI = 3.14159265358979323846264338327950288L;

/* the bootstrapping chain: the residual Q primes, then fresh primes of the
 * circuit's sizes (SlotsToCoeffs, EvalMod, CoeffsToSlots, bottom to top) and
 * of logP, each size from its own NTTFriendlyPrimesGenerator stream, skipping
 * every prime of the residual parameters (scheme_qp: their Q and P) */
int oracle_btp_chain(int logN, const u64 *scheme_qp, int n_scheme, int Lres, const int *logP, int lenP, u64 *out) {
  int bits[MAXMOD], nb = 0;
  for (int i = 0; i < BTP_STC; i++) bits[nb++] = BTP_STC_BITS;
  for (int i = 0; i < BTP_DEPTH + BTP_R; i++) bits[nb++] = BTP_MOD_BITS;
  for (int i = 0; i < BTP_CTS; i++) bits[nb++] = BTP_CTS_BITS;
  for (int i = 0; i < lenP; i++) bits[nb++] = logP[i];
  if (Lres + nb > MAXMOD) return -1;
  u64 taken[2 * MAXMOD];
  int nt = 0;
  for (int i = 0; i < n_scheme; i++) taken[nt++] = scheme_qp[i];
  primegen gens[MAXMOD];
  int gsize[MAXMOD], ng = 0;
  const u64 nthroot = (u64)2 << logN;
  for (int i = 0; i < Lres; i++) out[i] = scheme_qp[i];
  for (int i = 0; i < nb; i++) {
    int k;
    for (k = 0; k < ng; k++)
      if (gsize[k] == bits[i]) break;
    if (k == ng) {
      pg_init(&gens[ng], bits[i], nthroot);
      gsize[ng++] = bits[i];
    }
    u64 q;
    int dup;
    do {
      q = bits[i] == 61 ? pg_next_downstream(&gens[k]) : pg_next_alternating(&gens[k]);
      if (!q) return -1;
      dup = 0;
      for (int j = 0; j < nt; j++) dup |= taken[j] == q;
    } while (dup);
    taken[nt++] = q;
    out[Lres + i] = q;
  }
  return Lres + nb;
}

/* EvalMod's polynomial, Lattigo v6 mod1 CosDiscrete [U] (the default
 * Mod1Type; bootstrapper.go:33-38 leaves it at its default): a cos(2 pi (x -
 * 1/4) / 2^r), a = (2 pi)^(-1/2^r), interpolated at nodes on the integers
 * i in [-(K-1), K-1] the ModRaise overflow takes -- d_i Chebyshev nodes of the
 * first kind within dev = 2^-LogMessageRatio of i (i itself when d_i = 1), one
 * per integer and the remaining degree + 1 - (2K - 1) handed out greedily to
 * the largest bound dev^d_i / 2^(d_i - 1) prod_{j != i} |i - j|^d_j -- as
 * Chebyshev coefficients of u = x / K on [-1, 1].  Computed here in binary128
 * by Newton's divided differences and a change of basis (the library solves
 * the interpolation system instead, hostmath.cpp cos_discrete_cheb). */
typedef __float128 q128;
static const q128 Q_PI = (q128)3.141592653589793 + (q128)1.2246467991473532e-16 + (q128)-2.9947698097183397e-33;
static q128 q_cos(q128 x) { /* reduce into [-pi, pi], then Taylor */
  const long double k = roundl((long double)(x / (2 * Q_PI)));
  x -= (q128)k * 2 * Q_PI;
  q128 x2 = x * x, t = 1, s = 1;
  for (int i = 1; i < 60; i++) {
    t = -t * x2 / (q128)((2 * i - 1) * (2 * i));
    s += t;
    if ((t < 0 ? -t : t) < (q128)ldexpl(1.0L, -124)) break;
  }
  return s;
}
static q128 q_sqrt(q128 v) {
  q128 y = (q128)sqrtl((long double)v);
  for (int i = 0; i < 3; i++) y = (y + v / y) / 2;
  return y;
}
void oracle_btp_cos(int K, int degree, int r, long double *c) {
  const int n = degree + 1;
  const double dev = ldexp(1.0, -BTP_LOGMSG);
  int *d = (int *)malloc(sizeof(int) * K);
  for (int i = 0; i < K; i++) d[i] = 1;
  int tot = 2 * K - 1;
  while (tot < n) {
    int best = -1;
    long double bb = 0;
    for (int i = 0; i < K; i++) {
      if (i > 0 && tot + 2 > n) continue;
      long double lb = d[i] * log2l((long double)dev) - (d[i] - 1);
      for (int j = -(K - 1); j < K; j++)
        if (j != i) lb += d[j < 0 ? -j : j] * log2l((long double)(i > j ? i - j : j - i));
      if (best < 0 || lb > bb) best = i, bb = lb;
    }
    d[best] += 1;
    tot += best == 0 ? 1 : 2;
  }
  q128 *x = (q128 *)malloc(sizeof(q128) * n), *g = (q128 *)malloc(sizeof(q128) * n);
  int m = 0;
  for (int i = -(K - 1); i < K && m < n; i++) {
    const int di = d[i < 0 ? -i : i];
    for (int j = 0; j < di; j++)
      x[m++] = di == 1 ? (q128)i : (q128)i + (q128)dev * q_cos(Q_PI * (q128)(2 * j + 1) / (q128)(2 * di));
  }
  q128 a = 1 / (2 * Q_PI);
  for (int i = 0; i < r; i++) a = q_sqrt(a);
  for (int k = 0; k < n; k++) g[k] = a * q_cos(2 * Q_PI * (x[k] - (q128)0.25) / (q128)(1 << r));
  /* divided differences: g[k] = f[x_0 .. x_k] */
  for (int lvl = 1; lvl < n; lvl++)
    for (int k = n - 1; k >= lvl; k--) g[k] = (g[k] - g[k - 1]) / (x[k] - x[k - lvl]);
  /* Horner in the Chebyshev basis of u = x / K: P <- P (K u - x_k) + g_k,
   * u T_0 = T_1, u T_j = (T_{j+1} + T_{j-1}) / 2 */
  q128 *P = (q128 *)calloc(n + 1, sizeof(q128)), *T = (q128 *)calloc(n + 1, sizeof(q128));
  P[0] = g[n - 1];
  for (int k = n - 2; k >= 0; k--) {
    for (int j = 0; j <= n; j++) T[j] = 0;
    for (int j = 0; j < n - 1 - k; j++) { /* K u P */
      if (j == 0) {
        T[1] += (q128)K * P[0];
      } else {
        T[j + 1] += (q128)K * P[j] / 2;
        T[j - 1] += (q128)K * P[j] / 2;
      }
    }
    for (int j = 0; j < n - 1 - k; j++) T[j] -= x[k] * P[j];
    T[0] += g[k];
    for (int j = 0; j <= n; j++) P[j] = T[j];
  }
  for (int j = 0; j < n; j++) c[j] = (long double)P[j];
  free(d), free(x), free(g), free(P), free(T);
}

/* a diagonal map: offset (mod n slots) -> n complex values, NULL if absent;
 * walked in ascending offset order */
typedef struct {
  int n;
  cplx **d;
} dmap;
static dmap dm_new(int n) {
  dmap m = {n, (cplx **)calloc(n, sizeof(cplx *))};
  return m;
}
static cplx *dm_at(dmap *m, int off) {
  if (!m->d[off]) m->d[off] = (cplx *)calloc(m->n, sizeof(cplx));
  return m->d[off];
}
static void dm_free(dmap *m) {
  for (int i = 0; i < m->n; i++) free(m->d[i]);
  free(m->d);
  m->d = NULL;
}
/* the special FFT's twiddles for ns slots (SpecialFFT / SpecialiFFT):
 * tw[h + j] = roots[(rot[j] mod 4 len) M / (4 len)] (forward) or
 * roots[(4 len - rot[j] mod 4 len) M / (4 len)] (inverse), len = 2h, M = 4 ns */
static cplx *btp_twiddles(int ns, int inverse) {
  const int M = 4 * ns;
  int *rot;
  cplx *roots;
  special_tables(ns, M, &rot, &roots);
  cplx *tw = (cplx *)calloc(ns, sizeof(cplx));
  for (int h = 1; h < ns; h <<= 1) {
    const int lq = h << 3, gap = M / lq;
    for (int j = 0; j < h; j++) tw[h + j] = roots[(inverse ? lq - rot[j] % lq : rot[j] % lq) * gap];
  }
  free(rot);
  free(roots);
  return tw;
}
/* one butterfly stage of length len as diagonals on n slots: forward
 * (x_p + w x_{p+h}, x_{p-h} - w x_p), inverse (x_p + x_{p+h}, (x_{p-h} - x_p) w) */
static dmap btp_stage(int n, int len, int inverse, const cplx *tw) {
  const int h = len / 2;
  dmap m = dm_new(n);
  cplx *d0 = dm_at(&m, 0), *dp = dm_at(&m, h), *dn = dm_at(&m, n - h);
  for (int p = 0; p < n; p++) {
    const int j = p & (len - 1);
    if (j < h) {
      cplx w = tw[h + j];
      if (inverse) w.re = 1, w.im = 0;
      d0[p].re += 1.0;
      dp[p].re += w.re;
      dp[p].im += w.im;
    } else {
      const cplx w = tw[j];
      if (inverse) {
        dn[p].re += w.re;
        dn[p].im += w.im;
      } else {
        dn[p].re += 1.0;
      }
      d0[p].re -= w.re;
      d0[p].im -= w.im;
    }
  }
  return m;
}
/* A o B (B applied first): C[a + b] += A[a][p] B[b][p + a], offsets ascending */
static dmap btp_compose(const dmap *A, const dmap *B) {
  const int n = A->n;
  dmap C = dm_new(n);
  for (int a = 0; a < n; a++) {
    if (!A->d[a]) continue;
    for (int b = 0; b < n; b++) {
      if (!B->d[b]) continue;
      cplx *c = dm_at(&C, (a + b) % n);
      const cplx *x = A->d[a], *y = B->d[b];
      for (int p = 0; p < n; p++) {
        const cplx t = cmul(x[p], y[(p + a) % n]);
        c[p].re += t.re;
        c[p].im += t.im;
      }
    }
  }
  return C;
}
/* the stages of the ns-point transform in application order, over ng
 * transforms, the extra stages to the first ones */
static int btp_groups(int ns, int inverse, int ng, int lens[][16], int *cnt) {
  int all[32], tot = 0;
  if (inverse)
    for (int len = ns; len >= 2; len /= 2) all[tot++] = len;
  else
    for (int len = 2; len <= ns; len *= 2) all[tot++] = len;
  int at = 0;
  for (int k = 0; k < ng; k++) {
    cnt[k] = tot / ng + (k < tot % ng ? 1 : 0);
    for (int i = 0; i < cnt[k]; i++) lens[k][i] = all[at++];
  }
  return tot;
}

typedef struct {
  int level, n1, nd;
  int *idx;
  u64 **pts; /* [level+1+K][N] QP plaintexts, pre-rotated by the giant step */
} btp_lt;

struct oracle_btp_circuit {
  int slots, gap, K, r, degree, top, log_scale;
  u64 F;
  long double cos[BTP_DEG + 1], dac[BTP_R], t0, s_y;
  btp_lt lt[BTP_CTS + BTP_STC]; /* CoeffsToSlots, then SlotsToCoeffs */
  int ntrace;
  u64 trace[32];
  u64 *mono_i; /* X^(N/2) over the Q limbs (NTT), full slots only */
};

/* complex values on the N/2 slots encoded at scale over the limbs mods
 * (encoder.go Encode of a complex vector; oracle_encode's real-valued path
 * with the imaginary parts kept) */
static void encode_cplx(const oracle_ctx *c, const cplx *vals, double scale, const int *mods, int nm, u64 *out) {
  const int N = c->N, n = N / 2, M = 4 * n;
  int *rot;
  cplx *roots;
  special_tables(n, M, &rot, &roots);
  cplx *v = (cplx *)malloc(sizeof(cplx) * n);
  memcpy(v, vals, sizeof(cplx) * n);
  special_ifft(v, n, M, rot, roots);
  for (int i = 0; i < n; i++) {
    to_crt(v[i].re, scale, c, mods, nm, out + i, (size_t)N);
    to_crt(v[i].im, scale, c, mods, nm, out + i + n, (size_t)N);
  }
  for (int m = 0; m < nm; m++) oracle_ntt(c, mods[m], out + (size_t)m * N);
  free(v);
  free(rot);
  free(roots);
}

/* a BSGS transform from a diagonal map: N1 (FindBestBSGSRatio, LogBSGSRatio
 * 1), each diagonal rotated by minus its giant step and encoded at scale
 * q_level over QP (lineartransform.go:61-68's Encode, restated) */
static void btp_make_lt(const oracle_ctx *bc, const dmap *m, int level, btp_lt *T) {
  const int N = bc->N, n = N / 2, K = bc->K;
  T->level = level;
  T->nd = 0;
  T->idx = (int *)malloc(sizeof(int) * n);
  for (int off = 0; off < n; off++)
    if (m->d[off]) T->idx[T->nd++] = off;
  T->n1 = oracle_find_best_bsgs_n1(T->idx, T->nd, n, BTP_LOGBSGS);
  T->pts = (u64 **)malloc(sizeof(u64 *) * T->nd);
  int mods[MAXMOD], nm = 0;
  for (int j = 0; j <= level; j++) mods[nm++] = j;
  for (int k = 0; k < K; k++) mods[nm++] = bc->L + k;
  cplx *vec = (cplx *)malloc(sizeof(cplx) * n);
  for (int d = 0; d < T->nd; d++) {
    int gi, bi;
    bsgs_split(T->idx[d], n, T->n1, &gi, &bi);
    const cplx *src = m->d[T->idx[d]];
    for (int s = 0; s < n; s++) vec[s] = src[((s - gi) % n + n) % n];
    T->pts[d] = (u64 *)malloc(sizeof(u64) * (size_t)nm * N);
    encode_cplx(bc, vec, (double)bc->mod[level], mods, nm, T->pts[d]);
  }
  free(vec);
}

oracle_btp_circuit *oracle_btp_new(const oracle_ctx *bc, int log_scale, int slots) {
  const int N = bc->N, n = N / 2;
  if (bc->ci || slots < 2 || slots > n || (slots & (slots - 1))) return NULL;
  if (bc->L < BTP_CTS + BTP_DEPTH + BTP_R + BTP_STC + 1) return NULL;
  oracle_btp_circuit *C = (oracle_btp_circuit *)calloc(1, sizeof(oracle_btp_circuit));
  C->slots = slots;
  C->gap = n / slots;
  C->K = BTP_K;
  C->r = BTP_R;
  C->degree = BTP_DEG;
  C->log_scale = log_scale;
  C->top = bc->L - 1;
  oracle_btp_cos(C->K, C->degree, C->r, C->cos);
  {
    long double v = powl(2 * BTP_PI, -1.0L / (long double)(1 << C->r));
    for (int i = 0; i < C->r; i++) C->dac[i] = v = v * v;
  }
  {
    const long double f = roundl((long double)bc->mod[0] / ldexpl(1.0L, BTP_LOGMSG + log_scale));
    C->F = f < 1 ? 1 : (u64)f;
  }
  for (int s = slots; s < n; s *= 2) C->trace[C->ntrace++] = oracle_galois_element(bc, s);
  const int packed = slots < n;
  int lens[8][16], cnt[8];
  /* CoeffsToSlots: 2^-s and the 4th root of 1 / (2K) per transform */
  {
    cplx *twi = btp_twiddles(slots, 1);
    btp_groups(slots, 1, BTP_CTS, lens, cnt);
    const double kf = sqrt(sqrt(1.0 / (2.0 * C->K)));
    int level = C->top;
    for (int k = 0; k < BTP_CTS; k++) {
      dmap M = dm_new(n);
      cplx *m0 = dm_at(&M, 0);
      for (int p = 0; p < n; p++) m0[p].re = ldexp(kf, -cnt[k]), m0[p].im = 0;
      for (int i = 0; i < cnt[k]; i++) {
        dmap S = btp_stage(n, lens[k][i], 1, twi);
        dmap X = btp_compose(&S, &M);
        dm_free(&S);
        dm_free(&M);
        M = X;
      }
      if (packed && k == BTP_CTS - 1) { /* a = 1 on [0, n), -i on [n, 2n) of every 2n-period */
        dmap A = dm_new(n);
        cplx *a0 = dm_at(&A, 0);
        for (int p = 0; p < n; p++) {
          const int lo = (p % (2 * slots)) < slots;
          a0[p].re = lo ? 1 : 0;
          a0[p].im = lo ? 0 : -1;
        }
        dmap X = btp_compose(&A, &M);
        dm_free(&A);
        dm_free(&M);
        M = X;
      }
      btp_make_lt(bc, &M, level--, &C->lt[k]);
      dm_free(&M);
    }
    free(twi);
  }
  /* EvalMod scales: t0 such that the r double angles end on 2^60 */
  const int lp = C->top - BTP_CTS - BTP_DEPTH;
  {
    long double T = ldexpl(1.0L, BTP_MOD_BITS);
    for (int i = C->r - 1; i >= 0; i--) T = sqrtl(T * (long double)bc->mod[lp - i]);
    C->t0 = T;
    long double sc = T;
    for (int i = 0; i < C->r; i++) sc = sc * sc / (long double)bc->mod[lp - i];
    C->s_y = sc;
  }
  /* SlotsToCoeffs: forward stages times the cube root of q0 / (F s_y) each */
  {
    cplx *twf = btp_twiddles(slots, 0);
    btp_groups(slots, 0, BTP_STC, lens, cnt);
    const double cf = cbrt((double)((long double)bc->mod[0] / ((long double)C->F * C->s_y)));
    int level = lp - C->r;
    for (int k = 0; k < BTP_STC; k++) {
      dmap M = dm_new(n);
      if (packed && k == 0) { /* unpack real + i imag */
        cplx *m0 = dm_at(&M, 0), *m1 = dm_at(&M, slots);
        for (int p = 0; p < n; p++) {
          const int lo = (p % (2 * slots)) < slots;
          m0[p].re = lo ? cf : 0, m0[p].im = lo ? 0 : cf;
          m1[p].re = lo ? 0 : cf, m1[p].im = lo ? cf : 0;
        }
      } else {
        cplx *m0 = dm_at(&M, 0);
        for (int p = 0; p < n; p++) m0[p].re = cf, m0[p].im = 0;
      }
      for (int i = 0; i < cnt[k]; i++) {
        dmap S = btp_stage(n, lens[k][i], 0, twf);
        dmap X = btp_compose(&S, &M);
        dm_free(&S);
        dm_free(&M);
        M = X;
      }
      btp_make_lt(bc, &M, level--, &C->lt[BTP_CTS + k]);
      dm_free(&M);
    }
    free(twf);
  }
  if (!packed) { /* X^(N/2) */
    C->mono_i = (u64 *)calloc((size_t)bc->L * N, sizeof(u64));
    for (int l = 0; l < bc->L; l++) {
      C->mono_i[(size_t)l * N + N / 2] = 1;
      oracle_ntt(bc, l, C->mono_i + (size_t)l * N);
    }
  }
  return C;
}

void oracle_btp_free(oracle_btp_circuit *C) {
  if (!C) return;
  for (int k = 0; k < BTP_CTS + BTP_STC; k++) {
    for (int d = 0; d < C->lt[k].nd; d++) free(C->lt[k].pts[d]);
    free(C->lt[k].pts);
    free(C->lt[k].idx);
  }
  free(C->mono_i);
  free(C);
}

int oracle_btp_params(const oracle_btp_circuit *C, long double *out) {
  const long double v[] = {(long double)C->F, (long double)C->gap, (long double)C->K, (long double)C->r,
                           (long double)C->degree, (long double)C->slots, C->s_y, (long double)C->top,
                           (long double)C->ntrace, (long double)(BTP_CTS + BTP_STC), (long double)(C->degree + 1),
                           C->t0};
  const int cnt = (int)(sizeof(v) / sizeof(v[0]));
  if (out) memcpy(out, v, sizeof(v));
  return cnt;
}
int oracle_btp_lt_info(const oracle_btp_circuit *C, int k, int *level, int *n1, int *idx) {
  if (k < 0 || k >= BTP_CTS + BTP_STC) return -1;
  *level = C->lt[k].level;
  *n1 = C->lt[k].n1;
  if (idx) memcpy(idx, C->lt[k].idx, sizeof(int) * C->lt[k].nd);
  return C->lt[k].nd;
}
const u64 *oracle_btp_lt_diag(const oracle_btp_circuit *C, int k, int j) {
  if (k < 0 || k >= BTP_CTS + BTP_STC || j < 0 || j >= C->lt[k].nd) return NULL;
  return C->lt[k].pts[j];
}
const long double *oracle_btp_cos_of(const oracle_btp_circuit *C) { return C->cos; }

static const u64 *btp_key(const oracle_btp *P, u64 g) {
  for (int i = 0; i < P->ngk; i++)
    if (P->galEls[i] == g) return P->gks[i];
  return NULL;
}
/* sigma_g of a [2][level+1][N] ciphertext; returns -1 without a key */
static int btp_galois(const oracle_ctx *bc, const oracle_btp *P, pct *a, u64 g) {
  const u64 *gk = btp_key(P, g);
  if (!gk) return -1;
  pct o = pct_alloc(bc, a->level, a->scale);
  oracle_rotate(bc, a->level, a->v, g, gk, o.v);
  free(a->v);
  *a = o;
  return 0;
}
static pct pct_clone(const oracle_ctx *c, const pct *a) {
  pct o = pct_alloc(c, a->level, a->scale);
  memcpy(o.v, a->v, sizeof(u64) * 2 * (size_t)(a->level + 1) * c->N);
  return o;
}
/* a (+ or -) b at a's level and scale */
static void pct_addsub(const oracle_ctx *c, pct *a, const pct *b, int sub) {
  const size_t P = (size_t)(a->level + 1) * c->N, B = (size_t)(b->level + 1) * c->N;
  for (int comp = 0; comp < 2; comp++)
    for (int l = 0; l <= a->level; l++)
      for (int i = 0; i < c->N; i++) {
        u64 *x = a->v + comp * P + (size_t)l * c->N + i;
        const u64 y = b->v[comp * B + (size_t)l * c->N + i];
        *x = sub ? submod(*x, y, c->mod[l]) : addmod(*x, y, c->mod[l]);
      }
}
static void pct_mul_pt(const oracle_ctx *c, pct *a, const u64 *pt) {
  const size_t P = (size_t)(a->level + 1) * c->N;
  for (int comp = 0; comp < 2; comp++)
    for (int l = 0; l <= a->level; l++)
      for (int i = 0; i < c->N; i++) {
        u64 *x = a->v + comp * P + (size_t)l * c->N + i;
        *x = mulmod(*x, pt[(size_t)l * c->N + i], c->mod[l]);
      }
}
static int btp_lt_rescale(const oracle_ctx *bc, const oracle_btp *P, const btp_lt *T, pct *x) {
  if (T->level != x->level) return -1;
  pct y = pct_alloc(bc, x->level, x->scale);
  oracle_lt_bsgs(bc, x->level, x->v, T->nd, T->idx, (const u64 *const *)T->pts, T->n1, P->ngk, P->galEls, P->gks,
                 y.v);
  free(x->v);
  const long double s = x->scale;
  *x = y;
  pct_rescale(bc, x);
  x->scale = s; /* diagonals at scale q_level: the rescale restores the input scale */
  return 0;
}
static int btp_eval_mod(const oracle_ctx *bc, const oracle_btp_circuit *C, const oracle_btp *P, const pct *u, pct *y) {
  pct o = pct_alloc(bc, u->level, 0);
  long double sc = 0;
  const int lv = oracle_eval_poly_ld(bc, u->level, u->v, u->scale, C->cos, C->degree + 1, 1, C->t0, P->rlk, o.v, &sc);
  if (lv < 0) {
    free(o.v);
    return -1;
  }
  pct t = pct_alloc(bc, lv, sc);
  memcpy(t.v, o.v, sizeof(u64) * 2 * (size_t)(lv + 1) * bc->N);
  free(o.v);
  u64 k[MAXMOD];
  for (int j = 0; j < C->r; j++) { /* y <- 2 y^2 - a^(2^(j+1)), then the rescale */
    pct s2 = pct_mul_relin(bc, &t, &t, P->rlk);
    free(t.v);
    const size_t L = (size_t)(s2.level + 1) * bc->N;
    for (size_t i = 0; i < 2 * L; i++) {
      const int l = (int)((i % L) / bc->N);
      s2.v[i] = addmod(s2.v[i], s2.v[i], bc->mod[l]);
    }
    big_const_res(bc, -C->dac[j] * s2.scale, s2.level, k);
    for (int l = 0; l <= s2.level; l++)
      for (int i = 0; i < bc->N; i++) s2.v[(size_t)l * bc->N + i] = addmod(s2.v[(size_t)l * bc->N + i], k[l], bc->mod[l]);
    pct_rescale(bc, &s2);
    t = s2;
  }
  *y = t;
  return 0;
}

int oracle_bootstrap(const oracle_ctx *sc, const oracle_ctx *bc, const oracle_btp_circuit *C, const oracle_btp *P,
                     int level, long double scale, const u64 *ct, u64 *out, long double *out_scale) {
  const int N = bc->N, Ls = sc->L, top = bc->L - 1;
  if (sc->N != N || sc->mod[0] != bc->mod[0] || C->top != top) return -1;
  if (!P->d2s || !P->s2d || !P->rlk) return -1;
  const u64 q0 = bc->mod[0];
  /* ScaleDown (Lattigo ScaleDown [U]): F = round(q0 / (2^LogMessageRatio
   * scale)) from the input's own scale, so the message sits 2^-8 below q0
   * whatever its scale; the circuit's SlotsToCoeffs constant carries the
   * default scale's F, so the output scale is scale F / C->F (the input scale
   * exactly when it is the default) */
  const long double fr = roundl((long double)q0 / ldexpl(scale, BTP_LOGMSG));
  const u64 F = fr < 1 ? 1 : (u64)fr;
  if (out_scale) *out_scale = scale * (long double)F / (long double)C->F;
  u64 *x = (u64 *)malloc(sizeof(u64) * 2 * N);
  for (int comp = 0; comp < 2; comp++)
    for (int i = 0; i < N; i++) x[(size_t)comp * N + i] = mulmod(ct[(size_t)comp * (level + 1) * N + i], F % q0, q0);
  /* EvkDenseToSparse at level 0 */
  {
    u64 *k0 = (u64 *)malloc(sizeof(u64) * N), *k1 = (u64 *)malloc(sizeof(u64) * N);
    oracle_keyswitch(bc, 0, x + N, P->d2s, k0, k1);
    for (int i = 0; i < N; i++) {
      x[i] = addmod(x[i], k0[i], q0);
      x[N + i] = k1[i];
    }
    free(k0);
    free(k1);
  }
  /* ModRaise: the centred lift (x > q0 / 2 is x - q0) to every Q limb */
  pct m = pct_alloc(bc, top, (long double)q0);
  for (int comp = 0; comp < 2; comp++) {
    oracle_intt(bc, 0, x + (size_t)comp * N);
    for (int l = 0; l <= top; l++) {
      const u64 q = bc->mod[l];
      u64 *o = m.v + ((size_t)comp * (top + 1) + l) * N;
      for (int i = 0; i < N; i++) {
        const u64 v = x[(size_t)comp * N + i];
        const int neg = v > (q0 >> 1);
        const u64 r = (neg ? q0 - v : v) % q;
        o[i] = neg ? (r ? q - r : 0) : r;
      }
      oracle_ntt(bc, l, o);
    }
  }
  free(x);
  /* EvkSparseToDense at the top level */
  pct t = pct_alloc(bc, top, m.scale);
  {
    const size_t PQ = (size_t)(top + 1) * N;
    oracle_keyswitch(bc, top, m.v + PQ, P->s2d, t.v, t.v + PQ);
    for (int l = 0; l <= top; l++)
      for (int i = 0; i < N; i++) {
        const size_t j = (size_t)l * N + i;
        t.v[j] = addmod(t.v[j], m.v[j], bc->mod[l]);
      }
  }
  free(m.v);
  int rc = 0;
  if (C->gap > 1) { /* trace: gap^-1 t + its rotations by slots * 2^i */
    for (int l = 0; l <= top; l++) {
      const u64 q = bc->mod[l], gi = invmod((u64)C->gap % q, q);
      for (int comp = 0; comp < 2; comp++)
        for (int i = 0; i < N; i++) {
          u64 *v = t.v + ((size_t)comp * (top + 1) + l) * N + i;
          *v = mulmod(*v, gi, q);
        }
    }
    for (int j = 0; j < C->ntrace && !rc; j++) {
      pct r = pct_clone(bc, &t);
      rc = btp_galois(bc, P, &r, C->trace[j]);
      if (!rc) pct_addsub(bc, &t, &r, 0);
      free(r.v);
    }
  }
  for (int k = 0; k < BTP_CTS && !rc; k++) rc = btp_lt_rescale(bc, P, &C->lt[k], &t); /* CoeffsToSlots */
  pct y = {0, 0, NULL};
  if (!rc) {
    pct zc = pct_clone(bc, &t);
    rc = btp_galois(bc, P, &zc, 2 * (u64)N - 1);
    if (!rc && C->gap > 1) {
      pct u = pct_clone(bc, &t);
      pct_addsub(bc, &u, &zc, 0);
      rc = btp_eval_mod(bc, C, P, &u, &y);
      free(u.v);
    } else if (!rc) {
      pct re = pct_clone(bc, &t), im = pct_clone(bc, &zc);
      pct_addsub(bc, &re, &zc, 0);
      pct_addsub(bc, &im, &t, 1);
      pct_mul_pt(bc, &im, C->mono_i);
      pct yr, yi;
      rc = btp_eval_mod(bc, C, P, &re, &yr);
      if (!rc) rc = btp_eval_mod(bc, C, P, &im, &yi);
      if (!rc) {
        pct_mul_pt(bc, &yi, C->mono_i);
        if (yr.level != yi.level) rc = -1;
        else pct_addsub(bc, &yi, &yr, 0);
        y = yi;
        free(yr.v);
      }
      free(re.v);
      free(im.v);
    }
    free(zc.v);
  }
  free(t.v);
  for (int k = 0; k < BTP_STC && !rc; k++) rc = btp_lt_rescale(bc, P, &C->lt[BTP_CTS + k], &y); /* SlotsToCoeffs */
  if (!rc && y.level != Ls - 1) rc = -1;
  if (!rc) { /* post-scale gap (Orion bootstrapper.go:73-74), on the scheme's primes */
    for (int comp = 0; comp < 2; comp++)
      for (int l = 0; l < Ls; l++) {
        const u64 q = bc->mod[l], g = (u64)C->gap % q;
        for (int i = 0; i < N; i++)
          out[((size_t)comp * Ls + l) * N + i] = mulmod(y.v[((size_t)comp * (y.level + 1) + l) * N + i], g, q);
      }
  }
  free(y.v);
  return rc;
}
