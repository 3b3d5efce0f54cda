/*
 * ckks_oracle.h -- CPU restatement of the RNS-CKKS arithmetic that Orion's
 * Lattigo backend reaches (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity oracle for the HIP backend in orion_amd/.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * It is never linked into liborion_hip.so and never used as a fallback.
 *
 * Reference call sites it restates (all under /root/reference):
 *   orion/backend/lattigo/scheme.go:57-65     ckks.NewParametersFromLiteral (primes, NTT tables)
 *   orion/backend/lattigo/evaluator.go:61-99  Rotate/RotateNew/Rescale/RescaleNew
 *   orion/backend/lattigo/evaluator.go:101-294 scalar / plaintext / ciphertext add, sub, mul
 *   orion/backend/lattigo/evaluator.go:297-317 MulRelinCiphertext(New)
 *   orion/backend/lattigo/lineartransform.go:37-113 Generate/EvaluateLinearTransform (BSGS)
 *   orion/backend/lattigo/encoder.go:16-42    Encode/Decode
 * The algorithms themselves live in github.com/baahl-nyu/lattigo/v6 v6.2.0
 * (go.mod:5), which is NOT vendored in the reference and cannot be built here
 * (no Go toolchain).  This file restates Lattigo v6's published algorithms
 * (SURVEY.md Appendix A).  PARITY WITH LATTIGO ITSELF IS UNPINNED: the
 * reference holds no golden vectors for this path.  The
 * oracle is pinned by first-principles big-integer KATs (tests/golden/).
 *
 * Conventions shared with the HIP backend:
 *   - a polynomial is limb-major u64[nlimbs][N], every residue fully reduced;
 *   - NTT domain = Lattigo's: natural-order input, bit-reversed output,
 *     out[j] = a(psi^(2*brv(j)+1)) mod q, psi = g^((q-1)/2N), g the smallest
 *     primitive root of q;
 *   - QP moduli array = [q_0 .. q_{L-1}, p_0 .. p_{K-1}].
 */
#ifndef CKKS_ORACLE_H
#define CKKS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_ctx oracle_ctx;

/* Prime chain generation (Lattigo ckks GenModuli restated).
 * out must hold lenQ+lenP entries.  Returns 0 on success. */
int oracle_gen_moduli(int logN, const int *logQ, int lenQ, const int *logP,
                      int lenP, uint64_t *out);

oracle_ctx *oracle_new(int logN, const uint64_t *moduli, int L, int K);
/* ci = 1: Lattigo's ConjugateInvariant ring of degree 2^logN (NthRoot 4N,
 * N real slots; scheme.go:49-52); moduli must be 1 mod 4N */
oracle_ctx *oracle_new_ring(int logN, const uint64_t *moduli, int L, int K, int ci);
int oracle_is_ci(const oracle_ctx *ctx);
void oracle_free(oracle_ctx *ctx);
int oracle_N(const oracle_ctx *ctx);

/* NTT tables (for KATs): psi of modulus m, and the bit-reversed root table. */
uint64_t oracle_psi(const oracle_ctx *ctx, int m);
uint64_t oracle_primitive_root(uint64_t q);

/* In-place NTT / INTT of one limb under modulus index m. */
void oracle_ntt(const oracle_ctx *ctx, int m, uint64_t *a);
void oracle_intt(const oracle_ctx *ctx, int m, uint64_t *a);

/* Basis extension (Lattigo ModUpExact / reconstructRNS): x holds ns
 * coefficient-domain limbs (moduli src[0..ns)); writes nt limbs (moduli
 * dst[0..nt)) to out.  The quotient v is Lattigo's float64 sum of correctly
 * rounded divisions y_i / s_i in source order, truncated. */
void oracle_basis_extend(const oracle_ctx *ctx, const uint64_t *x,
                         const int *src, int ns, uint64_t *out,
                         const int *dst, int nt);
/* ModUp of one gadget digit (Lattigo Decomposer.DecomposeAndSplit): as
 * oracle_basis_extend, except that a single-prime digit (ns == 1) extends
 * its centered representative (x >= s >> 1 becomes x - s). */
void oracle_modup_digit(const oracle_ctx *ctx, const uint64_t *x,
                        const int *src, int ns, uint64_t *out,
                        const int *dst, int nt);

/* Rescale (DivRoundByLastModulusNTT): ct has ncomp components, each
 * [level+1][N] (NTT).  out gets [level][N] per component. */
void oracle_rescale(const oracle_ctx *ctx, int level, int ncomp,
                    const uint64_t *ct, uint64_t *out);

/* ModDown QP->Q of one poly: x is [level+1 + K][N] (Q limbs then P limbs,
 * NTT).  out is [level+1][N] = floor(x / P). */
void oracle_moddown(const oracle_ctx *ctx, int level, const uint64_t *x,
                    uint64_t *out);

/* Hybrid gadget product, lazy (no ModDown).  c: [level+1][N] NTT.
 * evk: [dnum][2][L+K][N] (NTT), dnum = ceil(L/K).
 * out0/out1: [level+1+K][N] in QP. */
void oracle_gadget_product_lazy(const oracle_ctx *ctx, int level,
                                const uint64_t *c, const uint64_t *evk,
                                uint64_t *out0, uint64_t *out1);
/* Same, followed by ModDown -> out0/out1 [level+1][N]. */
void oracle_keyswitch(const oracle_ctx *ctx, int level, const uint64_t *c,
                      const uint64_t *evk, uint64_t *out0, uint64_t *out1);

/* Galois element for a rotation by k slots (Standard ring): 5^k mod 2N. */
uint64_t oracle_galois_element(const oracle_ctx *ctx, int k);
/* NTT-domain automorphism: out[j] = in[index_g[j]] for nlimbs limbs. */
void oracle_automorphism_ntt(const oracle_ctx *ctx, uint64_t galEl,
                             const uint64_t *in, uint64_t *out, int nlimbs);

/* ct x ct with relinearisation (tensor + gadget product with rlk). a, b, out
 * are [2][level+1][N].  rlk layout as evk. */
void oracle_mul_relin(const oracle_ctx *ctx, int level, const uint64_t *a,
                      const uint64_t *b, const uint64_t *rlk, uint64_t *out);
/* Rotation: keyswitch c1 with gk, add c0, then automorphism. */
void oracle_rotate(const oracle_ctx *ctx, int level, const uint64_t *ct,
                   uint64_t galEl, const uint64_t *gk, uint64_t *out);

/* BSGS linear transform (lintrans MultiplyByDiagMatrixBSGS restated).
 *   ndiag diagonals, diag_idx[d] in [0, slots), pts[d] = [level+1+K][N]
 *   pre-rotated QP plaintexts (NTT), N1 baby-step size.
 *   gk_for(galEl) resolved through the (galEls, gks) table of ngk keys.
 * out: [2][level+1][N]. */
void oracle_lt_bsgs(const oracle_ctx *ctx, int level, const uint64_t *ct,
                    int ndiag, const int *diag_idx, const uint64_t *const *pts,
                    int N1, int ngk, const uint64_t *galEls,
                    const uint64_t *const *gks, uint64_t *out);
/* Lattigo FindBestBSGSRatio / BSGSIndex helpers. */
int oracle_find_best_bsgs_n1(const int *diag_idx, int ndiag, int slots,
                             int logMaxRatio);

/* ---- encoder (Standard ring, slots = N/2) ---- */
/* values: nvals <= N/2 reals (zero padded).  Encodes at scale into the limbs
 * listed in mods (NTT domain). */
void oracle_encode(const oracle_ctx *ctx, const double *values, int nvals,
                   double scale, const int *mods, int nmods, uint64_t *out);
/* Decode a [level+1][N] NTT plaintext at scale: writes N/2 reals. */
void oracle_decode(const oracle_ctx *ctx, int level, const uint64_t *pt,
                   double scale, double *values);

/* ---- test-only key generation (seeded, NOT the product keygen) ---- */
/* sk: [L+K][N] NTT ternary secret with Hamming weight h. */
void oracle_gen_secret(const oracle_ctx *ctx, uint64_t seed, int h,
                       uint64_t *sk);
/* evk switching s_in -> s_out: [dnum][2][L+K][N]. */
void oracle_gen_evk(const oracle_ctx *ctx, uint64_t seed, const uint64_t *s_in,
                    const uint64_t *s_out, uint64_t *evk);
/* Encrypt (secret key) a [level+1][N] NTT plaintext. */
void oracle_encrypt_sk(const oracle_ctx *ctx, uint64_t seed, int level,
                       const uint64_t *sk, const uint64_t *pt, uint64_t *ct);
void oracle_decrypt(const oracle_ctx *ctx, int level, const uint64_t *sk,
                    const uint64_t *ct, uint64_t *pt);

/* ---- public-key encryption sampler of the HIP backend (encoder.hip) ----
 * ChaCha20 block function (RFC 8439 §2.3); key from the scheme seed;
 * discrete Gaussian cumulative table (2 bound entries); samples of one
 * component (0 = u ternary, 1 = e0, 2 = e1) of one image; and
 * c0 = u pk0 + e0 + pt, c1 = u pk1 + e1 (pk: [2][L+K][N], ct: [2][level+1][N]). */
void oracle_chacha20_block(const uint32_t key[8], uint32_t counter,
                           const uint32_t nonce[3], uint32_t out[16]);
void oracle_enc_key(uint64_t seed, uint32_t key[8]);
void oracle_gauss_cdt(double sigma, int bound, uint64_t *t);
void oracle_enc_sample(int N, const uint32_t key[8], uint32_t enc, uint32_t image,
                       int comp, int64_t *out);
void oracle_encrypt_pk(const oracle_ctx *ctx, const uint32_t key[8], uint32_t enc,
                       uint32_t image, int level, const uint64_t *pk,
                       const uint64_t *pt, uint64_t *ct);

/* ---- polynomial evaluation: Lattigo v6 he.EvaluatePolynomial restated
 * (power basis + the recursePS Paterson-Stockmeyer tree and its scale rules,
 * as backend.hip eval_poly; parity with Lattigo itself unpinned) ----
 * p(x) (monomial or Chebyshev basis, coefficients lowest degree first) of a
 * [2][level+1][N] ciphertext at scale xscale; writes [2][out_level+1][N] at
 * scale *out_scale (= target) and returns out_level = level - bitlen(n-1),
 * or -1 when level < bitlen(n-1).  rlk layout as evk. */
int oracle_eval_poly(const oracle_ctx *ctx, int level, const uint64_t *ct,
                     long double xscale, const double *coeffs, int n, int cheb,
                     long double target, const uint64_t *rlk, uint64_t *out,
                     long double *out_scale);

int oracle_eval_poly_ldp(const oracle_ctx *ctx, int level, const uint64_t *ct,
                         const long double *xscale, const double *coeffs, int n, int cheb,
                         const long double *target, const uint64_t *rlk, uint64_t *out,
                         long double *out_scale);
int oracle_eval_poly_ld(const oracle_ctx *ctx, int level, const uint64_t *ct,
                        long double xscale, const long double *coeffs, int n, int cheb,
                        long double target, const uint64_t *rlk, uint64_t *out,
                        long double *out_scale);

/* ---- bootstrapping (bootstrapper.go:19-80 call site): Lattigo v6's default
 * bootstrapping.ParametersLiteral [U] restated, every constant, diagonal and
 * prime derived here from the parameters (nothing from the library under
 * test); the shared inputs are the keys and the input ciphertext.
 * sc: the scheme's context; bc: the bootstrapping chain (its first L_sc Q
 * primes are the scheme's). ---- */
/* the bootstrapping chain: scheme Q (Lres), circuit primes, then P of logP;
 * returns the prime count (Q count = Lres + 15), -1 when a stream runs out */
int oracle_btp_chain(int logN, const uint64_t *scheme_qp, int n_scheme, int Lres, const int *logP, int lenP,
                     uint64_t *out);
/* EvalMod's Chebyshev coefficients (degree+1, lowest first) */
void oracle_btp_cos(int K, int degree, int r, long double *c);
typedef struct oracle_btp_circuit oracle_btp_circuit;
/* the circuit for `slots` slots under bc, scheme default scale 2^log_scale */
oracle_btp_circuit *oracle_btp_new(const oracle_ctx *bc, int log_scale, int slots);
void oracle_btp_free(oracle_btp_circuit *C);
/* F, gap, K, r, degree, slots, s_y, top, #trace, #transforms, degree+1, t0 */
int oracle_btp_params(const oracle_btp_circuit *C, long double *out);
const long double *oracle_btp_cos_of(const oracle_btp_circuit *C);
/* transform k (0..3 CoeffsToSlots, 4..6 SlotsToCoeffs): level, N1, indices;
 * returns the diagonal count; diag j: [level+1+K][N] NTT, pre-rotated */
int oracle_btp_lt_info(const oracle_btp_circuit *C, int k, int *level, int *n1, int *idx);
const uint64_t *oracle_btp_lt_diag(const oracle_btp_circuit *C, int k, int j);
/* the keys of bc (full-chain layout [dnum][2][L+K][N]) */
typedef struct oracle_btp {
  const uint64_t *rlk;
  int ngk;
  const uint64_t *galEls;
  const uint64_t *const *gks;
  const uint64_t *d2s, *s2d; /* EvkDenseToSparse (level 0), EvkSparseToDense */
} oracle_btp;
/* ct: [2][level+1][N] (scheme) at `scale`; out: [2][L_scheme][N] at the
 * residual top level, at *out_scale (= scale when it is the default scale;
 * ScaleDown's F comes from the input scale).  Returns 0, or -1 when a key is
 * missing or a level does not match. */
int oracle_bootstrap(const oracle_ctx *sc, const oracle_ctx *bc, const oracle_btp_circuit *C, const oracle_btp *P,
                     int level, long double scale, const uint64_t *ct, uint64_t *out, long double *out_scale);

/* coefficient-wise helpers used by tests */
void oracle_mul_coeffs(const oracle_ctx *ctx, const int *mods, int nl,
                       const uint64_t *a, const uint64_t *b, uint64_t *out);

#ifdef __cplusplus
}
#endif
#endif
