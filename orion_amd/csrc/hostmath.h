// hostmath.h -- host-side setup math of the product library: NTT-friendly
// prime generation, primitive roots, CKKS special FFT, CRT helpers, seeded
// sampling.  None of this is on the per-inference hot path (it runs at
// NewScheme / Encode / keygen time); the hot path is the HIP kernels.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace orion {

typedef unsigned __int128 u128;
typedef uint64_t u64;

inline u64 hm_mulmod(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }
u64 hm_powmod(u64 b, u64 e, u64 q);
inline u64 hm_invmod(u64 a, u64 q) { return hm_powmod(a % q, q - 2, q); }
inline u64 hm_shoup(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }
u64 hm_bitrev(u64 x, int bits);

// Lattigo ckks GenModuli (Standard ring, NthRoot = 2N); throws on exhaustion
std::vector<u64> gen_moduli(int logN, const std::vector<int>& logQ, const std::vector<int>& logP);
// primes of the given bit sizes (in list order) from the same streams, none in `exclude`
std::vector<u64> gen_moduli_excluding(int logN, const std::vector<int>& bits, const std::vector<u64>& exclude);
u64 primitive_root(u64 q);

// CKKS canonical embedding helpers (n = N/2 slots, M = 2N)
struct Cplx {
  double re, im;
};
// special FFT twiddles, laid out per stage: tw[h + j] (h = half-length, j < h)
// is the factor of butterfly j of every block of length 2h; inverse = the
// conjugate-index table of SpecialiFFT, forward = SpecialFFT's (encoder.hip)
std::vector<Cplx> special_fft_twiddles(int logN, bool inverse);

// discrete Gaussian cumulative table: t[i] = floor(2^64 * P(X <= -bound + i)),
// i < 2 bound, P(x) proportional to exp(-x^2 / (2 sigma^2)) on |x| <= bound
void gauss_cdt(double sigma, int bound, u64* t);
// composite minimax sign approximation (Lattigo v6 GenMinimaxCompositePolynomial
// [U], restated in hostmath.cpp): one Chebyshev coefficient vector per degree;
// every fit absorbs a scheme error 2^-logerr, each stage but the last is
// divided by 1 + its maximum error, the last is halved and + 0.5 (orion,
// polyeval.go:136-143); stage_err (optional): each stage's maximum error
std::vector<std::vector<double>> minimax_sign_composite(const std::vector<int>& degrees, int logalpha, int logerr,
                                                        std::vector<double>* stage_err = nullptr, bool debug = false);
// 256-bit ChaCha20 key of the encryption sampler, from the scheme seed
void enc_key_from_seed(u64 seed, uint32_t key[8]);

// seeded PRNG (xoshiro256**)
class Prng {
 public:
  explicit Prng(u64 seed);
  u64 next();
  u64 uniform(u64 q);
  int64_t gaussian(double sigma, double bound);
  double unit();

 private:
  u64 s_[4];
};

// EvalMod's cosine polynomial (Lattigo v6 mod1 CosDiscrete [U], restated in
// hostmath.cpp): Chebyshev coefficients on [-1, 1] of u = x / K
std::vector<long double> cos_discrete_cheb(int K, int degree, int r, double dev);
}  // namespace orion
