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
u64 primitive_root(u64 q);

// CKKS canonical embedding helpers (n = N/2 slots, M = 2N)
struct Cplx {
  double re, im;
};
class SpecialFFT {
 public:
  explicit SpecialFFT(int logN);
  void inverse(std::vector<Cplx>& v) const;  // slots -> coefficient pairs
  void forward(std::vector<Cplx>& v) const;  // coefficient pairs -> slots
  int n() const { return n_; }

 private:
  int n_, M_;
  std::vector<int> rot_;
  std::vector<Cplx> roots_;
  void bitrev(std::vector<Cplx>& v) const;
};

// round(|v|*scale) as Lattigo's SingleFloat64ToFixedPointCRT, then residues
void fixed_point_crt(double v, double scale, const u64* mods, int nm, u64* out, size_t stride);

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

}  // namespace orion
