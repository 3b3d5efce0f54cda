// hostmath.cpp -- see hostmath.h.
#include "hostmath.h"

#include <math.h>

#include <algorithm>
#include <map>
#include <stdexcept>

namespace orion {

u64 hm_powmod(u64 b, u64 e, u64 q) {
  u64 r = 1 % q;
  b %= q;
  for (; e; e >>= 1) {
    if (e & 1) r = hm_mulmod(r, b, q);
    b = hm_mulmod(b, b, q);
  }
  return r;
}

u64 hm_bitrev(u64 x, int bits) {
  u64 r = 0;
  for (int i = 0; i < bits; ++i, x >>= 1) r = (r << 1) | (x & 1);
  return r;
}

// deterministic Miller-Rabin for 64-bit integers
static bool probably_prime(u64 n) {
  static const u64 bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return false;
  for (u64 p : bases)
    if (n % p == 0) return n == p;
  u64 d = n - 1;
  int s = 0;
  while (!(d & 1)) d >>= 1, ++s;
  for (u64 a : bases) {
    u64 x = hm_powmod(a, d, n);
    if (x == 1 || x == n - 1) continue;
    bool witness = true;
    for (int r = 1; r < s && witness; ++r) {
      x = hm_mulmod(x, x, n);
      if (x == n - 1) witness = false;
    }
    if (witness) return false;
  }
  return true;
}

// NTT-friendly prime stream around 2^bits (primes = 1 mod nthroot).  Mirrors
// Lattigo's NTTFriendlyPrimesGenerator: alternate between the next candidate
// above and below 2^bits + 1 while within half a bit of 2^bits; 61-bit
// requests walk downward only.
namespace {
struct PrimeStream {
  double size;
  u64 step, up, down;
  bool up_ok = true, down_ok = true;
  PrimeStream(int bits, u64 nthroot) : size(bits), step(nthroot), up((1ull << bits) + 1), down((1ull << bits) + 1) {}
  u64 below() {
    for (;;) {
      if (down < step) throw std::runtime_error("prime stream exhausted");
      down -= step;
      if (size - log2((double)down) >= 0.5) throw std::runtime_error("prime stream exhausted");
      if (probably_prime(down)) return down;
    }
  }
  u64 alternate() {
    for (;;) {
      if (!up_ok && !down_ok) throw std::runtime_error("prime stream exhausted");
      if (up_ok) {
        if (up > ~0ull - step || log2((double)up) - size >= 0.5) {
          up_ok = false;
        } else {
          up += step;
          if (probably_prime(up)) return up;
        }
      }
      if (down_ok) {
        if (down < step || size - log2((double)down) >= 0.5) {
          down_ok = false;
        } else {
          down -= step;
          if (probably_prime(down)) return down;
        }
      }
    }
  }
};
}  // namespace

std::vector<u64> gen_moduli(int logN, const std::vector<int>& logQ, const std::vector<int>& logP) {
  const u64 nthroot = 2ull << logN;
  std::map<int, int> need;
  for (int b : logQ) need[b]++;
  for (int b : logP) need[b]++;
  std::map<int, std::vector<u64>> pool;
  for (auto& kv : need) {
    PrimeStream ps(kv.first, nthroot);
    for (int i = 0; i < kv.second; ++i) pool[kv.first].push_back(kv.first == 61 ? ps.below() : ps.alternate());
  }
  std::map<int, size_t> used;
  std::vector<u64> out;
  for (int b : logQ) out.push_back(pool[b][used[b]++]);
  for (int b : logP) out.push_back(pool[b][used[b]++]);
  return out;
}

u64 primitive_root(u64 q) {
  std::vector<u64> fac;
  u64 m = q - 1;
  for (u64 f = 2; f * f <= m; f = (f == 2) ? 3 : f + 2) {
    if (m % f) continue;
    fac.push_back(f);
    while (m % f == 0) m /= f;
  }
  if (m > 1) fac.push_back(m);
  for (u64 g = 3;; ++g) {  // Lattigo: g starts at 2 and is incremented before the first test
    bool prim = std::all_of(fac.begin(), fac.end(), [&](u64 f) { return hm_powmod(g, (q - 1) / f, q) != 1; });
    if (prim) return g;
  }
}

// ---------------------------------------------------------------------------
// special FFT (HEAAN / Lattigo SpecialiFFT, SpecialFFT): slot j <-> X = zeta^(5^j)
// ---------------------------------------------------------------------------
SpecialFFT::SpecialFFT(int logN) : n_(1 << (logN - 1)), M_(2 << logN), rot_(n_), roots_(M_ + 1) {
  int r = 1;
  for (int i = 0; i < n_; ++i) {
    rot_[i] = r;
    r = (int)(((long)r * 5) % M_);
  }
  for (int i = 0; i <= M_; ++i) {
    double ang = 2.0 * M_PI * (double)i / (double)M_;
    roots_[i].re = cos(ang);
    roots_[i].im = sin(ang);
  }
}

void SpecialFFT::bitrev(std::vector<Cplx>& v) const {
  int logn = 0;
  while ((1 << logn) < n_) ++logn;
  for (int i = 0; i < n_; ++i) {
    int j = (int)hm_bitrev(i, logn);
    if (i < j) std::swap(v[i], v[j]);
  }
}

static inline Cplx cx_mul(const Cplx& a, const Cplx& b) {
  double ac = a.re * b.re, bd = a.im * b.im, ad = a.re * b.im, bc = a.im * b.re;
  return Cplx{ac - bd, ad + bc};
}

void SpecialFFT::inverse(std::vector<Cplx>& v) const {
  for (int len = n_; len >= 2; len >>= 1) {
    const int h = len >> 1, lq = len << 2, gap = M_ / lq;
    for (int i = 0; i < n_; i += len) {
      for (int j = 0; j < h; ++j) {
        Cplx& x = v[i + j];
        Cplx& y = v[i + j + h];
        Cplx u{x.re + y.re, x.im + y.im};
        Cplx w{x.re - y.re, x.im - y.im};
        x = u;
        y = cx_mul(w, roots_[(lq - (rot_[j] % lq)) * gap]);
      }
    }
  }
  bitrev(v);
  const double inv = 1.0 / (double)n_;
  for (auto& c : v) {
    c.re *= inv;
    c.im *= inv;
  }
}

void SpecialFFT::forward(std::vector<Cplx>& v) const {
  bitrev(v);
  for (int len = 2; len <= n_; len <<= 1) {
    const int h = len >> 1, lq = len << 2, gap = M_ / lq;
    for (int i = 0; i < n_; i += len) {
      for (int j = 0; j < h; ++j) {
        Cplx u = v[i + j];
        Cplx w = cx_mul(v[i + j + h], roots_[(rot_[j] % lq) * gap]);
        v[i + j] = Cplx{u.re + w.re, u.im + w.im};
        v[i + j + h] = Cplx{u.re - w.re, u.im - w.im};
      }
    }
  }
}

void fixed_point_crt(double v, double scale, const u64* mods, int nm, u64* out, size_t stride) {
  if (v == 0.0) {
    for (int m = 0; m < nm; ++m) out[m * stride] = 0;
    return;
  }
  const bool neg = v < 0;
  const double x = neg ? v * (-scale) : v * scale;
  if (!(x < 18446744073709551616.0)) throw std::runtime_error("encode: |value*scale| >= 2^64");
  const u64 c = (u64)(x + 0.5);
  for (int m = 0; m < nm; ++m) {
    const u64 r = c % mods[m];
    out[m * stride] = neg ? (r ? mods[m] - r : 0) : r;
  }
}

// ---------------------------------------------------------------------------
static inline u64 rotl(u64 x, int k) { return (x << k) | (x >> (64 - k)); }

Prng::Prng(u64 seed) {
  u64 z = seed;
  for (int i = 0; i < 4; ++i) {  // splitmix64 seeding
    z += 0x9E3779B97F4A7C15ull;
    u64 t = z;
    t = (t ^ (t >> 30)) * 0xBF58476D1CE4E5B9ull;
    t = (t ^ (t >> 27)) * 0x94D049BB133111EBull;
    s_[i] = t ^ (t >> 31);
  }
}

u64 Prng::next() {
  const u64 r = rotl(s_[1] * 5, 7) * 9;
  const u64 t = s_[1] << 17;
  s_[2] ^= s_[0];
  s_[3] ^= s_[1];
  s_[1] ^= s_[2];
  s_[0] ^= s_[3];
  s_[2] ^= t;
  s_[3] = rotl(s_[3], 45);
  return r;
}

u64 Prng::uniform(u64 q) {
  const int bits = 64 - __builtin_clzll(q);
  const u64 mask = bits == 64 ? ~0ull : ((1ull << bits) - 1);
  for (;;) {
    u64 r = next() & mask;
    if (r < q) return r;
  }
}

double Prng::unit() { return ((double)(next() >> 11) + 0.5) / 9007199254740992.0; }

int64_t Prng::gaussian(double sigma, double bound) {
  for (;;) {
    double z = sqrt(-2.0 * log(unit())) * cos(2.0 * M_PI * unit()) * sigma;
    if (fabs(z) <= bound) return (int64_t)llround(z);
  }
}

}  // namespace orion
