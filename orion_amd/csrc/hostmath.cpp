// hostmath.cpp -- see hostmath.h.
#include "hostmath.h"

#include <math.h>

#include <algorithm>
#include <map>
#include <set>
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

// Lattigo bootstrapping.NewParametersFromLiteral: the circuit's new primes
// (and its P primes) come from the same per-bit-size streams, skipping any
// prime of the residual parameters, so the residual Q chain is kept as is
std::vector<u64> gen_moduli_excluding(int logN, const std::vector<int>& bits, const std::vector<u64>& exclude) {
  const u64 nthroot = 2ull << logN;
  std::set<u64> taken(exclude.begin(), exclude.end());
  std::map<int, PrimeStream> streams;
  std::vector<u64> out;
  for (int b : bits) {
    auto it = streams.find(b);
    if (it == streams.end()) it = streams.emplace(b, PrimeStream(b, nthroot)).first;
    u64 q;
    do {
      q = b == 61 ? it->second.below() : it->second.alternate();
    } while (taken.count(q));
    taken.insert(q);
    out.push_back(q);
  }
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
// special FFT twiddles (HEAAN / Lattigo SpecialiFFT, SpecialFFT): slot j <->
// X = zeta^(5^j); butterfly j of a block of length len = 2h uses
// roots[(rot[j] mod 4len) * M / 4len] (forward) or roots[(4len - rot[j] mod
// 4len) * M / 4len] (inverse), roots[i] = exp(2 pi i / M), M = 2N
// ---------------------------------------------------------------------------
std::vector<Cplx> special_fft_twiddles(int logN, bool inverse) {
  const int n = 1 << (logN - 1), M = 2 << logN;
  std::vector<int> rot(n);
  int r = 1;
  for (int i = 0; i < n; ++i) {
    rot[i] = r;
    r = (int)(((long)r * 5) % M);
  }
  std::vector<Cplx> roots(M + 1);
  for (int i = 0; i <= M; ++i) {
    double ang = 2.0 * M_PI * (double)i / (double)M;
    roots[i].re = cos(ang);
    roots[i].im = sin(ang);
  }
  std::vector<Cplx> tw(n, Cplx{0.0, 0.0});
  for (int h = 1; h < n; h <<= 1) {
    const int lq = h << 3, gap = M / lq;
    for (int j = 0; j < h; ++j) tw[h + j] = roots[(inverse ? lq - rot[j] % lq : rot[j] % lq) * gap];
  }
  return tw;
}

void gauss_cdt(double sigma, int bound, u64* t) {
  std::vector<double> rho(2 * bound + 1);
  double sum = 0.0;
  for (int x = -bound; x <= bound; ++x) {
    rho[x + bound] = exp(-(double)(x * x) / (2.0 * sigma * sigma));
    sum += rho[x + bound];
  }
  double acc = 0.0;
  for (int i = 0; i < 2 * bound; ++i) {
    acc += rho[i];
    const double c = ldexp(acc / sum, 64);
    t[i] = c >= 18446744073709551616.0 ? ~0ull : (u64)c;
  }
}

void enc_key_from_seed(u64 seed, uint32_t key[8]) {
  u64 z = seed ^ 0x6a09e667f3bcc909ull;
  for (int i = 0; i < 4; ++i) {  // splitmix64
    z += 0x9E3779B97F4A7C15ull;
    u64 t = z;
    t = (t ^ (t >> 30)) * 0xBF58476D1CE4E5B9ull;
    t = (t ^ (t >> 27)) * 0x94D049BB133111EBull;
    t ^= t >> 31;
    key[2 * i] = (uint32_t)t;
    key[2 * i + 1] = (uint32_t)(t >> 32);
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

namespace orion {
// ---------------------------------------------------------------------------
// composite minimax approximation of sign (polyeval.go:91-167 ->
// Lattigo minimax.GenMinimaxCompositePolynomial), restated with the classic
// Remez exchange in long double.  sign is odd, so each stage is an odd
// Chebyshev series p(x) = sum_k c_k T_{2k+1}(x) fitted to 1 on [a, 1]; every
// stage but the last is divided by its maximum on [-1, 1] (times 1 + 2^-10),
// so the next stage's inputs stay inside [-1, 1], and the next stage is
// fitted on [min over [a, 1] of the scaled stage, 1].
// ---------------------------------------------------------------------------
namespace {
typedef long double ld;

ld cheb_odd_eval(const std::vector<ld>& c, ld x) {  // sum_k c_k T_{2k+1}(x)
  ld t0 = 1, t1 = x, s = 0;
  for (size_t n = 1, k = 0; k < c.size(); ++n) {
    if (n & 1) s += c[k++] * t1;
    const ld t2 = 2 * x * t1 - t0;
    t0 = t1;
    t1 = t2;
  }
  return s;
}
ld cheb_T(int n, ld x) {
  ld t0 = 1, t1 = x;
  if (n == 0) return t0;
  for (int i = 1; i < n; ++i) {
    const ld t2 = 2 * x * t1 - t0;
    t0 = t1;
    t1 = t2;
  }
  return t1;
}
// Gaussian elimination with partial pivoting, A is n x (n+1) augmented
std::vector<ld> solve(std::vector<std::vector<ld>> A) {
  const int n = (int)A.size();
  for (int col = 0; col < n; ++col) {
    int piv = col;
    for (int r = col + 1; r < n; ++r)
      if (fabsl(A[r][col]) > fabsl(A[piv][col])) piv = r;
    std::swap(A[col], A[piv]);
    if (A[col][col] == 0) throw std::runtime_error("minimax: singular Remez system");
    for (int r = 0; r < n; ++r) {
      if (r == col) continue;
      const ld f = A[r][col] / A[col][col];
      for (int k = col; k <= n; ++k) A[r][k] -= f * A[col][k];
    }
  }
  std::vector<ld> x(n);
  for (int i = 0; i < n; ++i) x[i] = A[i][n] / A[i][i];
  return x;
}
// best odd approximation of degree <= deg of 1 on [a, 1]; returns coefficients, sets err
std::vector<ld> remez_sign(int deg, ld a, ld& err) {
  const int n = (deg - 1) / 2 + 1;  // odd terms T_1, T_3, ..., T_{2n-1}
  std::vector<ld> xs(n + 1);
  for (int i = 0; i <= n; ++i) xs[i] = (a + 1) / 2 - (1 - a) / 2 * cosl(3.14159265358979323846264338327950288L * i / n);
  std::vector<ld> c(n, 0);
  const int G = 4000 * n;
  std::vector<ld> grid(G), eg(G);
  for (int j = 0; j < G; ++j) grid[j] = (a + 1) / 2 - (1 - a) / 2 * cosl(3.14159265358979323846264338327950288L * j / (G - 1));
  ld E = 0;
  for (int it = 0; it < 100; ++it) {
    std::vector<std::vector<ld>> A(n + 1, std::vector<ld>(n + 2));
    for (int i = 0; i <= n; ++i) {
      for (int k = 0; k < n; ++k) A[i][k] = cheb_T(2 * k + 1, xs[i]);
      A[i][n] = (i & 1) ? -1 : 1;
      A[i][n + 1] = 1;
    }
    std::vector<ld> sol = solve(A);
    for (int k = 0; k < n; ++k) c[k] = sol[k];
    E = fabsl(sol[n]);
    // local extrema of e(x) = p(x) - 1 on the grid, refined by ternary search
    for (int j = 0; j < G; ++j) eg[j] = cheb_odd_eval(c, grid[j]) - 1;
    std::vector<ld> ex, ev;
    for (int j = 0; j < G; ++j) {
      const bool l = j == 0 || fabsl(eg[j]) >= fabsl(eg[j - 1]);
      const bool r = j == G - 1 || fabsl(eg[j]) >= fabsl(eg[j + 1]);
      if (!(l && r)) continue;
      ld x = grid[j];
      if (j > 0 && j < G - 1) {
        ld lo = grid[j - 1], hi = grid[j + 1];
        const ld sg = eg[j] >= 0 ? 1 : -1;
        for (int t = 0; t < 60; ++t) {
          const ld m1 = lo + (hi - lo) / 3, m2 = hi - (hi - lo) / 3;
          if (sg * (cheb_odd_eval(c, m1) - 1) < sg * (cheb_odd_eval(c, m2) - 1))
            lo = m1;
          else
            hi = m2;
        }
        x = (lo + hi) / 2;
      }
      const ld v = cheb_odd_eval(c, x) - 1;
      if (!ex.empty() && ((v >= 0) == (ev.back() >= 0))) {  // same sign: keep the larger
        if (fabsl(v) > fabsl(ev.back())) ex.back() = x, ev.back() = v;
        continue;
      }
      ex.push_back(x);
      ev.push_back(v);
    }
    while ((int)ex.size() > n + 1) {  // drop the smaller end extremum
      if (fabsl(ev.front()) < fabsl(ev.back()))
        ex.erase(ex.begin()), ev.erase(ev.begin());
      else
        ex.pop_back(), ev.pop_back();
    }
    ld emax = 0;
    for (ld v : ev) emax = std::max(emax, fabsl(v));
    err = emax;
    if ((int)ex.size() < n + 1) break;  // cannot alternate further: keep the current solution
    xs = ex;
    if (emax - E <= 1e-12L * emax) break;
  }
  return c;
}
}  // namespace

std::vector<std::vector<double>> minimax_sign_composite(const std::vector<int>& degrees, int logalpha) {
  std::vector<std::vector<double>> out;
  ld a = ldexpl(1.0L, -logalpha);
  for (size_t i = 0; i < degrees.size(); ++i) {
    const int d = degrees[i];
    if (d < 1) throw std::runtime_error("minimax: degrees must be >= 1");
    ld err = 0;
    std::vector<ld> c = remez_sign(d, a, err);
    if (!(err < 1)) throw std::runtime_error("minimax: degree too small for the interval");
    const bool last = i + 1 == degrees.size();
    // a stage's image must stay inside the next stage's Chebyshev domain for
    // every input in [-1, 1], including the gap (-a, a) it is not fitted on,
    // with room for the float32 coefficients and the homomorphic noise: scale
    // by the true maximum of |p| on [0, 1] (p is odd), times 1 + 2^-10
    ld norm = 1;
    if (!last) {
      ld mx = 0, mn_fit = 2;
      const int G = 200000;
      for (int j = 0; j <= G; ++j) {
        const ld x = (ld)j / G;
        const ld v = fabsl(cheb_odd_eval(c, x));
        mx = std::max(mx, v);
        if (x >= a) mn_fit = std::min(mn_fit, v);
      }
      norm = mx * (1 + ldexpl(1.0L, -10));
      a = mn_fit / norm;
    }
    std::vector<double> p(d + 1, 0.0);
    for (size_t k = 0; k < c.size(); ++k) p[2 * k + 1] = (double)(c[k] / norm);
    out.push_back(p);
  }
  return out;
}
}  // namespace orion
