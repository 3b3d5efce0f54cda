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
// Lattigo v6 bignum.GenMinimaxCompositePolynomial [U], restated; the fixture
// tests/golden/minimax_sign.json is the same construction at `prec` = 128
// bits in mpmath, tools/gen_minimax.py):
//   stage i: p_i = the odd minimax fit of 1 on [a_i, 1] (= the minimax
//   approximation of sign on [-1, -a_i] U [a_i, 1], whose even Chebyshev
//   coefficients vanish), degree d_i, error E_i; p_i /= 1 + E_i;
//   a_{i+1} = (1 - E_i) / (1 + E_i); a_0 = 2^-logalpha.
// The Remez exchange runs in binary128 (__float128, 113 bits: every stage's
// minimax polynomial is unique, so once converged far below float64
// resolution each coefficient rounds to the same double as the 128-bit
// computation).
// ---------------------------------------------------------------------------
namespace {
typedef __float128 qf;

qf qabs(qf x) { return x < 0 ? -x : x; }
// sum_k c_k T_{2k+1}(x) and its derivative (T_m' = m U_{m-1})
void cheb_odd_eval(const std::vector<qf>& c, qf x, qf& s, qf& ds) {
  qf t0 = 1, t1 = x, u0 = 1, u1 = 2 * x;
  s = ds = 0;
  size_t k = 0;
  for (int m = 1; k < c.size(); ++m) {
    if (m & 1) {
      s += c[k] * t1;
      ds += c[k] * m * u0;
      ++k;
    }
    const qf t2 = 2 * x * t1 - t0, u2 = 2 * x * u1 - u0;
    t0 = t1, t1 = t2, u0 = u1, u1 = u2;
  }
}
// double-binary128 (~226 bits) for the Remez linear system alone: the last
// stages fit 1 on a short interval near 1 (a = 0.952 for orion's ReLU), where
// the Chebyshev columns are nearly dependent and binary128 loses the float64
// digits of the coefficients (mpmath at 128, 192 and 256 bits agree; binary128
// alone differs in 13 of 28 doubles).  Error-free transformations (Dekker
// split at 57 bits for the 113-bit significand).
struct dq {
  qf hi, lo;
};
inline dq qsum(qf a, qf b) {
  const qf s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
inline dq qfast(qf a, qf b) {
  const qf s = a + b;
  return {s, b - (s - a)};
}
inline dq qprod(qf a, qf b) {
  const qf p = a * b, C = (qf)144115188075855873.0L;  // 2^57 + 1
  const qf ca = C * a, ah = ca - (ca - a), al = a - ah;
  const qf cb = C * b, bh = cb - (cb - b), bl = b - bh;
  return {p, ((ah * bh - p) + ah * bl + al * bh) + al * bl};
}
inline dq operator+(dq a, dq b) {
  dq s = qsum(a.hi, b.hi);
  return qfast(s.hi, s.lo + a.lo + b.lo);
}
inline dq operator-(dq a) { return {-a.hi, -a.lo}; }
inline dq operator-(dq a, dq b) { return a + (-b); }
inline dq operator*(dq a, dq b) {
  dq p = qprod(a.hi, b.hi);
  return qfast(p.hi, p.lo + a.hi * b.lo + a.lo * b.hi);
}
inline dq operator/(dq a, dq b) {
  const qf q1 = a.hi / b.hi;
  dq r = a - b * dq{q1, 0};
  const qf q2 = r.hi / b.hi;
  r = r - b * dq{q2, 0};
  const qf q3 = r.hi / b.hi;
  return qfast(q1, q2) + dq{q3, 0};
}
inline dq to_dq(qf x) { return {x, 0}; }
dq cheb_T_dq(int n, qf x) {
  const dq x2 = to_dq(2 * x);
  dq t0 = to_dq(1), t1 = to_dq(x);
  if (n == 0) return t0;
  for (int i = 1; i < n; ++i) {
    const dq t2 = x2 * t1 - t0;
    t0 = t1, t1 = t2;
  }
  return t1;
}
// Gaussian elimination with partial pivoting, A is n x (n+1) augmented
std::vector<dq> solve(std::vector<std::vector<dq>> A) {
  const int n = (int)A.size();
  for (int col = 0; col < n; ++col) {
    int piv = col;
    for (int r = col + 1; r < n; ++r)
      if (qabs(A[r][col].hi) > qabs(A[piv][col].hi)) piv = r;
    std::swap(A[col], A[piv]);
    if (A[col][col].hi == 0) throw std::runtime_error("minimax: singular Remez system");
    for (int r = col + 1; r < n; ++r) {
      const dq f = A[r][col] / A[col][col];
      for (int k = col; k <= n; ++k) A[r][k] = A[r][k] - f * A[col][k];
    }
  }
  std::vector<dq> x(n);
  for (int i = n - 1; i >= 0; --i) {
    dq v = A[i][n];
    for (int k = i + 1; k < n; ++k) v = v - A[i][k] * x[k];
    x[i] = v / A[i][i];
  }
  return x;
}
// Chebyshev-spaced point j of m on [a, 1] (the starting reference and the scan grid)
qf cheb_pt(qf a, int j, int m) {
  return (a + 1) / 2 - (1 - a) / 2 * (qf)cosl(3.14159265358979323846264338327950288L * j / m);
}
// odd minimax fit of 1 on [a, 1] with n odd terms T_1 .. T_{2n-1}:
// coefficients (double-binary128), sets err
std::vector<dq> remez_sign(int n, qf a, qf& err) {
  std::vector<qf> xs(n + 1), c(n, 0);
  std::vector<dq> cd(n);
  for (int i = 0; i <= n; ++i) xs[i] = cheb_pt(a, i, n);
  const int G = 64 * n;
  std::vector<qf> grid(G + 1), dg(G + 1);
  for (int j = 0; j <= G; ++j) grid[j] = cheb_pt(a, j, G);
  const qf tol_rel = 1 / (qf)18446744073709551616.0L;  // 2^-64
  const qf tol_abs = tol_rel * tol_rel * 65536 * 2;    // 2^-111: binary128's floor
  int done = 0;
  for (int it = 0; it < 60; ++it) {
    std::vector<std::vector<dq>> A(n + 1, std::vector<dq>(n + 2));
    for (int i = 0; i <= n; ++i) {
      for (int k = 0; k < n; ++k) A[i][k] = cheb_T_dq(2 * k + 1, xs[i]);
      A[i][n] = to_dq((i & 1) ? -1 : 1);
      A[i][n + 1] = to_dq(1);
    }
    std::vector<dq> sol = solve(A);
    for (int k = 0; k < n; ++k) cd[k] = sol[k], c[k] = sol[k].hi + sol[k].lo;
    const qf E = qabs(sol[n].hi + sol[n].lo);
    // extrema of e = p - 1: the endpoints and the zeros of p' (bisection)
    qf s, ds;
    for (int j = 0; j <= G; ++j) cheb_odd_eval(c, grid[j], s, dg[j]);
    std::vector<qf> ex{grid[0]};
    for (int j = 0; j < G; ++j) {
      if (!(dg[j] == 0 || (dg[j] > 0) != (dg[j + 1] > 0))) continue;
      qf lo = grid[j], hi = grid[j + 1];
      const bool up = dg[j] > 0;
      for (int b = 0; b < 90; ++b) {
        const qf m = (lo + hi) / 2;
        cheb_odd_eval(c, m, s, ds);
        if ((ds > 0) == up) lo = m; else hi = m;
      }
      ex.push_back((lo + hi) / 2);
    }
    ex.push_back(grid[G]);
    std::vector<qf> px, pv;  // alternating points, the larger of equal-sign neighbours
    for (qf x : ex) {
      cheb_odd_eval(c, x, s, ds);
      const qf v = s - 1;
      if (!px.empty() && (v >= 0) == (pv.back() >= 0)) {
        if (qabs(v) > qabs(pv.back())) px.back() = x, pv.back() = v;
        continue;
      }
      px.push_back(x);
      pv.push_back(v);
    }
    while ((int)px.size() > n + 1) {  // drop the smaller end extremum
      if (qabs(pv.front()) < qabs(pv.back()))
        px.erase(px.begin()), pv.erase(pv.begin());
      else
        px.pop_back(), pv.pop_back();
    }
    if ((int)px.size() < n + 1) throw std::runtime_error("minimax: Remez lost the alternation");
    qf emax = 0;
    for (qf v : pv) emax = qabs(v) > emax ? qabs(v) : emax;
    err = emax;
    xs = px;
    // converged: the levelled error E matches the true maximum (relative,
    // or absolute for stages whose error is far below float64); two more
    // exchanges after the threshold (quadratic convergence)
    if (emax - E <= tol_rel * emax || emax - E <= tol_abs) {
      if (++done == 3) return cd;
    }
  }
  throw std::runtime_error("minimax: Remez did not converge");
}
}  // namespace

std::vector<std::vector<double>> minimax_sign_composite(const std::vector<int>& degrees, int logalpha) {
  std::vector<std::vector<double>> out;
  qf a = (qf)ldexpl(1.0L, -logalpha);
  for (size_t i = 0; i < degrees.size(); ++i) {
    const int d = degrees[i];
    if (d < 1) throw std::runtime_error("minimax: degrees must be >= 1");
    qf err = 0;
    std::vector<dq> c = remez_sign((d - 1) / 2 + 1, a, err);
    if (!(err < 1)) throw std::runtime_error("minimax: degree too small for the interval");
    const dq s = to_dq(1) + to_dq(err);
    std::vector<dq> p(d + 1, to_dq(0));
    for (size_t k = 0; k < c.size(); ++k) p[2 * k + 1] = c[k] / s;
    const dq an = (to_dq(1) - to_dq(err)) / s;
    a = an.hi + an.lo;
    if (i + 1 == degrees.size()) {  // orion (polyeval.go:136-143): halved, + 0.5 (in prec bits, then rounded)
      for (dq& v : p) v = v / to_dq(2);
      p[0] = p[0] + to_dq(0.5);
    }
    std::vector<double> pd(d + 1);
    for (int k = 0; k <= d; ++k) pd[k] = (double)(p[k].hi + p[k].lo);
    out.push_back(pd);
  }
  return out;
}
}  // namespace orion
