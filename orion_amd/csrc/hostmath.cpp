#include <cstdio>
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
// composite minimax approximation of sign (polyeval.go:91-167 -> Lattigo v6
// circuits/ckks/minimax.GenMinimaxCompositePolynomial and utils/bignum.Remez
// [U], restated below; the fixture tests/golden/minimax_sign.json is the same
// construction at `prec` = 128 bits in mpmath, tools/gen_minimax.py).  The
// Remez exchange runs in binary128 (__float128, 113 bits), its linear system
// in double-binary128.
// ---------------------------------------------------------------------------
namespace {
typedef __float128 qf;

qf qabs(qf x) { return x < 0 ? -x : x; }
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
// bignum.Remez [U] (Lattigo v6 utils/bignum/remez.go, the multi-interval
// Remez of Lee et al., eprint 2020/552), restated: the degree-D approximation
// of sign in the Chebyshev basis T_0 .. T_D evaluated at x itself (the basis
// orion's GenerateChebyshev evaluates on [-1, 1], polyeval.go:49-60), D =
// (nodes over all intervals) - 2:
//   start: each interval's `nodes` Chebyshev points of the first kind;
//   iterate (at most maxIters): solve p(x_i) + (-1)^i E = sign(x_i); take the
//   extreme points of p - sign (each interval's ends and the zeros of p');
//   drop same-signed neighbours but the larger; while more than D + 2 remain,
//   drop the smaller end point when one too many, else the adjacent pair with
//   the smallest |e_i| + |e_{i+1}|; MaxErr / MinErr = the largest / smallest
//   |e| of the new nodes; stop once (MaxErr - MinErr) / MinErr <= threshold.
// The coefficients returned are those of the last solve (the polynomial whose
// extreme points MaxErr measured).
struct RemezOut {
  std::vector<dq> coeffs;  // T_0 .. T_D
  qf maxerr = 0, minerr = 0;
  int iters = 0;
};
// sum_j c_j T_j(x) and its derivative (T_j' = j U_{j-1})
void cheb_eval_full(const std::vector<qf>& c, qf x, qf& s, qf& ds) {
  qf t0 = 1, t1 = x, u0 = 1, u1 = 2 * x;  // T_0, T_1, U_0, U_1
  s = c[0];
  ds = 0;
  for (size_t j = 1; j < c.size(); ++j) {
    s += c[j] * t1;
    ds += c[j] * (qf)(int)j * u0;
    const qf t2 = 2 * x * t1 - t0, u2 = 2 * x * u1 - u0;
    t0 = t1, t1 = t2, u0 = u1, u1 = u2;
  }
}
// pi and cos in binary128 (the nodes' positions must be exact to the
// format, or the early-stopped iterate moves: cosl has 64 bits)
const qf kPiQ = (qf)3.141592653589793 + (qf)1.2246467991473532e-16 + (qf)-2.9947698097183397e-33;
qf cosq_(qf x) {  // |x| <= pi: Taylor series, terms below 2^-120
  qf x2 = x * x, term = 1, sum = 1;
  for (int k = 1; k < 60; ++k) {
    term = -term * x2 / (qf)((2 * k - 1) * (2 * k));
    sum += term;
    if (qabs(term) < (qf)ldexpl(1.0L, -124)) break;
  }
  return sum;
}
RemezOut remez_sign_multi(const std::vector<std::pair<qf, qf>>& iv, int nodes_per, qf threshold, int max_iters,
                          bool debug) {
  const int nI = (int)iv.size(), nn = nodes_per * nI, D = nn - 2;
  std::vector<qf> xs;
  for (auto& I : iv)  // ascending: x_{n-k} = mid + half cos((k - 1/2) pi / n), k = 1..n
    for (int i = 0; i < nodes_per; ++i) {
      const int k = nodes_per - i;
      xs.push_back((I.first + I.second) / 2 +
                   (I.second - I.first) / 2 * cosq_(kPiQ * ((qf)k - (qf)0.5) / (qf)nodes_per));
    }
  auto sgn = [](qf x) -> qf { return x < 0 ? -1 : (x > 0 ? 1 : 0); };
  const int G = 64 * (D + 2);
  std::vector<std::vector<qf>> grids(nI);
  for (int t = 0; t < nI; ++t)
    for (int j = 0; j <= G; ++j)
      grids[t].push_back((iv[t].first + iv[t].second) / 2 -
                         (iv[t].second - iv[t].first) / 2 * cosq_(kPiQ * (qf)j / (qf)G));
  RemezOut out;
  std::vector<qf> c(D + 1, 0);
  for (int it = 0; it < max_iters; ++it) {
    std::vector<std::vector<dq>> A(nn, std::vector<dq>(nn + 1));
    for (int i = 0; i < nn; ++i) {
      for (int j = 0; j <= D; ++j) A[i][j] = cheb_T_dq(j, xs[i]);
      A[i][D + 1] = to_dq((i & 1) ? -1 : 1);
      A[i][nn] = to_dq(sgn(xs[i]));
    }
    std::vector<dq> sol = solve(A);
    out.coeffs.assign(sol.begin(), sol.begin() + D + 1);
    for (int j = 0; j <= D; ++j) c[j] = sol[j].hi + sol[j].lo;
    out.iters = it + 1;
    // extreme points of e = p - sign, interval by interval
    std::vector<qf> px, pv;
    qf s, ds;
    auto push = [&](qf x) {
      cheb_eval_full(c, x, s, ds);
      const qf v = s - sgn(x);
      if (!px.empty() && (v >= 0) == (pv.back() >= 0)) {  // same sign as the previous: keep the larger
        if (qabs(v) > qabs(pv.back())) px.back() = x, pv.back() = v;
        return;
      }
      px.push_back(x);
      pv.push_back(v);
    };
    for (int t = 0; t < nI; ++t) {
      const std::vector<qf>& g = grids[t];
      std::vector<qf> dg(G + 1);
      for (int j = 0; j <= G; ++j) cheb_eval_full(c, g[j], s, dg[j]);
      push(g[0]);
      for (int j = 0; j < G; ++j) {
        if (!(dg[j] == 0 || (dg[j] > 0) != (dg[j + 1] > 0))) continue;
        if (dg[j] == 0 && j == 0) continue;
        qf lo = g[j], hi = g[j + 1];
        const bool up = dg[j] > 0;
        for (int b = 0; b < 100; ++b) {
          const qf m = (lo + hi) / 2;
          cheb_eval_full(c, m, s, ds);
          if ((ds > 0) == up) lo = m; else hi = m;
        }
        push((lo + hi) / 2);
      }
      push(g[G]);
    }
    const size_t found = px.size();
    {  // the levelled error below the arithmetic's resolution (a constant fit
       // on a short interval near 1): converged as far as it can be measured
      qf E = qabs(sol[D + 1].hi + sol[D + 1].lo), vmax = 0;
      for (qf v : pv) vmax = qabs(v) > vmax ? qabs(v) : vmax;
      if (vmax < (qf)ldexpl(1.0L, -100)) {
        out.maxerr = vmax > E ? vmax : E, out.minerr = E;
        if (debug) fprintf(stderr, "Iteration: %2d - error %.3Le below 2^-100: stop\n", it, (long double)vmax);
        break;
      }
    }
    while ((int)px.size() > nn) {
      if ((int)px.size() == nn + 1) {  // one too many: the smaller end point
        if (qabs(pv.front()) < qabs(pv.back()))
          px.erase(px.begin()), pv.erase(pv.begin());
        else
          px.pop_back(), pv.pop_back();
        continue;
      }
      size_t m = 0;
      qf best = qabs(pv[0]) + qabs(pv[1]);
      for (size_t i = 1; i + 1 < px.size(); ++i)
        if (qabs(pv[i]) + qabs(pv[i + 1]) < best) best = qabs(pv[i]) + qabs(pv[i + 1]), m = i;
      px.erase(px.begin() + m, px.begin() + m + 2);
      pv.erase(pv.begin() + m, pv.begin() + m + 2);
    }
    if ((int)px.size() < nn) throw std::runtime_error("minimax: Remez lost the alternation");
    out.maxerr = 0, out.minerr = qabs(pv[0]);
    for (qf v : pv) {
      out.maxerr = qabs(v) > out.maxerr ? qabs(v) : out.maxerr;
      out.minerr = qabs(v) < out.minerr ? qabs(v) : out.minerr;
    }
    xs = px;
    const qf nerr = (out.maxerr - out.minerr) / out.minerr;
    if (debug) fprintf(stderr, "Iteration: %2d - %.6Le (nodes %d, alternating extreme points %zu)\n", it, (long double)nerr, nn, found);
    if (nerr <= threshold) break;
  }
  return out;
}
}  // namespace

// circuits/ckks/minimax.GenMinimaxCompositePolynomial [U], restated:
//   e = 2^-logerr (the scheme error the fit absorbs), a_0 = 2^-logalpha;
//   stage 0 fits sign on [-1 - e, -a_0 + e] U [a_0 - e, 1 + e];
//   stage i > 0: the previous stage's coefficients are divided by
//   1 + MaxErr (so its image [1 - MaxErr, 1 + MaxErr] lands in
//   [a_i, 1], a_i = (1 - MaxErr) / (1 + MaxErr)), and stage i fits sign on
//   [-1 - e, -a_i + e] U [a_i - e, 1 + e];
//   the last stage keeps its coefficients; every stage has
//   1 + (d + 1) / 2 nodes per interval, Remez threshold 2^-logalpha, at most
//   50 iterations; each coefficient vector is the first d + 1 of T_0 .. T_D.
// orion (polyeval.go:136-143): the last polynomial halved, + 0.5 on T_0.
std::vector<std::vector<double>> minimax_sign_composite(const std::vector<int>& degrees, int logalpha, int logerr,
                                                        std::vector<double>* stage_err, bool debug) {
  std::vector<std::vector<double>> out;
  const qf alpha = (qf)ldexpl(1.0L, -logalpha), e = (qf)ldexpl(1.0L, -logerr);
  qf a = alpha;
  RemezOut prev;
  std::vector<std::vector<dq>> polys;
  for (size_t i = 0; i < degrees.size(); ++i) {
    const int d = degrees[i];
    if (d < 1) throw std::runtime_error("minimax: degrees must be >= 1");
    if (i > 0) {
      const dq maxI = to_dq(1) + to_dq(prev.maxerr), minI = to_dq(1) - to_dq(prev.maxerr);
      for (dq& v : polys.back()) v = v / maxI;  // interval normalisation
      const dq an = minI / maxI;
      a = an.hi + an.lo;
    }
    std::vector<std::pair<qf, qf>> iv = {{-1 - e, -a + e}, {a - e, 1 + e}};
    if (debug)
      fprintf(stderr, "P[%zu]\nInterval: [%.12Lf, %.12Lf] U [%.12Lf, %.12Lf]\n", i, (long double)iv[0].first,
              (long double)iv[0].second, (long double)iv[1].first, (long double)iv[1].second);
    prev = remez_sign_multi(iv, 1 + ((d + 1) >> 1), alpha, 50, debug);
    if (debug) fprintf(stderr, "MaxErr %.6Le MinErr %.6Le\n", (long double)prev.maxerr, (long double)prev.minerr);
    if (!(prev.maxerr < 1)) throw std::runtime_error("minimax: degree too small for the interval");
    polys.emplace_back(prev.coeffs.begin(), prev.coeffs.begin() + d + 1);
    // sign is odd and the interval set symmetric: the even coefficients are
    // zero up to the exchange's rounding, and are set to zero
    for (int j = 0; j <= d; j += 2) polys.back()[j] = to_dq(0);
    if (stage_err) stage_err->push_back((double)prev.maxerr);
  }
  std::vector<dq>& last = polys.back();
  for (dq& v : last) v = v / to_dq(2);
  last[0] = last[0] + to_dq(0.5);
  for (auto& p : polys) {
    std::vector<double> pd;
    for (const dq& v : p) pd.push_back((double)(v.hi + v.lo));
    out.push_back(pd);
  }
  return out;
}

// ---------------------------------------------------------------------------
// EvalMod's cosine polynomial, Lattigo v6 mod1 CosDiscrete (the default
// Mod1Type; circuits/ckks/mod1 ApproximateCos, after Han-Ki [U]), restated:
// g(x) = a cos(2 pi (x - 1/4) / 2^r), a = (2 pi)^(-1/2^r), interpolated at
// nodes clustered on the integers the ModRaise overflow takes, i in
// [-(K-1), K-1]: d_i Chebyshev nodes of the first kind in [i - dev, i + dev]
// (the integer itself when d_i = 1), d_i = 1 each and the degree + 1 - (2K - 1)
// remaining nodes handed out greedily to the integer with the largest
// interpolation-error bound dev^d_i / 2^(d_i - 1) * prod_{j != i} |i - j|^d_j
// (d_{-i} = d_i; the centre takes single nodes); returned as Chebyshev
// coefficients of u = x / K on [-1, 1] (solved in double-binary128: the
// system at integer nodes has condition ~1e10), rounded to long double.
// ---------------------------------------------------------------------------
namespace {
qf cos_reduced(qf x) {  // any x: reduced into [-pi, pi] first
  const qf two_pi = 2 * kPiQ;
  const long double k = roundl((long double)(x / two_pi));
  return cosq_(x - (qf)k * two_pi);
}
qf sqrt_q(qf v) {  // binary128 square root: Newton from the long double one
  qf y = (qf)sqrtl((long double)v);
  for (int i = 0; i < 3; ++i) y = (y + v / y) / 2;
  return y;
}
}  // namespace
std::vector<long double> cos_discrete_cheb(int K, int degree, int r, double dev) {
  const int n = degree + 1;
  if (K < 1 || n < 2 * K - 1) throw std::runtime_error("CosDiscrete: degree + 1 must be >= 2K - 1");
  std::vector<int> d(K, 1);  // nodes at +-i (d[0]: the centre)
  int tot = 2 * K - 1;
  while (tot < n) {
    int best = -1;
    long double bb = 0;
    for (int i = 0; i < K; ++i) {
      if (i > 0 && tot + 2 > n) continue;
      long double lb = d[i] * log2l((long double)dev) - (d[i] - 1);
      for (int j = -(K - 1); j < K; ++j)
        if (j != i) lb += d[j < 0 ? -j : j] * log2l((long double)(i > j ? i - j : j - i));
      if (best < 0 || lb > bb) best = i, bb = lb;
    }
    d[best] += 1;
    tot += best == 0 ? 1 : 2;
  }
  std::vector<qf> xs;
  for (int i = -(K - 1); i < K; ++i) {
    const int di = d[i < 0 ? -i : i];
    for (int j = 0; j < di; ++j)
      xs.push_back(di == 1 ? (qf)i : (qf)i + (qf)dev * cosq_(kPiQ * (qf)(2 * j + 1) / (qf)(2 * di)));
  }
  qf a = 1 / (2 * kPiQ);
  for (int i = 0; i < r; ++i) a = sqrt_q(a);
  const qf sc = (qf)(1 << r);
  std::vector<std::vector<dq>> A(n, std::vector<dq>(n + 1));
  for (int k = 0; k < n; ++k) {
    const qf u = xs[k] / (qf)K;
    for (int j = 0; j < n; ++j) A[k][j] = cheb_T_dq(j, u);
    A[k][n] = to_dq(a * cos_reduced(2 * kPiQ * (xs[k] - (qf)0.25) / sc));
  }
  std::vector<dq> c = solve(A);
  std::vector<long double> out(n);
  for (int j = 0; j < n; ++j) out[j] = (long double)(c[j].hi + c[j].lo);
  return out;
}
}  // namespace orion
