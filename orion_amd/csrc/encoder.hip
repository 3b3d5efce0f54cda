// encoder.hip -- CKKS encoding, decoding and encryption sampling on the GPU
// (SURVEY.md §8f row 1).
//
//  * encode: slots -> special inverse FFT (HEAAN/Lattigo SpecialiFFT, the
//    butterfly order of oracle/ckks_oracle.c special_ifft) -> bit reversal and
//    1/n -> fixed-point CRT residues (Lattigo SingleFloat64ToFixedPointCRT,
//    including its exact path for |v*scale| >= 2^64) -> NTT (ntt.hip);
//  * decode: INTT -> centered CRT reconstruction (Garner digits, exact
//    multiword integer, one correctly rounded conversion) / scale -> bit
//    reversal -> special forward FFT;
//  * encryption: u (uniform ternary), e0, e1 (discrete Gaussian sigma 3.2,
//    |e| <= 19, by a 64-bit cumulative-table sampler) drawn from ChaCha20
//    (RFC 8439 block function) in counter mode, one block per 8 coefficients.
//
// Every float64 operation is written in the order of the CPU restatement and
// compiled with -ffp-contract=off, so encode and decode are bit-identical to
// oracle_encode / oracle_decode.
//
// FFT data: one image is n = N/2 complex doubles (256 KiB at N = 2^15), more
// than one CU's LDS.  The butterfly stages whose span exceeds 4096 elements
// (G = log2(n) - 12 of them) run in registers, 2^G strided elements per
// thread; the remaining 12 stages run in LDS on aligned 4096-element blocks
// (64 KiB, two workgroups per CU).  Twiddles of the stage with half-length h
// are tw[h + j], j < h (n doubles2 per direction, L2 resident).
#include <cstdio>

#include "common.h"

namespace {

constexpr int FFT_BLK = 4096;
constexpr int FFT_LDS_THREADS = 256;

__device__ __forceinline__ double2 cx_mul(double2 a, double2 b) {
  const double ac = a.x * b.x, bd = a.y * b.y, ad = a.x * b.y, bc = a.y * b.x;
  return make_double2(ac - bd, ad + bc);
}
// inverse (Gentleman-Sande) butterfly: x <- x + y, y <- (x - y) * w
__device__ __forceinline__ void bf_inv(double2& x, double2& y, double2 w) {
  const double2 u = make_double2(x.x + y.x, x.y + y.y);
  const double2 d = make_double2(x.x - y.x, x.y - y.y);
  x = u;
  y = cx_mul(d, w);
}
// forward (Cooley-Tukey) butterfly: x <- x + y w, y <- x - y w
__device__ __forceinline__ void bf_fwd(double2& x, double2& y, double2 w) {
  const double2 u = x, t = cx_mul(y, w);
  x = make_double2(u.x + t.x, u.y + t.y);
  y = make_double2(u.x - t.x, u.y - t.y);
}
__device__ __forceinline__ int brev(int i, int bits) { return (int)(__brev((unsigned)i) >> (32 - bits)); }

// stages with half-length >= FFT_BLK: thread t holds v[t + k S], S = n >> G
template <int G, bool INV>
__global__ void __launch_bounds__(256) fft_outer_kernel(double2* __restrict__ v, const double2* __restrict__ tw,
                                                        int logn) {
  const int n = 1 << logn, S = n >> G;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= S) return;
  double2* p = v + (size_t)blockIdx.y * n;
  double2 x[1 << G];
#pragma unroll
  for (int k = 0; k < (1 << G); ++k) x[k] = p[t + k * S];
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int s = INV ? i : G - 1 - i;  // stage s: length n >> s
    const int len = n >> s, h = len >> 1, span = 1 << (G - 1 - s);
#pragma unroll
    for (int k = 0; k < (1 << G); ++k) {
      if (k & span) continue;
      const int j = (t + k * S) & (len - 1);
      const double2 w = tw[h + j];
      if (INV)
        bf_inv(x[k], x[k + span], w);
      else
        bf_fwd(x[k], x[k + span], w);
    }
  }
#pragma unroll
  for (int k = 0; k < (1 << G); ++k) p[t + k * S] = x[k];
}

// stages with length <= blk (blk = min(n, FFT_BLK)) on one aligned block, in LDS
template <bool INV>
__global__ void __launch_bounds__(FFT_LDS_THREADS) fft_lds_kernel(double2* __restrict__ v,
                                                                  const double2* __restrict__ tw, int blk) {
  __shared__ double re[FFT_BLK], im[FFT_BLK];
  double2* p = v + (size_t)blockIdx.x * blk;
  for (int i = threadIdx.x; i < blk; i += FFT_LDS_THREADS) {
    const double2 a = p[i];
    re[i] = a.x;
    im[i] = a.y;
  }
  __syncthreads();
  const int half = blk >> 1;
  for (int len = INV ? blk : 2; INV ? len >= 2 : len <= blk; len = INV ? len >> 1 : len << 1) {
    const int h = len >> 1;
    for (int q = threadIdx.x; q < half; q += FFT_LDS_THREADS) {
      const int j = q & (h - 1);
      const int a = (q - j) * 2 + j, b = a + h;
      double2 x = make_double2(re[a], im[a]), y = make_double2(re[b], im[b]);
      if (INV)
        bf_inv(x, y, tw[h + j]);
      else
        bf_fwd(x, y, tw[h + j]);
      re[a] = x.x, im[a] = x.y, re[b] = y.x, im[b] = y.y;
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < blk; i += FFT_LDS_THREADS) p[i] = make_double2(re[i], im[i]);
}

// slots (float32, nvals per image) -> complex doubles, zero padded to n
__global__ void enc_load_kernel(const float* __restrict__ vals, int nvals, double2* __restrict__ v, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int b = blockIdx.y;
  v[(size_t)b * n + i] = make_double2(i < nvals ? (double)vals[(size_t)b * nvals + i] : 0.0, 0.0);
}

// coefficient i of image b: bit-reversed FFT output times 1/n, then
// round(|x| * scale) -> residues (negated for x < 0).  |x| * scale >= 2^64 is
// an exact integer mant * 2^e and is reduced exactly (Lattigo's big.Int path).
// Standard ring: N = 2n coefficients, real parts then imaginary parts; CI ring:
// N = n coefficients, the real parts (the imaginary parts are the degree-2N
// expansion's upper half, which the CI ring does not store).
__global__ void enc_crt_kernel(const double2* __restrict__ v, LimbSet out, double scale, double inv_n, int logn,
                               int ci, const DeviceTables* __restrict__ tb) {
  const int n = 1 << logn, N = ci ? n : 2 * n;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int b = blockIdx.y;
  const double2 s = v[(size_t)b * n + brev(i & (n - 1), logn)];
  double x = i < n ? s.x : s.y;
  x *= inv_n;
  const bool neg = x < 0;
  const double y = neg ? x * (-scale) : x * scale;
  u64 c = 0, mant = 0;
  int e = 0;
  const bool big = !(y < 18446744073709551616.0);
  if (!big) {
    c = (u64)(y + 0.5);
  } else {  // y = mant * 2^e exactly, e > 11
    int ex;
    const double fr = frexp(y, &ex);  // y = fr * 2^ex, fr in [0.5, 1)
    mant = (u64)ldexp(fr, 53);
    e = ex - 53;
  }
  u64* o = out.p + (size_t)b * out.batch_stride + i;
  for (int l = 0; l < out.nlimb; ++l) {
    const u64 q = tb->mc[out.mod[l]].q;
    u64 r;
    if (!big) {
      r = c % q;
    } else {
      r = mant % q;
      for (int k = 0; k < e; ++k) r = add_mod(r, r, q);
    }
    o[(size_t)out.pos[l] * out.limb_stride] = neg ? (r ? q - r : 0) : r;
  }
}

// decode: Garner digits of the centered value of coefficient i, exact integer
// value, one correctly rounded conversion to double, / scale, into the
// bit-reversed slot position of the forward FFT.
//   garner[j * nl + k] = (q_k mod q_j)^-1 mod q_j (k < j); garner[nl * nl + j]
//   = mixed-radix digit j of floor((Q - 1) / 2).
//   CI ring (N = n): slot input j is a_j - i a_{N-j} (a_0 real), so coefficient
//   i is the real part at slot i and, negated, the imaginary part at slot N - i
__global__ void dec_crt_kernel(LimbSet x, const u64* __restrict__ garner, double scale, int logn, int ci,
                               double2* __restrict__ v, const DeviceTables* __restrict__ tb) {
  const int n = 1 << logn, N = ci ? n : 2 * n;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int b = blockIdx.y, nl = x.nlimb;
  const u64* half = garner + nl * nl;
  u64 d[ORION_MAXLIMB];
  for (int j = 0; j < nl; ++j) {
    const ModConst& m = tb->mc[x.mod[j]];
    u64 r = x.p[(size_t)x.pos[j] * x.limb_stride + (size_t)b * x.batch_stride + i];
    for (int k = 0; k < j; ++k) r = mul_mod(sub_mod(r, d[k] % m.q, m.q), garner[j * nl + k], m);
    d[j] = r;
  }
  bool greater = false;
  for (int j = nl - 1; j >= 0; --j)
    if (d[j] != half[j]) {
      greater = d[j] > half[j];
      break;
    }
  if (greater) {  // Q - x: digits of (Q - 1 - x) + 1
    for (int j = 0; j < nl; ++j) d[j] = tb->mc[x.mod[j]].q - 1 - d[j];
    for (int j = 0; j < nl; ++j) {
      if (d[j] + 1 < tb->mc[x.mod[j]].q) {
        d[j] += 1;
        break;
      }
      d[j] = 0;
    }
  }
  int top = nl - 1;
  while (top > 0 && d[top] == 0) --top;
  // Horner from the top digit: w = w * q_j + d_j (little-endian u64 words)
  u64 w[ORION_MAXLIMB + 1];
  int nw = 1;
  w[0] = d[top];
  for (int j = top - 1; j >= 0; --j) {
    const u64 q = tb->mc[x.mod[j]].q;
    u64 carry = d[j];
    for (int t = 0; t < nw; ++t) {
      const u64 lo = w[t] * q, hi = mulhi64(w[t], q);
      const u64 s = lo + carry;
      carry = hi + (s < lo);
      w[t] = s;
    }
    if (carry) w[nw++] = carry;
  }
  double f;
  if (nw == 1) {
    f = (double)w[0];
  } else {
    const u64 tw = w[nw - 1];
    const int lz = __clzll(tw);
    u64 m = lz ? (tw << lz) | (w[nw - 2] >> (64 - lz)) : tw;
    bool sticky = lz ? (w[nw - 2] << lz) != 0 : w[nw - 2] != 0;
    for (int t = 0; t < nw - 2; ++t) sticky |= w[t] != 0;
    f = ldexp((double)(m | (u64)sticky), 64 * (nw - 1) - lz);
  }
  if (greater) f = -f;
  f = f / scale;
  double2* const vb = v + (size_t)b * n;
  if (ci) {
    reinterpret_cast<double*>(vb + brev(i, logn))[0] = f;
    reinterpret_cast<double*>(vb + brev((n - i) & (n - 1), logn))[1] = i ? -f : 0.0;
    return;
  }
  double* dst = reinterpret_cast<double*>(vb + brev(i & (n - 1), logn));
  dst[i < n ? 0 : 1] = f;
}

__global__ void dec_out_kernel(const double2* __restrict__ v, double* __restrict__ out, size_t total) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < total) out[i] = v[i].x;
}

// bootstrapping ModRaise: coefficient-domain residues mod q0 (row (c, 0, b) of
// in) -> centred integers in (-q0/2, q0/2] -> residues of every limb of out
__global__ void modraise_kernel(LimbSet out, LimbSet in, const DeviceTables* __restrict__ tb, int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int b = blockIdx.y % out.nbatch, c = blockIdx.y / out.nbatch;
  const u64 q0 = tb->mc[in.mod[0]].q;
  const u64 x = in.p[(size_t)c * in.comp_stride + (size_t)in.pos[0] * in.limb_stride + (size_t)b * in.batch_stride + i];
  const bool neg = x > (q0 >> 1);
  const u64 a = neg ? q0 - x : x;
  u64* o = out.p + (size_t)c * out.comp_stride + (size_t)b * out.batch_stride + i;
  for (int l = 0; l < out.nlimb; ++l) {
    const u64 q = tb->mc[out.mod[l]].q;
    const u64 r = a % q;
    o[(size_t)out.pos[l] * out.limb_stride] = neg ? (r ? q - r : 0) : r;
  }
}

// ---- ChaCha20 (RFC 8439 §2.3) ----
__device__ __forceinline__ u32 rotl32(u32 x, int k) { return (x << k) | (x >> (32 - k)); }
#define CHACHA_QR(a, b, c, d) \
  a += b, d ^= a, d = rotl32(d, 16), c += d, b ^= c, b = rotl32(b, 12), a += b, d ^= a, d = rotl32(d, 8), \
  c += d, b ^= c, b = rotl32(b, 7)
__device__ __forceinline__ void chacha20_block(const u32* key, u32 ctr, u32 n0, u32 n1, u32 n2, u32* out) {
  u32 s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
               key[4],      key[5],      key[6],      key[7],      ctr,    n0,     n1,     n2};
  u32 x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = s[i];
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    CHACHA_QR(x[0], x[4], x[8], x[12]);
    CHACHA_QR(x[1], x[5], x[9], x[13]);
    CHACHA_QR(x[2], x[6], x[10], x[14]);
    CHACHA_QR(x[3], x[7], x[11], x[15]);
    CHACHA_QR(x[0], x[5], x[10], x[15]);
    CHACHA_QR(x[1], x[6], x[11], x[12]);
    CHACHA_QR(x[2], x[7], x[8], x[13]);
    CHACHA_QR(x[3], x[4], x[9], x[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}

// u, e0, e1 of image b (component c = blockIdx.z) as residues of r at every limb
//   stream (enc, b, c): ChaCha20 nonce {enc, b, ENC_DOMAIN | c}, block counter =
//   coefficient / 8, coefficient i takes words 2(i%8), 2(i%8)+1 as a u64
__global__ void enc_sample_kernel(LimbSet r, EncSampler sp, const DeviceTables* __restrict__ tb, int N) {
  const int blk = blockIdx.x * blockDim.x + threadIdx.x;
  if (blk * 8 >= N) return;
  const int b = blockIdx.y, c = blockIdx.z;
  u32 w[16];
  chacha20_block(sp.key, (u32)blk, sp.enc, (u32)b, ORION_ENC_DOMAIN | (u32)c, w);
  int v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const u64 x = (u64)w[2 * k] | ((u64)w[2 * k + 1] << 32);
    if (c == 0) {
      v[k] = (int)(((x >> 32) * 3) >> 32) - 1;
    } else {
      int cnt = 0;
#pragma unroll
      for (int t = 0; t < 2 * ORION_GAUSS_BOUND; ++t) cnt += x >= sp.cdt[t];
      v[k] = cnt - ORION_GAUSS_BOUND;
    }
  }
  u64* o = r.p + (size_t)c * r.comp_stride + (size_t)b * r.batch_stride + (size_t)blk * 8;
  for (int l = 0; l < r.nlimb; ++l) {
    const u64 q = tb->mc[r.mod[l]].q;
    u64* ol = o + (size_t)r.pos[l] * r.limb_stride;
#pragma unroll
    for (int k = 0; k < 8; ++k) ol[k] = v[k] >= 0 ? (u64)v[k] : q - (u64)(-v[k]);
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// launchers (v: [B][n] double2 scratch; tw: [n] twiddles tw[h + j])
// ---------------------------------------------------------------------------
static int fft_run(double2* v, const double2* tw, int logn, int B, bool inverse, hipStream_t st) {
  const int n = 1 << logn, G = logn > 12 ? logn - 12 : 0, blk = n < FFT_BLK ? n : FFT_BLK;
  if (G > 4) return -1;
  const dim3 og((unsigned)(((n >> G) + 255) / 256), (unsigned)B);
  auto outer = [&]() {
    switch (G) {
      case 1: inverse ? fft_outer_kernel<1, true><<<og, 256, 0, st>>>(v, tw, logn)
                      : fft_outer_kernel<1, false><<<og, 256, 0, st>>>(v, tw, logn); break;
      case 2: inverse ? fft_outer_kernel<2, true><<<og, 256, 0, st>>>(v, tw, logn)
                      : fft_outer_kernel<2, false><<<og, 256, 0, st>>>(v, tw, logn); break;
      case 3: inverse ? fft_outer_kernel<3, true><<<og, 256, 0, st>>>(v, tw, logn)
                      : fft_outer_kernel<3, false><<<og, 256, 0, st>>>(v, tw, logn); break;
      case 4: inverse ? fft_outer_kernel<4, true><<<og, 256, 0, st>>>(v, tw, logn)
                      : fft_outer_kernel<4, false><<<og, 256, 0, st>>>(v, tw, logn); break;
    }
  };
  const unsigned nblk = (unsigned)((size_t)B * (n / blk));
  if (inverse) {
    if (G) outer();
    fft_lds_kernel<true><<<nblk, FFT_LDS_THREADS, 0, st>>>(v, tw, blk);
  } else {
    fft_lds_kernel<false><<<nblk, FFT_LDS_THREADS, 0, st>>>(v, tw, blk);
    if (G) outer();
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// logn: log2 of the slot count (N/2 Standard, N ConjugateInvariant)
int orion_launch_encode(const float* vals, int nvals, int B, double2* v, const double2* tw_inv, int logn, bool ci,
                        const LimbSet& out, double scale, const DeviceTables* tb, hipStream_t st) {
  const int n = 1 << logn, N = ci ? n : 2 * n;
  enc_load_kernel<<<dim3((unsigned)((n + 255) / 256), (unsigned)B), 256, 0, st>>>(vals, nvals, v, n);
  if (fft_run(v, tw_inv, logn, B, true, st)) return -1;
  enc_crt_kernel<<<dim3((unsigned)((N + 255) / 256), (unsigned)B), 256, 0, st>>>(v, out, scale, 1.0 / (double)n,
                                                                                logn, ci ? 1 : 0, tb);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int orion_launch_decode(const LimbSet& x, const u64* garner, double scale, int logn, bool ci, double2* v,
                        const double2* tw_fwd, double* out, const DeviceTables* tb, hipStream_t st) {
  const int n = 1 << logn, B = x.nbatch, N = ci ? n : 2 * n;
  dec_crt_kernel<<<dim3((unsigned)((N + 255) / 256), (unsigned)B), 256, 0, st>>>(x, garner, scale, logn, ci ? 1 : 0,
                                                                                v, tb);
  if (fft_run(v, tw_fwd, logn, B, false, st)) return -1;
  const size_t total = (size_t)B * n;
  dec_out_kernel<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(v, out, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// complex slots already in v ([B][n] double2, overwritten): FFT + CRT (no load step)
int orion_launch_encode_c(double2* v, int B, const double2* tw_inv, int logn, bool ci, const LimbSet& out,
                          double scale, const DeviceTables* tb, hipStream_t st) {
  const int n = 1 << logn, N = ci ? n : 2 * n;
  if (fft_run(v, tw_inv, logn, B, true, st)) return -1;
  enc_crt_kernel<<<dim3((unsigned)((N + 255) / 256), (unsigned)B), 256, 0, st>>>(v, out, scale, 1.0 / (double)n,
                                                                                logn, ci ? 1 : 0, tb);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int orion_launch_enc_sample(const LimbSet& r, const EncSampler& sp, const DeviceTables* tb, int N, hipStream_t st) {
  enc_sample_kernel<<<dim3((unsigned)((N / 8 + 255) / 256), (unsigned)r.nbatch, 3), 256, 0, st>>>(r, sp, tb, N);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int orion_launch_modraise(const LimbSet& out, const LimbSet& in, const DeviceTables* tb, int N, hipStream_t st) {
  modraise_kernel<<<dim3((unsigned)((N + 255) / 256), (unsigned)(out.ncomp * out.nbatch)), 256, 0, st>>>(out, in, tb, N);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fprintf(stderr, "orion_launch_modraise: %s\n", hipGetErrorString(e));
  return e == hipSuccess ? 0 : -1;
}
