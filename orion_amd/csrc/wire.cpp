// wire.cpp -- Lattigo v6 binary layouts (wire.h).  Host only, off the hot path.
#include "wire.h"

#include <string.h>

#include <stdexcept>

namespace orion {
namespace wire {

typedef unsigned __int128 u128;

namespace {
// x * c mod q with Shoup's precomputed quotient (c < q)
struct ShoupConst {
  u64 c, cs, q;
  ShoupConst(u64 c_, u64 q_) : c(c_), cs((u64)(((u128)c_ << 64) / q_)), q(q_) {}
  u64 mul(u64 x) const {
    const u64 hi = (u64)(((u128)x * cs) >> 64);
    u64 r = x * c - hi * q;
    return r >= q ? r - q : r;
  }
};
u64 pow_mod(u64 b, u64 e, u64 q) {
  u64 r = 1 % q;
  b %= q;
  while (e) {
    if (e & 1) r = (u64)(((u128)r * b) % q);
    b = (u64)(((u128)b * b) % q);
    e >>= 1;
  }
  return r;
}
}  // namespace

void put_u64(std::vector<char>& b, u64 v) {
  char t[8];
  memcpy(t, &v, 8);  // little endian host (x86-64), as Lattigo's buffer.WriteUint64
  b.insert(b.end(), t, t + 8);
}

void put_poly(std::vector<char>& b, const u64* data, const std::vector<u64>& mods, int N) {
  const size_t at = b.size();
  b.resize(at + poly_bytes((int)mods.size(), N));
  char* p = b.data() + at;
  const u64 rows = mods.size(), n = (u64)N;
  memcpy(p, &rows, 8);
  p += 8;
  for (size_t l = 0; l < mods.size(); ++l) {
    const u64 q = mods[l];
    const ShoupConst mf((u64)(((u128)1 << 64) % q), q);  // MForm: x 2^64 mod q
    memcpy(p, &n, 8);
    p += 8;
    u64* o = (u64*)p;
    const u64* s = data + l * (size_t)N;
    for (int i = 0; i < N; ++i) o[i] = mf.mul(s[i]);
    p += 8 * (size_t)N;
  }
}

u64 Reader::get_u64() {
  if (n_ - off_ < 8) throw std::runtime_error("serialized object truncated");
  u64 v;
  memcpy(&v, p_ + off_, 8);
  off_ += 8;
  return v;
}

void Reader::get_poly(u64* out, const std::vector<u64>& mods, int N, const char* what) {
  const u64 rows = get_u64();
  if (rows != mods.size())
    throw std::runtime_error(std::string(what) + ": " + std::to_string(rows) + " RNS limbs, expected " +
                             std::to_string(mods.size()));
  for (size_t l = 0; l < mods.size(); ++l) {
    const u64 n = get_u64();
    if (n != (u64)N)
      throw std::runtime_error(std::string(what) + ": ring degree " + std::to_string(n) + ", expected " +
                               std::to_string(N));
    if (n_ - off_ < 8 * (size_t)N) throw std::runtime_error(std::string(what) + ": truncated");
    const u64 q = mods[l];
    const u64 r = pow_mod((u64)(((u128)1 << 64) % q), q - 2, q);  // 2^-64 mod q
    const ShoupConst inv(r, q);
    const u64* s = (const u64*)(p_ + off_);
    u64* o = out + l * (size_t)N;
    for (int i = 0; i < N; ++i) {
      if (s[i] >= q) throw std::runtime_error(std::string(what) + ": coefficient not reduced mod q");
      o[i] = inv.mul(s[i]);
    }
    off_ += 8 * (size_t)N;
  }
}

}  // namespace wire
}  // namespace orion
