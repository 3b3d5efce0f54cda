// wire.h -- Lattigo v6 binary layouts for the io_mode save/load paths
// (keygenerator.go:38-58, lineartransform.go:131-193).
//
// The reference marshals Lattigo objects with their MarshalBinary methods and
// Orion stores the bytes in HDF5 unchanged (key_generator.py:17-31,
// lt_evaluator.py:283-315).  Layouts restated from Lattigo v6's WriteTo
// methods (github.com/baahl-nyu/lattigo/v6 v6.2.0, not vendored: parity
// unpinned):
//   structs.Vector[uint64]  u64 len, len x u64 (little endian)
//   structs.Matrix[T]       u64 rows, rows x Vector[T]
//   ring.Poly               Matrix[uint64] of the RNS limbs (one row per limb)
//   ringqp.Poly             ring.Poly Q, then ring.Poly P
//   rlwe.SecretKey          ringqp.Poly
//   rlwe.GadgetCiphertext   u64 BaseTwoDecomposition, Matrix[VectorQP]
//                           (dnum rows x 1 column, VectorQP = Vector of 2 ringqp.Poly)
//   rlwe.GaloisKey          u64 GaloisElement, u64 NthRoot, GadgetCiphertext
// Coefficients are in the NTT domain and in Montgomery form (x 2^64 mod q),
// as Lattigo keeps secret keys, evaluation keys and LT diagonals; this
// backend keeps them in plain form and converts at the boundary.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace orion {
namespace wire {

typedef uint64_t u64;

// bytes of a ring.Poly with nl limbs of N coefficients
inline size_t poly_bytes(int nl, int N) { return 8 + (size_t)nl * (8 + 8 * (size_t)N); }

void put_u64(std::vector<char>& b, u64 v);
// ring.Poly from host limbs data[l*N + n], l < mods.size(), converted to Montgomery form
void put_poly(std::vector<char>& b, const u64* data, const std::vector<u64>& mods, int N);

class Reader {
 public:
  Reader(const char* p, size_t n) : p_(p), n_(n) {}
  u64 get_u64();
  // ring.Poly of exactly mods.size() limbs of N coefficients into out[l*N + n],
  // converted back from Montgomery form; throws on any shape mismatch
  void get_poly(u64* out, const std::vector<u64>& mods, int N, const char* what);
  size_t left() const { return n_ - off_; }

 private:
  const char* p_;
  size_t n_, off_ = 0;
};

}  // namespace wire
}  // namespace orion
