"""ctypes wrapper of the CPU parity oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  The product path (orion_amd/) never does.

Restates Lattigo-v6 RNS-CKKS arithmetic reached from
/root/reference/orion/backend/lattigo/*.go (see ckks_oracle.h for the
function-by-function citations).  Parity with Lattigo itself is unpinned.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libckks_oracle.so")

_u64p = ctypes.POINTER(ctypes.c_uint64)
_intp = ctypes.POINTER(ctypes.c_int)
_dblp = ctypes.POINTER(ctypes.c_double)
_u32p = ctypes.POINTER(ctypes.c_uint32)


class OracleBtp(ctypes.Structure):
    """oracle_btp (ckks_oracle.h): the bootstrapping keys, the circuit's only
    shared inputs besides the input ciphertext."""
    _fields_ = [("rlk", _u64p), ("ngk", ctypes.c_int), ("galEls", _u64p), ("gks", ctypes.POINTER(_u64p)),
                ("d2s", _u64p), ("s2d", _u64p)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    if not os.path.exists(_LIB_PATH):
        build()
    lib = ctypes.CDLL(_LIB_PATH)
    vp = ctypes.c_void_p
    sig = {
        "oracle_gen_moduli": (ctypes.c_int, [ctypes.c_int, _intp, ctypes.c_int, _intp, ctypes.c_int, _u64p]),
        "oracle_new": (vp, [ctypes.c_int, _u64p, ctypes.c_int, ctypes.c_int]),
        "oracle_new_ring": (vp, [ctypes.c_int, _u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
        "oracle_free": (None, [vp]),
        "oracle_psi": (ctypes.c_uint64, [vp, ctypes.c_int]),
        "oracle_primitive_root": (ctypes.c_uint64, [ctypes.c_uint64]),
        "oracle_ntt": (None, [vp, ctypes.c_int, _u64p]),
        "oracle_intt": (None, [vp, ctypes.c_int, _u64p]),
        "oracle_basis_extend": (None, [vp, _u64p, _intp, ctypes.c_int, _u64p, _intp, ctypes.c_int]),
        "oracle_modup_digit": (None, [vp, _u64p, _intp, ctypes.c_int, _u64p, _intp, ctypes.c_int]),
        "oracle_rescale": (None, [vp, ctypes.c_int, ctypes.c_int, _u64p, _u64p]),
        "oracle_moddown": (None, [vp, ctypes.c_int, _u64p, _u64p]),
        "oracle_gadget_product_lazy": (None, [vp, ctypes.c_int, _u64p, _u64p, _u64p, _u64p]),
        "oracle_keyswitch": (None, [vp, ctypes.c_int, _u64p, _u64p, _u64p, _u64p]),
        "oracle_galois_element": (ctypes.c_uint64, [vp, ctypes.c_int]),
        "oracle_automorphism_ntt": (None, [vp, ctypes.c_uint64, _u64p, _u64p, ctypes.c_int]),
        "oracle_mul_relin": (None, [vp, ctypes.c_int, _u64p, _u64p, _u64p, _u64p]),
        "oracle_rotate": (None, [vp, ctypes.c_int, _u64p, ctypes.c_uint64, _u64p, _u64p]),
        "oracle_lt_bsgs": (None, [vp, ctypes.c_int, _u64p, ctypes.c_int, _intp,
                                  ctypes.POINTER(_u64p), ctypes.c_int, ctypes.c_int, _u64p,
                                  ctypes.POINTER(_u64p), _u64p]),
        "oracle_find_best_bsgs_n1": (ctypes.c_int, [_intp, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
        "oracle_encode": (None, [vp, _dblp, ctypes.c_int, ctypes.c_double, _intp, ctypes.c_int, _u64p]),
        "oracle_decode": (None, [vp, ctypes.c_int, _u64p, ctypes.c_double, _dblp]),
        "oracle_gen_secret": (None, [vp, ctypes.c_uint64, ctypes.c_int, _u64p]),
        "oracle_gen_evk": (None, [vp, ctypes.c_uint64, _u64p, _u64p, _u64p]),
        "oracle_encrypt_sk": (None, [vp, ctypes.c_uint64, ctypes.c_int, _u64p, _u64p, _u64p]),
        "oracle_decrypt": (None, [vp, ctypes.c_int, _u64p, _u64p, _u64p]),
        "oracle_mul_coeffs": (None, [vp, _intp, ctypes.c_int, _u64p, _u64p, _u64p]),
        "oracle_eval_poly": (ctypes.c_int, [vp, ctypes.c_int, _u64p, ctypes.c_longdouble, _dblp, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_longdouble, _u64p, _u64p,
                                            ctypes.POINTER(ctypes.c_longdouble)]),
        "oracle_eval_poly_ldp": (ctypes.c_int, [vp, ctypes.c_int, _u64p, ctypes.POINTER(ctypes.c_longdouble), _dblp,
                                                ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_longdouble), _u64p,
                                                _u64p, ctypes.POINTER(ctypes.c_longdouble)]),
        "oracle_bootstrap": (ctypes.c_int, [vp, vp, vp, ctypes.POINTER(OracleBtp), ctypes.c_int, ctypes.c_longdouble,
                                            _u64p, _u64p, ctypes.POINTER(ctypes.c_longdouble)]),
        "oracle_btp_chain": (ctypes.c_int, [ctypes.c_int, _u64p, ctypes.c_int, ctypes.c_int, _intp, ctypes.c_int,
                                            _u64p]),
        "oracle_btp_cos": (None, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_longdouble)]),
        "oracle_btp_new": (vp, [vp, ctypes.c_int, ctypes.c_int]),
        "oracle_btp_free": (None, [vp]),
        "oracle_btp_params": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_longdouble)]),
        "oracle_btp_cos_of": (ctypes.POINTER(ctypes.c_longdouble), [vp]),
        "oracle_btp_lt_info": (ctypes.c_int, [vp, ctypes.c_int, _intp, _intp, _intp]),
        "oracle_btp_lt_diag": (_u64p, [vp, ctypes.c_int, ctypes.c_int]),
        "oracle_chacha20_block": (None, [_u32p, ctypes.c_uint32, _u32p, _u32p]),
        "oracle_enc_key": (None, [ctypes.c_uint64, _u32p]),
        "oracle_gauss_cdt": (None, [ctypes.c_double, ctypes.c_int, _u64p]),
        "oracle_enc_sample": (None, [ctypes.c_int, _u32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_int64)]),
        "oracle_encrypt_pk": (None, [vp, _u32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, _u64p, _u64p,
                                     _u64p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _p(a):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(_u64p)


def _ip(lst):
    arr = (ctypes.c_int * max(1, len(lst)))(*lst)
    return arr


def gen_moduli(logN, logQ, logP):
    out = np.zeros(len(logQ) + len(logP), dtype=np.uint64)
    rc = lib().oracle_gen_moduli(logN, _ip(logQ), len(logQ), _ip(logP), len(logP), _p(out))
    if rc != 0:
        raise ValueError("prime generation exhausted")
    return [int(x) for x in out]


class Oracle:
    """One parameter set.  Arrays are numpy uint64, limb-major [limbs][N]."""

    def __init__(self, logN, moduli, L, K, ci=False):
        """ci: Lattigo's ConjugateInvariant ring of degree 2^logN (NthRoot 4N,
        N real slots; moduli = 1 mod 4N, i.e. gen_moduli(logN + 1, ...))."""
        self.logN, self.N, self.L, self.K = logN, 1 << logN, L, K
        self.ci = bool(ci)
        self.slots = self.N if self.ci else self.N // 2
        self.moduli = [int(m) for m in moduli]
        arr = np.array(self.moduli, dtype=np.uint64)
        self._h = lib().oracle_new_ring(logN, _p(arr), L, K, int(self.ci))
        self.dnum = (L + K - 1) // K if K else 0

    @classmethod
    def from_logs(cls, logN, logQ, logP):
        return cls(logN, gen_moduli(logN, logQ, logP), len(logQ), len(logP))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.oracle_free(self._h)
            self._h = None

    # -- single limb ------------------------------------------------------
    def ntt(self, m, a):
        a = np.ascontiguousarray(a, dtype=np.uint64).copy()
        lib().oracle_ntt(self._h, m, _p(a))
        return a

    def intt(self, m, a):
        a = np.ascontiguousarray(a, dtype=np.uint64).copy()
        lib().oracle_intt(self._h, m, _p(a))
        return a

    def psi(self, m):
        return int(lib().oracle_psi(self._h, m))

    def qp_mods(self, level):
        return list(range(level + 1)) + [self.L + k for k in range(self.K)]

    # -- polynomial ops ---------------------------------------------------
    def basis_extend(self, x, src, dst):
        x = np.ascontiguousarray(x, dtype=np.uint64)
        out = np.zeros((len(dst), self.N), dtype=np.uint64)
        lib().oracle_basis_extend(self._h, _p(x), _ip(src), len(src), _p(out), _ip(dst), len(dst))
        return out

    def modup_digit(self, x, src, dst):
        """ModUp of one gadget digit (DecomposeAndSplit: centered if one prime)."""
        x = np.ascontiguousarray(x, dtype=np.uint64)
        out = np.zeros((len(dst), self.N), dtype=np.uint64)
        lib().oracle_modup_digit(self._h, _p(x), _ip(src), len(src), _p(out), _ip(dst), len(dst))
        return out

    def rescale(self, ct, level):
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        ncomp = ct.shape[0]
        out = np.zeros((ncomp, level, self.N), dtype=np.uint64)
        lib().oracle_rescale(self._h, level, ncomp, _p(ct), _p(out))
        return out

    def moddown(self, x, level):
        x = np.ascontiguousarray(x, dtype=np.uint64)
        out = np.zeros((level + 1, self.N), dtype=np.uint64)
        lib().oracle_moddown(self._h, level, _p(x), _p(out))
        return out

    def gadget_product_lazy(self, c, evk, level):
        c = np.ascontiguousarray(c, dtype=np.uint64)
        evk = np.ascontiguousarray(evk, dtype=np.uint64)
        o0 = np.zeros((level + 1 + self.K, self.N), dtype=np.uint64)
        o1 = np.zeros_like(o0)
        lib().oracle_gadget_product_lazy(self._h, level, _p(c), _p(evk), _p(o0), _p(o1))
        return o0, o1

    def keyswitch(self, c, evk, level):
        c = np.ascontiguousarray(c, dtype=np.uint64)
        evk = np.ascontiguousarray(evk, dtype=np.uint64)
        o0 = np.zeros((level + 1, self.N), dtype=np.uint64)
        o1 = np.zeros_like(o0)
        lib().oracle_keyswitch(self._h, level, _p(c), _p(evk), _p(o0), _p(o1))
        return o0, o1

    def galois_element(self, k):
        return int(lib().oracle_galois_element(self._h, k))

    def automorphism_ntt(self, x, galEl):
        x = np.ascontiguousarray(x, dtype=np.uint64)
        out = np.zeros_like(x)
        lib().oracle_automorphism_ntt(self._h, galEl, _p(x), _p(out), x.shape[0])
        return out

    def mul_relin(self, a, b, rlk, level):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        b = np.ascontiguousarray(b, dtype=np.uint64)
        out = np.zeros((2, level + 1, self.N), dtype=np.uint64)
        lib().oracle_mul_relin(self._h, level, _p(a), _p(b), _p(np.ascontiguousarray(rlk)), _p(out))
        return out

    def rotate(self, ct, galEl, gk, level):
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        out = np.zeros((2, level + 1, self.N), dtype=np.uint64)
        lib().oracle_rotate(self._h, level, _p(ct), galEl, _p(np.ascontiguousarray(gk)), _p(out))
        return out

    def lt_bsgs(self, ct, level, diag_idx, pts, N1, gkeys):
        """gkeys: dict galEl -> evk array."""
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        out = np.zeros((2, level + 1, self.N), dtype=np.uint64)
        pts = [np.ascontiguousarray(p, dtype=np.uint64) for p in pts]
        ptarr = (_u64p * len(pts))(*[_p(p) for p in pts])
        gels = list(gkeys.keys())
        garr = np.array(gels if gels else [0], dtype=np.uint64)
        karrs = [np.ascontiguousarray(gkeys[g]) for g in gels]
        karr = (_u64p * max(1, len(karrs)))(*[_p(k) for k in karrs])
        lib().oracle_lt_bsgs(self._h, level, _p(ct), len(diag_idx), _ip(diag_idx), ptarr, N1,
                             len(gels), _p(garr), karr, _p(out))
        return out

    def find_best_bsgs_n1(self, diag_idx, log_ratio=0):
        return int(lib().oracle_find_best_bsgs_n1(_ip(diag_idx), len(diag_idx), self.slots, log_ratio))

    def encode(self, values, scale, mods):
        v = np.ascontiguousarray(values, dtype=np.float64)
        out = np.zeros((len(mods), self.N), dtype=np.uint64)
        lib().oracle_encode(self._h, v.ctypes.data_as(_dblp), len(v), float(scale), _ip(mods),
                            len(mods), _p(out))
        return out

    def decode(self, pt, level, scale):
        pt = np.ascontiguousarray(pt, dtype=np.uint64)
        out = np.zeros(self.slots, dtype=np.float64)
        lib().oracle_decode(self._h, level, _p(pt), float(scale), out.ctypes.data_as(_dblp))
        return out

    def gen_secret(self, seed, h):
        sk = np.zeros((self.L + self.K, self.N), dtype=np.uint64)
        lib().oracle_gen_secret(self._h, seed, h, _p(sk))
        return sk

    def gen_evk(self, seed, s_in, s_out):
        evk = np.zeros((self.dnum, 2, self.L + self.K, self.N), dtype=np.uint64)
        lib().oracle_gen_evk(self._h, seed, _p(np.ascontiguousarray(s_in)),
                             _p(np.ascontiguousarray(s_out)), _p(evk))
        return evk

    def encrypt_sk(self, seed, sk, pt, level):
        ct = np.zeros((2, level + 1, self.N), dtype=np.uint64)
        lib().oracle_encrypt_sk(self._h, seed, level, _p(np.ascontiguousarray(sk)),
                                _p(np.ascontiguousarray(pt)), _p(ct))
        return ct

    def decrypt(self, ct, sk, level):
        pt = np.zeros((level + 1, self.N), dtype=np.uint64)
        lib().oracle_decrypt(self._h, level, _p(np.ascontiguousarray(sk)),
                             _p(np.ascontiguousarray(ct)), _p(pt))
        return pt

    def mul_coeffs(self, a, b, mods):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        b = np.ascontiguousarray(b, dtype=np.uint64)
        out = np.zeros_like(a)
        lib().oracle_mul_coeffs(self._h, _ip(mods), len(mods), _p(a), _p(b), _p(out))
        return out

    def eval_poly(self, ct, level, scale, coeffs, cheb, target, rlk):
        """The HIP backend's EvaluatePolynomial restated: returns (ct_out,
        out_level, out_scale); coeffs lowest degree first."""
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        cf = np.ascontiguousarray(coeffs, dtype=np.float64)
        out = np.zeros(2 * (level + 1) * self.N, dtype=np.uint64)  # [2][out_level+1][N] written flat
        osc = ctypes.c_longdouble(0)
        lv = lib().oracle_eval_poly(self._h, level, _p(ct), scale, cf.ctypes.data_as(_dblp), len(cf), int(cheb),
                                    target, _p(np.ascontiguousarray(rlk)), _p(out), ctypes.byref(osc))
        if lv < 0:
            raise ValueError("level < depth")
        return out[:2 * (lv + 1) * self.N].reshape(2, lv + 1, self.N).copy(), lv, osc.value

    def bootstrap(self, boot, circuit, keys, ct, level, scale):
        """Bootstrap restated (oracle_bootstrap): self = the scheme's oracle,
        boot = the bootstrapping chain's oracle, circuit = BtpCircuit (the
        oracle's own constants and diagonals), keys = dict(rlk, gks {galEl:
        key}, d2s, s2d) of the bootstrapping chain, ct [2][level+1][N] at
        `scale`.  Returns ([2][L][N] at the residual top level, its scale as
        numpy longdouble)."""
        keep = []

        def u64arr(a):
            a = np.ascontiguousarray(a, dtype=np.uint64)
            keep.append(a)
            return _p(a)

        P = OracleBtp()
        gels = list(keys["gks"].keys())
        P.ngk, P.galEls = len(gels), u64arr(gels if gels else [0])
        ka = (_u64p * max(1, len(gels)))(*[u64arr(keys["gks"][g]) for g in gels])
        keep.append(ka)
        P.gks, P.rlk = ka, u64arr(keys["rlk"])
        P.d2s, P.s2d = u64arr(keys["d2s"]), u64arr(keys["s2d"])
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        out = np.zeros((2, self.L, self.N), dtype=np.uint64)
        osc = ctypes.c_longdouble(0)
        rc = lib().oracle_bootstrap(self._h, boot._h, circuit._h, ctypes.byref(P), level, ctypes.c_longdouble(scale),
                                    _p(ct), _p(out), ctypes.byref(osc))
        if rc != 0:
            raise ValueError("oracle_bootstrap: missing key or level mismatch")
        return out, np.longdouble(osc.value)

    def eval_poly_ld(self, ct, level, scale, coeffs, cheb, target, rlk):
        """eval_poly with 80-bit scales (numpy longdouble in and out, not via double)."""
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        cf = np.ascontiguousarray(coeffs, dtype=np.float64)
        out = np.zeros(2 * (level + 1) * self.N, dtype=np.uint64)
        xs = np.array([scale], dtype=np.longdouble)
        tg = np.array([target], dtype=np.longdouble)
        osc = np.zeros(1, dtype=np.longdouble)
        ldp = ctypes.POINTER(ctypes.c_longdouble)
        lv = lib().oracle_eval_poly_ldp(self._h, level, _p(ct), xs.ctypes.data_as(ldp), cf.ctypes.data_as(_dblp),
                                        len(cf), int(cheb), tg.ctypes.data_as(ldp), _p(np.ascontiguousarray(rlk)),
                                        _p(out), osc.ctypes.data_as(ldp))
        if lv < 0:
            raise ValueError("level < depth")
        return out[:2 * (lv + 1) * self.N].reshape(2, lv + 1, self.N).copy(), lv, osc[0]

    def encrypt_pk(self, seed, enc, image, pk, pt, level):
        """The HIP backend's public-key encryption of image `image` in
        encryption number `enc` (encoder.hip sampler, restated)."""
        ct = np.zeros((2, level + 1, self.N), dtype=np.uint64)
        lib().oracle_encrypt_pk(self._h, _u32(enc_key(seed)), enc, image, level,
                                _p(np.ascontiguousarray(pk)), _p(np.ascontiguousarray(pt)), _p(ct))
        return ct


def _u32(a):
    assert a.dtype == np.uint32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u32p)


def chacha20_block(key, counter, nonce):
    """RFC 8439 §2.3 block function: 8 key words, counter, 3 nonce words -> 16 words."""
    out = np.zeros(16, dtype=np.uint32)
    lib().oracle_chacha20_block(_u32(np.asarray(key, dtype=np.uint32)), counter,
                                _u32(np.asarray(nonce, dtype=np.uint32)), _u32(out))
    return out


def enc_key(seed):
    key = np.zeros(8, dtype=np.uint32)
    lib().oracle_enc_key(seed, _u32(key))
    return key


def gauss_cdt(sigma=3.2, bound=19):
    t = np.zeros(2 * bound, dtype=np.uint64)
    lib().oracle_gauss_cdt(sigma, bound, _p(t))
    return t


def enc_sample(N, seed, enc, image, comp):
    out = np.zeros(N, dtype=np.int64)
    lib().oracle_enc_sample(N, _u32(enc_key(seed)), enc, image, comp,
                            out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    return out


def btp_chain(logN, scheme_moduli, Lres, logP):
    """The bootstrapping chain (Q primes, P primes) derived by the oracle from
    the scheme's moduli and the bootstrapper's logPs (oracle_btp_chain)."""
    sm = np.array(scheme_moduli, dtype=np.uint64)
    out = np.zeros(128, dtype=np.uint64)
    n = lib().oracle_btp_chain(logN, _p(sm), len(sm), Lres, _ip(list(logP)), len(logP), _p(out))
    if n < 0:
        raise ValueError("prime stream exhausted")
    m = [int(x) for x in out[:n]]
    return m[:n - len(logP)], m[n - len(logP):]


def btp_cos(K, degree, r):
    """EvalMod's Chebyshev coefficients (oracle_btp_cos), as numpy longdouble."""
    out = np.zeros(degree + 1, dtype=np.longdouble)
    lib().oracle_btp_cos(K, degree, r, out.ctypes.data_as(ctypes.POINTER(ctypes.c_longdouble)))
    return out


class BtpCircuit:
    """The oracle's own bootstrapping circuit for `slots` slots under the
    bootstrapping chain `boot` (an Oracle), scheme default scale 2^log_scale:
    constants, diagonals and trace elements derived from the parameters."""

    def __init__(self, boot, log_scale, slots):
        self.boot = boot  # keeps the chain's context alive
        self._h = lib().oracle_btp_new(boot._h, log_scale, slots)
        if not self._h:
            raise ValueError("oracle_btp_new: unsupported slot count or chain")

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.oracle_btp_free(self._h)
            self._h = None

    def params(self):
        """dict: F, gap, K, r, degree, slots, s_y, top, ntrace, nlt, ncos, t0 (longdouble)."""
        out = np.zeros(16, dtype=np.longdouble)
        n = lib().oracle_btp_params(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_longdouble)))
        names = ["F", "gap", "K", "r", "degree", "slots", "s_y", "top", "ntrace", "nlt", "ncos", "t0"]
        return dict(zip(names, out[:n]))

    def cos(self):
        """The circuit's cosine coefficients as 80-bit values (read as bytes:
        indexing a ctypes c_longdouble pointer would round them to double)."""
        n = int(self.params()["ncos"])
        p = lib().oracle_btp_cos_of(self._h)
        ld = np.dtype(np.longdouble).itemsize
        return np.frombuffer(ctypes.string_at(p, n * ld), dtype=np.longdouble).copy()

    def lt(self, k):
        """(level, N1, diagonal indices, diagonals [level+1+K][N]) of transform k."""
        lv, n1 = ctypes.c_int(0), ctypes.c_int(0)
        nd = lib().oracle_btp_lt_info(self._h, k, ctypes.byref(lv), ctypes.byref(n1), None)
        idx = (ctypes.c_int * max(1, nd))()
        lib().oracle_btp_lt_info(self._h, k, ctypes.byref(lv), ctypes.byref(n1), idx)
        nl = lv.value + 1 + self.boot.K
        diags = []
        for j in range(nd):
            p = lib().oracle_btp_lt_diag(self._h, k, j)
            diags.append(np.ctypeslib.as_array(p, shape=(nl * self.boot.N,)).reshape(nl, self.boot.N).copy())
        return lv.value, n1.value, [idx[i] for i in range(nd)], diags

