"""Generate first-principles known-answer tests (tests/golden/kat_*.json) with
pure-Python big integers -- independent of the C oracle and of the HIP
backend.  The reference holds no golden vectors for this path (SURVEY.md §4,
§8c), so these pin the CPU restatement mathematically:

  * ntt:       negacyclic NTT by definition, out[j] = a(psi^(2*brv(j)+1)) mod q
  * rescale:   round(x / q_l) of the CRT-reconstructed, centered integer
  * moddown:   floor(x / P) of x in [0, Q*P)
  * basisext:  exact residues of x in [0, S) modulo other primes
  * bext_quotient: Lattigo's reconstructRNS quotient v = trunc(sum_i
               float64(y_i) / float64(s_i)) (correctly rounded divisions in
               source order), on coefficients x near 0 and near S where it
               is not floor(x / S) and where a reciprocal multiply
               y_i * (1/s_i) truncates to a different v
  * modup_single: DecomposeAndSplit's single-prime digit, extended from the
               centered representative (x >= s >> 1 -> x - s)
  * automorph: a(X^g) mod (X^N + 1) in the coefficient domain
  * primes:    NTT-friendly prime walk around 2^b (Lattigo GenModuli rule)

Usage: python tools/gen_kats.py
"""
import json
import math
import os
import random

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def is_prime(n):
    if n < 2:
        return False
    for p in [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37]:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37]:
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def prime_walk(bits, nthroot, count):
    """Alternate upward/downward from 2^bits+1 in steps of nthroot while within
    half a bit of 2^bits (61-bit: downward only)."""
    out = []
    up = down = (1 << bits) + 1
    up_ok = down_ok = True
    while len(out) < count:
        if bits == 61:
            down -= nthroot
            if bits - math.log2(down) >= 0.5:
                raise RuntimeError("exhausted")
            if is_prime(down):
                out.append(down)
            continue
        if not (up_ok or down_ok):
            raise RuntimeError("exhausted")
        if up_ok:
            if math.log2(up) - bits >= 0.5:
                up_ok = False
            else:
                up += nthroot
                if is_prime(up):
                    out.append(up)
                    continue
        if down_ok:
            if down < nthroot or bits - math.log2(down) >= 0.5:
                down_ok = False
            else:
                down -= nthroot
                if is_prime(down):
                    out.append(down)
    return out


def gen_moduli(logn, logq, logp):
    nth = 2 << logn
    need = {}
    for b in logq + logp:
        need[b] = need.get(b, 0) + 1
    pool = {b: prime_walk(b, nth, c) for b, c in need.items()}
    used = {b: 0 for b in need}
    out = []
    for b in logq + logp:
        out.append(pool[b][used[b]])
        used[b] += 1
    return out


def factor(n):
    f, d = [], 2
    while d * d <= n:
        if n % d == 0:
            f.append(d)
            while n % d == 0:
                n //= d
        d += 1 if d == 2 else 2
    if n > 1:
        f.append(n)
    return f


def prim_root(q):
    fs = factor(q - 1)
    g = 3
    while any(pow(g, (q - 1) // f, q) == 1 for f in fs):
        g += 1
    return g


def brv(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


def ntt_def(a, q, psi, logn):
    n = len(a)
    return [sum(a[k] * pow(psi, (2 * brv(j, logn) + 1) * k, q) for k in range(n)) % q for j in range(n)]


def crt(res, mods):
    Q = 1
    for m in mods:
        Q *= m
    x = 0
    for r, m in zip(res, mods):
        Mi = Q // m
        x += r * Mi * pow(Mi, -1, m)
    return x % Q, Q


def lattigo_v(ys, srcm):
    """reconstructRNS: vi += float64(y_i) / float64(Q[i]); v = uint64(vi)"""
    vf = 0.0
    for y, q in zip(ys, srcm):
        vf += float(y) / float(q)
    return int(vf)


def reciprocal_v(ys, srcm):
    """the same sum with y_i * (1/s_i) (the builder's round-2 form)"""
    vf = 0.0
    for y, q in zip(ys, srcm):
        vf += float(y) * (1.0 / float(q))
    return int(vf)


def bext_quotient_case(rng, mods, src, n):
    """n coefficients x of the sources' product S, at least half of them ones
    where the division form and the reciprocal form truncate differently;
    expected outputs follow the division form"""
    srcm = [mods[i] for i in src]
    dst = [j for j in range(len(mods)) if j not in src]
    S = 1
    for q in srcm:
        S *= q
    qhinv = [pow(S // q, -1, q) for q in srcm]

    def ys_of(x):
        return [(x % q) * h % q for q, h in zip(srcm, qhinv)]

    diff, same = [], []
    while len(diff) < n // 2 or len(same) < n - n // 2:
        k = rng.randrange(1 << 24)
        x = k if rng.random() < 0.5 else S - 1 - k
        ys = ys_of(x)
        vd, vr = lattigo_v(ys, srcm), reciprocal_v(ys, srcm)
        (diff if vd != vr else same).append(x)
    xs = diff[:n // 2] + same[:n - n // 2]
    outs, vds, vrs, vex = [], [], [], []
    for x in xs:
        ys = ys_of(x)
        vd = lattigo_v(ys, srcm)
        X = sum(y * (S // q) for y, q in zip(ys, srcm))
        vds.append(vd)
        vrs.append(reciprocal_v(ys, srcm))
        vex.append(X // S)
        outs.append([(X - vd * S) % mods[t] for t in dst])
    return dict(src=src, dst=dst, x=[[x % q for x in xs] for q in srcm],
                out=[[o[t] for o in outs] for t in range(len(dst))], v_div=vds, v_rcp=vrs, v_floor=vex)


def main():
    rng = random.Random(20251016)
    os.makedirs(OUT, exist_ok=True)
    kats = {}

    # primes (several parameter sets of the build's configs)
    kats["primes"] = []
    for logn, logq, logp in [(13, [55, 40, 40], [60, 60]), (15, [60] + [40] * 11, [60, 60]),
                             (13, [29, 26, 26, 26, 26, 26], [29, 29]), (14, [61, 50], [61])]:
        kats["primes"].append(dict(logn=logn, logq=logq, logp=logp, moduli=gen_moduli(logn, logq, logp)))

    # NTT by definition at small N
    kats["ntt"] = []
    for logn in (3, 5, 6):
        n = 1 << logn
        for bits in (40, 60):
            q = prime_walk(bits, 2 * n, 1)[0]
            g = prim_root(q)
            psi = pow(g, (q - 1) // (2 * n), q)
            a = [rng.randrange(q) for _ in range(n)]
            kats["ntt"].append(dict(logn=logn, q=q, g=g, psi=psi, a=a, out=ntt_def(a, q, psi, logn)))

    # basis extension / rescale / moddown at N=16 with the (logn=4) chain
    logn = 4
    n = 1 << logn
    mods = gen_moduli(logn, [50, 40, 40, 40], [60, 60])
    L, K = 4, 2
    kats["chain"] = dict(logn=logn, moduli=mods, L=L, K=K)
    # basis extension: x in [0, S), S = q0*q1, targets q2, q3, p0, p1
    src, dst = [0, 1], [2, 3, 4, 5]
    S = mods[0] * mods[1]
    xs = [rng.randrange(S) for _ in range(n)]
    kats["basisext"] = dict(src=src, dst=dst, x=[[x % mods[i] for x in xs] for i in src],
                            out=[[x % mods[t] for x in xs] for t in dst])
    # the float64 quotient of ModUpExact (Lattigo reconstructRNS [U]):
    # near-integer sums, where the division form decides the bits
    kats["bext_quotient"] = [bext_quotient_case(rng, mods, src, n)
                             for src in ([1, 2], [0, 1, 2], [4, 5], [1, 2, 3])]
    # single-prime digit (K = 1 digits, or the last digit of an odd level)
    src, dst = [1], [0, 2, 3, 4, 5]
    s1 = mods[1]
    xs = [rng.randrange(s1) for _ in range(n - 4)] + [s1 >> 1, (s1 >> 1) - 1, 0, s1 - 1]
    kats["modup_single"] = dict(src=src, dst=dst, x=[xs],
                                out=[[(x - s1 if x >= s1 >> 1 else x) % mods[t] for x in xs] for t in dst])
    # rescale at level 3: coefficient-domain residues of x, expected round(xc / q3) for centered xc
    lvl = 3
    Q = 1
    for m in mods[:lvl + 1]:
        Q *= m
    xs = [rng.randrange(Q) for _ in range(n)]
    exp = []
    for x in xs:
        xc = x - Q if x > Q // 2 else x
        # round half up, like floor((x + q/2)/q) of Lattigo's DivRoundByLastModulus
        r = (xc + mods[lvl] // 2) // mods[lvl]
        exp.append(r)
    kats["rescale"] = dict(level=lvl, x=[[x % m for x in xs] for m in mods[:lvl + 1]],
                           out=[[r % m for r in exp] for m in mods[:lvl]])
    # moddown at level 2: x in [0, Q2*P), expected floor(x / P) mod q_j
    lvl = 2
    QP = 1
    for m in mods[:lvl + 1] + mods[L:]:
        QP *= m
    P = mods[L] * mods[L + 1]
    xs = [rng.randrange(QP) for _ in range(n)]
    kats["moddown"] = dict(level=lvl, x=[[x % m for x in xs] for m in mods[:lvl + 1] + mods[L:]],
                           out=[[(x // P) % m for x in xs] for m in mods[:lvl + 1]])
    # automorphism X -> X^g in the coefficient domain (negacyclic)
    q = mods[1]
    a = [rng.randrange(q) for _ in range(n)]
    autos = []
    for g in (5, 25, 2 * n - 1):
        out = [0] * n
        for i, c in enumerate(a):
            e = (i * g) % (2 * n)
            if e < n:
                out[e] = (out[e] + c) % q
            else:
                out[e - n] = (out[e - n] - c) % q
        autos.append(dict(g=g, out=out))
    kats["automorph"] = dict(modidx=1, a=a, cases=autos)

    with open(os.path.join(OUT, "kat_ckks.json"), "w") as f:
        json.dump(kats, f)
    print("wrote", os.path.join(OUT, "kat_ckks.json"))


if __name__ == "__main__":
    main()
