"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the Pasta MSM hot path.

This module is the Python big-integer restatement used as the *checker* for the
HIP path.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it; the product library never does.

PARITY STATUS: parity unpinned by the reference.  The reference
(Trapdoor-Tech/halo2-aggregation) reaches its MSM through the un-vendored
halo2 fork ``kzg-agg2`` (``/root/reference/Cargo.toml:12``) and holds no test
vectors (``/root/reference/src/lib.rs:43-44`` is an empty test module).  The
restatement below is pinned instead by (a) curve constants checked at import
(primality-free checks: generator on curve, [r]G = O), (b) a known-discrete-log
identity (MSM of P_i = [a_i]G equals [sum s_i a_i]G), and (c) agreement with
the independent C restatement in ``oracle/msm_ref.c``.

Restated third-party algorithms (not present in /root/reference):
  * pasta_curves (Pallas / Vesta): short Weierstrass y^2 = x^3 + 5, Montgomery
    form with R = 2^256, affine identity encoded as (0, 0).
  * halo2 ``arithmetic::multiexp_serial`` / ``best_multiexp`` (reached from
    ``/root/reference/examples/simple-example.rs:606,620,638-640,702,722``):
    unsigned c-bit windows, c = 1 (n<4), 3 (n<32), else ceil(ln n);
    segments = 256 // c + 1; (2^c - 1) buckets; summation-by-parts; c doublings
    per segment; best_multiexp splits into ``num_threads`` contiguous chunks
    of ``n // num_threads`` and folds the partial results.
"""
from __future__ import annotations

import math

M64 = (1 << 64) - 1

# --- curve constants ---------------------------------
PALLAS_P = 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001
VESTA_P = 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001
BN254_P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
BN254_R = 21888242871839275222246405745257275088548364400416034343698204186575808495617

R_MONT = 1 << 256


class Curve:
    """Short Weierstrass curve y^2 = x^3 + b over F_p with group order r."""

    def __init__(self, name, p, r, b, gen, nbits):
        self.name, self.p, self.r, self.b, self.gen = name, p, r, b, gen
        self.scalar_bits = nbits

    # --- field helpers --------------------------------------------------------
    def to_mont(self, a):
        return (a * R_MONT) % self.p

    def from_mont(self, a):
        return (a * pow(R_MONT, -1, self.p)) % self.p

    def on_curve(self, P):
        if P is None:
            return True
        x, y = P
        return (y * y - x * x * x - self.b) % self.p == 0

    # --- affine group law (None = identity) ----------------------------------
    def neg(self, P):
        if P is None:
            return None
        return (P[0], (-P[1]) % self.p)

    def add(self, P, Q):
        p = self.p
        if P is None:
            return Q
        if Q is None:
            return P
        x1, y1 = P
        x2, y2 = Q
        if x1 == x2:
            if (y1 + y2) % p == 0:
                return None
            lam = (3 * x1 * x1) * pow(2 * y1, -1, p) % p
        else:
            lam = (y2 - y1) * pow(x2 - x1, -1, p) % p
        x3 = (lam * lam - x1 - x2) % p
        return (x3, (lam * (x1 - x3) - y1) % p)

    # --- Jacobian arithmetic (fast path for the restatement) -----------------
    # (X, Y, Z) with x = X/Z^2, y = Y/Z^3; Z == 0 is the identity.
    def jac(self, P):
        return (0, 1, 0) if P is None else (P[0], P[1], 1)

    def jdbl(self, A):
        p = self.p
        X, Y, Z = A
        if Z == 0 or Y == 0:
            return (0, 1, 0)
        XX = X * X % p
        YY = Y * Y % p
        YYYY = YY * YY % p
        S = 2 * ((X + YY) ** 2 - XX - YYYY) % p
        M = 3 * XX % p
        X3 = (M * M - 2 * S) % p
        Y3 = (M * (S - X3) - 8 * YYYY) % p
        Z3 = 2 * Y * Z % p
        return (X3, Y3, Z3)

    def jadd(self, A, B):
        p = self.p
        X1, Y1, Z1 = A
        X2, Y2, Z2 = B
        if Z1 == 0:
            return B
        if Z2 == 0:
            return A
        Z1Z1 = Z1 * Z1 % p
        Z2Z2 = Z2 * Z2 % p
        U1 = X1 * Z2Z2 % p
        U2 = X2 * Z1Z1 % p
        S1 = Y1 * Z2 * Z2Z2 % p
        S2 = Y2 * Z1 * Z1Z1 % p
        if U1 == U2:
            if S1 != S2:
                return (0, 1, 0)
            return self.jdbl(A)
        H = (U2 - U1) % p
        I = (2 * H) ** 2 % p
        J = H * I % p
        rr = 2 * (S2 - S1) % p
        V = U1 * I % p
        X3 = (rr * rr - J - 2 * V) % p
        Y3 = (rr * (V - X3) - 2 * S1 * J) % p
        Z3 = ((Z1 + Z2) ** 2 - Z1Z1 - Z2Z2) * H % p
        return (X3, Y3, Z3)

    def jaffine(self, A):
        X, Y, Z = A
        if Z == 0:
            return None
        zi = pow(Z, -1, self.p)
        zi2 = zi * zi % self.p
        return (X * zi2 % self.p, Y * zi2 * zi % self.p)

    def mul(self, k, P):
        """[k]P, affine in/out (double-and-add on Jacobian)."""
        k %= self.r
        acc = (0, 1, 0)
        base = self.jac(P)
        for bit in bin(k)[2:] if k else "":
            acc = self.jdbl(acc)
            if bit == "1":
                acc = self.jadd(acc, base)
        return self.jaffine(acc)

    # --- MSM restatements -----------------------------------------------------
    def msm_naive(self, scalars, points):
        acc = (0, 1, 0)
        for s, P in zip(scalars, points):
            if P is None or s % self.r == 0:
                continue
            acc = self.jadd(acc, self.jac(self.mul(s, P)))
        return self.jaffine(acc)

    def multiexp_serial(self, scalars, points):
        """Restatement of halo2 ``multiexp_serial`` (see module docstring).

        ``scalars`` are canonical integers (the ``to_repr`` value); windows are
        read from the 32-byte little-endian representation exactly like
        halo2's ``get_at`` (bits beyond byte 31 read as zero).
        """
        n = len(points)
        c = 1 if n < 4 else (3 if n < 32 else int(math.ceil(math.log(n))))
        segments = 256 // c + 1
        acc = (0, 1, 0)
        for seg in range(segments - 1, -1, -1):
            for _ in range(c):
                acc = self.jdbl(acc)
            buckets = [None] * ((1 << c) - 1)
            shift = seg * c
            for s, P in zip(scalars, points):
                if shift >= 256:
                    d = 0
                else:
                    d = (s >> shift) & ((1 << c) - 1)
                if d != 0 and P is not None:
                    b = buckets[d - 1]
                    buckets[d - 1] = self.jac(P) if b is None else self.jadd(b, self.jac(P))
            running = (0, 1, 0)
            for b in reversed(buckets):
                if b is not None:
                    running = self.jadd(running, b)
                acc = self.jadd(acc, running)
        return acc

    def best_multiexp(self, scalars, points, num_threads=8):
        """Restatement of halo2 ``best_multiexp``: contiguous chunks of
        ``n // num_threads`` points, one ``multiexp_serial`` per chunk, then a
        left fold of the partial results."""
        n = len(points)
        assert len(scalars) == n
        if n > num_threads:
            chunk = n // num_threads
            acc = (0, 1, 0)
            for lo in range(0, n, chunk):
                part = self.multiexp_serial(scalars[lo:lo + chunk], points[lo:lo + chunk])
                acc = self.jadd(acc, part)
            return self.jaffine(acc)
        return self.jaffine(self.multiexp_serial(scalars, points))


PALLAS = Curve("pallas", PALLAS_P, VESTA_P, 5, (PALLAS_P - 1, 2), 255)
VESTA = Curve("vesta", VESTA_P, PALLAS_P, 5, (VESTA_P - 1, 2), 255)
BN254 = Curve("bn254", BN254_P, BN254_R, 3, (1, 2), 254)
CURVES = {0: PALLAS, 1: VESTA, 2: BN254}


# --- deterministic synthetic inputs --------------------------
GOLDEN = 0x9E3779B97F4A7C15
SEED_BASES = 0xA11CE
SEED_SCALARS = 0x5EED


def mix64(x):
    """SplitMix64 step: advance by the golden gamma, then the finaliser."""
    z = (x + GOLDEN) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def synth_word(seed, i, j):
    return mix64((mix64((seed + i) & M64) + j) & M64)


def synth_scalar(seed, i, r, nbits=255):
    """Uniform in [0, r): 4 words, masked to ``nbits`` bits, rejection-sampled.
    Mirrors ``pm_synth_scalars`` in the HIP library bit for bit."""
    t = 0
    mask_top = (1 << (nbits - 192)) - 1
    while True:
        w = [synth_word(seed, i, 4 * t + k) for k in range(4)]
        w[3] &= mask_top
        v = w[0] | (w[1] << 64) | (w[2] << 128) | (w[3] << 192)
        if v < r:
            return v
        t += 1


def synth_base_dlog(curve, seed, i):
    """Discrete log a_i of synthetic base i: P_i = [a_i]G (a_i nonzero)."""
    a = synth_scalar(seed, i, curve.r, curve.scalar_bits)
    return a if a != 0 else 1


# --- limb packing helpers (C-ABI layout: little-endian u64 limbs) ------------
def to_limbs(v, n=4):
    return [(v >> (64 * k)) & M64 for k in range(n)]


def from_limbs(ls):
    return sum(int(x) << (64 * k) for k, x in enumerate(ls))


def point_to_limbs(curve, P, mont=True):
    """Affine point -> 8 u64 limbs (x then y), Montgomery by default; (0,0) = O."""
    if P is None:
        return [0] * 8
    x, y = P
    if mont:
        x, y = curve.to_mont(x), curve.to_mont(y)
    return to_limbs(x) + to_limbs(y)


def limbs_to_point(curve, ls, mont=True):
    x, y = from_limbs(ls[0:4]), from_limbs(ls[4:8])
    if x == 0 and y == 0:
        return None
    if mont:
        x, y = curve.from_mont(x), curve.from_mont(y)
    return (x, y)


def self_check():
    for c in (PALLAS, VESTA, BN254):
        assert c.on_curve(c.gen), c.name
        assert c.mul(c.r - 1, c.gen) == c.neg(c.gen), c.name
        # [r]G = O: (r-1)G + G
        assert c.add(c.mul(c.r - 1, c.gen), c.gen) is None, c.name
    # the Pasta cycle: Pallas scalar field = Vesta base field and vice versa
    assert PALLAS.r == VESTA.p and VESTA.r == PALLAS.p
    return True
