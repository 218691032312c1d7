"""CPU model of the accumulator ladder's quad doubling (coop29.hpp
jac29_dbl_q_ext, k_acc_powers): every lane's operands and results in the
radix-2^29 lazy representation, with the bounds fp29.hpp states checked at
each step (operand limb products <= 2^60, a b < R p, 64-bit column sums,
u32 limbs in add / sub / norm, reduce3's Norm < 16p input), and the 127-step
chain checked against affine doubling on BN254.  The limb constants (K6,
K8x3, QMAGIC) are read from fp29.hpp so the model checks the kernel's own.
The GPU tests (tests/test_accum_gpu.py) check the kernel's results against the
oracle; this one checks that no lazy bound is exceeded on the way.
"""
import os
import random
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 21888242871839275222246405745257275088696311157297823662689037894645226208583  # BN254 Fq
R = 1 << 261
M29 = (1 << 29) - 1


def _consts():
    txt = open(os.path.join(ROOT, "halo2-aggregation_amd", "csrc", "fp29.hpp")).read()
    blk = txt[txt.index("struct F29Consts<Bn254Fq>"):]
    blk = blk[:blk.index("\n};")]

    def arr(name):
        m = re.search(r"\b%s\[9\] = \{([^}]*)\}" % name, blk)
        return [int(x.strip().rstrip("u"), 16) for x in m.group(1).split(",")]

    q = int(re.search(r"QMAGIC = (0x[0-9a-f]+)u", blk).group(1), 16)
    return arr("P"), arr("K6"), arr("K8x3"), q, arr("ONE")


PL, K6, K8x3, QMAGIC, ONE = _consts()


def val(a):
    return sum(x << (29 * i) for i, x in enumerate(a))


def limbs(v):
    return [(v >> (29 * i)) & M29 for i in range(8)] + [v >> 232]


def mul(a, b):
    """f29_mul (additive form, fp29.hpp) with its stated preconditions and
    every 64-bit accumulator value checked."""
    assert max(a) * max(b) <= 1 << 60, "operand limb product"
    assert val(a) * val(b) < R * P, "a b < R p"
    inv = (-pow(P, -1, 1 << 29)) % (1 << 29)
    m, r, acc = [0] * 9, [0] * 9, 0
    for k in range(17):
        for i in range(9):
            j = k - i
            if 0 <= j < 9:
                acc += a[i] * b[j]
        for i in range(9):
            j = k - i
            if i < k and 1 <= j < 9:
                acc += m[i] * PL[j]
        if k < 9:
            m[k] = ((acc & 0xFFFFFFFF) * inv) & M29
            acc += m[k] * PL[0]
        else:
            r[k - 9] = acc & M29
        assert acc < 1 << 64, "column overflow"
        acc >>= 29
    r[8] = acc
    assert val(r) < 2 * P and max(r[:8]) <= M29
    return r


def add(a, b):
    r = [x + y for x, y in zip(a, b)]
    assert max(r) < 1 << 32
    return r


def sub(a, b, K):
    assert all(k >= y for k, y in zip(K, b)), "K must dominate b limb-wise"
    r = [x + k - y for x, k, y in zip(a, K, b)]
    assert max(r) < 1 << 32
    return r


def norm(a):
    assert max(a) < (1 << 32) - 8
    r, c = [0] * 9, 0
    for i in range(8):
        v = a[i] + c
        r[i], c = v & M29, v >> 29
    r[8] = a[8] + c
    return r


def reduce3(a):
    assert max(a[:8]) <= M29 and val(a) < 16 * P, "reduce3 input Norm < 16p"
    q = (a[8] * QMAGIC) >> 40
    r, c = [0] * 9, 0
    for i in range(9):
        v = a[i] - q * PL[i] + c
        r[i] = v & M29 if i < 8 else v
        c = v >> 29
    assert 0 <= val(r) < 3 * P and max(r[:8]) <= M29
    return r


def dbl_q_ext(X, Y, Z, beta):
    """jac29_dbl_q_ext, one quad: lanes 1, 2 hold Y (lanes 0, 3 a dummy);
    returns (X3, Y3 of lane 1, Z3, ZZ3, ZZZ3, beta X3)."""
    # L1: (X, X) / (Y, Y) / (Y, Z) / (3X, X)
    X3x = [x * 3 for x in X]
    B, YZ, E = mul(Y, Y), mul(Y, Z), mul(X3x, X)
    Z3 = add(YZ, YZ)
    # L2: (4B, B) / (4X, B) / (E, E) / (Z3, Z3)
    C4 = mul([x << 2 for x in B], B)
    D = mul([x << 2 for x in X], B)
    FF = mul(E, E)
    ZZ3 = mul(Z3, Z3)
    X3 = reduce3(norm(sub(FF, add(D, D), K8x3)))
    w = sub(D, X3, K6)
    C8 = add(C4, C4)
    # L3: (beta, X3) / (E, w) / (E, w) / (ZZ3, Z3); lanes 0 and 3 keep a dummy Y
    bx = mul(beta, X3)
    r3 = mul(E, w)
    ZZZ3 = mul(ZZ3, Z3)
    Y3 = reduce3(norm(sub(r3, C8, K8x3)))
    for dummy in (bx, ZZZ3):
        reduce3(norm(sub(dummy, C8, K8x3)))
    return X3, Y3, Z3, ZZ3, ZZZ3, bx


def to_mont(x):
    return limbs(x * R % P)


def from_mont(a):
    return val(a) * pow(R, -1, P) % P


def aff_dbl(x, y):
    lam = 3 * x * x * pow(2 * y, -1, P) % P
    x3 = (lam * lam - 2 * x) % P
    return x3, (lam * (x - x3) - y) % P


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_ladder_doubling_chain_bounds_and_values(seed):
    rng = random.Random(seed)
    # a random BN254 point (y^2 = x^3 + 3), both signs of y
    while True:
        x = rng.randrange(P)
        t = (x * x * x + 3) % P
        y = pow(t, (P + 1) // 4, P)
        if y * y % P == t:
            break
    if rng.random() < 0.5:
        y = P - y
    beta = to_mont(pow(2, (P - 1) // 3, P))  # any Norm constant < p exercises the bounds
    X, Y, Z = to_mont(x), to_mont(y), list(ONE)
    ax, ay = x, y
    for step in range(127):
        X, Y, Z, ZZ, ZZZ, bx = dbl_q_ext(X, Y, Z, beta)
        ax, ay = aff_dbl(ax, ay)
        z = from_mont(Z)
        assert from_mont(X) == ax * z * z % P, step
        assert from_mont(Y) == ay * z * z * z % P, step
        assert from_mont(ZZ) == z * z % P and from_mont(ZZZ) == z * z * z % P
        assert from_mont(bx) == from_mont(beta) * from_mont(X) % P
        assert max(Z) < 1 << 30 and val(Z) < 4 * P
