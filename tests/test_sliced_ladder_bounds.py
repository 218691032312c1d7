"""CPU: value-level model of the row-sliced ladder step of k_acc_powers_s
(csrc/accum_kernels.hpp, round 5: X3 and Y3 left unreduced) -- every product
is the Montgomery product's exact value (a b + M p) / 2^261 with M = -a b / p
mod 2^261 (what the CIOS of slice29.hpp and fp29.hpp computes), every
linear step the same sum of representatives.  Over 127 doublings from several
points of each curve it checks the bounds the kernel's comment states (X < 9.1p,
Y < 9.4p, w < 13.5p, products below 2.94p) and that every stored position is
[2^j] P as a point (X / ZZ, Y / ZZZ, with ZZ = Z^2, ZZZ = Z^3 from the rows'
ZZ3 = Z3^2 and ZZZ3 = ZZ3 Z3), and that k_acc_termadd's negation (12p - Y) and
store reduction take these representatives."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pasta as P  # noqa: E402

R = 1 << 261
CURVES = {"pallas": (P.PALLAS_P, 5, (P.PALLAS_P - 1, 2)), "bn254": (P.BN254_P, 3, (1, 2))}


def mont(p, a, b):
    t = a * b
    m = (-t * pow(p, -1, R)) % R
    assert (t + m * p) % R == 0
    return (t + m * p) // R


def aff_dbl(p, pt):
    x, y = pt
    lam = 3 * x * x * pow(2 * y, -1, p) % p
    x3 = (lam * lam - 2 * x) % p
    return x3, (lam * (x - x3) - y) % p


@pytest.mark.parametrize("curve", sorted(CURVES))
def test_unreduced_ladder_bounds(curve):
    p, b, G = CURVES[curve]
    rinv = pow(R, -1, p)
    to_m = lambda v: v * R % p  # noqa: E731
    def add(p1, p2):
        if p1 == p2:
            return aff_dbl(p, p1)
        lam = (p2[1] - p1[1]) * pow(p2[0] - p1[0], -1, p) % p
        x3 = (lam * lam - p1[0] - p2[0]) % p
        return x3, (lam * (p1[0] - x3) - p1[1]) % p

    pts, cur = [], G
    for k in range(2, 40):  # G, 2G, ... : take five of them
        if k in (2, 3, 6, 17, 39):
            pts.append(cur)
        cur = add(cur, G)
    assert all((y * y - x ** 3 - b) % p == 0 for x, y in pts)
    worst = {"X": 0, "Y": 0, "w": 0, "E": 0}
    for P0 in pts:
        X, Y, Z = to_m(P0[0]), to_m(P0[1]), to_m(1)
        true = P0
        for j in range(1, 128):
            B = mont(p, Y, Y)
            YZ = mont(p, Y, Z)
            E = mont(p, 3 * X, X)
            Z3 = 2 * YZ
            C4 = mont(p, 4 * B, B)
            D = mont(p, 4 * X, B)
            FF = mont(p, E, E)
            ZZ3 = mont(p, Z3, Z3)
            X3 = FF + 8 * p - 2 * D
            w = D + 12 * p - X3
            r3 = mont(p, E, w)
            ZZZ3 = mont(p, ZZ3, Z3)
            Y3 = r3 + 8 * p - 2 * C4
            for k, v in (("X", X3), ("Y", Y3), ("w", w), ("E", E)):
                worst[k] = max(worst[k], v / p)
            assert 0 < X3 < 9.1 * p and 0 < Y3 < 9.4 * p and 0 < w < 13.5 * p and E < 2.94 * p
            assert max(B, D, FF, C4, r3, ZZ3, ZZZ3) < 2 * p
            X, Y, Z = X3, Y3, Z3
            true = aff_dbl(p, true)
            zz, zzz = ZZ3 * rinv % p, ZZZ3 * rinv % p
            assert (X * rinv * pow(zz, -1, p) % p, Y * rinv * pow(zzz, -1, p) % p) == true
            # k_acc_termadd: 12p - Y (then normalised, reduced below 3p) and the store's reduction
            assert 0 < 12 * p - Y < 16 * p and X < 16 * p and Y < 16 * p
    assert worst["X"] < 9.1 and worst["Y"] < 9.4
