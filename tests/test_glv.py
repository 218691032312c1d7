"""CPU checks of the GLV constants compiled into the accumulator kernels
(halo2-aggregation_amd/csrc/accum_kernels.hpp, Glv<Curve>): beta is a cube
root of unity of the base field with phi(G) = (beta Gx, Gy) = [lambda]G, the
lattice vectors satisfy a + b lambda = 0 mod r, and the device's decomposition
(floor with 2^384-scaled g1, g2) gives |k1|, |k2| < 2^128 with
k = k1 + lambda k2 mod r on random and edge scalars."""
import os
import random
import re

import pytest

import pasta as P

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "halo2-aggregation_amd", "csrc",
                   "accum_kernels.hpp")
CURVES = {"PallasCurve": P.PALLAS, "VestaCurve": P.VESTA, "Bn254Curve": P.BN254}


def _parse():
    txt = open(HDR).read()
    out = {}
    for m in re.finditer(r"template <> struct Glv<(\w+)> \{(.*?)\n\};", txt, re.S):
        d = {}
        for a in re.finditer(r"static constexpr uint32_t (\w+)\[\d+\] = \{([^}]*)\}", m.group(2)):
            limbs = [int(x.strip().rstrip("u"), 16) for x in a.group(2).split(",")]
            d[a.group(1)] = sum(v << (32 * i) for i, v in enumerate(limbs))
        out[m.group(1)] = d
    return out


@pytest.mark.parametrize("name", list(CURVES))
def test_glv_constants(name):
    C = CURVES[name]
    g = _parse()[name]
    beta = g["BETA"] * pow(P.R_MONT, -1, C.p) % C.p
    assert pow(beta, 3, C.p) == 1 and beta != 1
    lam = None
    for cand in range(2, 50):
        l0 = pow(cand, (C.r - 1) // 3, C.r)
        for l in (l0, l0 * l0 % C.r):
            if l != 1 and C.mul(l, C.gen) == (beta * C.gen[0] % C.p, C.gen[1]):
                lam = l
        if lam:
            break
    assert lam is not None
    a1, b1, a2, b2 = g["A1"], -g["NB1"], g["A2"], g["B2"]
    assert (a1 + b1 * lam) % C.r == 0 and (a2 + b2 * lam) % C.r == 0
    rng = random.Random(7)
    ks = [0, 1, 2, C.r - 1, C.r - 2, lam, (C.r + 1) // 2, 1 << 253] + [rng.randrange(C.r) for _ in range(3000)]
    for k in ks:
        c1 = (k * g["G1"]) >> 384
        c2 = (k * g["G2"]) >> 384
        assert c1 < 1 << 128 and c2 < 1 << 128  # the device keeps 4 limbs
        k1 = k - c1 * a1 - c2 * a2
        k2 = c1 * -b1 - c2 * b2
        assert (k1 + k2 * lam - k) % C.r == 0
        assert abs(k1) < 1 << 128 and abs(k2) < 1 << 128
    # provable bound behind kGlvBits = 128: |k_i| <= (|a1| + |a2|) or (|b1| + |b2|), times (1 + 2^-120)
    assert max(abs(a1) + abs(a2), abs(b1) + abs(b2)) * (1 + 2.0 ** -100) < 2.0 ** 128
