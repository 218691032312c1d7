"""CPU checks of the GLV constants compiled into the accumulator kernels
(halo2-aggregation_amd/csrc/glv.hpp, Glv<Curve>): beta is a cube
root of unity of the base field with phi(G) = (beta Gx, Gy) = [lambda]G, the
lattice vectors satisfy a + b lambda = 0 mod r, and the device's decomposition
(floor with 2^384-scaled g1, g2) gives |k1|, |k2| < 2^128 with
k = k1 + lambda k2 mod r on random and edge scalars; with Babai rounding (the
MSM's GLV mode) |k1|, |k2| < 2^127."""
import os
import random
import re

import pytest

import pasta as P

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "halo2-aggregation_amd", "csrc",
                   "glv.hpp")
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


@pytest.mark.parametrize("name", list(CURVES))
def test_glv_rounded_split_below_2_127(name):
    """glv_split<Cv, ROUND=true> (mp_quot384 adds 2^383 before taking the
    quotient): |k1|, |k2| < 2^127, so the MSM's 8 signed 16-bit windows over
    128 bits never carry out of the top window."""
    C = CURVES[name]
    g = _parse()[name]
    a1, b1, a2, b2 = g["A1"], -g["NB1"], g["A2"], g["B2"]
    lam = None
    beta = g["BETA"] * pow(P.R_MONT, -1, C.p) % C.p
    for cand in range(2, 50):
        l0 = pow(cand, (C.r - 1) // 3, C.r)
        for l in (l0, l0 * l0 % C.r):
            if l != 1 and C.mul(l, C.gen) == (beta * C.gen[0] % C.p, C.gen[1]):
                lam = l
        if lam:
            break
    rng = random.Random(11)
    ks = [0, 1, 2, C.r - 1, C.r - 2, lam, (C.r + 1) // 2, 1 << 253, (1 << 254) % C.r] + [rng.randrange(C.r) for _ in range(5000)]
    # near the rounding boundaries of c1 / c2
    for t in range(1, 200):
        ks.append((t * (1 << 384) // g["G1"]) % C.r)
        ks.append((t * (1 << 384) // g["G2"] + 1) % C.r)
    # the provable bound: half the basis sum plus the rounding slack
    assert max(abs(a1) + abs(a2), abs(b1) + abs(b2)) / 2 + 2 < 2.0 ** 127 - 2.0 ** 112
    for k in ks:
        c1 = (k * g["G1"] + (1 << 383)) >> 384
        c2 = (k * g["G2"] + (1 << 383)) >> 384
        assert c1 < 1 << 128 and c2 < 1 << 128
        k1 = k - c1 * a1 - c2 * a2
        k2 = c1 * -b1 - c2 * b2
        assert (k1 + k2 * lam - k) % C.r == 0
        # the top 16-bit window of |k| plus a carry stays below 2^15 (msm_kernels.hpp signed_digit128)
        assert abs(k1) < (1 << 127) - (1 << 112) and abs(k2) < (1 << 127) - (1 << 112), (name, k)


def _digits128(k, W, flip):
    """Python restatement of msm_kernels.hpp signed_digit128 (GLV mode)."""
    base, extra = 128 // W, 128 % W
    out, carry, off = [], 0, 0
    for w in range(W):
        C = base + (1 if w < extra else 0)
        d = ((k >> off) & ((1 << C) - 1)) + carry
        off += C
        neg = 0
        if w != W - 1 and d + flip > (1 << (C - 1)):
            d, neg, carry = (1 << C) - d, 1, 1
        else:
            carry = 0
        out.append((C, -d if (neg ^ flip) else d))
    return out


@pytest.mark.parametrize("W", [7, 8, 9, 10, 11])
def test_glv_signed_digits(W):
    """The GLV-mode recoding of a 128-bit magnitude with the split's sign:
    digits sum to (-1)^flip k, the non-top windows stay within
    [-2^(C-1)+1, 2^(C-1)], every |d| <= 2^(cmax-1) (the bucket count) and, at
    cmax = 16, no digit is -2^15 (the 2-byte digit code has no room for it)."""
    rng = random.Random(W)
    top = (1 << 127) - (1 << 112) - 1
    ks = [0, 1, top, top - 1, (1 << 112) - 1, 1 << 111] + [rng.randrange(top) for _ in range(3000)]
    for k in ks:
        for flip in (0, 1):
            ds = _digits128(k, W, flip)
            cmax = max(C for C, _ in ds)
            val, off = 0, 0
            for i, (C, d) in enumerate(ds):
                if i < W - 1:
                    assert -(1 << (C - 1)) < d <= 1 << (C - 1), (k, flip, C, d)
                assert abs(d) <= 1 << (cmax - 1) and not (cmax == 16 and d == -(1 << 15)), (k, flip, C, d)
                val += d << off
                off += C
            assert val == (-k if flip else k)


def _naf128(k):
    """k_acc_termadd's naf128 (csrc/accum_kernels.hpp) on 32-bit words: with
    h = 3 k, digit i is h_{i+1} - k_{i+1}."""
    kw = [(k >> (32 * i)) & 0xFFFFFFFF for i in range(4)]
    h = 3 * k
    hw = [(h >> (32 * i)) & 0xFFFFFFFF for i in range(5)]
    nz, ng = [], []
    for i in range(4):
        hp = ((hw[i] >> 1) | (hw[i + 1] << 31)) & 0xFFFFFFFF
        kp = ((kw[i] >> 1) | ((kw[i + 1] << 31) if i < 3 else 0)) & 0xFFFFFFFF
        nz.append(hp ^ kp)
        ng.append(kp & ~hp & 0xFFFFFFFF)
    return nz, ng


def test_naf_of_rounded_glv_halves():
    """The term additions' digits: a non-adjacent form of every |k_i| < 2^127
    within 128 positions (the powers table's length), about a third nonzero,
    and the round-robin deal over S lanes gives each lane ceil(cnt / S) or
    fewer additions."""
    rng = random.Random(0x4AF)
    total = 0
    cases = [0, 1, 3, 7, (1 << 127) - 1, 0x5555555555555555555555555555555, 0x2AAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA]
    cases += [rng.getrandbits(127) for _ in range(400)]
    for k in cases:
        nz, ng = _naf128(k)
        digits = []
        for i in range(128):
            w, b = divmod(i, 32)
            d = ((nz[w] >> b) & 1) * (-1 if (ng[w] >> b) & 1 else 1)
            assert not ((ng[w] >> b) & 1) or ((nz[w] >> b) & 1)
            digits.append(d)
        assert sum(d << i for i, d in enumerate(digits)) == k
        assert all(not (digits[i] and digits[i + 1]) for i in range(127))
        cnt = sum(1 for d in digits if d)
        total += cnt
        for S in (8, 16, 32):
            per_lane = [len(range(j, cnt, S)) for j in range(S)]
            assert max(per_lane) == -(-cnt // S)
    assert 0.30 < total / (128 * len(cases)) < 0.36
