"""CPU: the generated per-column asm of csrc/fp29_asm.hpp (tools/gen_fp29_asm.py)
computes the radix-2^29 Montgomery product a b 2^-261 mod p.

The header is executed here by a small interpreter of exactly the constructs
the generator emits (v_mad_u64_u32 / v_mad_i64_i32 chains, v_lshrrev_b64 /
v_ashrrev_i64, and the C lines that
derive m_k / the output limbs from the accumulator's low word), with 64-bit
wrap-around checks, so a generator bug is caught without a GPU.  The device
self-test (tests/test_msm_gpu.py::test_radix29_field_selftest) checks the same
functions on the MI355X against the 32-bit arithmetic."""
import os
import random
import re

import pasta as P
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "halo2-aggregation_amd", "csrc", "fp29_asm.hpp")
M29 = (1 << 29) - 1
M64 = (1 << 64) - 1
FIELDS = {"PallasFp": P.PALLAS_P, "VestaFp": P.VESTA_P, "Bn254Fq": P.BN254_P, "Bn254Fr": P.BN254_R}


def _functions():
    src = open(HDR).read()
    out = {}
    for m in re.finditer(r"F29<(\w+)> (f29_(?:mul|sqr|mul2|mul2n|mul_sa|sqr_sa|mul2n_sb)_a)<\w+>\((.*?)\) \{\n(.*?)\n\}\n", src, re.S):
        out[(m.group(2), m.group(1))] = m.group(4)
    return out


def _run(body, a, b=None, u=None, v=None):
    env = {"a.l": list(a), "b.l": list(b) if b is not None else None, "m": [0] * 9, "r.l": [0] * 9, "d": [0] * 8,
           "u.l": list(u) if u is not None else None, "v.l": list(v) if v is not None else None, "nv": [0] * 9}
    acc = 0
    signed = False

    def val(expr):
        expr = expr.strip()
        mm = re.fullmatch(r"([a-z.]+)\[(\d+)\]", expr)
        if mm:
            return env[mm.group(1)][int(mm.group(2))]
        return int(expr.rstrip("ul"))

    stmts = re.findall(r'asm\("(.*?)"\s*:\s*"(?:\+|=&)v"\(acc\), "=&s"\(c\)\s*:\s*(.*?)\);|^  (?!asm)([^\n]*?);$', body,
                       re.S | re.M)
    for text, ins, cline in stmts:
        if text:
            ops = [val(x.split("(", 1)[1][:-1]) for x in re.findall(r'"[vs]"\([^)]*\)', ins)]
            for ins_text in text.split("\\n\\t"):
                f = [x.strip() for x in ins_text.replace(",", " ").split()]
                if f[0] in ("v_mad_u64_u32", "v_mad_i64_i32"):
                    assert f[1] == "%0" and f[2] == "%1" and f[5] in ("%0", "0")
                    if f[5] == "0":  # a product's first multiply-add: acc starts from 0
                        acc = 0
                    x = ops[int(f[3][1:]) - 2] if f[3].startswith("%") else int(f[3])
                    y = ops[int(f[4][1:]) - 2] if f[4].startswith("%") else int(f[4])
                    if f[0] == "v_mad_i64_i32":  # signed 32 x 32 + signed 64
                        x, y = (v - (1 << 32) if v >= 1 << 31 else v for v in (x % (1 << 32), y % (1 << 32)))
                    else:
                        assert 0 <= x < 2 ** 32 and 0 <= y < 2 ** 32
                    acc += x * y
                    # unsigned columns (additive form) or signed ones (subtractive)
                    assert -(1 << 63) <= acc <= M64, "column overflow"
                    assert not (signed and acc >= 1 << 63), "signed column overflow"
                elif f[0] == "v_lshl_add_u64":  # + a 64-bit SGPR-pair constant (p R limbs)
                    assert f[1] == "%0" and f[3] == "0" and f[4] == "%0"
                    acc += ops[int(f[2][1:]) - 2]
                    assert -(1 << 63) <= acc <= M64, "column overflow"
                    assert not (signed and acc >= 1 << 63), "signed column overflow"
                elif f[0] == "v_lshrrev_b64":
                    assert f[1:] == ["%0", "29", "%0"]
                    assert acc >= 0
                    acc >>= 29
                elif f[0] == "v_ashrrev_i64":
                    assert f[1:] == ["%0", "29", "%0"]
                    signed = True
                    acc >>= 29  # Python's >> floors: arithmetic shift
                else:
                    raise AssertionError(ins_text)
            continue
        c = cline
        if c.startswith("for (int i = 0; i < 8; i++) d[i] = a.l[i] << 1"):
            env["d"] = [(x << 1) & 0xFFFFFFFF for x in env["a.l"][:8]]
        elif c.startswith("for (int i = 0; i < 9; i++) nv[i] = 0u - v.l[i]"):
            env["nv"] = [(-x) & 0xFFFFFFFF for x in env["v.l"]]
        elif re.fullmatch(r"m\[\d\] = \(uint32_t\)acc & kM29", c):
            env["m"][int(c[2])] = acc & M29  # two's complement low bits
        elif re.fullmatch(r"m\[\d\] = \(0u - \(uint32_t\)acc\) & kM29", c):
            env["m"][int(c[2])] = (-(acc & 0xFFFFFFFF)) & M29
        elif re.fullmatch(r"m\[\d\] = \(\(uint32_t\)acc \* \d+u\) & kM29", c):
            inv = int(re.search(r"\* (\d+)u", c).group(1))
            env["m"][int(c[2])] = ((acc & 0xFFFFFFFF) * inv) & M29
        elif re.fullmatch(r"r\.l\[\d\] = \(uint32_t\)acc & kM29", c):
            env["r.l"][int(c[4])] = acc & M29
        elif c == "r.l[8] = (uint32_t)(acc >> 29)":
            assert acc >> 29 < 2 ** 32
            env["r.l"][8] = acc >> 29
        elif re.fullmatch(r"r\.l\[8\] = \(uint32_t\)\(\(int64_t\)acc >> 29\) \+ \d+u", c):
            top = (acc >> 29) + int(re.search(r"\+ (\d+)u", c).group(1))
            assert 0 <= top < 2 ** 32
            env["r.l"][8] = top
        elif not re.fullmatch(r"F29<\w+> r|uint32_t (m|d|nv)\[\d\]|uint64_t acc, c|\(void\)c|return r", c):
            raise AssertionError("unhandled line: " + c)
    return env["r.l"]


def _limbs(v):
    return [(v >> (29 * i)) & M29 for i in range(9)]


def _value(l):
    return sum(x << (29 * i) for i, x in enumerate(l))


def test_generated_header_is_current():
    import subprocess
    import sys

    gen = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_fp29_asm.py")], capture_output=True,
                         text=True, check=True).stdout
    assert gen == open(HDR).read(), "fp29_asm.hpp is stale: rerun tools/gen_fp29_asm.py"


@pytest.mark.parametrize("field", sorted(FIELDS))
def test_column_asm_products(field):
    p = FIELDS[field]
    fns = _functions()
    mul, sqr = fns[("f29_mul_a", field)], fns[("f29_sqr_a", field)]
    rinv = pow(1 << 261, -1, p)
    rng = random.Random(0xA5A5 + len(field))
    vals = [0, 1, p - 1, p - 2, 2 * p - 1, 3 * p + 7, 4 * p - 1] + [rng.randrange(4 * p) for _ in range(40)]
    for i, x in enumerate(vals):
        y = vals[(7 * i + 3) % len(vals)]
        r = _run(mul, _limbs(x), _limbs(y))
        assert all(l <= M29 for l in r[:8])
        assert _value(r) % p == x * y * rinv % p and _value(r) < 2 * p
        r = _run(sqr, _limbs(x))
        assert _value(r) % p == x * x * rinv % p and _value(r) < 2 * p
    # loose operand limbs (a + 6p limb-wise, the f29_sub form) on the mul path
    K6 = [l + (1 << 29) - 1 for l in _limbs(0)]  # stands in for a loose limb pattern < 2^30
    x = rng.randrange(p)
    lx = [a + b for a, b in zip(_limbs(x), K6)]
    y = rng.randrange(2 * p)
    r = _run(mul, lx, _limbs(y))
    assert _value(r) % p == _value(lx) * y * rinv % p


@pytest.mark.parametrize("field", sorted(FIELDS))
def test_column_asm_sum_of_products(field):
    """f29_mul2_a: (a b + u v) 2^-261 with one reduction, Norm operands up to
    the bounds the curve routines use (R, D < 8p; -Y < 6p; PPP < 2p)."""
    p = FIELDS[field]
    mul2 = _functions()[("f29_mul2_a", field)]
    rinv = pow(1 << 261, -1, p)
    rng = random.Random(0x5A5A + len(field))
    edge = [0, 1, p - 1, 2 * p - 1, 8 * p - 1, 6 * p - 1]
    for t in range(60):
        a = edge[t % len(edge)] if t < 12 else rng.randrange(8 * p)
        b = rng.randrange(8 * p) if t % 3 else 8 * p - 1
        u = rng.randrange(6 * p) if t % 5 else 6 * p - 1
        v = rng.randrange(2 * p) if t % 7 else 2 * p - 1
        r = _run(mul2, _limbs(a), _limbs(b), _limbs(u), _limbs(v))
        assert all(l <= M29 for l in r[:8])
        assert _value(r) % p == (a * b + u * v) * rinv % p
        assert _value(r) < 2 * p + p // 4  # < 2p for p < 2^254.7 (Pasta, BN254)


@pytest.mark.parametrize("field", sorted(FIELDS))
def test_column_asm_difference_of_products(field):
    """f29_mul2n_a: (a b - u v) 2^-261 with one reduction and signed columns,
    for the operand bounds of its callers (R, D < 10p / 8p; u, v < 4p:
    Y3 = R D - Y1 PPP of the bucket addition, M D - W Y of the doubling,
    R D - S1 PPP of the full addition), including a b = 0 with u v maximal
    (the most negative column sums) -> Norm, < 3p."""
    p = FIELDS[field]
    mul2n = _functions()[("f29_mul2n_a", field)]
    rinv = pow(1 << 261, -1, p)
    rng = random.Random(0x2A2A + len(field))
    for t in range(80):
        a = [0, 1, 10 * p - 1][t % 3] if t < 9 else rng.randrange(10 * p)
        b = [0, 8 * p - 1, 8 * p - 1][(t // 3) % 3] if t < 9 else rng.randrange(8 * p)
        u = rng.randrange(4 * p) if t % 4 else 4 * p - 1
        v = rng.randrange(4 * p) if t % 5 else 4 * p - 1
        r = _run(mul2n, _limbs(a), _limbs(b), _limbs(u), _limbs(v))
        assert all(0 <= l <= M29 for l in r[:8])
        assert _value(r) % p == (a * b - u * v) * rinv % p
        assert 0 <= _value(r) < 3 * p


def _f29_consts(field):
    src = open(os.path.join(ROOT, "halo2-aggregation_amd", "csrc", "fp29.hpp")).read()
    body = src[src.index("struct F29Consts<%s>" % field):]
    body = body[:body.index("\n};")]
    ks = [[int(x, 16) for x in re.search(r"%s\[9\] = \{(.*?)\}" % n, body).group(1).replace("u", "").split(",")]
          for n in ("K2", "K6")]
    qm = int(re.search(r"QMAGIC = (0x[0-9a-f]+)u", body).group(1), 16)
    return ks[0], ks[1], qm


@pytest.mark.parametrize("field", ["PallasFp", "VestaFp", "Bn254Fr"])
def test_ntt_operand_bounds(field):
    """The NTT's radix-4 unit (csrc/ntt_kernels.hpp lds_ntt4) in the
    radix-2^29 form: inputs Norm < 3p, twiddles canonical or negated (2p - w),
    the lazy sums / differences (limbs < 2^30 into the products, y3
    normalised), each output normalised and reduced to < 3p.  Every limb is
    checked against its 32-bit register, the products run through the
    interpreter with its column-overflow checks, and the outputs are the
    radix-4 butterfly of the inputs mod p."""
    p = FIELDS[field]
    mul = _functions()[("f29_mul_a", field)]
    K2, K6, qmagic = _f29_consts(field)
    P9 = _limbs(p)
    rinv = pow(1 << 261, -1, p)

    def add(a, b):
        r = [x + y for x, y in zip(a, b)]
        assert all(0 <= x < 2 ** 32 for x in r)
        return r

    def sub(a, b, K=K2):  # a + K - b, limb-wise (K = 2p or 6p)
        r = [x + k - y for x, k, y in zip(a, K, b)]
        assert all(0 <= x < 2 ** 32 for x in r)
        assert _value(r) == _value(a) + (2 if K is K2 else 6) * p - _value(b) >= 0
        return r

    def norm(a):
        r, c = [0] * 9, 0
        for i in range(8):
            v = a[i] + c
            assert v < 2 ** 32 - 8
            r[i], c = v & M29, v >> 29
        r[8] = a[8] + c
        assert r[8] < 2 ** 32
        return r

    def reduce3(a):
        assert _value(a) < 16 * p
        q = (a[8] * qmagic) >> 40
        r, c = [0] * 9, 0
        for i in range(9):
            v = a[i] - q * P9[i] + c
            r[i] = v & M29 if i < 8 else v % (1 << 32)
            c = v >> 29
        assert 0 <= _value(r) < 3 * p and all(x <= M29 for x in r[:8])
        return r

    def mmul(a, w):
        r = _run(mul, a, w)
        assert all(x <= M29 for x in r[:8]) and _value(r) < 2 * p
        assert _value(r) % p == _value(a) * _value(w) * rinv % p
        return r

    def twiddle(v, neg):
        w = _limbs(v)
        return norm(sub([0] * 9, w)) if neg else w

    rng = random.Random(0x7E7E + len(field))
    edge = [0, 1, p - 1, 2 * p, 3 * p - 1]
    one = [x % (1 << 32) for x in _limbs((1 << 261) % p)]  # R261 one: W = 1
    for t in range(80):
        first = t % 2 == 1  # stage 0 of the sub-transform: twiddle 1, x1 / x3 unmultiplied
        xs = [_limbs(edge[(t // 2 + k) % len(edge)] if t < 20 else rng.randrange(3 * p)) for k in range(4)]
        if t < 20 and first:
            xs[0], xs[2] = _limbs(0), _limbs(1)  # x1 > x0 + 2p: the case a + 2p - b would break
        ws = [twiddle(p - 1 if t < 20 else rng.randrange(1, p), (t >> k) & 1) for k in range(3)]
        x0, x1, x2, x3 = xs
        if first:
            ws[0] = one
            y1, y3 = sub(x0, x1, K6), norm(sub(x2, x3, K6))
        else:
            x1, x3 = mmul(x1, ws[0]), mmul(x3, ws[0])
            y1, y3 = sub(x0, x1), norm(sub(x2, x3))
        y0, y2 = add(x0, x1), add(x2, x3)
        assert all(x < 2 ** 30 for x in y2)
        z2, z3 = mmul(y2, ws[1]), mmul(y3, ws[2])
        outs = [reduce3(norm(add(y0, z2))), reduce3(norm(add(y1, z3))), reduce3(norm(sub(y0, z2))),
                reduce3(norm(sub(y1, z3)))]
        X = [_value(v) for v in xs]
        W = [_value(w) * rinv % p for w in ws]
        a1, a3 = X[1] * W[0] % p, X[3] * W[0] % p
        b0, b1, b2, b3 = X[0] + a1, X[0] - a1, X[2] + a3, X[2] - a3
        want = [b0 + b2 * W[1], b1 + b3 * W[2], b0 - b2 * W[1], b1 - b3 * W[2]]
        assert [_value(o) % p for o in outs] == [v % p for v in want]
        # the radix-2 stage 0 of an odd-length sub-transform: u + v, u - v + 6p
        u, v = xs[0], xs[1]
        o = [reduce3(norm(add(u, v))), reduce3(norm(sub(u, v, K6)))]
        assert [_value(x) % p for x in o] == [(X[0] + X[1]) % p, (X[0] - X[1]) % p]
        # the first radix-4 round fused into the load phase (ntt_load_first):
        # W_2 = W_4^0 = 1, no product; y2 and y3 normalised, 6p where the
        # subtrahend is unmultiplied (< 3p) or y2 (< 6p)
        y0, y1 = add(xs[0], xs[1]), sub(xs[0], xs[1], K6)
        y2, y3 = norm(add(xs[2], xs[3])), norm(sub(xs[2], xs[3], K6))
        z3 = mmul(y3, ws[2])
        outs = [reduce3(norm(add(y0, y2))), reduce3(norm(add(y1, z3))), reduce3(norm(sub(y0, y2, K6))),
                reduce3(norm(sub(y1, z3)))]
        b0, b1, b2, b3 = X[0] + X[1], X[0] - X[1], X[2] + X[3], X[2] - X[3]
        want = [b0 + b2, b1 + b3 * W[2], b0 - b2, b1 - b3 * W[2]]
        assert [_value(o) % p for o in outs] == [v % p for v in want]
        # lazy LDS rounds (lds_ntt4): a round on < 3p inputs leaves its outputs
        # normalised, < 7p; the next round takes < 7p inputs and reduces
        lazy_in = [_limbs(rng.randrange(7 * p) if t >= 20 else 7 * p - 1 - k) for k in range(4)]
        a0, a1, a2, a3 = lazy_in
        a1, a3 = mmul(a1, ws[0]), mmul(a3, ws[0])
        e0, e1, e2, e3 = add(a0, a1), sub(a0, a1), add(a2, a3), norm(sub(a2, a3))
        assert all(x < 2 ** 30 for x in e2)
        f2, f3 = mmul(e2, ws[1]), mmul(e3, ws[2])
        lz = [norm(add(e0, f2)), norm(add(e1, f3)), norm(sub(e0, f2)), norm(sub(e1, f3))]
        assert all(_value(o) < 11 * p and all(x <= M29 for x in o[:8]) for o in lz)
        assert all(_value(reduce3(o)) < 3 * p for o in lz)
        # and from < 3p inputs the unreduced outputs stay < 7p
        g1, g3 = mmul(xs[1], ws[0]), mmul(xs[3], ws[0])
        h0, h1, h2, h3 = add(xs[0], g1), sub(xs[0], g1), add(xs[2], g3), norm(sub(xs[2], g3))
        k2, k3 = mmul(h2, ws[1]), mmul(h3, ws[2])
        assert all(_value(norm(o)) < 7 * p for o in (add(h0, k2), sub(h0, k2), add(h1, k3), sub(h1, k3)))


def _k8x3(field):
    src = open(os.path.join(ROOT, "halo2-aggregation_amd", "csrc", "fp29.hpp")).read()
    body = src[src.index("struct F29Consts<%s>" % field):]
    body = body[:body.index("\n};")]
    return [int(x, 16) for x in re.search(r"K8x3\[9\] = \{(.*?)\}", body).group(1).replace("u", "").split(",")]


def _signed_limbs(v):
    """v (any sign) as 9 limbs with limbs 0..7 in [0, 2^29) and a signed top
    limb -- the limb pattern of a difference of two Norm values is any vector
    with |limb| < 2^29; this is one of them."""
    l = [(v >> (29 * i)) & M29 for i in range(8)]
    return l + [v >> 232]


MSM_FIELDS = {"PallasFp": 5, "VestaFp": 5, "Bn254Fq": 3}  # y^2 = x^3 + b


@pytest.mark.parametrize("field", sorted(MSM_FIELDS))
def test_signed_operand_products(field):
    """f29_mul_sa_a / f29_sqr_sa_a / f29_mul2n_sb_a: one operand with signed
    limbs (|limb| < 2^29), at the extremes k_accumulate's lazy step feeds them
    (P in (-9p, 2p), D in (-9p, 1.2p), R < 10p, Y1 < 3p, PPP < 2.1p), including
    limb patterns at -2^29 + 1 in every limb."""
    p = FIELDS[field]
    fns = _functions()
    mul_sa, sqr_sa, mul2n_sb = (fns[(n, field)] for n in ("f29_mul_sa_a", "f29_sqr_sa_a", "f29_mul2n_sb_a"))
    rinv = pow(1 << 261, -1, p)
    rng = random.Random(0x3C3C + len(field))
    worst = [-M29] * 8 + [1 - (9 * p >> 232)]  # every limb at its most negative, value > -9p
    for t in range(80):
        if t < 4:
            a = worst if t % 2 else _signed_limbs(-9 * p + 1)
        else:
            a = _signed_limbs(rng.randrange(-9 * p + 1, 2 * p))
        av = _value(a)
        assert -9 * p < av < 2 * p and all(abs(x) < 2 ** 29 for x in a)
        b = _limbs(rng.randrange(2 * p) if t % 3 else 2 * p - 1)
        r = _run(mul_sa, a, b)
        assert all(0 <= x <= M29 for x in r[:8])
        assert _value(r) % p == av * _value(b) * rinv % p and 0 <= _value(r) < 3 * p
        r = _run(sqr_sa, a)
        assert all(0 <= x <= M29 for x in r[:8])
        assert _value(r) % p == av * av * rinv % p and 0 <= _value(r) < 2 * p
        rr = _limbs(rng.randrange(10 * p) if t % 4 else 10 * p - 1)
        u = _limbs(rng.randrange(3 * p) if t % 5 else 3 * p - 1)
        v = _limbs(rng.randrange(3 * p) if t % 7 else 3 * p - 1)
        r = _run(mul2n_sb, rr, a, u, v)
        assert all(0 <= x <= M29 for x in r[:8])
        assert _value(r) % p == (_value(rr) * av - _value(u) * _value(v)) * rinv % p
        assert 0 <= _value(r) < 3 * p


def _aff_add(p, P1, P2):
    (x1, y1), (x2, y2) = P1, P2
    if x1 == x2:
        lam = 3 * x1 * x1 * pow(2 * y1, -1, p) % p
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, p) % p
    x3 = (lam * lam - x1 - x2) % p
    return x3, (lam * (x1 - x3) - y1) % p


@pytest.mark.parametrize("field", sorted(MSM_FIELDS))
def test_lazy_bucket_addition(field):
    """csrc/curve29.hpp xyzz29_madd_lazy, limb for limb: long chains of
    signed bucket additions (acc + (-1)^s B_i) through the generated products,
    with the accumulator's coordinates re-represented at the top of their
    lazy ranges (X1 + j p < 9p, Y1 + j p < 3p, ZZ / ZZZ + p < 2p) before
    steps, every intermediate checked against its 32-bit register and
    stated bound, and the affine result against the chord rule mod p."""
    p, bcoef = FIELDS[field], MSM_FIELDS[field]
    fns = _functions()
    mul, sqr = fns[("f29_mul_a", field)], fns[("f29_sqr_a", field)]
    mul_sa, sqr_sa, mul2n_sb = (fns[(n, field)] for n in ("f29_mul_sa_a", "f29_sqr_sa_a", "f29_mul2n_sb_a"))
    K8x3 = _k8x3(field)
    R = 1 << 261
    rinv = pow(R, -1, p)
    assert _value(K8x3) == 8 * p and all(k >= 3 * (2 ** 29 - 1) for k in K8x3[:8])

    def norm(a):
        r, c = [0] * 9, 0
        for i in range(8):
            v = a[i] + c
            assert 0 <= v < 2 ** 32
            r[i], c = v & M29, v >> 29
        r[8] = a[8] + c
        assert 0 <= r[8] < 2 ** 32
        return r

    def u32(a):
        assert all(0 <= x < 2 ** 32 for x in a)
        return a

    G = (p - 1, 2) if bcoef == 5 else (1, 2)
    assert (G[1] ** 2 - G[0] ** 3 - bcoef) % p == 0
    pts, cur = [], G
    for _ in range(24):
        pts.append(cur)
        cur = _aff_add(p, cur, G)
    rng = random.Random(0x1A2B + len(field))
    mont = lambda v: v * R % p  # noqa: E731
    for chain in range(6):
        start = pts[rng.randrange(len(pts))]
        X, Y = _limbs(mont(start[0])), _limbs(mont(start[1]))
        ZZ = ZZZ = _limbs(mont(1))
        true = start
        for step in range(30):
            if step % 3 == 0:  # push every coordinate to the top of its range
                X = _limbs(_value(X) % p + 8 * p)
                Y = _limbs(_value(Y) % p + 2 * p)
                ZZ, ZZZ = (_limbs(_value(z) % p + p) for z in (ZZ, ZZZ))
            k = rng.randrange(len(pts))
            neg = rng.randrange(2)
            bx, by = pts[k]
            add = (bx, (-by) % p if neg else by)
            if add[0] == true[0]:
                continue  # the exceptional case (xyzz29_madd_fix)
            x2, y2 = _limbs(mont(bx)), _limbs(mont(by))
            # --- xyzz29_madd_lazy
            U2, S2 = _run(mul, x2, ZZ), _run(mul, y2, ZZZ)
            assert _value(U2) < 2 * p and _value(S2) < 2 * p
            Pd = [a - b for a, b in zip(U2, X)]
            Rl = norm(u32([K8x3[i] + (-S2[i] if neg else S2[i]) - Y[i] for i in range(9)]))
            assert all(abs(x) < 2 ** 29 for x in Pd) and -9 * p < _value(Pd) < 2 * p
            assert 3 * p < _value(Rl) < 10 * p
            PP = _run(sqr_sa, Pd)
            PPP = _run(mul_sa, Pd, PP)
            Q = _run(mul, X, PP)
            assert _value(PP) < 1.76 * p and 0.86 * p < _value(PPP) <= 2.04 * p and _value(Q) < 1.14 * p
            R2 = _run(sqr, Rl)
            t = u32([a + b + b for a, b in zip(PPP, Q)])
            X3 = norm(u32([R2[i] + K8x3[i] - t[i] for i in range(9)]))
            assert 3.6 * p < _value(X3) < 9 * p
            D = [a - b for a, b in zip(Q, X3)]
            assert all(abs(x) < 2 ** 29 for x in D)
            Y3 = _run(mul2n_sb, Rl, D, Y, PPP)
            assert 0 <= _value(Y3) < 3 * p
            ZZ3, ZZZ3 = _run(mul, ZZ, PP), _run(mul, ZZZ, PPP)
            assert _value(ZZ3) < 2 * p and _value(ZZZ3) < 2 * p
            X, Y, ZZ, ZZZ = X3, Y3, ZZ3, ZZZ3
            true = _aff_add(p, true, add)
            zz, zzz = _value(ZZ) * rinv % p, _value(ZZZ) * rinv % p
            ax = _value(X) * rinv * pow(zz, -1, p) % p
            ay = _value(Y) * rinv * pow(zzz, -1, p) % p
            assert (ax, ay) == true
