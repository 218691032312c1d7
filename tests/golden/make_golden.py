"""Generate tests/golden/msm_vectors.npz with the Python oracle (oracle/pasta.py).

Every expected value is the oracle's restatement of halo2 best_multiexp and is
asserted equal to (a) the naive double-and-add sum and (b) the known-discrete-
log answer [sum s_i a_i]G before it is written.  Parity is unpinned by the
reference (it holds no MSM vectors); these fixtures pin the
HIP path to the restatement.

Layout: for case NAME the archive holds NAME.scalars (n,4) u64 Montgomery,
NAME.bases (n,8) u64 affine Montgomery ((0,0) = identity), NAME.expected (8,)
u64 affine Montgomery, NAME.curve () int.  Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pasta as P  # noqa: E402


def synth_case(curve, n, seed_s=P.SEED_SCALARS, seed_b=P.SEED_BASES):
    a = [P.synth_base_dlog(curve, seed_b, i) for i in range(n)]
    pts = [curve.mul(x, curve.gen) for x in a]
    s = [P.synth_scalar(seed_s, i, curve.r, curve.scalar_bits) for i in range(n)]
    return s, pts, a


def pack(curve, scalars, points, dlogs=None, check_naive=True):
    exp = curve.best_multiexp(scalars, points)
    if check_naive:
        assert exp == curve.msm_naive(scalars, points)
    if dlogs is not None:
        assert exp == curve.mul(sum(x * y for x, y in zip(scalars, dlogs)) % curve.r, curve.gen)
    # scalars in Montgomery form of the scalar field (R = 2^256 mod r)
    S = np.array([P.to_limbs((x % curve.r) * P.R_MONT % curve.r) for x in scalars],
                 dtype=np.uint64).reshape(-1, 4)
    B = np.array([P.point_to_limbs(curve, p) for p in points], dtype=np.uint64).reshape(-1, 8)
    E = np.array(P.point_to_limbs(curve, exp), dtype=np.uint64)
    return S, B, E


def main():
    P.self_check()
    cases = {}
    index = {}

    def add(name, curve_id, scalars, points, dlogs=None, note="", check_naive=True):
        C = P.CURVES[curve_id]
        S, B, E = pack(C, scalars, points, dlogs, check_naive)
        cases[f"{name}.scalars"] = S
        cases[f"{name}.bases"] = B
        cases[f"{name}.expected"] = E
        cases[f"{name}.curve"] = np.array(curve_id, dtype=np.int64)
        index[name] = {"curve": C.name, "n": len(points), "note": note}
        print(name, len(points), flush=True)

    C = P.PALLAS
    s, pts, a = synth_case(C, 4096)
    for n in (0, 1, 2, 3, 4, 31, 32, 33, 255, 1024, 4096):
        add(f"pallas_n{n}", 0, s[:n], pts[:n], a[:n], "synthetic seeds 0x5EED / 0xA11CE",
            check_naive=n <= 1024)
    m = 64
    s64, p64, a64 = s[:m], pts[:m], a[:m]
    add("pallas_zero_scalars", 0, [0] * m, p64, a64, "all scalars zero -> identity")
    add("pallas_r_minus_1", 0, [C.r - 1] * m, p64, a64, "all scalars r-1")
    add("pallas_dup_bases", 0, s64, [p64[0]] * m, [a64[0]] * m, "one base repeated (bucket doubling path)")
    add("pallas_neg_pairs", 0, s64[:32] + s64[:32], p64[:32] + [C.neg(p) for p in p64[:32]],
        a64[:32] + [C.r - x for x in a64[:32]], "P_i and -P_i with equal scalars -> identity")
    idb = [None if i % 3 == 0 else p for i, p in enumerate(p64)]
    ida = [0 if i % 3 == 0 else x for i, x in enumerate(a64)]
    add("pallas_identity_bases", 0, s64, idb, ida, "every third base is the identity (0,0)")
    add("pallas_equal_scalars", 0, [s[7]] * 4096, pts, a, "one scalar for all 4096 points (giant buckets)",
        check_naive=False)
    add("pallas_small_scalars", 0, [x % 16 for x in s64], p64, a64, "scalars < 16 (mostly empty windows)")
    top = [C.r - 1, C.r - 2, 1 << 254, (1 << 254) - 1, (1 << 254) + 1, 1, 2, (1 << 253)] * 8
    add("pallas_top_bits", 0, top, p64, a64, "scalars at the 2^254 / r boundary")
    add("pallas_same_point_same_scalar", 0, [s64[3]] * 8 + s64[8:], [p64[3]] * 8 + p64[8:],
        [a64[3]] * 8 + a64[8:], "equal (scalar, base) pairs: P + P inside one bucket")

    V = P.VESTA
    sv, pv, av = synth_case(V, 1024)
    for n in (1, 33, 1024):
        add(f"vesta_n{n}", 1, sv[:n], pv[:n], av[:n], "synthetic", check_naive=n <= 33)
    Bn = P.BN254
    sb, pb, ab = synth_case(Bn, 1024)
    for n in (1, 33, 1024):
        add(f"bn254_n{n}", 2, sb[:n], pb[:n], ab[:n], "synthetic", check_naive=n <= 33)

    np.savez_compressed(os.path.join(HERE, "msm_vectors.npz"), **cases)
    with open(os.path.join(HERE, "msm_vectors.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
