"""CPU tests: the oracle against the golden vectors and known answers, and the
host-side logic of the HIP pipeline (tests/pipeline_model.py)."""
import random

import numpy as np
import pytest

import msm_ref
import pasta as P
import pipeline_model as PM


def test_curve_constants():
    assert P.self_check()


def test_golden_python_oracle(golden):
    """Recompute the small golden cases with the Python restatement of
    best_multiexp (independent of the fixture generator's run)."""
    for name, case in golden.items():
        if case["scalars"].shape[0] > 255:
            continue
        C = P.CURVES[case["curve"]]
        sc = [P.from_limbs(s) * pow(P.R_MONT, -1, C.r) % C.r for s in case["scalars"]]
        pts = [P.limbs_to_point(C, list(b)) for b in case["bases"]]
        got = C.best_multiexp(sc, pts)
        assert P.point_to_limbs(C, got) == [int(x) for x in case["expected"]], name


def test_golden_c_oracle(golden):
    """The C restatement (independent field/curve code) reproduces every vector."""
    for name, case in golden.items():
        out = msm_ref.best_multiexp(case["curve"], case["scalars"], case["bases"], threads=4)
        assert np.array_equal(out, case["expected"]), name


def test_c_oracle_thread_count_invariant(golden):
    case = golden["pallas_n1024"]
    outs = {tuple(msm_ref.best_multiexp(0, case["scalars"], case["bases"], threads=t)) for t in (1, 3, 8, 17)}
    assert len(outs) == 1


def test_c_oracle_canonical_flag(golden):
    case = golden["pallas_n255"]
    C = P.PALLAS
    canon = np.array([P.to_limbs(P.from_limbs(s) * pow(P.R_MONT, -1, C.r) % C.r) for s in case["scalars"]],
                     dtype=np.uint64)
    assert np.array_equal(msm_ref.best_multiexp(0, canon, case["bases"], canonical=True), case["expected"])


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_synth_generators_match(curve):
    """The C synth generator (mirrored by the HIP one) matches the Python one."""
    C = P.CURVES[curve]
    idx = [0, 1, 2, 77, 1000]
    B = msm_ref.synth_bases(curve, P.SEED_BASES, 0, 1001, threads=4)
    S = msm_ref.synth_scalars(curve, P.SEED_SCALARS, 0, 1001, threads=4)
    for i in idx:
        a = P.synth_base_dlog(C, P.SEED_BASES, i)
        assert P.limbs_to_point(C, list(B[i])) == C.mul(a, C.gen)
        s = P.synth_scalar(P.SEED_SCALARS, i, C.r, C.scalar_bits)
        assert P.from_limbs(S[i]) == s * P.R_MONT % C.r


def test_halo2_window_formula():
    # 2^18 -> 13, 2^20 -> 14, 2^22 -> 16
    assert [PM.halo2_window(1 << k) for k in (18, 20, 22)] == [13, 14, 16]
    assert PM.halo2_window(3) == 1 and PM.halo2_window(31) == 3


@pytest.mark.parametrize("c", list(range(4, 21)))
def test_signed_digits_reconstruct(c):
    rng = random.Random(c)
    W = (256 + c - 1) // c
    widths = PM.window_widths(W)
    assert sum(widths) == 256 and max(widths) - min(widths) <= 1
    offs = [sum(widths[:w]) for w in range(W)]
    r = P.VESTA_P
    for s in [0, 1, r - 1, (1 << 254), (1 << 255) - 1] + [rng.randrange(r) for _ in range(200)]:
        ds = PM.digits(s, W)
        assert all(0 <= d <= (1 << (cw - 1)) for (d, _), cw in zip(ds, widths))
        assert sum((-d if neg else d) << o for o, (d, neg) in zip(offs, ds)) == s


def test_balanced_windows_no_giant_buckets():
    """Every window of a uniformly random scalar uses at least a quarter of
    the widest window's digit range (no few-bit top window)."""
    for c in range(4, 21):
        W = (256 + c - 1) // c
        widths = PM.window_widths(W)
        top_bits = 254 - sum(widths[:-1])  # Pasta/BN254 scalars are < 2^255, bit 254 ~never set
        assert top_bits >= max(widths) - 3, c


@pytest.mark.parametrize("n,c,chunk", [(1, 0, 0), (2, 4, 16), (7, 5, 3), (64, 6, 16), (200, 8, 5), (300, 4, 1000),
                                       (513, 7, 37), (1000, 0, 0), (1000, 10, 2), (900, 16, 3)])
def test_pipeline_model_random(n, c, chunk):
    rng = random.Random(n * 31 + c)
    r = P.VESTA_P
    s = [rng.randrange(r) for _ in range(n)]
    a = [rng.randrange(r) for _ in range(n)]
    assert PM.msm_model(s, a, r, c, chunk) == sum(x * y for x, y in zip(s, a)) % r


@pytest.mark.parametrize("chunk", [1, 2, 16, 100])
def test_pipeline_model_giant_bucket(chunk):
    """All scalars equal: one bucket per window spans many slices (chains
    longer than kSerialChain, folded wave-wide in k_bucket_seg_q)."""
    r = P.VESTA_P
    n = 500
    s = [0x1234567890ABCDEF << 100] * n
    a = list(range(1, n + 1))
    assert PM.msm_model(s, a, r, 6, chunk) == sum(x * y for x, y in zip(s, a)) % r


def test_pipeline_model_sparse():
    r = P.VESTA_P
    s = [0, 0, 5, 0, r - 1, 0, 1 << 200]
    a = [3, 4, 5, 6, 7, 8, 9]
    for c in (4, 9, 16):
        for chunk in (1, 3, 16):
            assert PM.msm_model(s, a, r, c, chunk) == sum(x * y for x, y in zip(s, a)) % r


@pytest.mark.parametrize("n,c,sort_b", [(100, 4, 16), (1000, 9, 128), (3000, 12, 512), (2500, 16, 300),
                                        (700, 18, 64), (50, 20, 2048)])
def test_two_level_sort_model(n, c, sort_b):
    """The LDS two-level bucket sort yields exactly the counting-sort offsets
    and the same (point, sign) multiset in every bucket."""
    rng = random.Random(n + c)
    r = P.VESTA_P
    pl = PM.make_plan(n, c)
    W, NB = pl["W"], pl["NB"]
    cmax = max(pl["widths"])
    dig = [PM.digits(rng.randrange(r), W) for _ in range(n)]
    offsets, sorted_ = PM.sort_model(dig, n, W, pl["K"], cmax, NB, sort_b)
    counts = [0] * (W * NB + 1)
    for i in range(n):
        for w, (d, _) in enumerate(dig[i]):
            if d:
                counts[w * NB + d] += 1
    ref, run = [], 0
    for x in counts:
        ref.append(run)
        run += x
    assert offsets == ref
    want = {}
    for i in range(n):
        for w, (d, neg) in enumerate(dig[i]):
            if d:
                want.setdefault((w, d), []).append((i, neg))
    for (w, slot), items in want.items():
        assert sorted(sorted_[ref[w * NB + slot]:ref[w * NB + slot + 1]]) == sorted(items)
