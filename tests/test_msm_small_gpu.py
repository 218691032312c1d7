"""GPU parity tests of the small-MSM path (msm_small.hpp: k_small_fused for
n <= 32, else k_small_table + k_small_sum; then the 33-window host Horner),
which pm_msm* take for n <= PM_SMALL_MSM_DEFAULT under the automatic window:

* every golden vector (Python restatement of halo2 best_multiexp) through
  the small path and, with the path disabled, through the sorting pipeline
* random sizes around every shape boundary (one term, one quad per term,
  several slices per window, several terms per quad) on all three curves
  against the C port of best_multiexp (oracle/msm_ref.c)
* edge inputs: identity bases, zero scalars, r - 1, canonical scalars >= r,
  duplicate bases, P and -P, all-equal terms
* the device, resident and resident-window entries on the same path
* which path ran (kernel timing stats), and the threshold setter's bounds
"""
import numpy as np
import pytest

import halo2_amd as H
import msm_ref
import pasta as P

pytestmark = pytest.mark.gpu


def _inputs(curve, n, seed=0x5A11):
    s = msm_ref.synth_scalars(curve, P.SEED_SCALARS ^ seed, 0, n, threads=4)
    b = msm_ref.synth_bases(curve, P.SEED_BASES ^ seed, 0, n, threads=4)
    return np.ascontiguousarray(s), np.ascontiguousarray(b)


def _ran_small(ctx):
    """the small-MSM kernels ran, or (a base set seen twice: the drop-in
    cache's small sets) the many-MSM sum"""
    two = ctx.kernel_stats("small_table")[0] > 0 and ctx.kernel_stats("small_sum")[0] > 0
    return two or ctx.kernel_stats("small_fused")[0] > 0 or ctx.kernel_stats("many_sum")[0] > 0


def test_golden_vectors_both_paths(golden, gpu_ctx):
    gpu_ctx.set_timing(True)
    try:
        for name, case in golden.items():
            for small in (H.SMALL_MSM_DEFAULT, 0):
                gpu_ctx.set_small_msm(small)
                gpu_ctx.reset_stats()
                got = gpu_ctx.msm(case["curve"], case["scalars"], case["bases"])
                assert np.array_equal(got, case["expected"]), (name, small)
                n = len(case["scalars"])
                if n:
                    assert _ran_small(gpu_ctx) == bool(small), (name, small)
    finally:
        gpu_ctx.set_small_msm(H.SMALL_MSM_DEFAULT)
        gpu_ctx.set_timing(False)


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_sizes_vs_c_port(gpu_ctx, curve):
    """n = 1 .. 4096 across the slice / quad boundaries (2n terms: <= 64 one
    block per window; > 512 several terms per quad)."""
    S, B = _inputs(curve, 4096, 0x11 + curve)
    for n in (1, 2, 3, 5, 16, 31, 32, 33, 63, 64, 65, 200, 256, 257, 511, 1000, 2049, 4095, 4096):
        s, b = S[:n], B[:n]
        want = msm_ref.best_multiexp(curve, s, b, threads=4)
        assert np.array_equal(gpu_ctx.msm(curve, s, b), want), (curve, n)


def test_edge_inputs(gpu_ctx):
    C = P.PALLAS
    S, B = _inputs(0, 300, 0x77)
    cases = {}
    b = B.copy()
    b[::3] = 0  # identity bases
    cases["identity_bases"] = (S, b)
    s = S.copy()
    s[1::2] = 0
    cases["zero_scalars"] = (s, B)
    cases["all_zero"] = (np.zeros_like(S), B)
    rm1 = np.array(P.to_limbs((C.r - 1) * P.R_MONT % C.r), dtype=np.uint64)
    cases["r_minus_1"] = (np.tile(rm1, (300, 1)), B)
    b = np.tile(B[:1], (300, 1))
    cases["one_base"] = (S, b)
    cases["equal_terms"] = (np.tile(S[:1], (300, 1)), b)
    neg = B.copy()
    for i in range(1, 300, 2):
        pt = P.limbs_to_point(C, [int(v) for v in B[i - 1]])
        neg[i] = np.array(P.point_to_limbs(C, C.neg(pt)), dtype=np.uint64)
    s = S.copy()
    s[1::2] = s[0::2]
    cases["neg_pairs"] = (s, neg)  # sum = 0
    for name, (s, b) in cases.items():
        want = msm_ref.best_multiexp(0, s, b, threads=4)
        assert np.array_equal(gpu_ctx.msm(0, s, b), want), name
    assert not gpu_ctx.msm(0, *cases["neg_pairs"]).any()
    assert not gpu_ctx.msm(0, *cases["all_zero"]).any()


@pytest.mark.parametrize("curve", [0, 2])
def test_canonical_scalars_above_r(gpu_ctx, curve):
    """Canonical-flag scalars are plain 256-bit integers: k and k + j r give
    the same point (reduced mod r before the GLV split)."""
    C = P.CURVES[curve]
    rng = np.random.default_rng(5)
    n = 100
    _, B = _inputs(curve, n, 0x99)
    ks = [int(rng.integers(0, 1 << 62)) << 190 | int(rng.integers(0, 1 << 62)) for _ in range(n)]
    ks = [k % C.r for k in ks]
    big = [k + ((2 ** 256 - 1 - k) // C.r) * C.r for k in ks]  # largest representative < 2^256
    a = np.array([P.to_limbs(k) for k in ks], dtype=np.uint64)
    a_big = np.array([P.to_limbs(k) for k in big], dtype=np.uint64)
    want = msm_ref.best_multiexp(curve, np.array([P.to_limbs(k * P.R_MONT % C.r) for k in ks], dtype=np.uint64), B,
                                 threads=4)
    assert np.array_equal(gpu_ctx.msm(curve, a, B, canonical=True), want)
    assert np.array_equal(gpu_ctx.msm(curve, a_big, B, canonical=True), want)


def test_device_and_resident_entries(gpu_ctx):
    import torch

    curve, n = 1, 3000
    S, B = _inputs(curve, n, 0x3E)
    dev = torch.device("cuda", gpu_ctx.device)
    ds = torch.from_numpy(S.view(np.int64)).to(dev)
    db = torch.from_numpy(B.view(np.int64)).to(dev)
    torch.cuda.synchronize()
    gpu_ctx.set_timing(True)
    try:
        for m, off in ((n, 0), (700, 0), (1000, 1234), (1, 2999)):
            want = msm_ref.best_multiexp(curve, S[off:off + m], B[off:off + m], threads=4)
            gpu_ctx.reset_stats()
            got = gpu_ctx.msm_device(curve, ds[off:].data_ptr(), db[off:].data_ptr(), m)
            assert np.array_equal(got, want), ("device", m, off)
            assert _ran_small(gpu_ctx)
        res = gpu_ctx.upload_bases(curve, B)
        try:
            for m, off in ((n, 0), (1000, 1234), (17, 2983)):
                want = msm_ref.best_multiexp(curve, S[off:off + m], B[off:off + m], threads=4)
                gpu_ctx.reset_stats()
                assert np.array_equal(gpu_ctx.msm_resident(res, off, S[off:off + m]), want), ("resident", m, off)
                assert _ran_small(gpu_ctx)
                got = gpu_ctx.msm_resident_device(res, off, ds[off:].data_ptr(), m)
                assert np.array_equal(got, want), ("resident_device", m, off)
        finally:
            res.release()
    finally:
        gpu_ctx.set_timing(False)


def test_threshold(gpu_ctx):
    """n above the threshold (or an explicit window) runs the pipeline; the
    setter refuses values above PM_SMALL_MSM_LIMIT."""
    S, B = _inputs(0, 600, 0x44)
    want = msm_ref.best_multiexp(0, S, B, threads=4)
    gpu_ctx.set_timing(True)
    try:
        for thr, small in ((599, False), (600, True), (H.SMALL_MSM_LIMIT, True)):
            gpu_ctx.set_small_msm(thr)
            gpu_ctx.reset_stats()
            assert np.array_equal(gpu_ctx.msm(0, S, B), want)
            assert _ran_small(gpu_ctx) == small, thr
        gpu_ctx.set_window(9)
        gpu_ctx.reset_stats()
        assert np.array_equal(gpu_ctx.msm(0, S, B), want)
        assert not _ran_small(gpu_ctx)
    finally:
        gpu_ctx.set_window(0)
        gpu_ctx.set_small_msm(H.SMALL_MSM_DEFAULT)
        gpu_ctx.set_timing(False)
    with pytest.raises(H.PmError, match="error -1"):
        gpu_ctx.set_small_msm(H.SMALL_MSM_LIMIT + 1)


def test_larger_threshold_sizes(gpu_ctx):
    """With the threshold raised to the limit: 2^13 .. 2^16 on the small path."""
    S, B = _inputs(2, 1 << 16, 0x65)
    gpu_ctx.set_small_msm(H.SMALL_MSM_LIMIT)
    try:
        for n in (8192, 20000, 1 << 16):
            want = msm_ref.best_multiexp(2, S[:n], B[:n], threads=8)
            assert np.array_equal(gpu_ctx.msm(2, S[:n], B[:n]), want), n
    finally:
        gpu_ctx.set_small_msm(H.SMALL_MSM_DEFAULT)


@pytest.mark.parametrize("curve", [0, 2])
def test_small_set_dropin_cache(curve):
    """A small base set seen twice is kept resident with a multiples table
    and later pm_msm calls with it run as one short MSM of the many-MSM path:
    every call (first sighting on the small path, admission, hits, a base
    changed in place, new scalars each time) against the C port."""
    ctx = H.Context(0)
    try:
        S, B = _inputs(curve, 8192, 0x5A5 + curve)
        admitted = 0
        for n in (1, 5, 32, 48, 64):
            b = np.ascontiguousarray(B[:n])
            for k in range(4):
                s = np.ascontiguousarray(S[k:k + n])
                want = msm_ref.best_multiexp(curve, s, b, threads=4)
                assert np.array_equal(ctx.msm(curve, s, b), want), (n, k)
            admitted += 1
            st = ctx.dropin_small_stats()
            assert st["admitted"] == admitted and st["entries"] == min(admitted, 8), (n, st)
            # a kept table costs 512 KiB per base (c = 8); only sets
            # of at most 64 points are kept, within the 256 MiB small-set cap
            assert st["device_bytes"] <= admitted * 64 * (2**19 + 64), st
        assert ctx.dropin_small_stats()["hits"] == 2 * 5
        # a base changed in place: a new key (first sighting, small path), still exact
        b = np.ascontiguousarray(B[:32]).copy()
        b[7] = B[100]
        s = np.ascontiguousarray(S[:32])
        assert np.array_equal(ctx.msm(curve, s, b), msm_ref.best_multiexp(curve, s, b, threads=4))
        assert ctx.dropin_small_stats()["hits"] == 10
        assert ctx.dropin_stats()["entries"] == 0   # the large-set cache is untouched
        # above the small-set limit: the small-MSM path, never kept
        for nb in (65, 300, 1000):
            b = np.ascontiguousarray(B[:nb])
            for k in range(3):
                s = np.ascontiguousarray(S[k:k + nb])
                assert np.array_equal(ctx.msm(curve, s, b), msm_ref.best_multiexp(curve, s, b, threads=4)), nb
        assert ctx.dropin_small_stats()["admitted"] == 5
        ctx.dropin_clear()
        assert ctx.dropin_small_stats()["entries"] == 0
    finally:
        ctx.close()
