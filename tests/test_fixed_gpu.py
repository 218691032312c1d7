"""GPU parity tests of the fixed-base MSM (pm_fixed_bases_create*,
pm_msm_fixed*): bit-identical to the oracle / variable-base MSM on the golden
vectors, every window width, prefixes of the table, padding rows, identity
bases, canonical scalars, and 2^20 against the known discrete log."""
import numpy as np
import pytest

import halo2_amd as H
import msm_ref
import pasta as P

pytestmark = pytest.mark.gpu


def test_golden_vectors_fixed(golden, gpu_ctx):
    for name, case in golden.items():
        if case["bases"].shape[0] == 0:
            continue
        fb = gpu_ctx.fixed_bases(case["curve"], case["bases"])
        try:
            assert np.array_equal(fb.msm(case["scalars"]), case["expected"]), name
        finally:
            fb.release()


@pytest.mark.parametrize("c", [4, 7, 11, 13, 16, 17, 18, 19, 20])
def test_fixed_window_widths(golden, gpu_ctx, c):
    for name in ("pallas_n4096", "pallas_top_bits", "pallas_equal_scalars", "pallas_neg_pairs", "bn254_n1024"):
        if name not in golden:
            continue
        case = golden[name]
        fb = gpu_ctx.fixed_bases(case["curve"], case["bases"], c=c)
        try:
            assert fb.windows == (256 + c - 1) // c and fb.c == c
            assert fb.table_bytes >= fb.windows * case["bases"].shape[0] * 64
            assert np.array_equal(fb.msm(case["scalars"]), case["expected"]), (name, c)
        finally:
            fb.release()


def test_prefix_and_padding(golden, gpu_ctx):
    """A table of 4096 bases serves any prefix n <= 4096 (commit of a shorter
    polynomial against params.g); rows past n and the padding are zero digits."""
    case = golden["pallas_n4096"]
    fb = gpu_ctx.fixed_bases(0, case["bases"])
    try:
        assert np.array_equal(fb.msm(case["scalars"][:1024]), golden["pallas_n1024"]["expected"])
        for n in (1, 3, 33, 2047, 2049, 4095):
            want = msm_ref.best_multiexp(0, case["scalars"][:n], case["bases"][:n])
            assert np.array_equal(fb.msm(case["scalars"][:n]), want), n
        assert np.array_equal(fb.msm(np.zeros((0, 4), np.uint64)), np.zeros(8, np.uint64))
        with pytest.raises(H.PmError):
            fb.msm(np.zeros((4097, 4), np.uint64))
    finally:
        fb.release()


def test_identity_bases_and_canonical(golden, gpu_ctx):
    case = golden["pallas_n1024"]
    b = case["bases"].copy()
    b[5] = 0
    b[700] = 0
    s = case["scalars"]
    want = msm_ref.best_multiexp(0, s, b)
    fb = gpu_ctx.fixed_bases(0, b, c=13)
    try:
        assert np.array_equal(fb.msm(s), want)
        C = P.PALLAS
        rinv = pow(P.R_MONT, -1, C.r)
        canon = np.array([P.to_limbs(P.from_limbs([int(x) for x in row]) * rinv % C.r) for row in s], np.uint64)
        assert np.array_equal(fb.msm(canon, canonical=True), want)
    finally:
        fb.release()


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_fixed_vs_variable_random(gpu_ctx, curve):
    import torch

    n = 50_000
    dev = torch.device("cuda", gpu_ctx.device)
    s = torch.empty((n, 4), dtype=torch.int64, device=dev)
    b = torch.empty((n, 8), dtype=torch.int64, device=dev)
    gpu_ctx.synth_scalars(curve, 0xF1 + curve, 0, n, s.data_ptr())
    gpu_ctx.synth_bases(curve, 0xF2 + curve, 0, n, b.data_ptr())
    torch.cuda.synchronize()
    want = gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n)
    fb = gpu_ctx.fixed_bases(curve, d_bases=b.data_ptr(), n=n)
    try:
        assert np.array_equal(fb.msm_device(s.data_ptr(), n), want)
        assert np.array_equal(want, msm_ref.best_multiexp(curve, s.cpu().numpy().view(np.uint64),
                                                          b.cpu().numpy().view(np.uint64)))
    finally:
        fb.release()


def test_fixed_known_dlog_2_20(gpu_ctx):
    """2^20 Pallas fixed-base MSM == the variable-base MSM == [sum s_i a_i]G
    (the latter is checked in test_msm_gpu.test_known_dlog_2_20)."""
    import torch

    n = 1 << 20
    dev = torch.device("cuda", gpu_ctx.device)
    s = torch.empty((n, 4), dtype=torch.int64, device=dev)
    b = torch.empty((n, 8), dtype=torch.int64, device=dev)
    gpu_ctx.synth_scalars(0, P.SEED_SCALARS, 0, n, s.data_ptr())
    gpu_ctx.synth_bases(0, P.SEED_BASES, 0, n, b.data_ptr())
    torch.cuda.synchronize()
    want = gpu_ctx.msm_device(0, s.data_ptr(), b.data_ptr(), n)
    fb = gpu_ctx.fixed_bases(0, d_bases=b.data_ptr(), n=n)
    try:
        assert np.array_equal(fb.msm_device(s.data_ptr(), n), want)
        s[:] = s[3]   # one bucket per window: long fixup chains in the merged bucket set
        want2 = gpu_ctx.msm_device(0, s.data_ptr(), b.data_ptr(), n)
        assert np.array_equal(fb.msm_device(s.data_ptr(), n), want2)
    finally:
        fb.release()


@pytest.mark.parametrize("curve", [0, 2])
def test_fixed_known_dlog_2_23(gpu_ctx, curve):
    """The outer prover's commit size (k = 23, examples/simple-example.rs:663,702):
    a 2^23 fixed-base table (auto c = 20: 13 windows, ~7 GB) on Pallas and
    BN254 == [sum s_i a_i]G, and == the variable-base MSM of the same inputs."""
    import torch

    from dlog_util import known_dlog_point

    n = 1 << 23
    dev = torch.device("cuda", gpu_ctx.device)
    s = torch.empty((n, 4), dtype=torch.int64, device=dev)
    b = torch.empty((n, 8), dtype=torch.int64, device=dev)
    gpu_ctx.synth_scalars(curve, P.SEED_SCALARS, 0, n, s.data_ptr())
    gpu_ctx.synth_bases(curve, P.SEED_BASES, 0, n, b.data_ptr())
    torch.cuda.synchronize()
    fb = gpu_ctx.fixed_bases(curve, d_bases=b.data_ptr(), n=n)
    try:
        assert fb.c == 20 and fb.windows == 13
        got = fb.msm_device(s.data_ptr(), n)
    finally:
        fb.release()
    assert np.array_equal(got, gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n))
    del s, b
    torch.cuda.empty_cache()
    C = P.CURVES[curve]
    assert P.limbs_to_point(C, [int(x) for x in got]) == known_dlog_point(curve, n)


def test_fixed_errors(gpu_ctx):
    with pytest.raises(H.PmError):
        gpu_ctx.fixed_bases(0, np.zeros((0, 8), np.uint64))
    with pytest.raises(H.PmError):
        gpu_ctx.fixed_bases(0, np.zeros((4, 8), np.uint64), c=21)
    with pytest.raises(H.PmError):
        gpu_ctx.fixed_bases(9, np.zeros((4, 8), np.uint64))


@pytest.mark.parametrize("c,rows", [(16, 2), (16, 4), (16, 8), (8, 4), (20, 13), (11, 24)])
def test_fixed_rows_golden(golden, gpu_ctx, c, rows):
    """Tables of `rows` rows (pm_fixed_bases_create_rows): windows w, w + W/rows,
    ... share W/rows bucket sets; every golden case bit for bit."""
    for name in ("pallas_n4096", "pallas_top_bits", "pallas_equal_scalars", "pallas_neg_pairs", "pallas_n1024",
                 "bn254_n1024"):
        if name not in golden:
            continue
        case = golden[name]
        fb = gpu_ctx.fixed_bases(case["curve"], case["bases"], c=c, rows=rows)
        try:
            assert fb.table_bytes >= rows * case["bases"].shape[0] * 64
            assert np.array_equal(fb.msm(case["scalars"]), case["expected"]), (name, c, rows)
            n = 1000
            want = msm_ref.best_multiexp(case["curve"], case["scalars"][:n], case["bases"][:n])
            assert np.array_equal(fb.msm(case["scalars"][:n]), want), (name, c, rows, n)
        finally:
            fb.release()


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_fixed_rows2_vs_variable(gpu_ctx, curve):
    """Two-row table ([2^128] P beside P) at 2^20 (Pallas, Vesta, BN254): equal
    to the variable-base MSM, also with identity bases and all-equal scalars."""
    import torch

    n = 1 << 20
    dev = torch.device("cuda", gpu_ctx.device)
    s = torch.empty((n, 4), dtype=torch.int64, device=dev)
    b = torch.empty((n, 8), dtype=torch.int64, device=dev)
    gpu_ctx.synth_scalars(curve, 0xF3 + curve, 0, n, s.data_ptr())
    gpu_ctx.synth_bases(curve, 0xF4 + curve, 0, n, b.data_ptr())
    b[17] = 0
    b[n - 5] = 0
    torch.cuda.synchronize()
    want = gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n)
    fb = gpu_ctx.fixed_bases(curve, d_bases=b.data_ptr(), n=n, c=16, rows=2)
    try:
        assert fb.windows == 16 and fb.table_bytes >= 2 * n * 64
        assert np.array_equal(fb.msm_device(s.data_ptr(), n), want)
        s[:] = s[3]
        torch.cuda.synchronize()
        assert np.array_equal(fb.msm_device(s.data_ptr(), n), gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n))
    finally:
        fb.release()


def test_fixed_rows_errors(gpu_ctx):
    b = np.zeros((4, 8), np.uint64)
    with pytest.raises(H.PmError):
        gpu_ctx.fixed_bases(0, b, c=16, rows=3)   # 3 does not divide W = 16
    with pytest.raises(H.PmError):
        gpu_ctx.fixed_bases(0, b, c=16, rows=-1)
    with pytest.raises(H.PmError):
        gpu_ctx.fixed_bases(0, b, c=13, rows=4)   # W = 20 windows of 12-13 bits: unequal widths
