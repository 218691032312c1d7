"""GPU parity tests of the NTT (pm_fft*) against the oracle (oracle/ntt.py):
golden vectors, every length 2^0 .. 2^14 on every field, scale (ifft),
device pointers, the three-pass form (forced at 2^15 .. 2^17) against the
oracle, and at 2^20 / 2^22 / 2^23 / 2^24 / 2^25 the size-independent
properties: ifft(fft(a)) == a, A_0, A_{n/2}, linearity, and spot outputs
A_k = sum_j a_j omega^{jk}."""
import json
import os
import random

import numpy as np
import pytest

import accum as A
import halo2_amd as H
import ntt as N
import pasta as P

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def mont(r, v):
    return P.to_limbs(v * P.R_MONT % r)


def unmont(r, row):
    return P.from_limbs([int(x) for x in row]) * pow(P.R_MONT, -1, r) % r


def test_golden_ntt(gpu_ctx):
    npz = np.load(os.path.join(GOLD, "ntt_vectors.npz"), allow_pickle=False)
    idx = json.load(open(os.path.join(GOLD, "ntt_vectors.json")))
    for name, meta in idx.items():
        got = gpu_ctx.fft(meta["curve"], npz[f"{name}.input"], npz[f"{name}.omega"])
        assert np.array_equal(got, npz[f"{name}.output"]), name


@pytest.mark.parametrize("cid", [0, 1, 2])
def test_every_length_vs_oracle(gpu_ctx, cid):
    r = P.CURVES[cid].r
    for k in range(0, 15):
        n = 1 << k
        rng = random.Random(1000 * cid + k)
        a = [rng.randrange(r) for _ in range(n)]
        w = A.domain_omega(r, k)
        want = N.serial_fft(list(a), w, k, r)
        arr = np.array([mont(r, v) for v in a], dtype=np.uint64).reshape(n, 4)
        got = gpu_ctx.fft(cid, arr, np.array(mont(r, w), np.uint64))
        assert np.array_equal(got, np.array([mont(r, v) for v in want], dtype=np.uint64).reshape(n, 4)), k
        # ifft = fft(omega^-1) * 1/n
        back = gpu_ctx.fft(cid, got, np.array(mont(r, pow(w, -1, r)), np.uint64),
                           scale=np.array(mont(r, pow(n, -1, r)), np.uint64))
        assert np.array_equal(back, arr), k


@pytest.mark.parametrize("cid", [0, 1, 2])
def test_three_pass_vs_oracle(gpu_ctx, cid):
    """The three-pass form (k_ntt_cols, k_ntt_mid, k_ntt_rows; the default
    above 2^22) forced at small sizes, factor shapes (5,5,5), (6,5,5), (6,6,5),
    against the oracle, with the ifft round trip."""
    os.environ["PM_NTT_PASSES"] = "3"
    try:
        ctx3 = H.Context(gpu_ctx.device)
    finally:
        del os.environ["PM_NTT_PASSES"]
    r = P.CURVES[cid].r
    for k in (15, 16, 17):
        n = 1 << k
        rng = random.Random(7000 * cid + k)
        a = [rng.randrange(r) for _ in range(n)]
        w = A.domain_omega(r, k)
        want = N.serial_fft(list(a), w, k, r)
        arr = np.array([mont(r, v) for v in a], dtype=np.uint64).reshape(n, 4)
        got = ctx3.fft(cid, arr, np.array(mont(r, w), np.uint64))
        assert np.array_equal(got, np.array([mont(r, v) for v in want], dtype=np.uint64).reshape(n, 4)), k
        back = ctx3.fft(cid, got, np.array(mont(r, pow(w, -1, r)), np.uint64),
                        scale=np.array(mont(r, pow(n, -1, r)), np.uint64))
        assert np.array_equal(back, arr), k


@pytest.mark.parametrize("k", [20, 22, 23, 24, 25])
def test_large_properties(gpu_ctx, k):
    import torch

    cid = 2
    r = P.CURVES[cid].r
    n = 1 << k
    dev = torch.device("cuda", gpu_ctx.device)
    a = torch.empty((n, 4), dtype=torch.int64, device=dev)
    gpu_ctx.synth_scalars(cid, 0xF7 + k, 0, n, a.data_ptr())
    torch.cuda.synchronize()
    orig = a.clone()
    w = A.domain_omega(r, k)
    gpu_ctx.fft_device(cid, a.data_ptr(), k, np.array(mont(r, w), np.uint64))
    torch.cuda.synchronize()
    out = a.cpu().numpy().view(np.uint64)
    src = orig.cpu().numpy().view(np.uint64)
    # A_0 = sum_j a_j and A_{n/2} = sum_j (-1)^j a_j, exact at any size (the
    # Montgomery map is linear, so the raw limbs are summed directly)
    def limb_sum(rows):
        tot = 0
        for l in range(4):
            col = rows[:, l]
            lo = int((col & np.uint64(0xFFFFFFFF)).sum(dtype=np.uint64))
            hi = int((col >> np.uint64(32)).sum(dtype=np.uint64))
            tot += (lo + (hi << 32)) << (64 * l)
        return tot

    ev, od = limb_sum(src[0::2]), limb_sum(src[1::2])
    as_int = lambda row: P.from_limbs([int(x) for x in row])  # noqa: E731
    assert as_int(out[0]) == (ev + od) % r
    assert as_int(out[n // 2]) == (ev - od) % r
    if k <= 20:   # spot outputs against the definition (O(n) each in Python)
        coeffs = [unmont(r, row) for row in src]
        for j in (1, n - 1, 12345):
            assert unmont(r, out[j]) == N.eval_at(coeffs, w, j, r), j
    gpu_ctx.fft_device(cid, a.data_ptr(), k, np.array(mont(r, pow(w, -1, r)), np.uint64),
                       scale=np.array(mont(r, pow(n, -1, r)), np.uint64))
    torch.cuda.synchronize()
    assert torch.equal(a, orig)


def test_linearity_2_18(gpu_ctx):
    import torch

    cid, k = 0, 18
    r = P.CURVES[cid].r
    n = 1 << k
    dev = torch.device("cuda", gpu_ctx.device)
    x = torch.empty((n, 4), dtype=torch.int64, device=dev)
    y = torch.empty((n, 4), dtype=torch.int64, device=dev)
    gpu_ctx.synth_scalars(cid, 1, 0, n, x.data_ptr())
    gpu_ctx.synth_scalars(cid, 2, 0, n, y.data_ptr())
    torch.cuda.synchronize()
    w = np.array(mont(r, A.domain_omega(r, k)), np.uint64)
    xs = x.cpu().numpy().view(np.uint64)
    ys = y.cpu().numpy().view(np.uint64)
    zs = np.array([mont(r, (unmont(r, p) + unmont(r, q)) % r) for p, q in zip(xs, ys)], dtype=np.uint64)
    fx, fy, fz = (gpu_ctx.fft(cid, v, w) for v in (xs, ys, zs))
    for j in range(0, n, 997):
        assert (unmont(r, fx[j]) + unmont(r, fy[j])) % r == unmont(r, fz[j]), j


def test_ntt_errors(gpu_ctx):
    with pytest.raises(H.PmError):
        gpu_ctx.fft(9, np.zeros((4, 4), np.uint64), np.zeros(4, np.uint64))
    with pytest.raises(ValueError):
        gpu_ctx.fft(0, np.zeros((3, 4), np.uint64), np.zeros(4, np.uint64))


@pytest.mark.parametrize("cid", [0, 1, 2])
def test_extreme_representations_vs_oracle(gpu_ctx, cid):
    """Inputs whose Montgomery representations sit at the top of [0, p)
    (p - 1, p - 2, alternating with 0 and 1, a lone p - 1): the lazy
    radix-2^29 butterflies see their largest limbs, and the intermediate
    values between passes land near the top of their < 3p bound.  Two-pass
    sizes and the forced three-pass form, against the oracle."""
    os.environ["PM_NTT_PASSES"] = "3"
    try:
        ctx3 = H.Context(gpu_ctx.device)
    finally:
        del os.environ["PM_NTT_PASSES"]
    r = P.CURVES[cid].r
    rinv = pow(P.R_MONT, -1, r)
    for k, ctx in ((10, gpu_ctx), (13, gpu_ctx), (15, ctx3)):
        n = 1 << k
        w = A.domain_omega(r, k)
        pats = [[r - 1] * n, [0 if j % 2 else r - 1 for j in range(n)], [r - 2 if j % 3 else 1 for j in range(n)],
                [r - 1 if j == n // 2 + 1 else 0 for j in range(n)]]
        for pi, reps in enumerate(pats):
            vals = [x * rinv % r for x in reps]
            want = N.serial_fft(list(vals), w, k, r)
            arr = np.array([P.to_limbs(x) for x in reps], dtype=np.uint64).reshape(n, 4)
            got = ctx.fft(cid, arr, np.array(mont(r, w), np.uint64))
            assert np.array_equal(got, np.array([mont(r, v) for v in want], dtype=np.uint64).reshape(n, 4)), (k, pi)
