"""CPU tests of the NTT oracle (oracle/ntt.py): serial_fft equals the DFT
definition, round-trips through ifft, obeys the convolution theorem; the
golden vectors re-derive from it; the library exports pm_fft*."""
import json
import os
import random

import numpy as np

import ntt as N
import pasta as P

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _root(r, k):
    import accum as A
    return A.domain_omega(r, k)


def test_fft_equals_dft_and_round_trip():
    for r in (P.VESTA_P, P.PALLAS_P, P.BN254_R):
        for k in range(0, 7):
            rng = random.Random(k * 7 + r % 97)
            a = [rng.randrange(r) for _ in range(1 << k)]
            w = _root(r, k)
            got = N.serial_fft(list(a), w, k, r)
            assert got == N.dft(a, w, r)
            assert N.ifft(list(got), w, k, r) == a
            for j in range(1 << k):
                assert N.eval_at(a, w, j, r) == got[j]


def test_convolution_theorem():
    r, k = P.BN254_R, 5
    n = 1 << k
    rng = random.Random(5)
    a = [rng.randrange(r) for _ in range(n)]
    b = [rng.randrange(r) for _ in range(n)]
    w = _root(r, k)
    A_ = N.serial_fft(list(a), w, k, r)
    B_ = N.serial_fft(list(b), w, k, r)
    conv = [sum(a[j] * b[(i - j) % n] for j in range(n)) % r for i in range(n)]
    assert N.serial_fft(conv, w, k, r) == [x * y % r for x, y in zip(A_, B_)]


def test_golden_ntt_vectors_match_oracle():
    npz = np.load(os.path.join(GOLD, "ntt_vectors.npz"), allow_pickle=False)
    idx = json.load(open(os.path.join(GOLD, "ntt_vectors.json")))
    for name, meta in idx.items():
        C = P.CURVES[meta["curve"]]
        r, k = C.r, meta["log_n"]
        rinv = pow(P.R_MONT, -1, r)
        a = [P.from_limbs([int(x) for x in row]) * rinv % r for row in npz[f"{name}.input"]]
        w = P.from_limbs([int(x) for x in npz[f"{name}.omega"]]) * rinv % r
        want = N.serial_fft(list(a), w, k, r)
        got = [P.from_limbs([int(x) for x in row]) * rinv % r for row in npz[f"{name}.output"]]
        assert got == want, name


def test_c_best_fft_matches_python_oracle():
    """The C port (serial and halo2's parallel_fft split) == oracle/ntt.py."""
    import msm_ref

    for cid in (0, 2):
        r = P.CURVES[cid].r
        for k in (0, 1, 4, 9):
            rng = random.Random(31 * k + cid)
            a = [rng.randrange(r) for _ in range(1 << k)]
            w = _root(r, k)
            want = N.serial_fft(list(a), w, k, r)
            arr = np.array([P.to_limbs(v * P.R_MONT % r) for v in a], dtype=np.uint64).reshape(-1, 4)
            wl = np.array(P.to_limbs(w * P.R_MONT % r), dtype=np.uint64)
            wantl = np.array([P.to_limbs(v * P.R_MONT % r) for v in want], dtype=np.uint64).reshape(-1, 4)
            for threads in (1, 2, 4, 8):
                assert np.array_equal(msm_ref.best_fft(cid, arr, k, wl, threads), wantl), (cid, k, threads)
