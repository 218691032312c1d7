"""GPU parity tests of pm_msm_resident_many* (msm_many.hpp): B short MSMs
against one resident base set in one launch -- the aggregator's per-proof
instance commitments, params_verifier.commit_lagrange(public_inputs)
(examples/simple-example.rs:632-641) -- each against the C port of halo2
best_multiexp (oracle/msm_ref.c) on the same scalars and base window:

* B in {1, 16, 256} with n_i from 1 to 4096, mixed in one call, prefix
  windows (offsets = NULL) and arbitrary offsets, on all three curves
* edge inputs: n_i = 0, identity bases, zero scalars, r - 1, canonical
  scalars >= r, the same base in every MSM, P and -P in one MSM
* the device-scalar entry, the table's growth (a later call reaching further
  into the set rebuilds it with a narrower window when the prefix needs it)
"""
import numpy as np
import pytest

import halo2_amd as H
import msm_ref
import pasta as P

pytestmark = pytest.mark.gpu


def _inputs(curve, n, seed):
    s = msm_ref.synth_scalars(curve, P.SEED_SCALARS ^ seed, 0, n, threads=4)
    b = msm_ref.synth_bases(curve, P.SEED_BASES ^ seed, 0, n, threads=4)
    return np.ascontiguousarray(s), np.ascontiguousarray(b)


def _want(curve, n, offsets, S, B):
    out, s0 = [], 0
    for i, k in enumerate(n):
        o = 0 if offsets is None else offsets[i]
        out.append(msm_ref.best_multiexp(curve, S[s0:s0 + k], B[o:o + k], threads=4) if k else np.zeros(8, np.uint64))
        s0 += k
    return np.array(out, dtype=np.uint64)


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_batches_vs_c_port(gpu_ctx, curve):
    nb = 4096
    S, B = _inputs(curve, 8192, 0x3A + curve)
    bases = gpu_ctx.upload_bases(curve, B[:nb])
    rng = np.random.default_rng(0xB5 + curve)
    for nbatch in (1, 16, 256):
        if nbatch == 1:
            n = [4096]
        elif nbatch == 16:
            n = [1, 2, 3, 31, 32, 33, 64, 100, 1, 0, 257, 1000, 4096, 5, 1, 2049]
        else:
            n = list(rng.choice([1, 1, 1, 2, 4, 8, 13, 64], size=nbatch))
        s = S[:sum(n)]
        got = gpu_ctx.msm_resident_many(bases, n, s)
        assert np.array_equal(got, _want(curve, n, None, s, B)), (curve, nbatch)
    # arbitrary windows of the set
    n = [int(x) for x in rng.integers(0, 300, size=40)]
    offs = [int(rng.integers(0, nb - k + 1)) for k in n]
    s = S[:sum(n)]
    got = gpu_ctx.msm_resident_many(bases, n, s, offsets=offs)
    assert np.array_equal(got, _want(curve, n, offs, s, B)), curve


def test_edge_inputs(gpu_ctx):
    C = P.PALLAS
    S, B = _inputs(0, 512, 0x77)
    Bi = B.copy()
    Bi[::5] = 0                       # identity bases
    Bi[7] = B[8]
    Bi[8] = P.point_to_limbs(C, C.neg(P.limbs_to_point(C, [int(v) for v in B[8]])))  # P and -P
    bases = gpu_ctx.upload_bases(0, Bi)
    s = S.copy()
    s[1::3] = 0                       # zero scalars
    rm1 = np.array(P.to_limbs((C.r - 1) * P.R_MONT % C.r), dtype=np.uint64)
    s[2] = rm1
    s[4] = s[9] = s[11]               # equal terms
    n = [0, 1, 9, 10, 0, 100, 256, 1, 1, 3]
    got = gpu_ctx.msm_resident_many(bases, n, s[:sum(n)])
    assert np.array_equal(got, _want(0, n, None, s, Bi))
    assert not got[0].any() and not got[4].any()
    # all-zero scalars and only identity bases give the identity
    got = gpu_ctx.msm_resident_many(bases, [5, 1], np.zeros((6, 4), np.uint64), offsets=[0, 5])
    assert not got.any()
    # canonical scalars, including values >= r (reduced mod r like best_multiexp's to_repr of a field element)
    sc = np.array([P.to_limbs(v) for v in (C.r - 1, C.r, C.r + 5, (1 << 256) - 1, 0, 1, 2, 12345)],
                  dtype=np.uint64)
    got = gpu_ctx.msm_resident_many(bases, [8, 3, 5], np.concatenate([sc, sc]), offsets=[16, 100, 200],
                                    canonical=True)
    want = []
    for k, o, ss in ((8, 16, sc), (3, 100, sc[:3]), (5, 200, sc[3:8])):
        ref = [P.to_limbs(int(P.from_limbs([int(v) for v in row])) % C.r * P.R_MONT % C.r) for row in ss]
        want.append(msm_ref.best_multiexp(0, np.array(ref, dtype=np.uint64), Bi[o:o + k]))
    assert np.array_equal(got, np.array(want, dtype=np.uint64))


def test_device_entry_and_table_growth():
    import torch

    ctx = H.Context(0)
    curve = 2
    S, B = _inputs(curve, 4096, 0x99)
    B = B[:2048]
    bases = ctx.upload_bases(curve, B)
    assert bases.many_info() == (0, 0, 0)
    n = [1] * 64
    got = ctx.msm_resident_many(bases, n, S[:64])
    assert np.array_equal(got, _want(curve, n, None, S, B))
    pre, c, nbytes = bases.many_info()
    assert pre == 64 and c == 8 and nbytes == 64 * 32 * 128 * 128
    # device scalars, reaching further: the table grows (to a power of two)
    n = [700, 1, 2047, 0, 33]
    d = torch.from_numpy(S[:sum(n)].view(np.int64)).cuda()
    torch.cuda.synchronize()
    got = ctx.msm_resident_many_device(bases, n, d.data_ptr())
    assert np.array_equal(got, _want(curve, n, None, S, B))
    assert bases.many_info()[0] == 2048
    # explicit preparation is a no-op when the table already covers the prefix
    ctx.bases_many_prepare(bases, 1000)
    assert bases.many_info()[0] == 2048
    with pytest.raises(H.PmError):   # window beyond the set
        ctx.msm_resident_many(bases, [10], S[:10], offsets=[2040])
    with pytest.raises(H.PmError):   # prefix beyond the set
        ctx.bases_many_prepare(bases, 4096)


def test_pipeline_order_independent(gpu_ctx):
    """The same MSMs in another order (and split over two calls) give the
    same points: no state leaks between MSMs or calls."""
    curve = 1
    S, B = _inputs(curve, 1000, 0x1234)
    bases = gpu_ctx.upload_bases(curve, B[:256])
    n = [1, 5, 17, 64, 1, 2, 100, 3] * 4
    offs = [(7 * i) % 100 for i in range(len(n))]
    s = S[:sum(n)]
    got = gpu_ctx.msm_resident_many(bases, n, s, offsets=offs)
    starts = np.cumsum([0] + n[:-1])
    perm = list(reversed(range(len(n))))
    s2 = np.concatenate([s[starts[i]:starts[i] + n[i]] for i in perm])
    got2 = gpu_ctx.msm_resident_many(bases, [n[i] for i in perm], s2, offsets=[offs[i] for i in perm])
    assert np.array_equal(got2, got[perm])
    h = len(n) // 2
    a = gpu_ctx.msm_resident_many(bases, n[:h], s[:starts[h]], offsets=offs[:h])
    b = gpu_ctx.msm_resident_many(bases, n[h:], s[starts[h]:], offsets=offs[h:])
    assert np.array_equal(np.concatenate([a, b]), got)
