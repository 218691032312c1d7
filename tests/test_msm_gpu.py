"""GPU parity tests: the HIP MSM (through the C-ABI) against the oracle.

* golden vectors (Python restatement of halo2 best_multiexp), every case
* every window width 4..20 on one vector (exercises all k_digits instances)
* larger random sizes against the C restatement (oracle/msm_ref.c)
* 2^20 against the known-discrete-log answer (size-independent property)
* API surface: resident bases, multi-GPU entry, device pointers, errors
"""
import numpy as np
import pytest

import halo2_amd as H
from dlog_util import known_dlog_point
import msm_ref
import pasta as P

pytestmark = pytest.mark.gpu


def test_golden_vectors(golden):
    for name, case in golden.items():
        got = H.best_multiexp(case["curve"], case["scalars"], case["bases"])
        assert np.array_equal(got, case["expected"]), name


@pytest.mark.parametrize("c", list(range(4, 21)))
def test_every_window_width(golden, gpu_ctx, c):
    gpu_ctx.set_window(c)
    try:
        for name in ("pallas_n1024", "pallas_top_bits", "pallas_equal_scalars", "pallas_neg_pairs"):
            case = golden[name]
            got = gpu_ctx.msm(case["curve"], case["scalars"], case["bases"])
            assert np.array_equal(got, case["expected"]), (name, c)
    finally:
        gpu_ctx.set_window(0)


def test_retired_options(gpu_ctx):
    """The A/B paths measured slower (GLV mode, window groups, pinned staging
    threads) are retired: their setters accept only the default and refuse
    the rest with PM_ERR_UNSUPPORTED (-4) instead of silently ignoring it."""
    gpu_ctx.set_glv(False)
    gpu_ctx.set_pipeline(0, 0)
    gpu_ctx.set_pipeline(1, 0)
    gpu_ctx.set_h2d_threads(0)
    for call in (lambda: gpu_ctx.set_glv(True), lambda: gpu_ctx.set_pipeline(2, 0),
                 lambda: gpu_ctx.set_h2d_threads(4)):
        with pytest.raises(H.PmError, match="error -4"):
            call()
    with pytest.raises(H.PmError, match="error -1"):
        gpu_ctx.set_h2d_threads(-1)


@pytest.mark.parametrize("min_chunk", [1, 2, 7, 64])
def test_slice_lengths(golden, gpu_ctx, min_chunk):
    """The accumulate slice length (every chain shape, from one-entry slices
    to whole buckets per lane) does not change results."""
    gpu_ctx.set_pipeline(0, min_chunk)
    try:
        for name in ("pallas_n4096", "pallas_equal_scalars", "pallas_neg_pairs", "vesta_n1024", "bn254_n1024"):
            if name not in golden:
                continue
            case = golden[name]
            for c in (0, 5, 11):
                gpu_ctx.set_window(c)
                got = gpu_ctx.msm(case["curve"], case["scalars"], case["bases"])
                assert np.array_equal(got, case["expected"]), (name, min_chunk, c)
    finally:
        gpu_ctx.set_window(0)
        gpu_ctx.set_pipeline(0, 0)


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_radix29_field_selftest(gpu_ctx, curve):
    """The MSM pipeline's radix-2^29 lazy Montgomery arithmetic agrees with the
    32-bit arithmetic on 2^16 random + edge operand pairs, including loose
    operands at the limb bound and the 16p -> 3p reduction."""
    assert gpu_ctx.selftest_field(curve, 0x29 + curve, 1 << 16) == 0


def test_canonical_scalars(golden):
    case = golden["pallas_n4096"]
    C = P.PALLAS
    rinv = pow(P.R_MONT, -1, C.r)
    canon = np.array([P.to_limbs(P.from_limbs(s) * rinv % C.r) for s in case["scalars"]], dtype=np.uint64)
    got = H.best_multiexp(0, canon, case["bases"], canonical=True)
    assert np.array_equal(got, case["expected"])


def _torch_inputs(ctx, curve, n, i0=0):
    import torch

    dev = torch.device("cuda", ctx.device)
    s = torch.empty((n, 4), dtype=torch.int64, device=dev)
    b = torch.empty((n, 8), dtype=torch.int64, device=dev)
    ctx.synth_scalars(curve, P.SEED_SCALARS, i0, n, s.data_ptr())
    ctx.synth_bases(curve, P.SEED_BASES, i0, n, b.data_ptr())
    torch.cuda.synchronize()
    return s, b


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_synth_on_device_matches_oracle(gpu_ctx, curve):
    n = 3000
    s, b = _torch_inputs(gpu_ctx, curve, n, i0=12345)
    S = s.cpu().numpy().view(np.uint64)
    B = b.cpu().numpy().view(np.uint64)
    assert np.array_equal(S, msm_ref.synth_scalars(curve, P.SEED_SCALARS, 12345, n))
    assert np.array_equal(B, msm_ref.synth_bases(curve, P.SEED_BASES, 12345, n))


# sizes cover every sort block shape (1024 threads x ppt points: ppt 1 below
# 2^18, 2 from 2^18, 4 from 2^19, 8 from 2^20), ragged tails included
@pytest.mark.parametrize("curve,n", [(0, 5000), (0, (1 << 16) + 123), (1, 1 << 16), (2, 40000), (0, 1 << 18),
                                     (1, (1 << 19) + 777), (2, (1 << 20) + 5)])
def test_vs_c_oracle(gpu_ctx, curve, n):
    s, b = _torch_inputs(gpu_ctx, curve, n)
    got = gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n)
    S = s.cpu().numpy().view(np.uint64)
    B = b.cpu().numpy().view(np.uint64)
    want = msm_ref.best_multiexp(curve, S, B)
    assert np.array_equal(got, want)
    if n <= H.SMALL_MSM_DEFAULT:  # that ran the small-MSM path: the sorting pipeline too
        gpu_ctx.set_small_msm(0)
        try:
            assert np.array_equal(gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n), want)
        finally:
            gpu_ctx.set_small_msm(H.SMALL_MSM_DEFAULT)


@pytest.mark.parametrize("curve,logn", [(0, 20), (0, 22), (1, 22)])
def test_known_dlog(gpu_ctx, curve, logn):
    """2^k MSM == [sum s_i a_i]G (a_i = discrete log of synthetic base i).
    2^22 Pallas is the north-star size; 2^22 Vesta is SURVEY config 4 on
    one GPU.  At 2^22 the bases (256 MB) + their R = 2^261 copy exceed the
    Infinity Cache, so the gathers take the HBM path."""
    n = 1 << logn
    s, b = _torch_inputs(gpu_ctx, curve, n)
    got = gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n)
    C = P.CURVES[curve]
    assert P.limbs_to_point(C, [int(x) for x in got]) == known_dlog_point(curve, n)
    if logn >= 22:
        # and bit for bit against the C restatement of best_multiexp
        assert np.array_equal(got, msm_ref.best_multiexp(curve, s.cpu().numpy().view(np.uint64),
                                                         b.cpu().numpy().view(np.uint64)))


@pytest.mark.parametrize("cache_kb,chunk_kb", [(4, 4), (8, 8), (68, 8), (136, 16)])
def test_fine_sort_lds_modes(monkeypatch, cache_kb, chunk_kb):
    """k_sort_fine with its segment cache and chunk buffer forced (PM_FINE_*,
    read when a context is created): 4-8 KiB re-read every segment from HBM
    in many chunks, 68 / 136 KiB hold whole segments in LDS and sort them in
    8 / 16 KiB chunks.  2^18 resident (8-row table: 16 K-entry segments) and
    2^20 raw bases, against the C restatement."""
    monkeypatch.setenv("PM_FINE_CACHE_KB", str(cache_kb))
    monkeypatch.setenv("PM_FINE_CHUNK_KB", str(chunk_kb))
    ctx = H.Context(0)
    for curve, n in [(0, (1 << 18) + 5), (1, 1 << 20)]:
        s, b = _torch_inputs(ctx, curve, n)
        want = msm_ref.best_multiexp(curve, s.cpu().numpy().view(np.uint64), b.cpu().numpy().view(np.uint64))
        assert np.array_equal(ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n), want)
        rb = H.Bases(ctx, curve, d_bases=b.data_ptr(), n=n)
        try:
            assert np.array_equal(ctx.msm_resident_device(rb, 0, s.data_ptr(), n), want)
        finally:
            rb.release()


def test_all_equal_scalars_large(gpu_ctx):
    """One bucket per window holds every point: long fixup chains."""
    n = 1 << 16
    s, b = _torch_inputs(gpu_ctx, 0, n)
    s[:] = s[7]
    got = gpu_ctx.msm_device(0, s.data_ptr(), b.data_ptr(), n)
    assert np.array_equal(got, msm_ref.best_multiexp(0, s.cpu().numpy().view(np.uint64),
                                                     b.cpu().numpy().view(np.uint64)))


@pytest.mark.parametrize("distinct", [3, 40, 700])
def test_few_distinct_scalars(gpu_ctx, distinct):
    """Scalars from a small set: buckets of ~n/distinct points whose runs
    cross a few accumulate slices (chains folded by the bucket's own lane in
    k_bucket_seg_q) or more than kSerialChain of them (folded wave-wide)."""
    import torch

    n = 1 << 16
    s, b = _torch_inputs(gpu_ctx, 0, n)
    idx = torch.arange(n, device=s.device) % distinct
    s[:] = s[idx]
    torch.cuda.synchronize()
    got = gpu_ctx.msm_device(0, s.data_ptr(), b.data_ptr(), n)
    assert np.array_equal(got, msm_ref.best_multiexp(0, s.cpu().numpy().view(np.uint64),
                                                     b.cpu().numpy().view(np.uint64)))


def test_resident_bases_window(golden, gpu_ctx):
    case = golden["pallas_n4096"]
    rb = gpu_ctx.upload_bases(0, case["bases"])
    try:
        got = gpu_ctx.msm_resident(rb, 0, case["scalars"])
        assert np.array_equal(got, case["expected"])
        sub = golden["pallas_n1024"]
        assert np.array_equal(gpu_ctx.msm_resident(rb, 0, case["scalars"][:1024]), sub["expected"])
        with pytest.raises(H.PmError):
            gpu_ctx.msm_resident(rb, 4000, case["scalars"][:200])
    finally:
        rb.release()


def test_multi_entry_and_point_add(golden):
    case = golden["pallas_n4096"]
    ngpu = H.device_count()
    got = H.msm_multi(0, case["scalars"], case["bases"], ngpu)
    assert np.array_equal(got, case["expected"])
    a = H.best_multiexp(0, case["scalars"][:2000], case["bases"][:2000])
    b = H.best_multiexp(0, case["scalars"][2000:], case["bases"][2000:])
    assert np.array_equal(H.point_add(0, a, b), case["expected"])


def test_errors():
    with pytest.raises(H.PmError):
        H.best_multiexp(7, np.zeros((1, 4), np.uint64), np.zeros((1, 8), np.uint64))
    with pytest.raises(ValueError):
        H.best_multiexp(0, np.zeros((2, 4), np.uint64), np.zeros((1, 8), np.uint64))
    assert np.array_equal(H.best_multiexp(0, np.zeros((0, 4), np.uint64), np.zeros((0, 8), np.uint64)),
                          np.zeros(8, np.uint64))


@pytest.mark.parametrize("curve,n", [(0, (1 << 20) + 3), (1, 70001), (2, 5000)])
def test_resident_device_and_host_paths(gpu_ctx, curve, n):
    """Resident bases (converted to the pipeline form at upload, from device
    or host memory) give the raw-bases result, with device and host scalars,
    and for windows at an offset."""
    s, b = _torch_inputs(gpu_ctx, curve, n)
    want = gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n)
    S = s.cpu().numpy().view(np.uint64)
    B = b.cpu().numpy().view(np.uint64)
    rb = gpu_ctx.upload_bases(curve, d_bases=b.data_ptr(), n=n)
    rh = gpu_ctx.upload_bases(curve, B)
    try:
        assert np.array_equal(gpu_ctx.msm_resident_device(rb, 0, s.data_ptr(), n), want)
        assert np.array_equal(gpu_ctx.msm_resident_device(rh, 0, s.data_ptr(), n), want)
        assert np.array_equal(gpu_ctx.msm_resident(rb, 0, S), want)
        assert np.array_equal(gpu_ctx.msm(curve, S, B), want)
        k = n // 3
        part = gpu_ctx.msm_device(curve, s[k:].data_ptr(), b[k:].data_ptr(), n - k)
        assert np.array_equal(gpu_ctx.msm_resident(rb, k, S[k:]), part)
    finally:
        rb.release()
        rh.release()
    if n < (1 << 20):
        assert np.array_equal(want, msm_ref.best_multiexp(curve, S, B))


@pytest.mark.parametrize("k", [1, 2, 5])
def test_resident_batch(gpu_ctx, k):
    """pm_msm_resident_batch (copies of MSM j+1 and the host tail of MSM j-1
    overlapping MSM j's kernels) == k single pm_msm_resident calls, also with
    canonical scalars and an offset window."""
    import torch

    n = (1 << 16) + 7
    s, b = _torch_inputs(gpu_ctx, 0, n + 100)
    B = b.cpu().numpy().view(np.uint64)
    rb = gpu_ctx.upload_bases(0, B)
    try:
        lists = []
        for j in range(k):
            sj = torch.empty((n, 4), dtype=torch.int64, device=s.device)
            gpu_ctx.synth_scalars(0, 0x5EED + 17 * j, 0, n, sj.data_ptr())
            torch.cuda.synchronize()
            lists.append(sj.cpu().numpy().view(np.uint64).copy())
        got = gpu_ctx.msm_resident_batch(rb, 50, lists)
        for j in range(k):
            assert np.array_equal(got[j], gpu_ctx.msm_resident(rb, 50, lists[j])), j
        assert np.array_equal(got[0], msm_ref.best_multiexp(0, lists[0], B[50:50 + n]))
        C = P.PALLAS
        rinv = pow(P.R_MONT, -1, C.r)
        canon = [np.array([P.to_limbs(P.from_limbs([int(x) for x in row]) * rinv % C.r) for row in L[:300]],
                          dtype=np.uint64) for L in lists[:2]]
        got_c = gpu_ctx.msm_resident_batch(rb, 0, canon, canonical=True)
        for j in range(len(canon)):
            assert np.array_equal(got_c[j], gpu_ctx.msm_resident(rb, 0, lists[j][:300])), j
        with pytest.raises(ValueError):
            gpu_ctx.msm_resident_batch(rb, 0, [lists[0], lists[0][:5]])
        with pytest.raises(H.PmError):
            gpu_ctx.msm_resident_batch(rb, 200, lists[:1])   # window past the resident bases
    finally:
        rb.release()


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_resident_row_table(gpu_ctx, curve):
    """Resident bases from 2^18 on keep [2^{64 j}] P rows (pm_bases_upload*):
    full-length MSMs and batches take the row-table path, offset windows the
    plain pipeline on row 0; all equal the raw-bases MSM."""
    import torch

    n = (1 << 20) + 3
    s, b = _torch_inputs(gpu_ctx, curve, n)
    rb = gpu_ctx.upload_bases(curve, d_bases=b.data_ptr(), n=n)
    try:
        want = gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n)
        assert np.array_equal(gpu_ctx.msm_resident_device(rb, 0, s.data_ptr(), n), want)
        m = (1 << 19) + 17   # covers more than half of the table: row-table path
        assert np.array_equal(gpu_ctx.msm_resident_device(rb, 0, s.data_ptr(), m),
                              gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), m))
        # offset window: plain pipeline on row 0
        o = 5
        assert np.array_equal(gpu_ctx.msm_resident_device(rb, o, s.data_ptr(), m),
                              gpu_ctx.msm_device(curve, s.data_ptr(), b[o:].data_ptr(), m))
        S = s.cpu().numpy().view(np.uint64)
        lists = [S[:m], np.roll(S[:m], 1, axis=0)]
        got = gpu_ctx.msm_resident_batch(rb, 0, lists)
        for j, L in enumerate(lists):
            assert np.array_equal(got[j], gpu_ctx.msm_resident(rb, 0, L)), j
    finally:
        rb.release()


@pytest.mark.parametrize("curve,min_chunk", [(1, 0), (0, 16), (2, 3)])
def test_adjacent_giant_buckets(gpu_ctx, curve, min_chunk):
    """Scalars 1 .. 64 (canonical): window 0's buckets 1 .. 64 hold n/64
    points each and lie in ONE wave of k_bucket_seg_q, so almost every lane
    of that wave owns a chain longer than kSerialChain slices: the wave's
    rule picks the lanes' own walks over 64 wave-wide folds.  (A single giant
    bucket, test_all_equal_scalars_large, takes the wave-wide fold.)"""
    import torch

    n = (1 << 17) + 99
    s, b = _torch_inputs(gpu_ctx, curve, n)
    small = (torch.arange(n, device=s.device) % 64) + 1
    s.zero_()
    s[:, 0] = small
    torch.cuda.synchronize()
    gpu_ctx.set_pipeline(0, min_chunk)
    try:
        got = gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n, canonical=True)
    finally:
        gpu_ctx.set_pipeline(0, 0)
    C = P.CURVES[curve]
    B = b.cpu().numpy().view(np.uint64)
    # sum_i (i % 64 + 1) P_i == the C port on the Montgomery form of the scalars
    mont = np.array([P.to_limbs((i % 64 + 1) * P.R_MONT % C.r) for i in range(64)], dtype=np.uint64)
    S = mont[np.arange(n) % 64]
    assert np.array_equal(got, msm_ref.best_multiexp(curve, S, B))


@pytest.mark.parametrize("curve", [0, 2])
def test_dropin_base_cache(curve):
    """pm_msm_ctx (host scalars + host bases, the transparent best_multiexp
    drop-in) keeps repeated base sets resident keyed by a keyed content
    digest: the first sighting runs the plain pipeline and is not admitted,
    the second admits the set, later calls hit (also for other scalars);
    bytes changed in place at the same address miss and stay bit-exact;
    small MSMs bypass the cache; at most 4 sets stay; clear() releases them;
    two contexts hold different digest keys."""
    ctx = H.Context(0)
    ctx2 = H.Context(0)
    try:
        assert ctx.dropin_key_id() != ctx2.dropin_key_id()
        n = (1 << 14) + 3
        s, b = _torch_inputs(ctx, curve, 2 * n)
        S = s.cpu().numpy().view(np.uint64).copy()
        B = b.cpu().numpy().view(np.uint64).copy()
        Bn = np.ascontiguousarray(B[:n])
        want = msm_ref.best_multiexp(curve, S[:n], Bn)
        assert np.array_equal(ctx.msm(curve, S[:n], Bn), want)
        st = ctx.dropin_stats()
        assert st["misses"] == 1 and st["hits"] == 0 and st["entries"] == 0   # seen once: not admitted
        assert np.array_equal(ctx.msm(curve, S[n:], Bn), msm_ref.best_multiexp(curve, S[n:], Bn))
        st = ctx.dropin_stats()
        assert st["misses"] == 2 and st["hits"] == 0 and st["entries"] == 1   # second sighting: admitted
        assert np.array_equal(ctx.msm(curve, S[:n], Bn), want)
        st = ctx.dropin_stats()
        assert st["hits"] == 1 and st["entries"] == 1
        # the other context's cache is its own
        assert np.array_equal(ctx2.msm(curve, S[:n], Bn), want)
        assert ctx2.dropin_stats()["hits"] == 0
        # mutate one base in place (same pointer): must miss and stay exact
        Bn[5] = B[n + 5]
        want2 = msm_ref.best_multiexp(curve, S[:n], Bn)
        for _ in range(2):
            assert np.array_equal(ctx.msm(curve, S[:n], Bn), want2)
        st = ctx.dropin_stats()
        assert st["misses"] == 4 and st["entries"] == 2 and st["hits"] == 1
        assert np.array_equal(ctx.msm(curve, S[:n], Bn), want2)
        assert ctx.dropin_stats()["hits"] == 2
        # warm hits start the predicted set's MSM behind the scalar copy
        kept, drained = ctx.dropin_spec_stats()
        assert kept >= 2 and drained == 0
        # a change the prediction cannot see (a middle base: the first and
        # last 8 points are equal): the predicted set's MSM starts, the full
        # digest names no set, the speculative result is dropped
        Bm = Bn.copy()
        Bm[n // 2] = B[n + 7]
        wm = msm_ref.best_multiexp(curve, S[:n], Bm)
        assert np.array_equal(ctx.msm(curve, S[:n], Bm), wm)
        assert ctx.dropin_spec_stats() == (kept, 1)
        assert ctx.dropin_stats()["hits"] == 2
        assert ctx.dropin_oom_stats() == (0, 0)   # no out-of-memory event at these sizes
        # small MSMs bypass the cache
        ctx.msm(curve, S[:100], B[:100])
        assert ctx.dropin_stats()["entries"] == 2
        # LRU bound
        for k in range(4):
            Bk = np.ascontiguousarray(B[k + 1:k + 1 + n])
            wk = msm_ref.best_multiexp(curve, S[:n], Bk)
            for _ in range(2):
                assert np.array_equal(ctx.msm(curve, S[:n], Bk), wk)
        assert ctx.dropin_stats()["entries"] == 4
        ctx.dropin_clear()
        assert ctx.dropin_stats()["entries"] == 0
    finally:
        ctx.close()
        ctx2.close()


def test_dropin_row_table(gpu_ctx):
    """A full-length repeated set from 2^18 points runs as a resident
    row-table MSM once admitted (second call); pm_msm_resident / pm_msm_fixed
    with host scalars; all equal the device-input MSM."""
    import torch

    n = (1 << 18) + 11
    s, b = _torch_inputs(gpu_ctx, 0, n)
    want = gpu_ctx.msm_device(0, s.data_ptr(), b.data_ptr(), n)
    S = s.cpu().numpy().view(np.uint64).copy()
    B = b.cpu().numpy().view(np.uint64).copy()
    ctx = H.Context(0)
    try:
        for _ in range(4):
            assert np.array_equal(ctx.msm(0, S, B), want)
        st = ctx.dropin_stats()
        assert st["hits"] == 2 and st["misses"] == 2 and st["entries"] == 1
        # a middle base changed: the speculative row-table MSM (split scalar
        # copy) starts on the predicted set, the digest names no set, the
        # speculative result is drained and the call runs as a miss
        kept, drained = ctx.dropin_spec_stats()
        Bm = B.copy()
        Bm[n // 2] = B[3]
        wm = gpu_ctx.msm_device(0, s.data_ptr(), torch.from_numpy(Bm.view(np.int64)).to(b.device).data_ptr(), n)
        assert np.array_equal(ctx.msm(0, S, Bm), wm)
        assert ctx.dropin_spec_stats() == (kept, drained + 1)
        rb = ctx.upload_bases(0, d_bases=b.data_ptr(), n=n)
        assert rb.rows > 1
        assert np.array_equal(ctx.msm_resident(rb, 0, S), want)
        rb.release()
        fb = ctx.fixed_bases(0, d_bases=b.data_ptr(), n=n)
        assert np.array_equal(fb.msm(S), want)
        fb.release()
    finally:
        ctx.close()


@pytest.mark.parametrize("curve", [0, 2])
def test_split_scalar_copy(gpu_ctx, curve):
    """Row-table MSMs with host scalars from PM_SPLIT_COPY_MIN_N points copy
    the scalars in two parts (3/8, 5/8; three from 2^21 points), each sorted
    and accumulated on its own, with one bucket reduction over the parts'
    sorted lists (k_bucket_seg_q<F, 2 | 3>): ragged parts, lengths at and just
    above the threshold, a giant bucket that spans both parts, three parts,
    the fixed-base MSM, and
    the one-copy schedule (pm_ctx_set_msm_option MSM_OPT_SPLIT_COPY = 0) all
    equal the device-input MSM."""
    import torch

    n = (1 << 19) + 8195
    s, b = _torch_inputs(gpu_ctx, curve, n)
    S = s.cpu().numpy().view(np.uint64).copy()
    rb = gpu_ctx.upload_bases(curve, d_bases=b.data_ptr(), n=n)
    try:
        assert rb.rows > 1
        for m in (n, (1 << 19) + 17, n - 8192):   # > n / 2: the row-table path
            want = gpu_ctx.msm_resident_device(rb, 0, s.data_ptr(), m)
            assert np.array_equal(gpu_ctx.msm_resident(rb, 0, S[:m]), want), m
            gpu_ctx.set_msm_option(H.MSM_OPT_SPLIT_COPY, 0)
            try:
                assert np.array_equal(gpu_ctx.msm_resident(rb, 0, S[:m]), want), m
            finally:
                gpu_ctx.set_msm_option(H.MSM_OPT_SPLIT_COPY, -1)
        # canonical scalars (PM_SCALARS_CANONICAL) through both parts
        want = gpu_ctx.msm_resident_device(rb, 0, s.data_ptr(), n, canonical=True)
        assert np.array_equal(gpu_ctx.msm_resident(rb, 0, S, canonical=True), want)
        # every scalar equal: one giant bucket per window, in both parts' lists
        e = s[7:8].repeat(n, 1).contiguous()
        torch.cuda.synchronize()
        want = gpu_ctx.msm_resident_device(rb, 0, e.data_ptr(), n)
        assert np.array_equal(gpu_ctx.msm_resident(rb, 0, e.cpu().numpy().view(np.uint64).copy()), want)
    finally:
        rb.release()
    # at the threshold: a fresh table of exactly PM_SPLIT_COPY_MIN_N (+ 1) points
    for m in (H.SPLIT_COPY_MIN_N, H.SPLIT_COPY_MIN_N + 1):
        rb = gpu_ctx.upload_bases(curve, d_bases=b.data_ptr(), n=m)
        try:
            assert rb.rows > 1
            want = gpu_ctx.msm_resident_device(rb, 0, s.data_ptr(), m)
            assert np.array_equal(gpu_ctx.msm_resident(rb, 0, S[:m]), want), m
        finally:
            rb.release()
    # three parts from 2^21 points (ragged last part); and the fixed-base
    # table past 2^21 points (c = 20, 13 merged windows: 8-B sort entries)
    m = (1 << 21) + 77
    s3, b3 = _torch_inputs(gpu_ctx, curve, m)
    S3 = s3.cpu().numpy().view(np.uint64).copy()
    rb = gpu_ctx.upload_bases(curve, d_bases=b3.data_ptr(), n=m)
    try:
        want = gpu_ctx.msm_resident_device(rb, 0, s3.data_ptr(), m)
        assert np.array_equal(gpu_ctx.msm_resident(rb, 0, S3), want)
    finally:
        rb.release()
    fb = gpu_ctx.fixed_bases(curve, d_bases=b3.data_ptr(), n=m)
    try:
        assert fb.c == 20
        assert np.array_equal(fb.msm(S3), want)
    finally:
        fb.release()
    del s3, b3
    # the fixed-base MSM (one merged bucket set) with host scalars
    m = (1 << 18) + 5
    fb = gpu_ctx.fixed_bases(curve, d_bases=b.data_ptr(), n=m)
    try:
        assert np.array_equal(fb.msm(S[:m]), gpu_ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), m))
    finally:
        fb.release()


def test_msm_option_arguments(gpu_ctx):
    """pm_ctx_set_msm_option: -1 and 0 accepted, anything else refused."""
    for v in (0, -1):
        gpu_ctx.set_msm_option(H.MSM_OPT_SPLIT_COPY, v)
    for opt, v in ((H.MSM_OPT_SPLIT_COPY, 1), (H.MSM_OPT_SPLIT_COPY, -2), (99, 0)):
        with pytest.raises(H.PmError):
            gpu_ctx.set_msm_option(opt, v)


@pytest.mark.parametrize("logn,rows", [(20, 8), (22, 4)])
def test_headline_path_vs_c_port(gpu_ctx, logn, rows):
    """The bench's exact headline path with default knobs: Pallas 2^20
    (2^22) synthetic pairs, bases uploaded once with pm_bases_upload_device
    (the 8-row (4-row) resident table), scalars resident, pm_msm_resident_device
    -- against the C restatement of halo2 best_multiexp (oracle/msm_ref.c).
    At 2^20 the same call also runs through pm_msm with the drop-in cache
    warm (host scalars + host bases), the literal Rust-shim call."""
    n = 1 << logn
    s, b = _torch_inputs(gpu_ctx, 0, n)
    S = s.cpu().numpy().view(np.uint64).copy()
    B = b.cpu().numpy().view(np.uint64).copy()
    want = msm_ref.best_multiexp(0, S, B)
    rb = gpu_ctx.upload_bases(0, d_bases=b.data_ptr(), n=n)
    try:
        assert rb.rows == rows
        for _ in range(2):
            assert np.array_equal(gpu_ctx.msm_resident_device(rb, 0, s.data_ptr(), n), want)
    finally:
        rb.release()
    if logn == 20:
        ctx = H.Context(0)
        try:
            for _ in range(3):
                assert np.array_equal(ctx.msm(0, S, B), want)
            assert ctx.dropin_stats()["hits"] == 1
        finally:
            ctx.close()


@pytest.mark.parametrize("threads", [1, 3])
def test_split_host_tail_pool_sizes(threads):
    """The host tail split by bucket set (>= 8 sets: the variable-base MSM's
    16 windows) with a pool smaller than the set count: 1 thread computes
    every set inline in the chain, 3 threads leave the caller several sets.
    Run in a child process (the pool size is read from OMP_NUM_THREADS when a
    context first uses it) against the C port."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys, numpy as np\n"
        f"sys.path[:0] = [{os.path.join(root, 'halo2-aggregation_amd')!r}, {os.path.join(root, 'oracle')!r}]\n"
        "import halo2_amd as H, msm_ref, pasta as P\n"
        "n = (1 << 16) + 5\n"
        "S = msm_ref.synth_scalars(1, P.SEED_SCALARS ^ 0x77, 0, n, threads=4)\n"
        "B = msm_ref.synth_bases(1, P.SEED_BASES ^ 0x77, 0, n, threads=4)\n"
        "ctx = H.Context(0)\n"
        "got = ctx.msm(1, S, B)\n"
        "assert np.array_equal(got, msm_ref.best_multiexp(1, S, B, threads=4))\n"
        "ctx.set_window(5)\n"
        "assert np.array_equal(ctx.msm(1, S[:3000], B[:3000]), msm_ref.best_multiexp(1, S[:3000], B[:3000], threads=4))\n"
        "ctx.close()\n"
        "print('ok')\n")
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]
