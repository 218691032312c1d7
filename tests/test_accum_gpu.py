"""GPU parity tests of the batch multiopen accumulator (pm_accum_batch*)
against the oracle (oracle/accum.py): committed golden vectors, fresh random
proofs on every curve and both shapes, the device-pointer entry, and errors."""
import json
import os

import numpy as np
import pytest

import accum as A
import accum_util as U
import halo2_amd as H
import pasta as P

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden():
    npz = np.load(os.path.join(GOLD, "accum_vectors.npz"), allow_pickle=False)
    idx = json.load(open(os.path.join(GOLD, "accum_vectors.json")))
    return npz, idx


def test_golden_accumulator(gpu_ctx):
    npz, idx = _golden()
    for name, meta in idx.items():
        C = P.CURVES[meta["curve"]]
        sh = A.synth_vk_points(C, U.SHAPES[meta["shape"]](C, meta["log_n"]), seed=meta["seed"] ^ 0x7EC)
        ps = U.to_product_shape(meta["curve"], sh)
        quads, h = gpu_ctx.accum_batch(ps, npz[f"{name}.points"], npz[f"{name}.scalars"], npz[f"{name}.challenges"])
        assert np.array_equal(h, npz[f"{name}.h_eval"]), name
        assert np.array_equal(quads, npz[f"{name}.quads"]), name


@pytest.mark.parametrize("lg", [0, 1, 2, 3, 4, 5])
def test_split_ladder_widths(gpu_ctx, lg):
    """Every split of the term multiplication (2^lg lanes per term,
    k_acc_powers + k_acc_termadd; lg = 0 is the one-lane GLV kernel)
    reproduces the golden vectors, including the identity / W_1 = -W_0 edge
    case, and random rich-shape proofs on Pallas."""
    gpu_ctx.set_accum_split(lg)
    try:
        test_golden_accumulator(gpu_ctx)
        C, sh, proofs = U.make_case(0, "rich", 12, 3, 0x5917 + lg)
        ps = U.to_product_shape(0, sh)
        pts, scs, chs = A.pack_proofs(C, sh, proofs)
        quads, h = gpu_ctx.accum_batch(ps, pts, scs, chs)
        for b, pf in enumerate(proofs):
            q, hh = A.pack_result(C, A.accumulate_msm(C, sh, pf))
            assert np.array_equal(h[b], hh) and np.array_equal(quads[b], q), b
    finally:
        gpu_ctx.set_accum_split(-1)


@pytest.mark.parametrize("tpl", ["1", "2"])
def test_one_lane_windows_terms_per_lane(gpu_ctx, tpl):
    """The one-lane form's GLV products by signed 3-bit windows with one term
    per lane and with two terms of one output per lane (shared doublings, the
    pair's sum at its first row and the identity at its second; chosen
    automatically for large batches, forced here with
    PM_ACC_OPT_TERMS_PER_LANE) reproduce the golden vectors and random
    rich-shape proofs on Pallas and BN254."""
    gpu_ctx.set_accum_split(0)
    gpu_ctx.set_accum_option(H.ACC_OPT_TERMS_PER_LANE, int(tpl))
    try:
        test_golden_accumulator(gpu_ctx)
        for cid in (0, 2):
            C, sh, proofs = U.make_case(cid, "rich", 12, 5, 0x7B1 + cid)
            ps = U.to_product_shape(cid, sh)
            pts, scs, chs = A.pack_proofs(C, sh, proofs)
            quads, h = gpu_ctx.accum_batch(ps, pts, scs, chs)
            for b, pf in enumerate(proofs):
                q, hh = A.pack_result(C, A.accumulate_msm(C, sh, pf))
                assert np.array_equal(h[b], hh) and np.array_equal(quads[b], q), (cid, b)
    finally:
        gpu_ctx.set_accum_option(H.ACC_OPT_TERMS_PER_LANE, -1)
        gpu_ctx.set_accum_split(-1)


@pytest.mark.parametrize("mode", [0, 1])
def test_ladder_modes(gpu_ctx, mode):
    """Both forms of the powers-of-two table chains (0: a quad of lanes per
    chain, k_acc_powers; 1: a row-sliced wave per chain, k_acc_powers_s)
    reproduce the golden vectors (identity and W_1 = -W_0 edge cases) and
    random proofs of both shapes on every curve; with the VK tables rebuilt
    by the mode under test (a fresh context)."""
    ctx = H.Context(0)
    ctx.set_accum_ladder(mode)
    test_golden_accumulator(ctx)
    for cid in (0, 1, 2):
        for shape in ("simple", "rich"):
            C, sh, proofs = U.make_case(cid, shape, 12, 6, 0x1ADD + 13 * cid + mode)
            ps = U.to_product_shape(cid, sh)
            pts, scs, chs = A.pack_proofs(C, sh, proofs)
            quads, h = ctx.accum_batch(ps, pts, scs, chs)
            for b in (0, 5):
                q, hh = A.pack_result(C, A.accumulate_msm(C, sh, proofs[b]))
                assert np.array_equal(h[b], hh) and np.array_equal(quads[b], q), (cid, shape, b)
    with pytest.raises(H.PmError):
        ctx.set_accum_ladder(2)


@pytest.mark.parametrize("cid", [0, 1, 2])
@pytest.mark.parametrize("shape", ["simple", "rich"])
def test_random_proofs_vs_oracle(gpu_ctx, cid, shape):
    C, sh, proofs = U.make_case(cid, shape, 13, 5, 0xD00D + 7 * cid)
    ps = U.to_product_shape(cid, sh)
    pts, scs, chs = A.pack_proofs(C, sh, proofs)
    quads, h = gpu_ctx.accum_batch(ps, pts, scs, chs)
    for b, pf in enumerate(proofs):
        q, hh = A.pack_result(C, A.accumulate_msm(C, sh, pf))
        assert np.array_equal(h[b], hh), b
        assert np.array_equal(quads[b], q), b


def test_batch_of_64_and_order_independence(gpu_ctx):
    """B = 64: each proof's result is independent of its batch position."""
    C, sh, proofs = U.make_case(2, "simple", 17, 64, 0x64)
    ps = U.to_product_shape(2, sh)
    pts, scs, chs = A.pack_proofs(C, sh, proofs)
    quads, h = gpu_ctx.accum_batch(ps, pts, scs, chs)
    perm = np.random.default_rng(1).permutation(64)
    q2, h2 = gpu_ctx.accum_batch(ps, pts[perm], scs[perm], chs[perm])
    assert np.array_equal(q2, quads[perm]) and np.array_equal(h2, h[perm])
    for b in (0, 17, 63):
        q, hh = A.pack_result(C, A.accumulate_msm(C, sh, proofs[b]))
        assert np.array_equal(quads[b], q) and np.array_equal(h[b], hh)


def test_device_pointer_entry(gpu_ctx):
    import torch

    npz, idx = _golden()
    name = "bn254_simple_k14"
    meta = idx[name]
    C = P.CURVES[meta["curve"]]
    sh = A.synth_vk_points(C, U.SHAPES[meta["shape"]](C, meta["log_n"]), seed=meta["seed"] ^ 0x7EC)
    ps = U.to_product_shape(meta["curve"], sh)
    dev = torch.device("cuda", gpu_ctx.device)
    t = {k: torch.from_numpy(npz[f"{name}.{k}"].view(np.int64)).to(dev) for k in ("points", "scalars", "challenges")}
    B = meta["B"]
    dq = torch.zeros((B, 4, 8), dtype=torch.int64, device=dev)
    dh = torch.zeros((B, 4), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    gpu_ctx.accum_batch_device(ps, B, t["points"].data_ptr(), t["scalars"].data_ptr(), t["challenges"].data_ptr(),
                               dq.data_ptr(), dh.data_ptr())
    assert np.array_equal(dq.cpu().numpy().view(np.uint64), npz[f"{name}.quads"])
    assert np.array_equal(dh.cpu().numpy().view(np.uint64), npz[f"{name}.h_eval"])


def test_empty_batch_and_bad_shape(gpu_ctx):
    C, sh, proofs = U.make_case(2, "simple", 12, 1, 9)
    ps = U.to_product_shape(2, sh)
    npts, nsc, _ = ps.layout()
    q, h = gpu_ctx.accum_batch(ps, np.zeros((0, npts, 8), np.uint64), np.zeros((0, nsc, 4), np.uint64),
                               np.zeros((0, 7, 4), np.uint64))
    assert q.shape == (0, 4, 8)
    sh.gates = [A.Advice(42)]
    with pytest.raises(H.PmError):
        bad = U.to_product_shape(2, sh)
        gpu_ctx.accum_batch(bad, np.zeros((1, npts, 8), np.uint64), np.zeros((1, nsc, 4), np.uint64),
                            np.zeros((1, 7, 4), np.uint64))


@pytest.mark.parametrize("cid", [2, 0])
def test_zero_denominator_status(gpu_ctx, cid):
    """x an n-th root of unity (x = 1, x = omega^-3; then x^n = 1 and a
    Lagrange denominator x - omega^-i vanishes): the reference's
    main_gate.div fails there (vanishing.rs:175, verifier.rs:580), so the
    proof is flagged PM_ACCUM_DENOM_ZERO and the rest of the batch is
    untouched (bit-exact vs the oracle)."""
    C, sh, proofs = U.make_case(cid, "simple", 11, 5, 0xDE0 + cid)
    w_inv = pow(sh.omega, -1, C.r)
    proofs[1].challenges[4] = 1
    proofs[3].challenges[4] = pow(w_inv, 3, C.r)
    ps = U.to_product_shape(cid, sh)
    pts, scs, chs = A.pack_proofs(C, sh, proofs)
    quads, h, st = gpu_ctx.accum_batch_status(ps, pts, scs, chs)
    want = [A.proof_status(C, sh, pf.challenges) for pf in proofs]
    assert want == [0, A.STATUS_DENOM_ZERO, 0, A.STATUS_DENOM_ZERO, 0]
    assert [int(x) for x in st] == want
    for b in (0, 2, 4):
        q, hh = A.pack_result(C, A.accumulate_msm(C, sh, proofs[b]))
        assert np.array_equal(quads[b], q) and np.array_equal(h[b], hh), b
    # the same through the fused transcript entry (x is then the replayed
    # challenge, so only the status OR of the clean proofs is checked)
    vk = np.array(A.to_limbs_mont(C.r, 77), dtype=np.uint64)
    _, _, _, st2 = gpu_ctx.accum_batch_transcript(ps, pts, scs, vk)
    assert not st2.any()


def test_lookup_z_identity_status(gpu_ctx):
    """An identity lookup-Z commitment: the reference aborts (lookup.rs:100
    propagates common_point's error), status = IDENTITY_SKIPPED |
    LOOKUP_Z_IDENTITY; an identity advice commitment only skips (status 1)."""
    import transcript as T

    C, sh, proofs = U.make_case(2, "rich", 10, 3, 0x12C)
    po = sh.point_offsets()
    proofs[0].points[po["lk_z"][0]] = None
    proofs[2].points[po["adv"][0]] = None
    ps = U.to_product_shape(2, sh)
    vkr = T.vk_repr(C.r, b"lkz")
    vk = np.array(A.to_limbs_mont(C.r, vkr), dtype=np.uint64)
    pts, scs, _ = A.pack_proofs(C, sh, proofs)
    _, _, ch, st = gpu_ctx.accum_batch_transcript(ps, pts, scs, vk)
    want = [T.replay_challenges(C, sh, pf, vkr)[1] for pf in proofs]
    assert want == [T.STATUS_IDENTITY_SKIPPED | T.STATUS_LOOKUP_Z_IDENTITY, 0, T.STATUS_IDENTITY_SKIPPED]
    assert [int(x) for x in st] == want
    ch2, st2 = gpu_ctx.transcript_batch(ps, pts, scs, vk)
    assert np.array_equal(ch, ch2) and np.array_equal(st, st2)


def test_accum_batch_multi(gpu_ctx):
    """pm_accum_batch_multi shards the proofs over contexts (here: several
    contexts on the one device of the box, ragged split) and equals the
    single-context calls, with caller challenges and with the replay."""
    import transcript as T

    C, sh, proofs = U.make_case(2, "simple", 12, 11, 0x3417)
    ps = U.to_product_shape(2, sh)
    pts, scs, chs = A.pack_proofs(C, sh, proofs)
    q1, h1, s1 = gpu_ctx.accum_batch_status(ps, pts, scs, chs)
    vkr = T.vk_repr(C.r, b"multi")
    vk = np.array(A.to_limbs_mont(C.r, vkr), dtype=np.uint64)
    qt, ht, cht, stt = gpu_ctx.accum_batch_transcript(ps, pts, scs, vk)
    extra = [H.Context(0) for _ in range(2)]
    try:
        for ctxs in ([gpu_ctx], [gpu_ctx] + extra, extra + [gpu_ctx, extra[0]]):
            ch, q, h, st = H.accum_batch_multi(ctxs, ps, pts, scs, challenges=chs)
            assert np.array_equal(q, q1) and np.array_equal(h, h1) and np.array_equal(st, s1)
            assert np.array_equal(ch, chs)
            ch, q, h, st = H.accum_batch_multi(ctxs, ps, pts, scs, vk_repr=vk)
            assert np.array_equal(q, qt) and np.array_equal(h, ht) and np.array_equal(ch, cht)
            assert np.array_equal(st, stt)
    finally:
        for c in extra:
            c.close()
    for b in (0, 10):
        q, hh = A.pack_result(C, A.accumulate_msm(C, sh, proofs[b]))
        assert np.array_equal(q1[b], q) and np.array_equal(h1[b], hh)


@pytest.mark.parametrize("lg", [2, 3])
def test_vk_tables_follow_the_vk(gpu_ctx, lg):
    """The per-VK powers tables (k_acc_powers' VK quads, cached in the
    context) are rebuilt whenever the verifying key's points or the curve
    change: alternate two VKs of the same shape on Pallas, then the same VK
    bytes' shape on Vesta, and back, each call against the oracle."""
    gpu_ctx.set_accum_split(lg)
    try:
        cases = [(0, 0xA1), (0, 0xB2), (0, 0xA1), (1, 0xA1), (0, 0xA1), (0, 0xA1)]
        for cid, seed in cases:
            C, sh, proofs = U.make_case(cid, "simple", 12, 3, seed)
            ps = U.to_product_shape(cid, sh)
            pts, scs, chs = A.pack_proofs(C, sh, proofs)
            quads, h = gpu_ctx.accum_batch(ps, pts, scs, chs)
            for b, pf in enumerate(proofs):
                q, hh = A.pack_result(C, A.accumulate_msm(C, sh, pf))
                assert np.array_equal(h[b], hh), (cid, seed, b)
                assert np.array_equal(quads[b], q), (cid, seed, b)
    finally:
        gpu_ctx.set_accum_split(-1)
