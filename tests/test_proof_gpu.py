"""GPU parity tests of the proof-byte boundary (pm_decode_proofs*,
pm_accum_batch_proofs*): the device's read_point / read_scalar (point
decompression by square root, canonical checks) against the oracle
(oracle/proof_bytes.py), bit for bit, on valid proofs of both shapes on all
three curves and on proofs with every kind of invalid encoding; then the fused
decode + transcript replay + accumulator against the oracle's accumulator."""
import random

import numpy as np
import pytest

import accum as A
import accum_util as U
import halo2_amd as H
import pasta as P
import proof_bytes as PB
import transcript as T

pytestmark = pytest.mark.gpu


def _pack(C, sh, rows):
    """oracle parse results [(points, scalars, status)] -> packed arrays"""
    proofs = [A.Proof(points=p, scalars=s, challenges=[0] * 7) for p, s, _ in rows]
    pts, scs, _ = A.pack_proofs(C, sh, proofs)
    return pts, scs, np.array([st for _, _, st in rows], dtype=np.uint32)


def _non_residue_x(C, rng):
    while True:
        x = rng.randrange(1, C.p)
        if PB.sqrt_mod(x ** 3 + C.b, C.p) is None:
            return x


def _corrupt(C, sh, data, rng, kind):
    """One invalid (or edge) encoding at a random item of the right kind."""
    data = bytearray(data)
    items = PB.proof_items(sh)
    pts = [j for j, (k, _) in enumerate(items) if k == "pt"]
    scs = [j for j, (k, _) in enumerate(items) if k == "sc"]
    if kind == "x_ge_p":
        j = rng.choice(pts)
        data[32 * j:32 * j + 32] = (C.p + rng.randrange(0, 1000)).to_bytes(32, "little")
    elif kind == "x_ge_p_signed":
        j = rng.choice(pts)
        data[32 * j:32 * j + 32] = (C.p | (1 << 255)).to_bytes(32, "little")
    elif kind == "non_residue":
        j = rng.choice(pts)
        x = _non_residue_x(C, rng) | (rng.randrange(2) << 255)
        data[32 * j:32 * j + 32] = x.to_bytes(32, "little")
    elif kind == "identity":
        j = rng.choice(pts)
        data[32 * j:32 * j + 32] = bytes(32)
    elif kind == "flip_sign":       # valid: the negated point
        j = rng.choice(pts)
        data[32 * j + 31] ^= 0x80
    elif kind == "zero_x_signed":   # x = 0 with the sign bit: (0, sqrt(b)) or invalid
        j = rng.choice(pts)
        data[32 * j:32 * j + 32] = (1 << 255).to_bytes(32, "little")
    elif kind == "scalar_ge_r":
        j = rng.choice(scs)
        data[32 * j:32 * j + 32] = (C.r + rng.randrange(0, 1 << 40)).to_bytes(32, "little")
    elif kind == "scalar_max":
        j = rng.choice(scs)
        data[32 * j:32 * j + 32] = b"\xff" * 32
    elif kind == "scalar_r_minus_1":  # valid
        j = rng.choice(scs)
        data[32 * j:32 * j + 32] = (C.r - 1).to_bytes(32, "little")
    return bytes(data)


KINDS = ["x_ge_p", "x_ge_p_signed", "non_residue", "identity", "flip_sign", "zero_x_signed", "scalar_ge_r",
         "scalar_max", "scalar_r_minus_1"]


@pytest.mark.parametrize("cid", [0, 1, 2])
@pytest.mark.parametrize("shape", ["simple", "rich"])
def test_decode_vs_oracle(gpu_ctx, cid, shape):
    """B = 37 proofs (ragged 64-lane blocks): the first 27 untouched, the
    other 10 each with one encoding of every kind above; decoded points,
    scalars and status words equal the oracle's."""
    C, sh, proofs = U.make_case(cid, shape, 10, 37, 0xDEC0 + cid)
    ps = U.to_product_shape(cid, sh)
    rng = random.Random(0xC0 + cid)
    ni = sh.num_instance_columns
    datas = [PB.serialize(C, sh, pf) for pf in proofs]
    for b in range(27, 37):
        datas[b] = _corrupt(C, sh, datas[b], rng, KINDS[(b - 27) % len(KINDS)])
    inst = np.array([[P.point_to_limbs(C, q) for q in pf.points[:ni]] for pf in proofs], dtype=np.uint64)
    pts, scs, st = gpu_ctx.decode_proofs(ps, datas, inst)
    want = _pack(C, sh, [PB.parse(C, sh, d, pf.points[:ni]) for d, pf in zip(datas, proofs)])
    assert np.array_equal(st, want[2])
    assert not st[:27].any()
    assert np.array_equal(pts, want[0])
    assert np.array_equal(scs, want[1])
    # the valid proofs decode to the proofs themselves
    p0, s0, _ = A.pack_proofs(C, sh, proofs[:27])
    assert np.array_equal(pts[:27], p0) and np.array_equal(scs[:27], s0)


@pytest.mark.parametrize("cid,mode", [(0, -1), (1, -1), (2, -1), (2, 0), (2, 1)])
def test_decode_many_points(gpu_ctx, cid, mode):
    """Decompression of 2000 random curve points and their negations (random
    square roots in both Tonelli-Shanks windows / the (p+1)/4 power), plus
    random x (about half non-residues): every output against the oracle.
    BN254 also with each square-root form forced (mode 0: one lane per point;
    1: one row-sliced row per point, k_proof_decode<Cv, true>)."""
    if mode >= 0:
        gpu_ctx = H.Context(0)
        gpu_ctx.set_accum_ladder(mode)
    C = P.CURVES[cid]
    rng = random.Random(0x5027 + cid)
    sh = A.synth_vk_points(C, U.SHAPES["simple"](C, 10), seed=0x11)
    ps = U.to_product_shape(cid, sh)
    items = PB.proof_items(sh)
    slots = [j for j, (k, _) in enumerate(items) if k == "pt"]
    ni = sh.num_instance_columns
    B = 2000 // len(slots) + 1
    base = PB.serialize(C, sh, A.synth_proof(C, sh, 0x11, 0))
    datas = []
    for b in range(B):
        d = bytearray(base)
        for j in slots:
            if rng.random() < 0.5:
                pt = C.mul(rng.randrange(1, C.r), C.gen)
                enc = PB.encode_point(C, pt if rng.random() < 0.5 else C.neg(pt))
            else:
                enc = (rng.randrange(C.p) | (rng.randrange(2) << 255)).to_bytes(32, "little")
            d[32 * j:32 * j + 32] = enc
        datas.append(bytes(d))
    inst = np.zeros((B, ni, 8), dtype=np.uint64)
    pts, scs, st = gpu_ctx.decode_proofs(ps, datas, inst)
    rows = [PB.parse(C, sh, d, [None] * ni) for d in datas]
    want = _pack(C, sh, rows)
    assert np.array_equal(st, want[2])
    assert np.array_equal(pts, want[0])


@pytest.mark.parametrize("cid,shape", [(2, "simple"), (0, "rich"), (1, "simple")])
def test_accum_from_bytes(gpu_ctx, cid, shape):
    """pm_accum_batch_proofs == pm_accum_batch_transcript on the decoded
    inputs == the oracle accumulator on the transcript's challenges; a proof
    with a bad encoding only flags itself."""
    C, sh, proofs = U.make_case(cid, shape, 14, 9, 0xAB0 + cid)
    ps = U.to_product_shape(cid, sh)
    ni = sh.num_instance_columns
    vkr = T.vk_repr(C.r, b"pinned-bytes")
    vk = np.array(A.to_limbs_mont(C.r, vkr), dtype=np.uint64)
    datas = [PB.serialize(C, sh, pf) for pf in proofs]
    rng = random.Random(0xAB)
    datas[4] = _corrupt(C, sh, datas[4], rng, "non_residue")
    datas[7] = _corrupt(C, sh, datas[7], rng, "scalar_ge_r")
    inst = np.array([[P.point_to_limbs(C, q) for q in pf.points[:ni]] for pf in proofs], dtype=np.uint64)
    quads, h, ch, st = gpu_ctx.accum_batch_proofs(ps, datas, inst, vk)
    assert st[4] & H.PROOF_BAD_POINT and st[7] & H.PROOF_BAD_SCALAR
    good = [b for b in range(9) if b not in (4, 7)]
    assert not st[good].any()
    pts, scs, _ = A.pack_proofs(C, sh, proofs)
    q2, h2, ch2, st2 = gpu_ctx.accum_batch_transcript(ps, pts, scs, vk)
    assert np.array_equal(quads[good], q2[good]) and np.array_equal(h[good], h2[good])
    assert np.array_equal(ch[good], ch2[good])
    T.with_replayed_challenges(C, sh, proofs, vkr)
    for b in (0, 8):
        q, hh = A.pack_result(C, A.accumulate_msm(C, sh, proofs[b]))
        assert np.array_equal(quads[b], q) and np.array_equal(h[b], hh), b


def test_device_entries_and_stride(gpu_ctx):
    """The device variants, proofs at a padded stride (psize + 96 bytes),
    equal the host entries."""
    import torch

    cid = 2
    C, sh, proofs = U.make_case(cid, "simple", 12, 21, 0xD5)
    ps = U.to_product_shape(cid, sh)
    ni = sh.num_instance_columns
    npts, nsc, _ = ps.layout()
    psize = H.proof_size(ps)
    stride = psize + 96
    buf = np.zeros((21, stride), dtype=np.uint8)
    for b, pf in enumerate(proofs):
        buf[b, :psize] = np.frombuffer(PB.serialize(C, sh, pf), dtype=np.uint8)
        buf[b, psize:] = 0xEE   # trailing bytes are never read
    inst = np.array([[P.point_to_limbs(C, q) for q in pf.points[:ni]] for pf in proofs], dtype=np.uint64)
    vk = np.array(A.to_limbs_mont(C.r, T.vk_repr(C.r, b"dev")), dtype=np.uint64)
    hp, hs, hst = gpu_ctx.decode_proofs(ps, buf, inst)
    hq, hh, hc, hst2 = gpu_ctx.accum_batch_proofs(ps, buf, inst, vk)
    dev = torch.device("cuda", gpu_ctx.device)
    dpf = torch.from_numpy(buf).to(dev)
    din = torch.from_numpy(inst.view(np.int64)).to(dev)
    dp = torch.zeros((21, npts, 8), dtype=torch.int64, device=dev)
    ds = torch.zeros((21, nsc, 4), dtype=torch.int64, device=dev)
    dst = torch.full((21,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    gpu_ctx.decode_proofs_device(ps, 21, dpf.data_ptr(), stride, din.data_ptr(), dp.data_ptr(), ds.data_ptr(),
                                 dst.data_ptr())
    assert np.array_equal(dp.cpu().numpy().view(np.uint64), hp)
    assert np.array_equal(ds.cpu().numpy().view(np.uint64), hs)
    assert not dst.cpu().numpy().any() and not hst.any()
    dc = torch.zeros((21, 7, 4), dtype=torch.int64, device=dev)
    dq = torch.zeros((21, 4, 8), dtype=torch.int64, device=dev)
    dh = torch.zeros((21, 4), dtype=torch.int64, device=dev)
    gpu_ctx.accum_batch_proofs_device(ps, 21, vk, dpf.data_ptr(), stride, din.data_ptr(), dc.data_ptr(),
                                      dq.data_ptr(), dh.data_ptr(), dst.data_ptr())
    assert np.array_equal(dq.cpu().numpy().view(np.uint64), hq)
    assert np.array_equal(dh.cpu().numpy().view(np.uint64), hh)
    assert np.array_equal(dc.cpu().numpy().view(np.uint64), hc)
    assert not hst2.any() and not dst.cpu().numpy().any()
    with pytest.raises(H.PmError):   # stride below the proof size
        gpu_ctx.decode_proofs_device(ps, 21, dpf.data_ptr(), psize - 4, din.data_ptr(), dp.data_ptr(),
                                     ds.data_ptr(), dst.data_ptr())


def test_alternating_shapes_one_context():
    """on one untimed context, batches from proof bytes that
    alternate between two shapes and two VKs re-send the program / constants /
    VK words behind the decode; each result must still equal the fused
    transcript entry on the decoded inputs, computed on a second context (a
    stale read would see the previous shape's program words)."""
    ctx = H.Context(0)
    cases = []
    for i, (cid, shape) in enumerate([(2, "simple"), (2, "rich"), (0, "simple"), (2, "simple")]):
        C, sh, proofs = U.make_case(cid, shape, 11 + i, 12, 0xA17 + 31 * i)
        ps = U.to_product_shape(cid, sh)
        ni = sh.num_instance_columns
        vk = np.array(A.to_limbs_mont(C.r, T.vk_repr(C.r, b"alt-%d" % i)), dtype=np.uint64)
        datas = [PB.serialize(C, sh, pf) for pf in proofs]
        inst = np.array([[P.point_to_limbs(C, q) for q in pf.points[:ni]] for pf in proofs], dtype=np.uint64)
        pts, scs, _ = A.pack_proofs(C, sh, proofs)
        cases.append((ps, datas, inst, vk, pts, scs))
    want = []
    ref = H.Context(0)
    for ps, datas, inst, vk, pts, scs in cases:
        want.append(ref.accum_batch_transcript(ps, pts, scs, vk))
    for rep in range(3):
        for (ps, datas, inst, vk, _, _), w in zip(cases, want):
            q, h, ch, st = ctx.accum_batch_proofs(ps, datas, inst, vk)
            assert not st.any()
            assert np.array_equal(q, w[0]) and np.array_equal(h, w[1]) and np.array_equal(ch, w[2]), rep


def test_bn254_hand_derived_edges(gpu_ctx):
    """The hand-derived BN254 G1 encodings of tests/test_proof_bytes_oracle.py
    (generator, its negation, x = 0 with and without the sign bit, x = p - 1
    with both parities, a non-residue x, x = p) through the device decoder:
    each in the first point slot of its own proof."""
    from test_proof_bytes_oracle import BN254_EDGE, bn254_edge_bytes

    cid = 2
    C, sh, proofs = U.make_case(cid, "simple", 10, len(BN254_EDGE), 0xED6E)
    ps = U.to_product_shape(cid, sh)
    items = PB.proof_items(sh)
    j = next(k for k, (kind, _) in enumerate(items) if kind == "pt")
    slot = items[j][1]
    ni = sh.num_instance_columns
    datas = []
    for pf, ((x, sign), _) in zip(proofs, BN254_EDGE):
        d = bytearray(PB.serialize(C, sh, pf))
        d[32 * j:32 * j + 32] = bn254_edge_bytes(x, sign)
        datas.append(bytes(d))
    inst = np.array([[P.point_to_limbs(C, q) for q in pf.points[:ni]] for pf in proofs], dtype=np.uint64)
    pts, _, st = gpu_ctx.decode_proofs(ps, datas, inst)
    for b, (_, want) in enumerate(BN254_EDGE):
        if want is None:
            assert st[b] & H.PROOF_BAD_POINT, b
        else:
            assert st[b] == 0, b
            assert P.limbs_to_point(C, [int(v) for v in pts[b, slot]]) == want, b


def test_large_batch_vs_c_port():
    """A 1000-proof batch from bytes (simple-example shape, BN254, k = 17: the
    one-lane term-product path above the table budget) in ONE
    pm_accum_batch_proofs_device call, against oracle/accum_ref.c on the same
    bytes (decode + Blake2b replay + accumulator): every challenge, quad and
    h_eval; and its first 256 proofs as a batch of their own give the same
    quads (no cross-proof state)."""
    import torch

    import accum_ref
    import workloads as Wk

    ctx = H.Context(0)
    B = 1000
    shape = Wk.simple_example_shape(ctx, H.BN254, 17)
    batch = Wk.SyntheticBatch(ctx, shape, B, seed=0xB16)
    batch.to_proof_bytes(shape)
    batch.run_bytes(ctx, shape)
    torch.cuda.synchronize()
    proofs = batch.proofs.cpu().numpy()
    inst = batch.inst.cpu().numpy().view(np.uint64)
    o = accum_ref.batch_proofs(H.BN254, shape.c, proofs, inst, vk_repr=np.asarray(batch.vk_repr, dtype=np.uint64),
                               threads=8)
    ch = batch.challenges.cpu().numpy().view(np.uint64)
    quads = batch.quads.cpu().numpy().view(np.uint64)
    hev = batch.h_eval.cpu().numpy().view(np.uint64)
    assert not o["status"].any() and not batch.status.cpu().numpy().any()
    assert np.array_equal(o["challenges"].reshape(ch.shape), ch)
    assert np.array_equal(o["quads"].reshape(quads.shape), quads)
    assert np.array_equal(o["h_eval"].reshape(hev.shape), hev)
    sub = 256
    dev = batch.proofs.device
    q = torch.empty((sub, 4, 8), dtype=torch.int64, device=dev)
    h = torch.empty((sub, 4), dtype=torch.int64, device=dev)
    c = torch.empty((sub, 7, 4), dtype=torch.int64, device=dev)
    st = torch.empty((sub,), dtype=torch.int32, device=dev)
    ctx.accum_batch_proofs_device(shape, sub, batch.vk_repr, batch.proofs.data_ptr(), batch.psize,
                                  batch.inst.data_ptr(), c.data_ptr(), q.data_ptr(), h.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(q, batch.quads[:sub]) and torch.equal(h, batch.h_eval[:sub])


@pytest.mark.parametrize("B,logn", [(16, 14), (200, 17)])
def test_schedule_options_vs_c_port(B, logn):
    """Config 3 (16 simple-example proofs at k = 14) and a B = 200 batch at
    k = 17 through the proof-bytes entry the bench times, against
    oracle/accum_ref.c on the same bytes; then the same batch under every
    accumulator schedule option (pm_ctx_set_accum_option: twisted ladder off
    and forced,
    term additions on the main stream, per-record transcript, one / two terms
    per lane with the one-lane form, both ladder forms), each bit-identical
    (no env-gated path left untested)."""
    import torch

    import accum_ref
    import workloads as Wk

    ctx = H.Context(0)
    shape = Wk.simple_example_shape(ctx, H.BN254, logn)
    batch = Wk.SyntheticBatch(ctx, shape, B, seed=0xC3 + B)
    batch.to_proof_bytes(shape)
    batch.run_bytes(ctx, shape)
    torch.cuda.synchronize()
    o = accum_ref.batch_proofs(H.BN254, shape.c, batch.proofs.cpu().numpy(), batch.inst.cpu().numpy().view(np.uint64),
                               vk_repr=np.asarray(batch.vk_repr, dtype=np.uint64), threads=8)
    want_q, want_h = batch.quads.clone(), batch.h_eval.clone()
    assert not o["status"].any() and not batch.status.cpu().numpy().any()
    assert np.array_equal(o["challenges"].reshape(B, 7, 4), batch.challenges.cpu().numpy().view(np.uint64))
    assert np.array_equal(o["quads"].reshape(B, 4, 8), want_q.cpu().numpy().view(np.uint64))
    assert np.array_equal(o["h_eval"].reshape(B, 4), want_h.cpu().numpy().view(np.uint64))
    settings = [
        [(H.ACC_OPT_TWIST, 0)],
        [(H.ACC_OPT_TWIST, 1)],
        [(H.ACC_OPT_TWIST, 2)],
        [(H.ACC_OPT_TAIL_STREAM, 0)],
        [(H.ACC_OPT_TWIST, 0), (H.ACC_OPT_TAIL_STREAM, 0)],
        [(H.ACC_OPT_TRANSCRIPT, 0)],
        [("ladder", 0)],
        [("ladder", 1)],
        [("split", 0), (H.ACC_OPT_TERMS_PER_LANE, 1)],
        [("split", 0), (H.ACC_OPT_TERMS_PER_LANE, 2)],
    ]
    for opts in settings:
        c2 = H.Context(0)
        for k, v in opts:
            if k == "ladder":
                c2.set_accum_ladder(v)
            elif k == "split":
                c2.set_accum_split(v)
            else:
                c2.set_accum_option(k, v)
        batch.quads.zero_()
        batch.h_eval.zero_()
        batch.run_bytes(c2, shape)
        torch.cuda.synchronize()
        assert not batch.status.cpu().numpy().any(), opts
        assert torch.equal(batch.quads, want_q) and torch.equal(batch.h_eval, want_h), opts
        c2.close()


def test_accum_option_arguments(gpu_ctx):
    """Unknown options and out-of-range values are refused (PM_ERR_ARG)."""
    for opt, val in [(0, 0), (99, -1), (H.ACC_OPT_TWIST, 3), (H.ACC_OPT_TAIL_STREAM, 1), (H.ACC_OPT_TERMS_PER_LANE, 0),
                     (H.ACC_OPT_TERMS_PER_LANE, 3), (H.ACC_OPT_TRANSCRIPT, -2)]:
        with pytest.raises(H.PmError):
            gpu_ctx.set_accum_option(opt, val)
    for opt in (H.ACC_OPT_TWIST, H.ACC_OPT_TAIL_STREAM, H.ACC_OPT_TERMS_PER_LANE, H.ACC_OPT_TRANSCRIPT):
        gpu_ctx.set_accum_option(opt, -1)
