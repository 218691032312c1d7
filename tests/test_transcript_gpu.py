"""GPU parity tests of the batched Blake2b transcript replay
(pm_transcript_batch*, pm_accum_batch_transcript*) against the oracle
(oracle/transcript.py) and its committed golden vectors."""
import json
import os

import numpy as np
import pytest

import accum as A
import accum_util as U
import halo2_amd as H
import pasta as P
import transcript as T

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden():
    npz = np.load(os.path.join(GOLD, "transcript_vectors.npz"), allow_pickle=False)
    idx = json.load(open(os.path.join(GOLD, "transcript_vectors.json")))
    return npz, idx


def _shape(meta):
    C = P.CURVES[meta["curve"]]
    sh = A.synth_vk_points(C, U.SHAPES[meta["shape"]](C, meta["log_n"]), seed=meta["seed"] ^ 0x7EC)
    return C, sh, U.to_product_shape(meta["curve"], sh)


def test_golden_transcript(gpu_ctx):
    npz, idx = _golden()
    for name, meta in idx.items():
        _, _, ps = _shape(meta)
        ch, st = gpu_ctx.transcript_batch(ps, npz[f"{name}.points"], npz[f"{name}.scalars"],
                                          npz[f"{name}.vk_repr"])
        assert np.array_equal(ch, npz[f"{name}.challenges"]), name
        assert np.array_equal(st, npz[f"{name}.status"]), name


@pytest.mark.parametrize("cid", [0, 1, 2])
@pytest.mark.parametrize("shape", ["simple", "rich"])
def test_random_transcripts_vs_oracle(gpu_ctx, cid, shape):
    C, sh, proofs = U.make_case(cid, shape, 12, 67, 0x7C0 + cid)   # 67: five 16-proof blocks, ragged tail
    ps = U.to_product_shape(cid, sh)
    vkr = T.vk_repr(C.r, b"vk-%d-%s" % (cid, shape.encode()))
    vk = np.array(A.to_limbs_mont(C.r, vkr), dtype=np.uint64)
    pts, scs, _ = A.pack_proofs(C, sh, proofs)
    ch, st = gpu_ctx.transcript_batch(ps, pts, scs, vk)
    assert not st.any()
    for b in range(67):  # every quad slot of every block
        want, _ = T.replay_challenges(C, sh, proofs[b], vkr)
        assert np.array_equal(ch[b], np.array([A.to_limbs_mont(C.r, c) for c in want], dtype=np.uint64)), b


def test_streamed_and_record_blocks_mixed(gpu_ctx):
    """k_transcript_s: a block of 16 proofs with an identity commitment (its
    record is skipped, so the stream shifts) runs the per-record replay while
    the other blocks run the streamed chain; every proof against the oracle."""
    C, sh, proofs = U.make_case(2, "simple", 10, 40, 0x7C9)
    k, _ = sh.point_offsets()["adv"]
    proofs[20].points[k] = None                    # block 1
    ps = U.to_product_shape(2, sh)
    vkr = T.vk_repr(C.r, b"vk-mixed")
    vk = np.array(A.to_limbs_mont(C.r, vkr), dtype=np.uint64)
    pts, scs, _ = A.pack_proofs(C, sh, proofs)
    ch, st = gpu_ctx.transcript_batch(ps, pts, scs, vk)
    assert st.tolist() == [1 if b == 20 else 0 for b in range(40)]
    for b in range(40):
        want, skipped = T.replay_challenges(C, sh, proofs[b], vkr)
        assert skipped == (b == 20)
        assert np.array_equal(ch[b], np.array([A.to_limbs_mont(C.r, c) for c in want], dtype=np.uint64)), b


def test_accum_with_replayed_challenges(gpu_ctx):
    """Transcript + accumulator in one call == oracle accumulate on the
    transcript's challenges; also == pm_accum_batch fed those challenges."""
    for cid, shape in ((2, "simple"), (0, "rich")):
        C, sh, proofs = U.make_case(cid, shape, 14, 6, 0x7D0 + cid)
        ps = U.to_product_shape(cid, sh)
        vkr = T.vk_repr(C.r, b"pinned")
        vk = np.array(A.to_limbs_mont(C.r, vkr), dtype=np.uint64)
        T.with_replayed_challenges(C, sh, proofs, vkr)
        pts, scs, chs = A.pack_proofs(C, sh, proofs)
        quads, h, ch, st = gpu_ctx.accum_batch_transcript(ps, pts, scs, vk)
        assert np.array_equal(ch, chs) and not st.any()
        q2, h2 = gpu_ctx.accum_batch(ps, pts, scs, chs)
        assert np.array_equal(quads, q2) and np.array_equal(h, h2)
        for b in (0, 5):
            q, hh = A.pack_result(C, A.accumulate_msm(C, sh, proofs[b]))
            assert np.array_equal(quads[b], q) and np.array_equal(h[b], hh), (cid, b)


def test_device_entries(gpu_ctx):
    import torch

    npz, idx = _golden()
    name = "bn254_simple_k14"
    meta = idx[name]
    C, sh, ps = _shape(meta)
    dev = torch.device("cuda", gpu_ctx.device)
    B = meta["B"]
    dp = torch.from_numpy(npz[f"{name}.points"].view(np.int64)).to(dev)
    ds = torch.from_numpy(npz[f"{name}.scalars"].view(np.int64)).to(dev)
    dc = torch.zeros((B, 7, 4), dtype=torch.int64, device=dev)
    dst = torch.full((B,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    gpu_ctx.transcript_batch_device(ps, B, npz[f"{name}.vk_repr"], dp.data_ptr(), ds.data_ptr(), dc.data_ptr(),
                                    dst.data_ptr())
    assert np.array_equal(dc.cpu().numpy().view(np.uint64), npz[f"{name}.challenges"])
    assert np.array_equal(dst.cpu().numpy().view(np.uint32), npz[f"{name}.status"])
    # fused device entry: quads equal the host-buffer fused call
    dq = torch.zeros((B, 4, 8), dtype=torch.int64, device=dev)
    dh = torch.zeros((B, 4), dtype=torch.int64, device=dev)
    gpu_ctx.accum_batch_transcript_device(ps, B, npz[f"{name}.vk_repr"], dp.data_ptr(), ds.data_ptr(),
                                          dc.data_ptr(), dq.data_ptr(), dh.data_ptr())
    quads, h, _, _ = gpu_ctx.accum_batch_transcript(ps, npz[f"{name}.points"], npz[f"{name}.scalars"],
                                                    npz[f"{name}.vk_repr"])
    assert np.array_equal(dq.cpu().numpy().view(np.uint64), quads)
    assert np.array_equal(dh.cpu().numpy().view(np.uint64), h)


def test_empty_batch_and_errors(gpu_ctx):
    C, sh, _ = U.make_case(0, "simple", 10, 1, 1)
    ps = U.to_product_shape(0, sh)
    npts, nsc, _ = ps.layout()
    ch, st = gpu_ctx.transcript_batch(ps, np.zeros((0, npts, 8), np.uint64), np.zeros((0, nsc, 4), np.uint64),
                                      np.zeros(4, np.uint64))
    assert ch.shape == (0, 7, 4)
    assert H.lib().pm_transcript_batch(gpu_ctx.h, 0, None, 1, None, None, None, None, None) == -1
    vk = np.zeros(4, np.uint64)
    import ctypes
    assert H.lib().pm_transcript_batch(gpu_ctx.h, 9, ctypes.byref(ps.c), 0, vk.ctypes.data_as(H._u64p), None, None,
                                       None, None) == -1   # unknown curve


@pytest.mark.parametrize("cid", [2, 0])
def test_single_proof_k9_fused(gpu_ctx, cid):
    """The reference's only real configuration: ONE simple-example proof at
    k = 9 (examples/simple-example.rs:561,620-626) -- B = 1 through the fused
    transcript replay + accumulator, against the oracle."""
    C, sh, proofs = U.make_case(cid, "simple", 9, 1, 0x9009 + cid)
    ps = U.to_product_shape(cid, sh)
    vkr = T.vk_repr(C.r, b"simple-example k=9")
    vk = np.array(A.to_limbs_mont(C.r, vkr), dtype=np.uint64)
    T.with_replayed_challenges(C, sh, proofs, vkr)
    pts, scs, chs = A.pack_proofs(C, sh, proofs)
    quads, h, ch, st = gpu_ctx.accum_batch_transcript(ps, pts, scs, vk)
    assert np.array_equal(ch, chs) and not st.any()
    q, hh = A.pack_result(C, A.accumulate_msm(C, sh, proofs[0]))
    assert np.array_equal(quads[0], q) and np.array_equal(h[0], hh)


@pytest.mark.parametrize("cid", [0, 2])
def test_config3_sixteen_proofs_k14(gpu_ctx, cid):
    """BASELINE config 3 at its exact size: 16 simple-example proofs at k = 14
    (examples/simple-example.rs:99-159, 561) through the fused transcript
    replay + accumulator, every proof's challenges, quad and h_eval bit for
    bit against the C port (oracle/accum_ref.c), two of them also against the
    literal Python restatement."""
    import accum_ref as R

    C, sh, proofs = U.make_case(cid, "simple", 14, 16, 0xC3 + cid)
    ps = U.to_product_shape(cid, sh)
    vkr = T.vk_repr(C.r, b"simple-example")
    vk = np.array(A.to_limbs_mont(C.r, vkr), dtype=np.uint64)
    pts, scs, _ = A.pack_proofs(C, sh, proofs)
    quads, h, ch, st = gpu_ctx.accum_batch_transcript(ps, pts, scs, vk)
    assert not st.any()
    rch, rq, rh, rst = R.accum_batch(cid, ps.c, pts, scs, vk_repr=vk, threads=4)
    assert not rst.any()
    assert np.array_equal(ch, rch.reshape(ch.shape))
    assert np.array_equal(quads, rq.reshape(quads.shape))
    assert np.array_equal(h, rh.reshape(h.shape))
    T.with_replayed_challenges(C, sh, proofs, vkr)
    for b in (0, 15):
        q, hh = A.pack_result(C, A.accumulate_msm(C, sh, proofs[b]))
        assert np.array_equal(quads[b], q) and np.array_equal(h[b], hh), b
