"""CPU tests of the Blake2b transcript oracle (oracle/transcript.py) and of
the library's host-side BLAKE2b (pm_vk_transcript_repr shares
blake2b_compress with the device kernel), plus the committed golden vectors."""
import hashlib
import json
import os

import numpy as np
import pytest

import accum as A
import accum_util as U
import halo2_amd as H
import pasta as P
import transcript as T

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_blake2b_rfc7693_vector():
    # RFC 7693 Appendix A: BLAKE2b-512("abc")
    want = ("ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
            "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923")
    assert hashlib.blake2b(b"abc").hexdigest() == want


@pytest.mark.parametrize("cid", [0, 1, 2])
@pytest.mark.parametrize("n", [0, 1, 55, 119, 120, 127, 128, 129, 255, 256, 1000])
def test_host_vk_repr_matches_oracle(cid, n):
    """Crosses block boundaries: the 8-byte length prefix makes 120 bytes of
    payload exactly one full block (buffered until finalisation)."""
    C = P.CURVES[cid]
    rng = np.random.default_rng(n + 100 * cid)
    pinned = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    got = H.vk_transcript_repr(cid, pinned)
    want = T.vk_repr(C.r, pinned)
    assert P.from_limbs([int(x) for x in got]) == want * P.R_MONT % C.r


def test_vk_repr_rejects_bad_curve():
    with pytest.raises(H.PmError):
        H.vk_transcript_repr(7, b"x")


def test_replay_is_order_sensitive():
    C, sh, proofs = U.make_case(0, "simple", 10, 2, 0xAB)
    ch0, _ = T.replay_challenges(C, sh, proofs[0], 5)
    assert len(set(ch0)) == 7 and all(0 <= c < C.r for c in ch0)
    assert T.replay_challenges(C, sh, proofs[0], 5)[0] == ch0
    assert T.replay_challenges(C, sh, proofs[0], 6)[0][0] != ch0[0]
    # W_j are absorbed after the last squeeze: changing them changes nothing
    pf = proofs[0]
    k, n = sh.point_offsets()["W"]
    pf2 = A.Proof(points=pf.points[:k] + [proofs[1].points[k]] * n, scalars=pf.scalars, challenges=None)
    assert T.replay_challenges(C, sh, pf2, 5)[0] == ch0
    # the last scalar feeds v and u only
    pf3 = A.Proof(points=pf.points, scalars=pf.scalars[:-1] + [pf.scalars[-1] + 1], challenges=None)
    ch3 = T.replay_challenges(C, sh, pf3, 5)[0]
    assert ch3[:5] == ch0[:5] and ch3[5] != ch0[5]


def test_identity_point_is_skipped():
    """An identity commitment is not hashed (transcript.rs:101-110): theta
    equals the theta of the same stream with that point left out."""
    C, sh, proofs = U.make_case(1, "simple", 10, 1, 0xAC)
    pf = proofs[0]
    k, n_adv = sh.point_offsets()["adv"]
    pts = list(pf.points)
    pts[k] = None
    ch, skipped = T.replay_challenges(C, sh, A.Proof(points=pts, scalars=pf.scalars, challenges=None), 9)
    assert skipped
    t = T.Blake2bTranscript(C.r)
    t.common_scalar(9)
    for q in pts[:k] + pts[k + 1:k + n_adv]:   # instance + remaining advice commitments
        t.common_point(q)
    assert ch[0] == t.squeeze_challenge()


def test_golden_transcript_vectors_match_oracle():
    npz = np.load(os.path.join(GOLD, "transcript_vectors.npz"), allow_pickle=False)
    idx = json.load(open(os.path.join(GOLD, "transcript_vectors.json")))
    for name, meta in idx.items():
        C = P.CURVES[meta["curve"]]
        sh = A.synth_vk_points(C, U.SHAPES[meta["shape"]](C, meta["log_n"]), seed=meta["seed"] ^ 0x7EC)
        pts, scs = npz[f"{name}.points"], npz[f"{name}.scalars"]
        vkr = P.from_limbs([int(x) for x in npz[f"{name}.vk_repr"]]) * pow(P.R_MONT, -1, C.r) % C.r
        for b in range(pts.shape[0]):
            pf = A.Proof(points=[P.limbs_to_point(C, [int(x) for x in row]) for row in pts[b]],
                         scalars=[P.from_limbs([int(x) for x in row]) * pow(P.R_MONT, -1, C.r) % C.r
                                  for row in scs[b]], challenges=None)
            ch, skipped = T.replay_challenges(C, sh, pf, vkr)
            want = np.array([A.to_limbs_mont(C.r, c) for c in ch], dtype=np.uint64)
            assert np.array_equal(npz[f"{name}.challenges"][b], want), (name, b)
            assert int(npz[f"{name}.status"][b]) == int(skipped), (name, b)
