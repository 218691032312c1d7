"""CPU tests of the multiopen-accumulator oracle (oracle/accum.py) and of the
host side of the C-ABI (shape layout / validation; no GPU calls)."""
import json
import os

import numpy as np
import pytest

import accum as A
import accum_util as U
import halo2_amd as H
import pasta as P

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_field_constants_match_published():
    """ROOT_OF_UNITY / DELTA as published by pasta_curves (Fp, Fq) and
    halo2curves / pairing_bn256 (bn256 Fr); omega of a k-domain is
    ROOT_OF_UNITY^(2^(S-k)) (halo2 EvaluationDomain::new)."""
    root, delta, s = A.two_adic(P.PALLAS_P)
    assert s == 32 and root == 0x2bce74deac30ebda362120830561f81aea322bf2b7bb7584bdad6fabd87ea32f
    root, delta, s = A.two_adic(P.VESTA_P)
    assert s == 32 and root == 0x2de6a9b8746d3f589e5c4dfd492ae26e9bb97ea3c106f049a70e2c1102b6d05f
    root, delta, s = A.two_adic(P.BN254_R)
    assert s == 28 and root == 0x03ddb9f5166d18b798865ea93dd31f743215cf6dd39329c8d34f1ed960c37c9c
    assert delta == 0x09226b6e22c6f0ca64ec26aad4c86e715b5f898e5e963f25870e56bbe533e9a2
    for r in (P.PALLAS_P, P.VESTA_P, P.BN254_R):
        w = A.domain_omega(r, 14)
        assert pow(w, 1 << 14, r) == 1 and pow(w, 1 << 13, r) != 1


@pytest.mark.parametrize("cid", [0, 1, 2])
@pytest.mark.parametrize("shape", ["simple", "rich"])
def test_two_restatements_agree(cid, shape):
    C, sh, proofs = U.make_case(cid, shape, 11, 2, 0xBEEF + cid)
    for pf in proofs:
        assert A.accumulate(C, sh, pf) == A.accumulate_msm(C, sh, pf)


def test_query_order_and_sets_simple_shape():
    """verifier.rs:705-712 order; BTreeMap set order (multiopen.rs:25-44)."""
    C, sh, proofs = U.make_case(2, "simple", 14, 1, 1)
    d = A._split(sh, proofs[0])
    q = A.build_queries(sh, d, 0)
    assert len(q) == 24  # Q ~ 24
    rots = [r for _, r, _ in q]
    # instance, advice (cur, cur, next), perm (cur, next, cur, next, last), lookup, fixed, sigma, vanishing
    assert rots[:4] == [0, 0, 0, 1]
    assert rots[4:9] == [0, 1, 0, 1, -6]
    assert rots[9:14] == [0, 0, 0, -1, 1]
    sets = A.construct_intermediate_sets(q)
    assert [r for r, _ in sets] == [-6, -1, 0, 1]
    assert q[-2][0] == A.H_POINT


@pytest.mark.parametrize("shape", ["simple", "rich"])
def test_c_layout_matches_oracle(shape):
    for cid in (0, 1, 2):
        C, sh, _ = U.make_case(cid, shape, 12, 0, 3)
        ps = U.to_product_shape(cid, sh)
        assert ps.layout() == (sh.points_per_proof(), sh.scalars_per_proof(), sh.num_sets())


def test_compile_expressions_postfix():
    consts = []
    code = H.compile_expressions([A.Prod(A.Fixed(2), A.Sum(A.Advice(0), A.Neg(A.Scaled(A.Instance(1), 9))))],
                                 consts)
    assert code == [2 | 2 << 8, 3 | 0 << 8, 4 | 1 << 8, 8 | 0 << 8, 5, 6, 7, 0]
    assert consts == [9]


def _bad(sh_kwargs_edit):
    C, sh, _ = U.make_case(2, "simple", 12, 0, 3)
    sh_kwargs_edit(sh)
    return U.to_product_shape(2, sh)


@pytest.mark.parametrize("edit,msg", [
    (lambda sh: setattr(sh, "advice_queries", sh.advice_queries + [(7, 0)]), "advice query column"),
    (lambda sh: setattr(sh, "gates", [A.Prod(A.Advice(0), A.Advice(99))]), "ADVICE query index"),
    (lambda sh: setattr(sh, "perm_columns", sh.perm_columns + [(A.KIND_FIXED, 50)]), "permutation column"),
    (lambda sh: setattr(sh, "blinding_factors", 100), "blinding_factors"),
    (lambda sh: setattr(sh, "quotient_degree", 0), "quotient_degree"),
])
def test_c_shape_validation(edit, msg):
    ps = _bad(edit)
    with pytest.raises(H.PmError, match=msg):
        ps.layout()


def test_golden_vectors_reproduce():
    """The committed fixtures equal a fresh run of the literal restatement."""
    npz = np.load(os.path.join(GOLD, "accum_vectors.npz"), allow_pickle=False)
    idx = json.load(open(os.path.join(GOLD, "accum_vectors.json")))
    for name, meta in idx.items():
        C = P.CURVES[meta["curve"]]
        sh = A.synth_vk_points(C, U.SHAPES[meta["shape"]](C, meta["log_n"]), seed=meta["seed"] ^ 0x7EC)
        assert np.array_equal(npz[f"{name}.fixed"],
                              np.array([P.point_to_limbs(C, q) for q in sh.fixed_commitments], dtype=np.uint64))
        pts, scs, chs = npz[f"{name}.points"], npz[f"{name}.scalars"], npz[f"{name}.challenges"]
        rinv = pow(P.R_MONT, -1, C.r)
        for b in range(meta["B"]):
            pf = A.Proof(points=[P.limbs_to_point(C, [int(x) for x in p]) for p in pts[b]],
                         scalars=[P.from_limbs([int(x) for x in s]) * rinv % C.r for s in scs[b]],
                         challenges=[P.from_limbs([int(x) for x in s]) * rinv % C.r for s in chs[b]])
            q, h = A.pack_result(C, A.accumulate(C, sh, pf))
            assert np.array_equal(q, npz[f"{name}.quads"][b]), (name, b)
            assert np.array_equal(h, npz[f"{name}.h_eval"][b]), (name, b)


# ------------------------------------------- C restatement (oracle/accum_ref.c)
def _c_case(cid, shape, log_n, B, seed):
    import accum_util as U

    C, sh, proofs = U.make_case(cid, shape, log_n, B, seed)
    return C, sh, proofs, U.to_product_shape(cid, sh)


def test_c_accumulator_matches_golden():
    """The C restatement reproduces every golden quad / h_eval bit for bit."""
    import json
    import os

    import numpy as np

    import accum_ref as R
    import accum_util as U

    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    npz = np.load(os.path.join(gold, "accum_vectors.npz"), allow_pickle=False)
    idx = json.load(open(os.path.join(gold, "accum_vectors.json")))
    for name, meta in idx.items():
        C = P.CURVES[meta["curve"]]
        sh = A.synth_vk_points(C, U.SHAPES[meta["shape"]](C, meta["log_n"]), seed=meta["seed"] ^ 0x7EC)
        ps = U.to_product_shape(meta["curve"], sh)
        _, q, h, st = R.accum_batch(meta["curve"], ps.c, npz[f"{name}.points"], npz[f"{name}.scalars"],
                                    npz[f"{name}.challenges"], threads=3)
        assert np.array_equal(q, npz[f"{name}.quads"]) and np.array_equal(h, npz[f"{name}.h_eval"]), name
        assert not st.any(), name


@pytest.mark.parametrize("cid", [0, 1, 2])
@pytest.mark.parametrize("shape", ["simple", "rich"])
def test_c_transcript_and_accumulator_vs_python(cid, shape):
    """C transcript replay + accumulator == oracle/transcript.py +
    oracle/accum.py on random proofs, with identity commitments (an advice
    one: status 1; a lookup Z: status 3) and a zero denominator (x = 1:
    status 4 with caller challenges)."""
    import numpy as np

    import accum_ref as R
    import transcript as T

    C, sh, proofs, ps = _c_case(cid, shape, 10, 5, 0xCC0 + cid)
    po = sh.point_offsets()
    proofs[1].points[po["adv"][0]] = None
    proofs[3].points[po["lk_z"][0]] = None
    vkr = T.vk_repr(C.r, b"c-port")
    vk = np.array(A.to_limbs_mont(C.r, vkr), dtype=np.uint64)
    want_st = [T.replay_challenges(C, sh, pf, vkr)[1] for pf in proofs]
    assert want_st == [0, 1, 0, 3, 0]
    T.with_replayed_challenges(C, sh, proofs, vkr)
    pts, scs, chs = A.pack_proofs(C, sh, proofs)
    ch, q, h, st = R.accum_batch(cid, ps.c, pts, scs, vk_repr=vk, threads=2)
    assert np.array_equal(ch, chs)
    assert [int(x) for x in st] == want_st
    for b in range(5):
        qq, hh = A.pack_result(C, A.accumulate_msm(C, sh, proofs[b]))
        assert np.array_equal(q[b], qq) and np.array_equal(h[b], hh), b
    chs[2, 4] = A.to_limbs_mont(C.r, 1)  # x = 1
    _, _, _, st2 = R.accum_batch(cid, ps.c, pts, scs, challenges=chs, threads=2)
    assert [int(x) for x in st2] == [0, 0, A.STATUS_DENOM_ZERO, 0, 0]
