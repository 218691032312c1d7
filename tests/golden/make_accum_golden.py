"""Generate tests/golden/accum_vectors.npz with the Python accumulator oracle
(oracle/accum.py).  Every expected value is produced by the literal Horner
restatement (``accumulate``) and asserted equal to the closed-form MSM
restatement (``accumulate_msm``) before it is written.  Parity is unpinned by
the reference (no vectors for this path); these fixtures pin
the HIP path to the restatement.

Case NAME holds NAME.points (B, npts, 8), NAME.scalars (B, nsc, 4),
NAME.challenges (B, 7, 4), NAME.quads (B, 4, 8) = (w, zw, f, e) affine,
NAME.h_eval (B, 4), NAME.fixed (nf, 8), NAME.sigma (np, 8); all u64 Montgomery.
The JSON index records curve, shape builder, log_n and seed.
Run: python tests/golden/make_accum_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "..", "oracle"), os.path.join(HERE, "..")]
import accum as A  # noqa: E402
import pasta as P  # noqa: E402

SHAPES = {"simple": A.simple_example_shape, "rich": A.rich_shape}

CASES = [
    # name, curve id, shape, log_n, B, seed, edit
    ("bn254_simple_k14", 2, "simple", 14, 4, 0xACC1, None),
    ("pallas_simple_k14", 0, "simple", 14, 2, 0xACC2, None),
    ("vesta_rich_k10", 1, "rich", 10, 2, 0xACC3, None),
    ("bn254_rich_k17", 2, "rich", 17, 2, 0xACC4, None),
    ("bn254_simple_edge", 2, "simple", 14, 3, 0xACC5, "edge"),
    # the reference's only real configuration: ONE inner simple-example proof
    # at k = 9 (examples/simple-example.rs:561,620-626), B = 1
    ("bn254_simple_k9_single", 2, "simple", 9, 1, 0xACC6, None),
]


def edit_edge(C, sh, proofs):
    """Identity commitments / witnesses, zero and equal evals, repeated points:
    exercises the identity and P == Q branches of the group law."""
    po = sh.point_offsets()
    p0 = proofs[0]
    p0.points[po["W"][0]] = None                  # W_0 = identity
    p0.points[po["adv"][0]] = None                # an advice commitment = identity
    p0.scalars = [0] * len(p0.scalars)            # all evals zero
    p1 = proofs[1]
    same = p1.points[po["adv"][0]]
    p1.points[po["adv"][0] + 1] = same            # two columns commit to the same point
    p1.points[po["W"][0] + 1] = C.neg(p1.points[po["W"][0]])  # W_1 = -W_0
    p2 = proofs[2]
    p2.challenges[5] = 1                          # v = 1
    p2.challenges[6] = 0                          # u = 0 (only the last set survives)
    return proofs


def main():
    arrays, index = {}, {}
    for name, cid, shp, log_n, B, seed, edit in CASES:
        C = P.CURVES[cid]
        sh = A.synth_vk_points(C, SHAPES[shp](C, log_n), seed=seed ^ 0x7EC)
        proofs = [A.synth_proof(C, sh, seed, b) for b in range(B)]
        if edit == "edge":
            proofs = edit_edge(C, sh, proofs)
        quads, hs = [], []
        for pf in proofs:
            res = A.accumulate(C, sh, pf)
            assert res == A.accumulate_msm(C, sh, pf), name
            q, h = A.pack_result(C, res)
            quads.append(q)
            hs.append(h)
        pts, scs, chs = A.pack_proofs(C, sh, proofs)
        arrays[f"{name}.points"] = pts
        arrays[f"{name}.scalars"] = scs
        arrays[f"{name}.challenges"] = chs
        arrays[f"{name}.quads"] = np.array(quads, dtype=np.uint64)
        arrays[f"{name}.h_eval"] = np.array(hs, dtype=np.uint64)
        arrays[f"{name}.fixed"] = np.array([P.point_to_limbs(C, q) for q in sh.fixed_commitments], dtype=np.uint64)
        arrays[f"{name}.sigma"] = np.array([P.point_to_limbs(C, q) for q in sh.sigma_commitments], dtype=np.uint64)
        index[name] = {"curve": cid, "shape": shp, "log_n": log_n, "B": B, "seed": seed, "edit": edit}
        print(name, pts.shape, flush=True)
    np.savez_compressed(os.path.join(HERE, "accum_vectors.npz"), **arrays)
    with open(os.path.join(HERE, "accum_vectors.json"), "w") as f:
        json.dump(index, f, indent=1)


if __name__ == "__main__":
    main()
