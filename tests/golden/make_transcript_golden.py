"""Regenerates tests/golden/transcript_vectors.{npz,json} from the oracle
(oracle/transcript.py).  Run from the repo root:
    python tests/golden/make_transcript_golden.py
Cases: every curve, both synthetic shapes, ragged batch sizes, one proof with
an identity commitment (skipped by the transcript, status bit 0)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "halo2-aggregation_amd")]

import accum as A  # noqa: E402
import accum_util as U  # noqa: E402
import pasta as P  # noqa: E402
import transcript as T  # noqa: E402

CASES = [
    ("pallas_simple_k11", 0, "simple", 11, 3, 0x7A1, None),
    ("vesta_rich_k12", 1, "rich", 12, 2, 0x7A2, None),
    ("bn254_simple_k14", 2, "simple", 14, 5, 0x7A3, (1, "adv")),
    ("bn254_rich_k9", 2, "rich", 9, 1, 0x7A4, None),
]


def main():
    arrays, index = {}, {}
    for name, cid, shape, log_n, B, seed, ident in CASES:
        C, sh, proofs = U.make_case(cid, shape, log_n, B, seed)
        if ident is not None:
            b, grp = ident
            k, _ = sh.point_offsets()[grp]
            proofs[b].points[k] = None
        vkr = T.vk_repr(C.r, f"pinned-vk-{name}".encode())
        status = []
        for pf in proofs:
            pf.challenges, skipped = T.replay_challenges(C, sh, pf, vkr)
            status.append(int(skipped))
        pts, scs, chs = A.pack_proofs(C, sh, proofs)
        arrays[f"{name}.points"] = pts
        arrays[f"{name}.scalars"] = scs
        arrays[f"{name}.challenges"] = chs
        arrays[f"{name}.status"] = np.array(status, dtype=np.uint32)
        arrays[f"{name}.vk_repr"] = np.array(A.to_limbs_mont(C.r, vkr), dtype=np.uint64)
        index[name] = {"curve": cid, "shape": shape, "log_n": log_n, "B": B, "seed": seed}
    out = os.path.join(ROOT, "tests", "golden")
    np.savez_compressed(os.path.join(out, "transcript_vectors.npz"), **arrays)
    json.dump(index, open(os.path.join(out, "transcript_vectors.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
