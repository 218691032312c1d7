"""Regenerates tests/golden/ntt_vectors.{npz,json} from the oracle
(oracle/ntt.py).  Run from the repo root: python tests/golden/make_ntt_golden.py
Cases: every scalar field; log_n 0..11 (one pass on the GPU) and 13 (two
passes); edge inputs (all zero, delta at 0 and at n-1, constant, r-1)."""
import json
import os
import random
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle")]

import accum as A  # noqa: E402
import ntt as N  # noqa: E402
import pasta as P  # noqa: E402


def mont(r, v):
    return P.to_limbs(v * P.R_MONT % r)


def main():
    arrays, index = {}, {}
    cases = []
    for cid in (0, 1, 2):
        for k in (0, 1, 2, 3, 5, 8, 11):
            cases.append((f"c{cid}_k{k}_rand", cid, k, "rand"))
    cases.append(("c2_k13_rand", 2, 13, "rand"))   # two passes on the GPU
    for kind in ("zero", "delta0", "deltalast", "const", "rminus1"):
        cases.append((f"c2_k6_{kind}", 2, 6, kind))
    for name, cid, k, kind in cases:
        C = P.CURVES[cid]
        r, n = C.r, 1 << k
        rng = random.Random(zlib.crc32(name.encode()))
        if kind == "rand":
            a = [rng.randrange(r) for _ in range(n)]
        elif kind == "zero":
            a = [0] * n
        elif kind == "delta0":
            a = [1] + [0] * (n - 1)
        elif kind == "deltalast":
            a = [0] * (n - 1) + [1]
        elif kind == "const":
            a = [12345] * n
        else:
            a = [r - 1] * n
        w = A.domain_omega(r, k)
        out = N.serial_fft(list(a), w, k, r)
        arrays[f"{name}.input"] = np.array([mont(r, v) for v in a], dtype=np.uint64).reshape(n, 4)
        arrays[f"{name}.output"] = np.array([mont(r, v) for v in out], dtype=np.uint64).reshape(n, 4)
        arrays[f"{name}.omega"] = np.array(mont(r, w), dtype=np.uint64)
        index[name] = {"curve": cid, "log_n": k, "kind": kind}
    out = os.path.join(ROOT, "tests", "golden")
    np.savez_compressed(os.path.join(out, "ntt_vectors.npz"), **arrays)
    json.dump(index, open(os.path.join(out, "ntt_vectors.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
