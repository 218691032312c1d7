"""Config 5 projection (BASELINE.json configs[4]: 256 proofs, 8 x MI355X)
from a one-GPU batch-size sweep (tools/accum_scaling.py output): with N ranks
each rank decodes and accumulates 256 / N proofs from bytes, then the ranks
all-gather the B x 4 affine quads (64 B each).  The per-rank time is the
measured batch time at B = 256 / N; the all-gather is not measured here (no
multi-GPU box): it is listed as a separate term, a 1-hop RCCL all-gather of
at most 64 KiB, bounded by GATHER_US (default 25 us, an assumption stated in
the output).  Usage: python tools/accum_projection.py sweep.jsonl > out.jsonl"""
import json
import os
import sys


def main():
    rows = {}
    for line in open(sys.argv[1]):
        line = line.strip()
        if line.startswith("{"):
            r = json.loads(line)
            rows[r["B"]] = r
    gather_us = float(os.environ.get("GATHER_US", "25"))
    base = rows[256]["ms_per_batch"]
    for n in (1, 2, 4, 8):
        b = 256 // n
        if b not in rows:
            continue
        ms = rows[b]["ms_per_batch"] + (gather_us * 1e-3 if n > 1 else 0.0)
        print(json.dumps({"gpus": n, "proofs_per_rank": b, "rank_batch_ms": rows[b]["ms_per_batch"],
                          "allgather_ms_assumed": gather_us * 1e-3 if n > 1 else 0.0,
                          "batch_ms": round(ms, 4), "speedup_vs_1": round(base / ms, 3),
                          "throughput_many_batches_per_rank": "B = 4096 per rank: see accumulator_b4096",
                          "source": sys.argv[1]}))


if __name__ == "__main__":
    main()
