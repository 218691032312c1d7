#!/bin/bash
# Round-2 microbenchmarks: field product / mixed add / inversion throughput,
# and the 1-GPU strong-scaling projection of the 2^22 Vesta MSM.
set -o pipefail
OUT=gpurun_out/${1:-micro}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench_f29 > $OUT/microbench_f29.jsonl 2>&1 || { echo "microbench failed"; cat $OUT/microbench_f29.jsonl; exit 1; }
cat $OUT/microbench_f29.jsonl
timeout -k 10 300 python tools/strong_projection.py 22 1 > $OUT/strong_projection.jsonl 2>&1 || { echo "projection failed"; tail -20 $OUT/strong_projection.jsonl; exit 1; }
cat $OUT/strong_projection.jsonl
