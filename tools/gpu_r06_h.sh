#!/bin/bash
# Round 6: decode form beside the twisted ladder (auto: one-lane decode when
# the sliced grid does not fit beside the ladder) vs the forced fences that
# keep the sliced decode; interleaved, twice; then the accumulator tests.
set -o pipefail
OUT=gpurun_out/r06_h
mkdir -p $OUT
for rep in 1 2; do
  for tw in -1 2 1; do
    BS=64,128,192,256,320 TWIST=$tw REPS=30 timeout -k 10 200 python -u tools/accum_scaling.py >> $OUT/sweep.jsonl 2>> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_proof_gpu.py tests/test_accum_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
