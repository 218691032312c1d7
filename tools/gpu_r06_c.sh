#!/bin/bash
# Round 6: twisted-ladder decode fence A/B (1 unfenced, 2 two blocks per CU,
# 0 off), interleaved, and the small-MSM phases with a settled GPU.
set -o pipefail
OUT=gpurun_out/r06_c
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_proof_gpu.py -k "schedule_options or option_arguments" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for tw in 1 2 0; do
    BS=128,192,256,384,512,768,1024 TWIST=$tw REPS=20 timeout -k 10 200 python -u tools/accum_scaling.py >> $OUT/sweep.jsonl 2>> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
  done
done
timeout -k 10 200 python -u tools/small_phases.py > $OUT/small_phases.jsonl 2> $OUT/small.err || { tail -20 $OUT/small.err; exit 1; }
cat $OUT/small_phases.jsonl
