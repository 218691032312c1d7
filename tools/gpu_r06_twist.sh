#!/bin/bash
# Round 6: forced twisted ladder (decode unfenced beside the quad ladder) vs
# auto at mid batch sizes, interleaved; plus the schedule-option parity tests.
set -o pipefail
OUT=gpurun_out/r06_twist
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_proof_gpu.py -k "schedule_options or option_arguments" tests/test_accum_gpu.py -k "schedule_options or option_arguments or terms_per_lane" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
for rep in 1 2; do
  for tw in -1 1; do
    BS=${BS:-256,512,768,1024,1536} TWIST=$tw REPS=20 timeout -k 10 200 python -u tools/accum_scaling.py >> $OUT/sweep.jsonl 2>> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
  done
done
tail -5 $OUT/tests.log
