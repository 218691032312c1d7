#!/bin/bash
# Round 6: k_acc_sum row step after two-term lanes; accumulator tests + large-B sweep.
set -o pipefail
OUT=gpurun_out/r06_i
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_proof_gpu.py tests/test_accum_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
BS=2048,3072,4096 REPS=20 timeout -k 10 200 python -u tools/accum_scaling.py > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
