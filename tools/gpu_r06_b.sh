#!/bin/bash
# Round 6 step: GPU suite, accumulator sweep (auto schedule), small-MSM phases.
set -o pipefail
OUT=gpurun_out/r06_b
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
BS=16,32,64,128,192,256,384,512,768,1024,1536,2048,3072,4096 REPS=20 timeout -k 10 300 python -u tools/accum_scaling.py > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
timeout -k 10 200 python -u tools/small_phases.py > $OUT/small_phases.jsonl 2> $OUT/small.err || { tail -20 $OUT/small.err; exit 1; }
cat $OUT/small_phases.jsonl
