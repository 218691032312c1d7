#!/bin/bash
set -o pipefail
OUT=gpurun_out/pipe2; mkdir -p $OUT
LOGN=20,22 PM_SWEEP_GROUPS=1,2,4 PM_SWEEP_MINCHUNK=16,32,64 timeout -k 10 600 python tools/msm_timing.py > $OUT/sweep.jsonl 2>&1 || { tail -30 $OUT/sweep.jsonl; exit 1; }
cat $OUT/sweep.jsonl
