#!/bin/bash
set -o pipefail
OUT=gpurun_out/accum1
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python tools/accum_timing.py > $OUT/accum_timing.jsonl 2>&1 || { tail -30 $OUT/accum_timing.jsonl; exit 1; }
cat $OUT/accum_timing.jsonl
LOGN=20,22 timeout -k 10 300 python tools/msm_timing.py > $OUT/msm_timing.jsonl 2>&1 || { tail -30 $OUT/msm_timing.jsonl; exit 1; }
cat $OUT/msm_timing.jsonl
