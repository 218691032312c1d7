#!/bin/bash
# Quick GPU iteration: field self-test + MSM parity tests, then per-size
# timing.  Usage (through gpurun): bash tools/gpu_quick.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-quick}
K=${2:-"msm or selftest"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
if [ "$LOGN" != "none" ]; then
  LOGN=${LOGN:-18,20,22} timeout -k 10 300 python tools/msm_timing.py > $OUT/timing.jsonl 2>&1 || { echo "timing failed"; tail -30 $OUT/timing.jsonl; exit 1; }
  cat $OUT/timing.jsonl
fi
if [ -n "$ACCUM" ]; then
  timeout -k 10 300 python tools/accum_timing.py > $OUT/accum_timing.jsonl 2>&1 || { tail -30 $OUT/accum_timing.jsonl; exit 1; }
  cat $OUT/accum_timing.jsonl
fi
