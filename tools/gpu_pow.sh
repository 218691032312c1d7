#!/bin/bash
# accumulator: parity of the powers-of-two path, then per-kernel timing
set -o pipefail
OUT=gpurun_out/${1:-pow}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_accum_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_accum.log 2>&1 || { echo "pytest accum failed"; tail -40 $OUT/pytest_accum.log; exit 1; }
tail -2 $OUT/pytest_accum.log
SPLITS=${SPLITS:--1} CASES=${CASES:-all} timeout -k 10 300 python tools/accum_timing.py > $OUT/timing.jsonl 2>&1 || { tail -30 $OUT/timing.jsonl; exit 1; }
cat $OUT/timing.jsonl
