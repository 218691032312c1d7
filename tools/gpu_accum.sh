#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-accum2}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_accum_gpu.py -x -q > $OUT/pytest_accum.log 2>&1 || { echo "pytest accum failed"; tail -40 $OUT/pytest_accum.log; exit 1; }
tail -2 $OUT/pytest_accum.log
timeout -k 10 300 python tools/accum_timing.py > $OUT/accum_timing.jsonl 2>&1 || { tail -30 $OUT/accum_timing.jsonl; exit 1; }
cat $OUT/accum_timing.jsonl
