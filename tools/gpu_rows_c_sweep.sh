#!/bin/bash
# 2^20 sweep: resident rows 4 / 8 x fine bits, then the fixed-base MSM over
# window widths 16-22.  Usage (through gpurun): bash tools/gpu_rows_c_sweep.sh
set -o pipefail
OUT=gpurun_out/rows_c
mkdir -p $OUT
export TMPDIR=/tmp
for rows in 4 8; do
  for fb in 0 6 8; do
    PM_RESIDENT_ROWS=$rows PM_SORT_FB=$fb RESIDENT=1 LOGN=20 timeout -k 10 120 python tools/msm_timing.py > $OUT/rows${rows}_fb${fb}.jsonl 2>&1 || { echo "rows $rows fb $fb failed"; tail -20 $OUT/rows${rows}_fb${fb}.jsonl; exit 1; }
    grep wall_ms $OUT/rows${rows}_fb${fb}.jsonl | cut -c1-160
  done
done
FIXED_C=16,17,18,19,20,22 LOGN=20 WINDOWS=16 timeout -k 10 300 python tools/msm_timing.py > $OUT/fixed_c.jsonl 2>&1 || { echo "fixed failed"; tail -20 $OUT/fixed_c.jsonl; exit 1; }
grep wall_ms $OUT/fixed_c.jsonl | cut -c1-200
