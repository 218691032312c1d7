#!/bin/bash
# Row-table sweep of the resident MSM (PM_RESIDENT_ROWS) with the in-tree lib:
#   bash tools/gpu_rows_r03.sh TAG "4 8 16" 19,20,22
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
for R in $2; do
  echo "rows=$R"
  PM_RESIDENT_ROWS=$R RESIDENT=1 LOGN=${3:-19,20} timeout -k 10 180 python tools/msm_timing.py 2>/dev/null \
    | grep logn | tee -a $OUT/rows_$R.jsonl | cut -c1-420 || { echo "rows $R failed"; exit 1; }
done
