#!/bin/bash
# Diagnose the large-n accumulate slowdown: prefetch on/off, window widths.
set -o pipefail
OUT=gpurun_out/diag22
mkdir -p $OUT
for pf in 0 1; do
  PM_PREFETCH=$pf LOGN=20,21,22 WINDOWS=0,16,20 timeout -k 10 300 python tools/msm_timing.py > $OUT/pf$pf.jsonl 2>&1 || { tail $OUT/pf$pf.jsonl; exit 1; }
  cat $OUT/pf$pf.jsonl
done
