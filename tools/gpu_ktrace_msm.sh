#!/bin/bash
# Kernel timeline of repeated 2^LOGN Pallas MSMs (gap analysis, tools/ktrace_gaps.py).
set -o pipefail
OUT=gpurun_out/${1:-ktrm}; mkdir -p $OUT; export TMPDIR=/tmp
LOGN=${LOGN:-20} timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/p -o run -- python3 tools/msm_timing.py > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
find $OUT/p -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
python3 tools/ktrace_gaps.py $OUT/kernel_trace.csv k_bases_to_r261
