#!/bin/bash
# Host + kernel timeline of repeated resident 2^LOGN MSMs (tools/htrace_gaps.py)
set -o pipefail
OUT=gpurun_out/${1:-htr}; mkdir -p $OUT; export TMPDIR=/tmp
RESIDENT=1 LOGN=${LOGN:-20} timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace -f csv -d $OUT/p -o run -- python3 tools/msm_timing.py > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
find $OUT/p -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
find $OUT/p -name '*hip_api_trace.csv' -exec cp {} $OUT/hip_api_trace.csv \;
rm -rf $OUT/p
python3 tools/htrace_gaps.py $OUT/kernel_trace.csv $OUT/hip_api_trace.csv k_sort_hist 2,3
