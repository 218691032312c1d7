#!/bin/bash
# Kernel timeline (rocprofv3 --kernel-trace) of repeated accumulator calls:
# per-kernel start/end for the gap analysis in tools/ktrace_gaps.py.
# Usage (through gpurun): bash tools/gpu_ktrace.sh TAG [CASES] [first kernel of a call]
set -o pipefail
OUT=gpurun_out/${1:-ktr}; mkdir -p $OUT; export TMPDIR=/tmp
CASES=${2:-simple:256} REPS=10 timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/p -o run -- python3 tools/accum_timing.py > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
find $OUT/p -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
python3 tools/ktrace_gaps.py $OUT/kernel_trace.csv ${3:-k_acc_ladder}
