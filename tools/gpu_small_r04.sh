#!/bin/bash
# Round-4 small-MSM session (through gpurun): kernel traces of the small path
# at n = 1, 32, 4096 and the completion-flag vs event A/B.
set -o pipefail
OUT=gpurun_out/${1:-sm4}
mkdir -p $OUT
export TMPDIR=/tmp
for n in 1 32 4096; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/k$n -o run -- python3 tools/small_msm_timing.py only $n 300 \
    > $OUT/k$n.log 2>&1 || { echo "trace $n failed"; tail -5 $OUT/k$n.log; exit 1; }
done
for n in 1 32 4096; do
  timeout -k 10 100 python3 tools/small_msm_timing.py only $n 400 > $OUT/flag$n.log 2>&1 || exit 1
  PM_SMALL_EVENT=1 timeout -k 10 100 python3 tools/small_msm_timing.py only $n 400 > $OUT/event$n.log 2>&1 || exit 1
done
grep -h small_us $OUT/*.log
