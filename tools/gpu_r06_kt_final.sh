#!/bin/bash
# Round 6 (final tree): the headline-only bench under rocprofv3 --kernel-trace
# --stats -- the k_accumulate summary the roofline's HIP-event average must
# agree with.  Since the split scalar copy the same run's host-scalar legs
# launch k_accumulate on parts of the points too, so the summary of the
# headline leg's own launches is taken from the trace (tools/kt_headline_summary.py).
set -o pipefail
OUT=gpurun_out/r06_kt_final
mkdir -p $OUT
export TMPDIR=/tmp
HEAD="--no-cpu --logn22 0 --strong-logn 0 --fixed 0 --fixed23 0 --ntt-logn 0 --ntt-large-logn 0 --accum-batch 0 --accum-b16 0 --accum-b32 0 --accum-large 0 --inst-batch 0 --small-n 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o run -- python3 bench.py $HEAD --detail $OUT/kt_headline_detail.json > $OUT/kt_headline.log 2>&1 || { tail -20 $OUT/kt_headline.log; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/kt_headline_kernel_stats.csv \;
find $OUT/kt -name '*kernel_trace.csv' -exec cp {} $OUT/kt_headline_kernel_trace.csv \;
rm -rf $OUT/kt
tail -1 $OUT/kt_headline.log | cut -c1-300
