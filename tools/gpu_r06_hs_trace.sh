#!/bin/bash
# Round 6: kernel + memory-copy trace of the reduced bench (MSM legs only) to
# see the split scalar copy inside the bench's own context.
set -o pipefail
OUT=gpurun_out/${TAG:-r06_hs_trace}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof -o trace -- python3 bench.py --no-cpu --fixed 0 --ntt-logn 0 --ntt-large-logn 0 --accum-batch 0 --logn22 0 --fixed23 0 --strong-logn 0 --small-n 0 --inst-batch 0 --accum-b32 0 --accum-large 0 --accum-b16 0 --detail $OUT/d.json > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
find $OUT/prof -name "*.csv" -exec mv {} $OUT/ \;
rm -rf $OUT/prof
ls $OUT
