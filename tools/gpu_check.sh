#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel stats, PMC traffic of
# k_accumulate, per-size timing.
# Usage (from the repo root, through gpurun): bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --no-cpu --fixed 0 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
head -12 $OUT/kernel_stats.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_accumulate -f csv -d $OUT/pmc_$C -o run -- python3 bench.py --no-cpu --fixed 0 --steps 5 --warmup 1 --accum-batch 0 > $OUT/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -20 $OUT/pmc_$C.log; exit 1; }
  find $OUT/pmc_$C -name '*counter_collection.csv' -exec cp {} $OUT/pmc_$C.csv \;
done
LOGN=${LOGN:-18,20,22} timeout -k 10 300 python tools/msm_timing.py > $OUT/timing.jsonl 2>&1 || { echo "timing failed"; tail -30 $OUT/timing.jsonl; exit 1; }
cat $OUT/timing.jsonl
timeout -k 10 300 python tools/accum_timing.py > $OUT/accum_timing.jsonl 2>&1 || { tail -30 $OUT/accum_timing.jsonl; exit 1; }
cat $OUT/accum_timing.jsonl
