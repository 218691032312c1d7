#!/bin/bash
# Round-2 GPU session: full parity suite, the bench line, a rocprofv3 kernel
# trace summary of the same bench command.
# Usage (through gpurun, from the repo root): bash tools/gpu_r02.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-r02}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$K" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v ${K:+-k "$K"} --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --no-cpu --fixed 0 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
  find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
  head -16 $OUT/kernel_stats.csv
fi
