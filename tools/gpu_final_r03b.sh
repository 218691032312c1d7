#!/bin/bash
# Round-3 final evidence for the tree as committed: GPU tests, smoke, default
# bench, then the headline-only kernel trace (tools/gpu_prof_r03.sh kt).
# Usage (through gpurun): bash tools/gpu_final_r03b.sh TAG
set -o pipefail
TAG=${1:-fin}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
bash tools/gpu_prof_r03.sh $TAG/prof kt
