#!/bin/bash
# Round-3 GPU session (through gpurun, from the repo root):
#   TESTS="<pytest paths/-k>" AB="xp ids" LOGN=19,20,22 BENCH=1 PROF=1 bash tools/gpu_r03.sh TAG
# TESTS: GPU parity tests to run first (default: the whole -m gpu suite; "none" skips)
# AB:    msm_timing A/B of lib_xp/libxp<id>.so builds against the in-tree lib ("0"), alternated
# BENCH: the bench line; PROF: rocprofv3 kernel-trace summary of a headline-only bench run
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-all}" != "none" ]; then
  if [ "${TESTS:-all}" = "all" ]; then T="tests"; else T="$TESTS"; fi
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
for X in ${AB:-}; do
  if [ "$X" = 0 ]; then L=halo2-aggregation_amd/lib/libpasta_msm.so; else L=halo2-aggregation_amd/lib_xp/libxp$X.so; fi
  echo "xp=$X"
  PM_LIB=$L RESIDENT=${RESIDENT:-1} LOGN=${LOGN:-19,20,22} timeout -k 10 180 python tools/msm_timing.py 2>/dev/null \
    | grep logn | tee -a $OUT/ab_$X.jsonl | cut -c1-420 || { echo "timing $X failed"; exit 1; }
done
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 500 python bench.py ${BENCHARGS:-} > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
  cut -c1-3000 $OUT/bench.json
fi
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --no-cpu \
    --logn22 0 --strong-logn 0 --fixed 0 --ntt-logn 0 --ntt-large-logn 0 --accum-batch 0 > $OUT/prof.log 2>&1 \
    || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
  find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
  cut -c1-160 $OUT/kernel_stats.csv | head -16
fi
