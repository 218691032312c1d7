#!/bin/bash
# A/B of the host wait (PM_SPIN_WAIT 0/1): full GPU tests once, then
# interleaved MSM / accumulator timings and the headline bench per mode.
# Usage (through gpurun): bash tools/gpu_spin_ab.sh
set -o pipefail
OUT=gpurun_out/spin_ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for rep in 1 2; do
  for sw in 0 1; do
    echo "spin=$sw rep=$rep"
    PM_SPIN_WAIT=$sw RESIDENT=1 LOGN=19,20,22 timeout -k 10 200 python tools/msm_timing.py > $OUT/msm_s${sw}_r${rep}.jsonl 2>&1 || { echo "msm timing failed"; tail -20 $OUT/msm_s${sw}_r${rep}.jsonl; exit 1; }
    PM_SPIN_WAIT=$sw CASES=simple:16,simple:256 timeout -k 10 200 python tools/accum_timing.py > $OUT/acc_s${sw}_r${rep}.jsonl 2>&1 || { echo "accum timing failed"; tail -20 $OUT/acc_s${sw}_r${rep}.jsonl; exit 1; }
    PM_SPIN_WAIT=$sw timeout -k 10 300 python bench.py > $OUT/bench_s${sw}_r${rep}.json 2> $OUT/bench_s${sw}_r${rep}.err || { echo "bench failed"; tail -20 $OUT/bench_s${sw}_r${rep}.err; exit 1; }
  done
done
echo done
