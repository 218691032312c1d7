#!/bin/bash
# Round 6 final evidence: GPU suite + smoke, the default bench (its detail
# record), the bench under rocprofv3 --kernel-trace --stats (the headline
# kernel's summary), the small-MSM phases, and the k_accumulate PMC passes of
# the headline workload (resident row table, 2^20).
set -o pipefail
OUT=gpurun_out/${TAG:-r06_final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --detail $OUT/bench_detail.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -c 600 $OUT/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o run -- python3 bench.py --steps 20 --warmup 5 --detail $OUT/kt_bench_detail.json > $OUT/kt_bench.log 2>&1 || { tail -20 $OUT/kt_bench.log; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/kt_kernel_stats.csv \;
rm -rf $OUT/kt
timeout -k 10 200 python -u tools/small_phases.py > $OUT/small_phases.jsonl 2> $OUT/small.err || { tail -20 $OUT/small.err; exit 1; }
RESIDENT=1 LOGNS="20 22" bash tools/gpu_pmc_r02.sh ${TAG:-r06_final}/pmc > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
ls $OUT $OUT/pmc
