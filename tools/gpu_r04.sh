#!/bin/bash
# Round-4 GPU session (through gpurun, from the repo root): bash tools/gpu_r04.sh TAG [parts]
#   test   pytest -m gpu (one process) [TESTS="tests/x.py ..." to restrict, K="expr" for -k]
#   smoke  __graft_entry__.smoke()
#   bench  the default bench.py line -> bench.json
#   quick  headline + accumulator legs only -> bench_quick.json
#   kt     rocprofv3 --kernel-trace --stats of the headline-only bench
#   acckt  rocprofv3 --kernel-trace --stats of the accumulator-only bench
#   micro  tools/microbench_chain (built here beforehand): single-wave step latencies
set -o pipefail
TAG=${1:-r04}
PARTS=${2:-"test smoke bench"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
QUICK="--logn22 0 --strong-logn 0 --fixed 0 --ntt-logn 0 --ntt-large-logn 0 --small-n 0"
for P in $PARTS; do
  echo "== $P $(date +%T)"
  case $P in
    test)
      KARG=()
      [ -n "$K" ] && KARG=(-k "$K")
      timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
        "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1
      rc=$?
      tail -5 $OUT/pytest_gpu.log
      [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | head -20; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
      cat $OUT/smoke.log ;;
    bench)
      timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
      cut -c1-400 $OUT/bench.json ;;
    quick)
      timeout -k 10 600 python -u bench.py --no-cpu $QUICK > $OUT/bench_quick.json 2> $OUT/bench_quick.err || { tail -20 $OUT/bench_quick.err; exit 1; }
      cut -c1-400 $OUT/bench_quick.json ;;
    kt)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o run -- python3 bench.py --no-cpu \
        $QUICK --accum-batch 0 --accum-b16 0 > $OUT/kt.log 2>&1 || { echo "kernel trace failed"; tail -20 $OUT/kt.log; exit 1; }
      find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
      cut -c1-150 $OUT/kernel_stats.csv | head -14 ;;
    acckt)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/acckt -o run -- python3 bench.py --no-cpu \
        $QUICK --logn 15 --accum-b16 1 > $OUT/acckt.log 2>&1 || { echo "kernel trace failed"; tail -20 $OUT/acckt.log; exit 1; }
      find $OUT/acckt -name '*kernel_stats.csv' -exec cp {} $OUT/acc_kernel_stats.csv \;
      cut -c1-150 $OUT/acc_kernel_stats.csv | head -20 ;;
    micro)
      timeout -k 10 300 ./tools/microbench_chain > $OUT/chain_latency.jsonl 2>&1 || { cat $OUT/chain_latency.jsonl; exit 1; }
      cat $OUT/chain_latency.jsonl ;;
  esac
done
echo "== done $(date +%T)"
