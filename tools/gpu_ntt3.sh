#!/bin/bash
# NTT: parity of the two- and three-pass forms, then A/B timing (PM_NTT_PASSES)
set -o pipefail
OUT=gpurun_out/${1:-ntt3}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ntt_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_ntt.log 2>&1 || { echo "pytest ntt failed"; tail -40 $OUT/pytest_ntt.log; exit 1; }
tail -2 $OUT/pytest_ntt.log
for P in 2 3; do
  PM_NTT_PASSES=$P LOGN=${LOGN:-20,22,23,24} timeout -k 10 300 python tools/ntt_timing.py > $OUT/timing_p$P.jsonl 2>&1 || { tail -20 $OUT/timing_p$P.jsonl; exit 1; }
  echo "passes=$P"; grep log_n $OUT/timing_p$P.jsonl
done
LOGN=25,26 timeout -k 10 300 python tools/ntt_timing.py > $OUT/timing_auto.jsonl 2>&1 || { tail -20 $OUT/timing_auto.jsonl; exit 1; }
echo auto; grep log_n $OUT/timing_auto.jsonl
