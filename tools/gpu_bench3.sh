#!/bin/bash
# MSM parity tests, then the MSM-only bench three times (box noise check).
set -o pipefail
OUT=gpurun_out/${1:-b2}
mkdir -p $OUT
timeout -k 10 120 python -u -m pytest tests -m gpu -x -q -k "msm" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu --fixed 0 --ntt-logn 0 --accum-batch 0 > $OUT/bench$i.json 2> $OUT/err$i.log || { tail -20 $OUT/err$i.log; exit 1; }
done
cat $OUT/bench*.json
