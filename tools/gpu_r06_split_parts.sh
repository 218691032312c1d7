#!/bin/bash
# Round 6: split scalar copy in two parts (3/8 + 5/8) against three (1/4 + 3/8
# + 3/8) from 2^20 points (PM_SPLIT_PARTS: an A/B switch of round 6, since removed:
# three parts from 2^21 points).
set -o pipefail
OUT=gpurun_out/${TAG:-r06_split_parts}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
PM_SPLIT_PARTS=3 timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests3.log 2>&1 || { tail -30 $OUT/tests3.log; exit 1; }
tail -1 $OUT/tests3.log
for rep in 1 2; do
  for parts in 2 3; do
    PM_SPLIT_PARTS=$parts LOGN=20,22 ROUNDS=1 timeout -k 10 300 python -u tools/split_copy_ab.py | grep -v dropin_stats | sed "s/^{/{\"parts\": $parts, /" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
  done
done
cat $OUT/ab.jsonl
