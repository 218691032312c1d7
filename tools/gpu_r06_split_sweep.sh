#!/bin/bash
# Round 6: split scalar copy sweep -- the first part's share (PM_SPLIT_FRAC16
# sixteenths) with the parts' own slice plans (PM_SPLIT_OWN_PLAN=1): A/B builds of round 6
# only -- both switches were removed once the sweep had picked 3/8 with own plans.
set -o pipefail
OUT=gpurun_out/${TAG:-r06_split_sweep2}
mkdir -p $OUT
for rep in 1 2; do
  for f in 5 6 7; do
    PM_SPLIT_FRAC16=$f PM_SPLIT_OWN_PLAN=1 LOGN=${LOGN:-20,22} ROUNDS=1 timeout -k 10 300 python -u tools/split_copy_ab.py | grep -v dropin_stats | sed "s/^{/{\"frac16\": $f, /" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
  done
done
cat $OUT/ab.jsonl
