#!/bin/bash
# Round 6: the split scalar copy -- parity (MSM GPU tests), then the A/B of
# pm_msm_resident / drop-in pm_msm with host scalars, one copy vs split
# (PM_SPLIT_OWN_PLAN: the halves' slice length, an A/B switch of round 6 since removed).
set -o pipefail
OUT=gpurun_out/${TAG:-r06_splitcopy}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_msm_gpu.py tests/test_fixed_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
PM_SPLIT_OWN_PLAN=1 timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -k "split_scalar_copy or dropin_row_table or headline" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_own.log 2>&1 || { tail -30 $OUT/tests_own.log; exit 1; }
tail -1 $OUT/tests_own.log
for own in 0 1 0 1; do
  PM_SPLIT_OWN_PLAN=$own LOGN=${LOGN:-20,22} ROUNDS=2 timeout -k 10 300 python -u tools/split_copy_ab.py | sed "s/^{/{\"own_plan\": $own, /" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
done
cat $OUT/ab.jsonl
