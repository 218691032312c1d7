#!/bin/bash
# Round 6: the split copy's two-list bucket fold side by side (k_bucket_seg_q2)
# against the serial fold (k_bucket_seg_q<F, 2>); PM_SEG_PAR2 is an A/B switch.
set -o pipefail
OUT=gpurun_out/${TAG:-r06_seg2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -k "split_scalar_copy or dropin_row_table or headline" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for par in 0 1; do
    PM_SEG_PAR2=$par LOGN=20 ROUNDS=1 REPS=30 timeout -k 10 300 python -u tools/split_copy_ab.py | grep -v dropin_stats | grep auto | sed "s/^{/{\"seg_par2\": $par, /" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
  done
done
cat $OUT/ab.jsonl
