#!/bin/bash
# MSM: parity with the fused chain + segment kernel, then A/B (PM_SEGQ)
set -o pipefail
OUT=gpurun_out/${1:-segq}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_fixed_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for V in 1 0 1; do
  PM_SEGQ=$V RESIDENT=1 LOGN=19,20,22 timeout -k 10 200 python tools/msm_timing.py 2>/dev/null | grep logn > $OUT/t.jsonl || exit 1
  echo "== PM_SEGQ=$V"; cat $OUT/t.jsonl; cat $OUT/t.jsonl >> $OUT/timing_all.jsonl
done
PM_SEGQ=1 LOGN=20 FIXED_C=16 WINDOWS=0 timeout -k 10 200 python tools/msm_timing.py 2>/dev/null | grep fixed | tee -a $OUT/timing_all.jsonl
PM_SEGQ=0 LOGN=20 FIXED_C=16 WINDOWS=0 timeout -k 10 200 python tools/msm_timing.py 2>/dev/null | grep fixed | tee -a $OUT/timing_all.jsonl
