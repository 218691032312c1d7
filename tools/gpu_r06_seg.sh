#!/bin/bash
# Round 6: k_bucket_seg_q with a quad per bucket -- MSM parity, then the
# per-kernel timing of the resident (row-table), raw and fixed-base paths.
set -o pipefail
OUT=gpurun_out/${TAG:-r06_seg}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py tests/test_fixed_gpu.py tests/test_msm_many_gpu.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
RESIDENT=1 LOGN=20,22 REPS=20 timeout -k 10 200 python -u tools/msm_timing.py > $OUT/resident.jsonl 2>&1 || { tail -20 $OUT/resident.jsonl; exit 1; }
RESIDENT=0 LOGN=20 REPS=20 FIXED_C=16 timeout -k 10 200 python -u tools/msm_timing.py > $OUT/raw.jsonl 2>&1 || { tail -20 $OUT/raw.jsonl; exit 1; }
cut -c1-400 $OUT/resident.jsonl $OUT/raw.jsonl
