#!/bin/bash
# A/B MSM timing of experiment builds (PM_LIB), repeated: bash tools/gpu_xp_msm.sh "0 old 0 old"
set -o pipefail
for X in $1; do
  if [ $X = 0 ]; then L=halo2-aggregation_amd/lib/libpasta_msm.so; else L=halo2-aggregation_amd/lib_xp/libxp$X.so; fi
  echo "xp=$X"
  mkdir -p gpurun_out/xpmsm; PM_LIB=$L RESIDENT=1 LOGN=${LOGN:-20} timeout -k 10 120 python tools/msm_timing.py 2>/dev/null | grep logn | tee -a gpurun_out/xpmsm/timing_$X.jsonl | cut -c1-400 || exit 1
done
