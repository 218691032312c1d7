#!/bin/bash
# NTT VALU PMC (round 4): SQ_INSTS_VALU / _INT64 / _INT32 + GRBM_GUI_ACTIVE of
# every pass at 2^20 and 2^25 (one --pmc pass each, driver tools/ntt_timing.py),
# reduced by tools/ntt_valu.py into the "valu" entries of profiles/pmc_ntt.json.
# Usage (through gpurun, from the repo root): bash tools/gpu_ntt_valu_r04.sh TAG
set -o pipefail
TAG=${1:-ntt_valu}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
for L in 20 25; do
  D=$OUT/v$L
  LOGN=$L timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex k_ntt -f csv -d $D -o run -- python3 tools/ntt_timing.py > $D.log 2>&1 || { echo "pmc $L failed"; tail -20 $D.log; exit 1; }
  find $D -name '*counter_collection.csv' -exec cp {} $OUT/valu_n$L.csv \;
done
ls $OUT
