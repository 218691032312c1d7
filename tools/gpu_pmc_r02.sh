#!/bin/bash
# PMC passes of k_accumulate (each its own rocprofv3 run, --pmc only):
#   SQ pass: VALU instruction counts (all / INT64 / INT32), VALU-active and
#   busy cycles, waves + GRBM_GUI_ACTIVE; then FETCH_SIZE and WRITE_SIZE.
# Sizes: LOGNS (default "20 22"), Pallas, driver tools/msm_timing.py.
# Usage (through gpurun): bash tools/gpu_pmc_r02.sh TAG
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || { echo "rocprofv3 -L failed"; tail -5 $OUT/counters.txt; }
want="SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU"
sq=""
for c in $want; do grep -qw "$c" $OUT/counters.txt && sq="$sq $c"; done
echo "SQ pass:$sq"
for LG in ${LOGNS:-20 22}; do
  i=0
  for P in "$sq GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    D=$OUT/n${LG}_p$i
    LOGN=$LG RESIDENT=${RESIDENT:-0} timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex k_accumulate -f csv -d $D -o run -- python3 tools/msm_timing.py > $D.log 2>&1 || { echo "pmc pass $i at 2^$LG failed"; tail -20 $D.log; exit 1; }
    find $D -name '*counter_collection.csv' -exec cp {} $OUT/n${LG}_p$i.csv \;
  done
done
ls $OUT
