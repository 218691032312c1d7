#!/bin/bash
# SQ counter passes of k_accumulate for A/B builds (PM_LIB), 2^20 Pallas.
# Usage (through gpurun): bash tools/gpu_pmc_sq.sh TAG "libA libB ..."
set -o pipefail
TAG=${1:-pmcsq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
P2="SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_IFETCH SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS"
for L in $2; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    D=$OUT/$(basename $L .so)_p$i
    PM_LIB=$L LOGN=${LOGN:-20} timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex k_accumulate -f csv -d $D -o run -- python3 tools/msm_timing.py > $D.log 2>&1 || { echo "pmc pass $i $L failed"; tail -20 $D.log; exit 1; }
    find $D -name '*counter_collection.csv' -exec cp {} $D.csv \;
  done
done
ls $OUT
