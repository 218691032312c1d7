#!/bin/bash
# Where k_accumulate's non-issuing cycles go: wait / active-instruction
# counters, address-translation and L2-read-latency counters, at 2^20 and
# 2^22 on the resident-bases path the bench times.  One rocprofv3 run per
# pass (--pmc only, within the per-block limits: 8 SQ, 4 TCP).
# Usage (through gpurun): bash tools/gpu_pmc_stall.sh TAG
set -o pipefail
TAG=${1:-stall}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY"
P3="SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"
for LG in ${LOGNS:-20 22}; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    D=$OUT/n${LG}_s$i
    LOGN=$LG RESIDENT=1 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex k_accumulate -f csv -d $D -o run -- python3 tools/msm_timing.py > $D.log 2>&1 || { echo "pmc pass $i at 2^$LG failed"; tail -20 $D.log; exit 1; }
    find $D -name '*counter_collection.csv' -exec cp {} $OUT/n${LG}_s$i.csv \;
  done
done
ls $OUT
