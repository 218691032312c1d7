#!/bin/bash
# Instruction-fetch PMC passes of the bucket-reduction kernels (and k_accumulate
# for reference), each its own rocprofv3 --pmc run: bash tools/gpu_pmc_icache.sh TAG
set -o pipefail
TAG=${1:-icache}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_WAVES SQ_INSTS_SALU" \
         "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ"; do
  i=$((i+1))
  D=$OUT/p$i
  LOGN=${LG:-20} RESIDENT=1 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "${KRE:-k_bucket|k_accumulate}" -f csv -d $D -o run \
    -- python3 tools/msm_timing.py > $D.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $D.log; exit 1; }
  find $D -name '*counter_collection.csv' -exec cp {} $OUT/p$i.csv \;
done
ls $OUT
