#!/bin/bash
# PMC passes of the accumulator kernels on bench.py's accumulator leg (B = 256
# simple-example proofs from bytes, BN254, k = 17; driver
# tools/accum_bytes_run.py), each pass its own rocprofv3 run (--pmc only,
# within the per-block limits: 8 SQ, 2 GRBM).  Reduced by tools/pmc_acc.py.
# Usage (through gpurun, from the repo root): bash tools/gpu_pmc_acc.sh TAG
set -o pipefail
TAG=${1:-pmc_acc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
RE='k_acc_|k_transcript|k_proof_decode'
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  D=$OUT/p$i
  REPS=10 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$RE" -f csv -d $D -o run -- python3 tools/accum_bytes_run.py > $D.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $D.log; exit 1; }
  find $D -name '*counter_collection.csv' -exec cp {} $OUT/p$i.csv \;
done
REPS=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o run -- python3 tools/accum_bytes_run.py > $OUT/kt.log 2>&1 || { echo "kernel trace failed"; tail -20 $OUT/kt.log; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/kt -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
ls $OUT
