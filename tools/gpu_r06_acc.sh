#!/bin/bash
# Round 6: accumulator profiles per batch size (BN254 simple-example proofs
# from bytes, k = 17, tools/accum_bytes_run.py): for each B a kernel trace
# (--kernel-trace --stats) and one SQ counter pass (the VALU roofline of the
# throughput legs: VALU / INT64 wave-instructions, issue cycles, busy cycles).
# Reduced by tools/acc_valu.py.  Usage (gpurun, repo root):
#   bash tools/gpu_r06_acc.sh TAG "1024 4096"
set -o pipefail
TAG=${1:-r06_acc}
BS=${2:-"1024 4096"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
RE='k_acc_|k_transcript|k_proof_decode'
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for B in $BS; do
  D=$OUT/b$B
  mkdir -p $D
  B=$B REPS=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $D/kt -o run -- python3 tools/accum_bytes_run.py > $D/kt.log 2>&1 || { echo "kernel trace B=$B failed"; tail -20 $D/kt.log; exit 1; }
  find $D/kt -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats.csv \;
  find $D/kt -name '*kernel_trace.csv' -exec cp {} $D/kernel_trace.csv \;
  rm -rf $D/kt
  B=$B REPS=6 timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex "$RE" -f csv -d $D/p1 -o run -- python3 tools/accum_bytes_run.py > $D/p1.log 2>&1 || { echo "pmc B=$B failed"; tail -20 $D/p1.log; exit 1; }
  find $D/p1 -name '*counter_collection.csv' -exec cp {} $D/p1.csv \;
  rm -rf $D/p1
  echo "B=$B done"
done
ls -R $OUT | head -40
