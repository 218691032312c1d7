#!/bin/bash
# Where the NTT passes' cycles go (SQ wait / active counters, one rocprofv3
# run per pass within the 8-SQ-counter limit), tools/ntt_timing.py at 2^LOGN.
# Usage (through gpurun): LOGN=20 bash tools/gpu_ntt_stall.sh TAG
set -o pipefail
TAG=${1:-ntt_stall}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INST_CYCLES_VMEM_RD"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MAD_U64 SQ_BUSY_CU_CYCLES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  D=$OUT/s$i
  LOGN=${LOGN:-20} timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "k_ntt_(cols|mid|rows)" -f csv -d $D -o run -- python3 tools/ntt_timing.py > $D.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $D.log; exit 1; }
  find $D -name '*counter_collection.csv' -exec cp {} $OUT/s$i.csv \;
done
python3 - $OUT <<'PY'
import csv, sys, statistics, collections
out = sys.argv[1]
for i in (1, 2, 3):
    try:
        rows = list(csv.DictReader(open(f"{out}/s{i}.csv")))
    except FileNotFoundError:
        continue
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        kn = next((x for x in ("k_ntt_cols", "k_ntt_mid", "k_ntt_rows") if x in r["Kernel_Name"]), "?")
        by[kn][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for kn, c in sorted(by.items()):
        print(i, kn, {k: statistics.median(v) for k, v in c.items()})
PY
