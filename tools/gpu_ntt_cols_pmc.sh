#!/bin/bash
# Why pass A (k_ntt_cols) at 2^25 is slower than the other passes: SQ wait
# counters and TCP address-translation / read-latency counters of every NTT
# pass, one rocprofv3 --pmc run per counter set.  Usage: bash tools/gpu_ntt_cols_pmc.sh TAG
set -o pipefail
TAG=${1:-ntt_cols}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"
P2="TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  D=$OUT/s$i
  LOGN=${LOGN:-25} timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex k_ntt -f csv -d $D -o run -- python3 tools/ntt_timing.py > $D.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $D.log; exit 1; }
  find $D -name '*counter_collection.csv' -exec cp {} $OUT/s$i.csv \;
done
python3 - $OUT <<'PY'
import csv, sys, statistics, collections, re
out = sys.argv[1]
for i in (1, 2, 3):
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{out}/s{i}.csv")):
        k = re.search(r"k_ntt_\w+", r["Kernel_Name"]).group(0)
        by[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in sorted(by.items()):
        print(i, k, {n: int(statistics.median(v)) for n, v in c.items()})
PY
