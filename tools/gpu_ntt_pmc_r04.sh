#!/bin/bash
# NTT 2^25 (three passes) PMC: FETCH_SIZE, WRITE_SIZE (separate passes, for
# profiles/pmc_ntt.json), the SQ wait / issue set and the TCP translation /
# L2-read counters of every pass; driver tools/ntt_timing.py (LOGN=25).
# Usage (through gpurun, from the repo root): bash tools/gpu_ntt_pmc_r04.sh TAG
set -o pipefail
TAG=${1:-ntt_pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="FETCH_SIZE"
P2="WRITE_SIZE"
P3="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"
P4="TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  D=$OUT/s$i
  LOGN=${LOGN:-25} timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex k_ntt -f csv -d $D -o run -- python3 tools/ntt_timing.py > $D.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $D.log; exit 1; }
  find $D -name '*counter_collection.csv' -exec cp {} $OUT/s$i.csv \;
done
LOGN=${LOGN:-25} timeout -k 10 120 python3 tools/ntt_timing.py > $OUT/timing.jsonl 2>&1 || exit 1
cat $OUT/timing.jsonl
python3 - $OUT <<'PY'
import csv, sys, statistics, collections, re
out = sys.argv[1]
for i in (1, 2, 3, 4):
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{out}/s{i}.csv")):
        k = re.search(r"k_ntt_\w+", r["Kernel_Name"]).group(0)
        by[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in sorted(by.items()):
        print(i, k, {n: int(statistics.median(v)) for n, v in c.items()})
PY
