#!/bin/bash
# SQ counters of k_accumulate (one pass, SQ block: up to 8 counters)
set -o pipefail
OUT=gpurun_out/${1:-pmc_sq}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex k_accumulate -f csv -d $OUT/p -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 --accum-batch 0 > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
find $OUT/p -name '*counter_collection.csv' -exec cp {} $OUT/sq.csv \;
python3 - <<'PY'
import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq/sq.csv")))
agg = collections.defaultdict(list)
for r in rows: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items(): print(k, sorted(v)[len(v)//2])
PY
