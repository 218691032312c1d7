#!/bin/bash
# PMC HBM traffic of the NTT kernels (separate --pmc passes, kernel trace
# stats alongside) for bench.py's ntt leg.  Usage: bash tools/gpu_ntt_pmc.sh TAG
set -o pipefail
TAG=${1:-ntt}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# NTT_ARGS: which legs run (default the 2^20 leg); e.g. "--ntt-logn 0 --ntt-large-logn 25" for 2^25
BENCH="python3 bench.py --no-cpu --fixed 0 --accum-batch 0 --accum-b16 0 --logn22 0 --strong-logn 0 --small-n 0 --steps 5 --warmup 1 ${NTT_ARGS:---ntt-large-logn 0}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- $BENCH > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_ntt -f csv -d $OUT/pmc_$C -o run -- $BENCH > $OUT/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -20 $OUT/pmc_$C.log; exit 1; }
  find $OUT/pmc_$C -name '*counter_collection.csv' -exec cp {} $OUT/pmc_$C.csv \;
done
python3 - "$OUT" <<'PY'
import csv, sys, statistics, json
out = sys.argv[1]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = list(csv.DictReader(open(f"{out}/pmc_{c}.csv")))
    by = {}
    for r in rows:
        if r["Counter_Name"] != c:
            continue
        k = next((x for x in ("k_ntt_cols", "k_ntt_mid", "k_ntt_rows") if x in r["Kernel_Name"]), None)
        if k:
            by.setdefault(k, []).append(float(r["Counter_Value"]))
    res[c] = {k: statistics.median(v) for k, v in by.items()}
print(json.dumps(res))
json.dump(res, open(f"{out}/pmc_summary.json", "w"))
PY
