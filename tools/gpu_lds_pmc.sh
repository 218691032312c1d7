#!/bin/bash
# LDS bank conflicts / waits of every kernel: the resident 2^20 MSM
# (tools/msm_timing.py) and the B = 256 accumulator (tools/accum_timing.py),
# one rocprofv3 --pmc pass each.  Usage (through gpurun): bash tools/gpu_lds_pmc.sh TAG
set -o pipefail
TAG=${1:-lds}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
LOGN=20 RESIDENT=1 REPS=3 timeout -s KILL 120 rocprofv3 --pmc $P -f csv -d $OUT/msm -o run -- python3 tools/msm_timing.py > $OUT/msm.log 2>&1 || { echo "msm pass failed"; tail -20 $OUT/msm.log; exit 1; }
find $OUT/msm -name '*counter_collection.csv' -exec cp {} $OUT/msm.csv \;
timeout -s KILL 120 rocprofv3 --pmc $P -f csv -d $OUT/acc -o run -- python3 tools/accum_timing.py > $OUT/acc.log 2>&1 || { echo "acc pass failed"; tail -20 $OUT/acc.log; exit 1; }
find $OUT/acc -name '*counter_collection.csv' -exec cp {} $OUT/acc.csv \;
python3 - $OUT <<'PY'
import csv, sys, statistics, collections, re
out = sys.argv[1]
for f in ("msm", "acc"):
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{out}/{f}.csv")):
        k = re.sub(r"<.*", "", r["Kernel_Name"].replace("void ", "").replace("pm::", ""))[:28]
        by[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in by.items():
        m = {n: statistics.median(v) for n, v in c.items()}
        if m.get("SQ_INSTS_LDS", 0) == 0: continue
        print(f, k, "conflict/idx=%.2f" % (m["SQ_LDS_BANK_CONFLICT"] / max(1, m["SQ_LDS_IDX_ACTIVE"])),
              "ldswait/wave=%.2f" % (m["SQ_WAIT_INST_LDS"] / max(1, m["SQ_WAVE_CYCLES"])),
              "valu_active/wave=%.2f" % (m["SQ_ACTIVE_INST_VALU"] / max(1, m["SQ_WAVE_CYCLES"])), {n: int(v) for n, v in m.items()})
PY
