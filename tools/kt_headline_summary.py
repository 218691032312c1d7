"""k_accumulate<PallasFp> launches of the headline leg in a rocprofv3 kernel
trace of bench.py (tools/gpu_r06_kt_final.sh): the launches before the first
k_bases_to_r261 (the variable-base leg's first kernel) are the headline leg's
(settle, warmup, timed steps, breakdown).  argv: kernel_trace.csv"""
import csv
import json
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
acc = []
for r in rows:
    name = r["Kernel_Name"]
    if "k_bases_to_r261" in name:
        break
    if "k_accumulate<pm::PallasFp>" in name:
        acc.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
acc.sort()
n = len(acc)
print(json.dumps({"kernel": "k_accumulate<pm::PallasFp>", "leg": "headline (2^20, resident 8-row table)",
                  "launches": n, "mean_ms": round(sum(acc) / n, 4), "median_ms": round(acc[n // 2], 4),
                  "min_ms": round(acc[0], 4), "max_ms": round(acc[-1], 4)}))
