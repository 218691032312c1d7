"""Gap analysis of a rocprofv3 kernel trace: for the last calls of a repeated
workload, every kernel's start / end relative to the first kernel of its call
(a call starts at each `first` kernel name)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "k_tr_canon"
calls, cur = [], None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("pm::", "")
    if first in name:
        cur = []
        calls.append(cur)
    if cur is not None:
        cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for c in calls[-3:]:
    t0 = c[0][1]
    print("call: %.1f us" % ((max(e for _, _, e in c) - t0) / 1e3))
    for name, s, e in c:
        print("  %-28s %8.1f %8.1f  (%6.1f)" % (name[:28], (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
if len(calls) > 2:
    prev_end = max(e for _, _, e in calls[-2])
    print("idle between calls: %.1f us" % ((calls[-1][0][1] - prev_end) / 1e3))
