"""Gap analysis of a rocprofv3 kernel trace: for some calls of a repeated
workload, every kernel's start / end relative to the first kernel of its call
(a call starts at each `first` kernel name).  argv: trace.csv [first kernel]
[call indices, default "3,4" -- the timing tools run untimed calls first and
then calls with per-kernel HIP events, whose event pairs add ~10 us gaps]."""
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
idx = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "3,4").split(",")]
for c in [calls[i] for i in idx if -len(calls) <= i < len(calls)]:
    t0 = c[0][1]
    print("call: %.1f us" % ((max(e for _, _, e in c) - t0) / 1e3))
    for name, s, e in c:
        print("  %-28s %8.1f %8.1f  (%6.1f)" % (name[:28], (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
if len(calls) > max(idx) + 1:
    prev_end = max(e for _, _, e in calls[max(idx)])
    print("idle between calls: %.1f us" % ((calls[max(idx) + 1][0][1] - prev_end) / 1e3))
