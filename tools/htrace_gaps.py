"""Host-side view of the gap between consecutive MSM calls: from a rocprofv3
kernel trace + HIP API trace, for call i (a call starts at each `first`
kernel), list the HIP API calls issued between the end of call i's last
kernel and the start of call i+1's first kernel, and the API time spent
while call i's kernels ran.  argv: kernel_trace.csv hip_api_trace.csv
[first kernel] [call indices]."""
import csv
import sys

kt = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
api = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[3] if len(sys.argv) > 3 else "k_sort_hist"
idx = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "2,3").split(",")]
calls, cur = [], None
for r in kt:
    name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("pm::", "")
    if first in name:
        cur = []
        calls.append(cur)
    if cur is not None:
        cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for i in idx:
    if i + 1 >= len(calls):
        break
    c, nx = calls[i], calls[i + 1]
    k0, kend, n0 = c[0][1], max(e for _, _, e in c), nx[0][1]
    print("call %d: kernels %.1f us, idle until next call %.1f us" % (i, (kend - k0) / 1e3, (n0 - kend) / 1e3))
    tot = {}
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < k0 - 200000 or s > n0:
            continue
        f = r["Function"]
        if s >= kend - 1000 or e >= kend:
            print("   %-32s %9.1f %9.1f  (%7.1f)" % (f[:32], (s - kend) / 1e3, (e - kend) / 1e3, (e - s) / 1e3))
        else:
            tot[f] = tot.get(f, 0) + (e - s)
    print("   API time before the last kernel ended (us):",
          {k: round(v / 1e3, 1) for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:12]})
