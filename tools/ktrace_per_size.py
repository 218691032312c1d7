"""Per-kernel duration summary (mean, median, deciles) from a rocprofv3
kernel_trace.csv. The median of a headline-only bench run (`--logn22 0 ...`)
is the resident 2^20 launch that bench.py's roofline averages with HIP
events; the mean also holds the settle ramp and the raw-bases leg.
Usage: python tools/ktrace_per_size.py <kernel_trace.csv> [name-substring ...]"""
import collections
import csv
import json
import statistics
import sys


def main():
    path, names = sys.argv[1], sys.argv[2:] or ["k_accumulate"]
    groups = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not any(s in name for s in names):
            continue
        grid = int(r.get("Grid_Size") or 0)
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        groups[(name.split("(")[0], grid)].append(dur)
    for (name, grid), d in sorted(groups.items()):
        print(json.dumps({"kernel": name, "grid": grid, "launches": len(d), "mean_ms": round(statistics.mean(d), 4),
                          "median_ms": round(statistics.median(d), 4),
                          "p10_ms": round(sorted(d)[len(d) // 10], 4), "p90_ms": round(sorted(d)[9 * len(d) // 10], 4),
                          "min_ms": round(min(d), 4), "max_ms": round(max(d), 4)}))


if __name__ == "__main__":
    main()
