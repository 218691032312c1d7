"""Reduce tools/gpu_r06_acc.sh's accumulator passes to profiles/pmc_acc_valu.json
(the throughput legs' VALU roofline that bench.py accum_valu_roofline reads).

Per batch size B (one pm_accum_batch_proofs_device call = one launch of each
accumulator kernel): per kernel the median SQ_INSTS_VALU / SQ_INSTS_VALU_INT64
wave-instructions per dispatch (the --pmc pass, p1.csv), its mean duration
from the kernel trace of the same workload (kernel_stats.csv), and the issue
time those instructions need at the measured peaks -- the INT64 class at the
v_mad_u64_u32 peak (33.944 T lane-ops/s), every other VALU instruction at the
simple-op peak (61.164 T/s), profiles/valu_peak.json -- over that duration
(issue_frac).  Per batch: the sums over the kernels.

Usage: python tools/acc_valu.py profiles/r06/acc   (directories b<B>/ inside)
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INT64_PEAK_T = 33.944
SIMPLE_PEAK_T = 61.164


def short(name):
    name = name.replace("void ", "").replace("pm::", "")
    return name.split("<")[0].split("(")[0].strip()


def median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def reduce_b(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    kname = {}
    for r in csv.DictReader(open(os.path.join(d, "p1.csv"))):
        k = r["Dispatch_Id"]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        kname[k] = short(r["Kernel_Name"])
    per = collections.defaultdict(list)
    for k, c in agg.items():
        per[kname[k]].append(c)
    dur = {}
    for r in csv.DictReader(open(os.path.join(d, "kernel_stats.csv"))):
        dur[short(r["Name"])] = float(r["AverageNs"]) * 1e-9
    kernels, tot_issue, tot_lane = {}, 0.0, 0.0
    for name, rows in sorted(per.items()):
        valu = median([x.get("SQ_INSTS_VALU", 0.0) for x in rows])
        i64 = median([x.get("SQ_INSTS_VALU_INT64", 0.0) for x in rows])
        issue = i64 * 64 / (INT64_PEAK_T * 1e12) + (valu - i64) * 64 / (SIMPLE_PEAK_T * 1e12)
        t = dur.get(name)
        kernels[name] = {"valu_insts": valu, "int64_insts": i64, "waves": median([x.get("SQ_WAVES", 0.0) for x in rows]),
                         "avg_ms": round(t * 1e3, 4) if t else None, "issue_us": round(issue * 1e6, 2),
                         "issue_frac": issue / t if t else None}
        tot_issue += issue
        tot_lane += valu * 64
    return kernels, tot_issue, tot_lane


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r06", "acc")
    out = os.path.join(ROOT, "profiles", "pmc_acc_valu.json")
    res = {"what": __doc__.strip().splitlines()[0], "batches": {}}
    for e in sorted(os.listdir(src)):
        m = re.fullmatch(r"b(\d+)", e)
        if not m or not os.path.exists(os.path.join(src, e, "p1.csv")):
            continue
        kernels, issue, lane = reduce_b(os.path.join(src, e))
        res["batches"][m.group(1)] = {
            "kernels": {k: v for k, v in kernels.items() if v["issue_frac"] is not None},
            "issue_seconds_per_batch": issue, "valu_lane_insts_per_batch": lane,
            "int64_peak_Tops": INT64_PEAK_T, "simple_peak_Tops": SIMPLE_PEAK_T,
            "source": os.path.relpath(os.path.join(src, e), ROOT) + "/{p1.csv,kernel_stats.csv} (tools/gpu_r06_acc.sh)"}
    json.dump(res, open(out, "w"), indent=1)
    for b, d in res["batches"].items():
        print(b, {k: (v["avg_ms"], round(v["issue_frac"], 3)) for k, v in d["kernels"].items()},
              "issue_ms", round(d["issue_seconds_per_batch"] * 1e3, 4))


if __name__ == "__main__":
    main()
