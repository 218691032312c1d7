"""Reduce the NTT VALU PMC passes (tools/gpu_ntt_valu_r04.sh; CSV copies in
profiles/r04/ntt_valu/valu_n{20,25}.csv) to the "valu" entry of each NTT
workload in profiles/pmc_ntt.json, which bench.py adds to the ntt legs'
roofline as valu_int.  Same issue model as tools/pmc_valu.py: the INT64 class
issues at 33.944 T lane-ops/s, the rest at 61.164 T (measured peaks,
profiles/r01_s3/microbench_isa.jsonl), so
issue_frac = (INT64 * 64 / 33.944T + (VALU - INT64) * 64 / 61.164T) / (sum of the passes' durations).

Usage: python tools/ntt_valu.py profiles/r04/ntt_valu"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INT64_PEAK_T = 33.944
SIMPLE_PEAK_T = 61.164


def median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def main():
    src = sys.argv[1]
    rel = os.path.relpath(src, ROOT)
    p = os.path.join(ROOT, "profiles", "pmc_ntt.json")
    d = json.load(open(p))
    for lg in (20, 25):
        f = os.path.join(src, f"valu_n{lg}.csv")
        if not os.path.exists(f):
            continue
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        dur, kern = {}, {}
        for r in csv.DictReader(open(f)):
            dd = r["Dispatch_Id"]
            agg[dd][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[dd] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            kern[dd] = re.search(r"k_ntt_\w+", r["Kernel_Name"]).group(0)
        per = {}
        for k in sorted(set(kern.values())):
            ds = [dd for dd in agg if kern[dd] == k and k != "k_ntt_twiddles"]
            if not ds:
                continue
            v = median([agg[dd]["SQ_INSTS_VALU"] for dd in ds])
            i64 = median([agg[dd]["SQ_INSTS_VALU_INT64"] for dd in ds])
            s = median([dur[dd] for dd in ds])
            need = i64 * 64 / (INT64_PEAK_T * 1e12) + (v - i64) * 64 / (SIMPLE_PEAK_T * 1e12)
            per[k] = {"valu_insts": int(v), "int64_insts": int(i64), "profiled_ms": round(s * 1e3, 4),
                      "issue_frac": round(need / s, 4)}
        tot_need = sum(x["int64_insts"] * 64 / (INT64_PEAK_T * 1e12)
                       + (x["valu_insts"] - x["int64_insts"]) * 64 / (SIMPLE_PEAK_T * 1e12) for x in per.values())
        tot_s = sum(x["profiled_ms"] for x in per.values()) * 1e-3
        i64_all = sum(x["int64_insts"] for x in per.values())
        wl = f"ntt_bn254_2^{lg}"
        d.setdefault("workloads", {}).setdefault(wl, {})["valu"] = {
            "per_kernel": per, "issue_frac": round(tot_need / tot_s, 4),
            "int64_Tops": round(i64_all * 64 / tot_s / 1e12, 3), "int64_peak_Tops": INT64_PEAK_T,
            "int64_frac": round(i64_all * 64 / tot_s / 1e12 / INT64_PEAK_T, 4),
            "source": f"{rel}/valu_n{lg}.csv (rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 ...; "
                      "tools/gpu_ntt_valu_r04.sh, tools/ntt_valu.py)"}
        print(wl, json.dumps(d["workloads"][wl]["valu"]))
    json.dump(d, open(p, "w"), indent=1)


if __name__ == "__main__":
    main()
