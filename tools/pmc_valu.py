"""Reduce the k_accumulate PMC passes of tools/gpu_pmc_r02.sh (CSV copies under
profiles/<round>/pmc/) to the two JSON files bench.py reads:

  profiles/pmc_valu.json        per workload: VALU wave-instructions per launch
                                (all / INT64 / INT32), the issue-slot fraction
                                they occupy, and the measured issue peaks;
  profiles/pmc_accumulate.json  per workload: FETCH_SIZE + WRITE_SIZE bytes per
                                launch (HBM-side traffic, MI355X_MICROARCH.md).

Issue peaks (profiles/r01_s3/microbench_isa.jsonl, 4 waves per SIMD = the
occupancy of k_accumulate): v_mad_u64_u32 33.944 T lane-ops/s (8 independent
chains), v_and_b32 61.164 T/s.  The INT64 class (multiply-adds, 64-bit shifts
and adds) issues at the former, every other VALU instruction at the latter, so
issue_frac = (INT64 * 64 / 33.944T + (VALU - INT64) * 64 / 61.164T) / duration.

Usage: python tools/pmc_valu.py profiles/r03/pmc [per_gpu|raw]
  (per_gpu: the headline's resident row-table MSM, RESIDENT=1; raw: the
  plain pipeline from raw device bases, bench.py's variable_base leg)
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INT64_PEAK_T = 33.944
SIMPLE_PEAK_T = 61.164


def kernel_label(path):
    """'k_accumulate<PallasFp,true>' from the CSV's kernel name"""
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("void ", "").replace("pm::", "").split("(")[0]
        return name.replace(", ", ",")
    return "k_accumulate"


def per_dispatch(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(path)):
        d = r["Dispatch_Id"]
        agg[d][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return agg, dur


def median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r02", "pmc")
    suffix = sys.argv[2] if len(sys.argv) > 2 else "per_gpu"  # workload key: pallas_msm_2^lg_<suffix>
    rel = os.path.relpath(src, ROOT)
    pv = os.path.join(ROOT, "profiles", "pmc_valu.json")
    pa = os.path.join(ROOT, "profiles", "pmc_accumulate.json")
    # merge into the existing files: other workloads' entries stay
    valu = json.load(open(pv)) if os.path.exists(pv) else {}
    traffic = json.load(open(pa)).get("workloads", {}) if os.path.exists(pa) else {}
    for lg in (19, 20, 22):
        f1 = os.path.join(src, f"n{lg}_p1.csv")
        if not os.path.exists(f1):
            continue
        wl = f"pallas_msm_2^{lg}_{suffix}"
        agg, dur = per_dispatch(f1)
        # the first dispatch of the driver is a warm-up with cold caches; take medians
        c = {k: median([agg[d][k] for d in agg]) for k in next(iter(agg.values()))}
        s = median(list(dur.values()))
        v, i64 = c["SQ_INSTS_VALU"], c["SQ_INSTS_VALU_INT64"]
        need = i64 * 64 / (INT64_PEAK_T * 1e12) + (v - i64) * 64 / (SIMPLE_PEAK_T * 1e12)
        adds = (1 << lg) * 16  # n x W bucket additions (W = 16 windows at c = 16)
        valu[wl] = {"kernel": kernel_label(f1),
                    "valu_insts_per_launch": int(v), "int64_insts_per_launch": int(i64),
                    "int32_insts_per_launch": int(c["SQ_INSTS_VALU_INT32"]),
                    "salu_insts_per_launch": int(c.get("SQ_INSTS_SALU", 0)),
                    "valu_lane_insts_per_bucket_add": round(v * 64 / adds, 1),
                    "int64_lane_insts_per_bucket_add": round(i64 * 64 / adds, 1),
                    "profiled_launch_ms": round(s * 1e3, 4),
                    "grbm_gui_active_per_xcd": int(c["GRBM_GUI_ACTIVE"] / 8),
                    "issue_frac": round(need / s, 4),
                    "int64_peak_Tops": INT64_PEAK_T, "simple_peak_Tops": SIMPLE_PEAK_T,
                    "source": f"{rel}/n{lg}_p1.csv (rocprofv3 --pmc, SQ pass; tools/gpu_pmc_r02.sh)"}
        if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
            valu[wl]["wait_inst_frac"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
        fe, _ = per_dispatch(os.path.join(src, f"n{lg}_p2.csv"))
        wr, _ = per_dispatch(os.path.join(src, f"n{lg}_p3.csv"))
        fkb = median([fe[d]["FETCH_SIZE"] for d in fe])
        wkb = median([wr[d]["WRITE_SIZE"] for d in wr])
        traffic[wl] = {"kernel": kernel_label(f1), "fetch_size_kb_median": fkb,
                       "write_size_kb_median": wkb, "hbm_bytes_per_launch": int((fkb + wkb) * 1024),
                       "launches_per_msm": 1,
                       "source": f"{rel}/n{lg}_p2.csv, n{lg}_p3.csv (separate --pmc FETCH_SIZE / WRITE_SIZE passes)",
                       "note": "L2 memory-side requests (Infinity-Cache hits included); no x2 streaming "
                               "correction: the dominant reads are random 64-B base gathers, one 128-B line "
                               "each. Algorithmic bytes are 96 B x n (SURVEY 8d)."}
    json.dump(valu, open(pv, "w"), indent=1)
    json.dump({"workloads": traffic}, open(pa, "w"), indent=1)
    print(json.dumps(valu, indent=1))
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
