"""Hardware latency floor of the accumulator's dependent steps (round 5,
VERDICT r4 item 1): each step's loop body in the gfx950 listing of the
microbenchmarks that time it in isolation, counted by instruction class, times
the single-wave issue cost of that class measured on MI355X (one wave per
SIMD, profiles/r01_s3/microbench_isa.jsonl):

  v_mad_u64_u32 / v_mad_i64_i32   3.815 ns  (mad_8chain, 17.18 T lane-op/s / 65536 lanes)
  every other VALU op (incl. DPP) 2.206 ns  (and_b32, 29.70 T/s)
  s_nop N                         (N + 1) cycles at 2.4 GHz
  other SALU / branch             1 cycle
  LDS (ds_*)                      2.206 ns issue (its latency is not counted)

A lone wave cannot retire a chain faster than it can issue the chain's
instructions, so sum(count x cost) is a floor set by the hardware, not by this
code's own step latency (the round-4 floor).  The measured step latency
(chain_latency.jsonl / microbench_slice.jsonl) over this floor says how much
of a step is dependency stalls on top of issue.

Usage: python tools/hw_floor.py > profiles/r05/hw_floor.json
  (compiles tools/microbench_chain.hip and tools/microbench_slice.hip to gfx950
  assembly with hipcc -S; no GPU needed)"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLK_NS = 1 / 2.4


def issue_costs():
    """ns per instruction of one lone wave, by class: the round-5 measurement
    in the chains' own configuration (tools/microbench_issue.hip, one wave per
    CU) when present, else round 1's one-wave-per-SIMD figures"""
    c = {"mad64": 65536 / 17.180e12 * 1e9, "valu": 65536 / 29.702e12 * 1e9, "dpp": 65536 / 29.702e12 * 1e9,
         "lds": 65536 / 29.702e12 * 1e9, "salu": CLK_NS}
    src = "profiles/r01_s3/microbench_isa.jsonl (waves_per_simd 1)"
    p = os.path.join(ROOT, "profiles", "r05", "issue_costs.jsonl")
    if os.path.exists(p):
        m = {}
        for line in open(p):
            if line.startswith("{"):
                d = json.loads(line)
                if "form" in d:
                    m[d["form"]] = d["ns_per_instruction"]
        c["mad64"] = m.get("v_mad_u64_u32 independent", c["mad64"])
        c["valu"] = m.get("v_and_b32 independent", c["valu"])
        c["dpp"] = m.get("v_mov_b32_dpp row_newbcast independent", c["valu"])
        c["lds"] = c["valu"]  # issue only; the exchange latency is in the measured step
        src = "profiles/r05/issue_costs.jsonl (tools/microbench_issue.hip, one wave per CU)"
    return c, src


COST_NS, COST_SRC = issue_costs()

# (step, listing, kernel-name regex, what one loop iteration is)
STEPS = [
    ("f29_mul", "chain", r"k_chainIN2pm10Bn254CurveELi0E", "one radix-2^29 product, one lane"),
    ("f29_sqr", "chain", r"k_chainIN2pm10Bn254CurveELi1E", "one radix-2^29 square, one lane"),
    ("fe_mul", "chain", r"k_chainIN2pm10Bn254CurveELi2E", "one 8x32-bit FIPS product (k_acc_scalars)"),
    ("ladder_dbl", "chain", r"k_chainIN2pm10Bn254CurveELi3E", "one quad-cooperative Jacobian doubling"),
    ("xyzz_add", "chain", r"k_chainIN2pm10Bn254CurveELi4E", "one XYZZ addition, one lane (k_acc_termadd)"),
    ("xyzz_add_q", "chain", r"k_chainIN2pm10Bn254CurveELi5E", "one quad-cooperative XYZZ addition (k_acc_sum)"),
    ("b2_compress_q", "chain", r"k_chainIN2pm10Bn254CurveELi9E", "one quad Blake2b compression (k_transcript)"),
    ("s29_mul", "slice", r"k_sliceIN2pm7Bn254FqE", "one row-sliced product (decode sqrt, sliced ladder)"),
]


def listing(src):
    out = os.path.join(tempfile.gettempdir(), os.path.basename(src) + ".s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-w", "--offload-arch=gfx950", "--cuda-device-only",
                    "-S", "-o", out, src], check=True, capture_output=True)
    return open(out).read().split("\n")


def loop_body(lines, pat):
    """instructions of the outermost loop of the first kernel matching pat"""
    i = next(k for k, l in enumerate(lines) if re.match(r"^_Z\w*" + pat + r"\w*:", l))
    j = i
    while not lines[j].startswith(".Lfunc_end"):
        j += 1
    body = lines[i:j]
    labels = {l.split(":")[0]: k for k, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
    best = None
    for k, l in enumerate(body):
        m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            span = (labels[m.group(1)], k)
            if best is None or span[1] - span[0] > best[1] - best[0]:
                best = span
    ops = []
    for l in body[best[0]:best[1] + 1]:
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        ops.append(t)
    inner = sum(1 for k, l in enumerate(body[best[0] + 1:best[1]])
                if re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
                and labels.get(re.match(r"\s+s_\w+\s+(\.LBB\d+_\d+)", l).group(1), 1 << 30) <= best[0] + 1 + k
                and labels.get(re.match(r"\s+s_\w+\s+(\.LBB\d+_\d+)", l).group(1), -1) > best[0])
    return ops, inner


def classify(ops):
    c = collections.Counter()
    ns = 0.0
    for t in ops:
        op = t.split()[0]
        if op.startswith(("v_mad_u64_u32", "v_mad_i64_i32")):
            k = "mad64"
        elif op.startswith("v_") and ("_dpp" in op or "row_" in t or "quad_perm" in t):
            k = "dpp"
        elif op.startswith("v_"):
            k = "valu"
        elif op.startswith("ds_"):
            k = "lds"
        elif op == "s_nop":
            c["s_nop_cycles"] += int(t.split()[1]) + 1
            ns += (int(t.split()[1]) + 1) * CLK_NS
            continue
        elif op.startswith("s_"):
            k = "salu"
        else:
            k = "other"
        c[k] += 1
        ns += COST_NS.get(k, 0.0)
    return c, ns


def measured():
    m = {}
    for p in ("profiles/r04/chain_latency.jsonl", "profiles/r05/chain_latency.jsonl"):
        p = os.path.join(ROOT, p)
        if os.path.exists(p):
            for line in open(p):
                if line.startswith("{"):
                    d = json.loads(line)
                    if "step" in d:
                        m[d["step"]] = d["us_per_step"]
    p = os.path.join(ROOT, "profiles", "r05", "microbench_slice.jsonl")
    if os.path.exists(p):
        for line in open(p):
            if line.startswith("{"):
                d = json.loads(line)
                if d.get("field") == "bn254_fq" and "sliced_us_per_mul" in d:
                    m["s29_mul"] = d["sliced_us_per_mul"]
    return m


def sqrt_products():
    """row-sliced products of one BN254 decompression (proof_kernels.hpp
    sqrt_pow_s over make_schedule's 4-bit sliding window of (p + 1) / 4):
    a^2, 7 odd powers, then the schedule's squarings and multiplications"""
    p = 21888242871839275222246405745257275088696311157297823662689037894645226208583
    e = (p + 1) // 4
    bits = [(e >> i) & 1 for i in range(256)]
    i = 255
    while i >= 0 and not bits[i]:
        i -= 1
    sq = mul = 0
    first = True
    while i >= 0:
        if not bits[i]:
            sq += 1
            i -= 1
            continue
        j = max(i - 3, 0)
        while not bits[j]:
            j += 1
        if not first:
            sq += i - j + 1
            mul += 1
        first = False
        i = j - 1
    return {"squarings": sq, "multiplications": mul, "table": 8, "total": sq + mul + 8}


def main():
    srcs = {"chain": listing(os.path.join(ROOT, "tools", "microbench_chain.hip")),
            "slice": listing(os.path.join(ROOT, "tools", "microbench_slice.hip"))}
    meas = measured()
    out = {"what": __doc__.split("\n\n")[0].replace("\n", " "), "cost_ns": COST_NS, "cost_source": COST_SRC,
           "clock_GHz": 2.4, "steps": {}, "bn254_sqrt_products": sqrt_products()}
    for step, src, pat, what in STEPS:
        ops, inner = loop_body(srcs[src], pat)
        c, ns = classify(ops)
        row = {"what": what, "counts": dict(c), "issue_floor_us": round(ns / 1e3, 4)}
        if inner:
            row["note"] = "the loop body holds inner loops: static count, not a floor"
        if step in meas:
            row["measured_us"] = meas[step]
            row["measured_over_floor"] = round(meas[step] / (ns / 1e3), 2)
        out["steps"][step] = row
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
