"""bench.py -- Pallas MSM throughput on MI355X (BASELINE.json metric).

python bench.py --gpus N --steps K --warmup W   (N>1: launched by torch.distributed.run)

One step = one Pallas MSM over this rank's slice of 2^20 (scalar, base) pairs
(rank r owns pairs [r*2^20, (r+1)*2^20) of an N*2^20-point MSM, weak scaling),
with scalars and bases already resident in HBM, plus the exchange step: an
all-gather of the per-rank partial points over RCCL and their fold on the host
(EC addition is not limb-wise, so no all-reduce).  `value` = N*2^20 / step time.

`roofline` is for the dominant kernel (k_accumulate), its duration measured
live with HIP events on the context stream over the timed region.  The
headline runs against the resident SRS bases (their row table, like
params.g in halo2); `variable_base` is the same MSM from raw bases (non-SRS
bases, e.g. the verifier's proof commitments) with its own roofline,
`dropin_pm_msm` the literal pm_msm_ctx drop-in call with host inputs (first, admitting and
warm), `small_n` its latency against the C port for n = 2^0 .. 2^16.
`cpu_baseline` times the C restatement of halo2 best_multiexp (oracle/msm_ref.c)
on the host cores of the same box, on the same inputs, at N=1 on rank 0.

`accumulator` is the second half of the BASELINE metric ("aggregated proofs
verified/s"): each rank takes its own B = 256 synthetic simple-example proofs
as serialized bytes in HBM, decodes them on the device (point decompression,
canonical checks: halo2's read_point / read_scalar), replays the Blake2b
transcript and runs the batch multiopen accumulator on the replayed challenges
(pm_accum_batch_proofs_device, SURVEY §8 rows a-3..a-9 + §8f-2; BN254, k = 17;
weak scaling, proofs are independent), followed by an all-gather of the B x 4
accumulator points over RCCL.  Its cpu_baseline is the C restatement of the
same work from the same bytes (oracle/accum_ref.c, all host threads) over the
GPU's whole batch, with a bit-exact check of every proof's challenges, quad and
h_eval.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "halo2-aggregation_amd"))

METRIC = "Pallas MSM Mscalar/s at 2^20 (1/2/4/8 GPU); aggregated proofs verified/s"
LOGN = 20
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_PAIR = 96            # 32 B scalar + 64 B affine base
SEED_SCALARS, SEED_BASES = 0x5EED, 0xA11CE


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--logn", type=int, default=LOGN)
    ap.add_argument("--window", type=int, default=0, help="force window width c (0 = auto)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--fixed", type=int, default=1, help="also time the fixed-base MSM (1) or skip it (0)")
    ap.add_argument("--ntt-logn", type=int, default=20, help="NTT leg size (0 = skip)")
    ap.add_argument("--ntt-large-logn", type=int, default=25,
                    help="second NTT leg, three-pass form (create_proof at k = 23 transforms 2^25) (0 = skip)")
    ap.add_argument("--accum-batch", type=int, default=256, help="proofs per GPU for the accumulator leg (0 = skip)")
    ap.add_argument("--accum-logn", type=int, default=17)
    ap.add_argument("--logn22", type=int, default=1,
                    help="also time the 2^22 Pallas MSM per GPU (north-star size, weak scaling) (1) or skip it (0)")
    ap.add_argument("--fixed23", type=int, default=1,
                    help="also time the fixed-base MSM at 2^23 per GPU (the outer prover's k = 23 commit) (1) or skip (0)")
    ap.add_argument("--strong-logn", type=int, default=22,
                    help="strong-scaling leg: a fixed 2^k Vesta MSM split over the ranks (SURVEY config 4); 0 = skip")
    ap.add_argument("--small-n", type=int, default=1, help="drop-in latency curve n = 2^0..2^16 vs the C port (1/0)")
    ap.add_argument("--inst-batch", type=int, default=256,
                    help="instance-commitment leg: proofs per GPU (pm_msm_resident_many, 0 = skip)")
    ap.add_argument("--inst-npub", type=int, default=1, help="public inputs per proof (simple-example: 1)")
    ap.add_argument("--accum-b32", type=int, default=1,
                    help="config 5's per-rank share: 32 proofs at k = 17 per GPU (1/0)")
    ap.add_argument("--accum-large", type=int, default=4096,
                    help="throughput leg: one batch of this many proofs per GPU in ONE call (0 = skip)")
    ap.add_argument("--accum-b16", type=int, default=1,
                    help="also time BASELINE config 3: 16 simple-example proofs at k = 14 per GPU (1) or skip (0)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rendezvous check only: no GPU work (gloo), prints the JSON skeleton")
    ap.add_argument("--detail", default=DETAIL_DEFAULT,
                    help="file for the full per-leg record (kernel breakdowns, small_n curve, configs); "
                         "the stdout line carries only compact leg summaries ('' = do not write it)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# output: ONE compact stdout line (the driver parses it; round 5's 22 KB line
# was not parsed) + the full record in a JSON file beside it
# ---------------------------------------------------------------------------
DETAIL_DEFAULT = os.path.join("profiles", "bench_detail_last.json")
LINE_LIMIT = 12000                 # bytes; tests/test_bench_line.py holds the line to it
CONTRACT_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                 "scaling", "vs_baseline", "dtype", "data")
ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "avg_launch_ms",
             "alg_bytes_per_launch")
CPU_KEYS = ("value", "unit", "cores", "kind", "sample", "matches_gpu")


def _r(v, nd=4):
    return round(v, nd) if isinstance(v, float) else v


def leg_summary(leg):
    """value / unit / ms / frac / matches of one sub-leg (the verbose fields
    stay in the detail file)."""
    s = {"value": _r(leg.get("value")), "unit": leg.get("unit")}
    for k in ("ms_per_step", "ms_per_batch", "ms_per_ntt", "warm_ms_per_msm"):
        if k in leg:
            s["ms"] = _r(leg[k])
            break
    roof = leg.get("roofline")
    if isinstance(roof, dict):
        s["frac"] = _r(roof.get("frac"), 5)
        s["bound"] = roof.get("bound")
    matches = [v for k, v in leg.items() if (k.startswith("matches") or k.startswith("quads_match"))
               and isinstance(v, bool)]
    for sub in ("from_decoded", "per_proof_loop"):
        if isinstance(leg.get(sub), dict):
            matches += [v for k, v in leg[sub].items() if k.startswith(("matches", "quads_match"))
                        and isinstance(v, bool)]
    if isinstance(leg.get("cpu_baseline"), dict):
        cb = leg["cpu_baseline"]
        s["cpu"] = {"value": _r(cb.get("value")), "cores": cb.get("cores"), "kind": cb.get("kind")}
        for k in ("matches_gpu", "matches"):
            if isinstance(cb.get(k), bool):
                matches.append(cb[k])
    if "status_nonzero" in leg:
        matches.append(leg["status_nonzero"] == 0)
    two = leg.get("two_in_flight")
    if isinstance(two, dict) and two.get("value") is not None:
        s["two_in_flight"] = _r(two["value"])
        if isinstance(two.get("quads_match_single_runs"), bool):
            matches.append(two["quads_match_single_runs"])
    if matches:
        s["matches"] = all(matches)
    return {k: v for k, v in s.items() if v is not None}


def compact_line(out, detail_path=None):
    """The stdout JSON line: the contract keys, `config` (workload names only),
    `roofline` and `cpu_baseline` of the headline, and one compact summary per
    sub-leg.  Guaranteed under LINE_LIMIT bytes: if the summaries ever grow past
    it, the least important fields go first and the legs last."""
    line = {k: out.get(k) for k in CONTRACT_KEYS}
    cfg = out.get("config") or {}
    line["config"] = {k: cfg[k] for k in ("workload", "curve", "n_per_gpu", "n_total", "parallelism")
                      if k in cfg}
    roof = out.get("roofline")
    if isinstance(roof, dict):
        r = {k: roof.get(k) for k in ROOF_KEYS if k in roof}
        v = roof.get("valu_int")
        if isinstance(v, dict):
            r["valu_int"] = {k: v.get(k) for k in ("achieved", "peak", "unit", "frac", "issue_frac")}
        line["roofline"] = r
    cpu = out.get("cpu_baseline")
    if isinstance(cpu, dict):
        line["cpu_baseline"] = {k: cpu.get(k) for k in CPU_KEYS if k in cpu}
    legs = {}
    for k, v in out.items():
        if k in CONTRACT_KEYS or k in ("config", "roofline", "cpu_baseline", "kernels_ms"):
            continue
        if isinstance(v, dict) and "value" in v:
            legs[k] = leg_summary(v)
        elif k == "small_n" and isinstance(v, dict):
            rows = {r["n"]: r for r in v.get("curve", [])}
            legs[k] = {"gpu_us": {n: rows[n].get("gpu_us") for n in (1, 32, 4096) if n in rows},
                       "gpu_us_fresh_bases": {n: rows[n].get("gpu_us_fresh_bases") for n in (1, 32, 4096)
                                              if n in rows},
                       "matches": all(r.get("match", True) for r in rows.values())}
        elif k == "dropin_pm_msm" and isinstance(v, dict):
            legs[k] = {"value": v.get("warm_Mscalar_s"), "unit": "Mscalar/s", "ms": v.get("warm_ms_per_msm"),
                       "one_copy_ms": v.get("warm_ms_one_copy"), "first_ms": v.get("first_ms"),
                       "matches": v.get("matches")}
        elif k == "host_scalars" and isinstance(v, dict) and isinstance(v.get("pageable"), dict):
            p = v["pageable"]
            one = v.get("pageable_one_copy") if isinstance(v.get("pageable_one_copy"), dict) else {}
            legs[k] = {"value": p.get("Mscalar_s"), "unit": "Mscalar/s", "ms": p.get("ms_per_msm"),
                       "one_copy_ms": one.get("ms_per_msm"), "matches": bool(p.get("matches") and
                                                                             one.get("matches", True))}
    if legs:
        line["legs"] = legs
    if detail_path:
        line["detail"] = detail_path
    s = json.dumps(line, separators=(",", ":"))
    for drop in (("bound", "two_in_flight"), ("cpu",), ("frac", "ms")):
        if len(s) < LINE_LIMIT:
            break
        for leg in legs.values():
            for k in drop:
                leg.pop(k, None)
        s = json.dumps(line, separators=(",", ":"))
    if len(s) >= LINE_LIMIT:
        line.pop("legs", None)
        s = json.dumps(line, separators=(",", ":"))
    return s


def emit(out, detail_path):
    """Write the full record to `detail_path` (when set), then print the
    compact line as the LAST line of stdout."""
    if detail_path:
        try:
            d = os.path.dirname(detail_path)
            if d:
                os.makedirs(d, exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(out, f, indent=1)
        except OSError as e:  # a read-only tree must not cost the headline
            print(f"bench.py: detail file not written: {e}", file=sys.stderr)
            detail_path = None
    print(compact_line(out, detail_path), flush=True)


def cpu_threads():
    """Host threads for the CPU baselines: the CPUs this process may run on
    (sched_getaffinity), capped by OMP_NUM_THREADS when the box sets it (the
    GPU pool gives each 1-GPU job a 16-CPU share while os.cpu_count() reports
    the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_info():
    return {"threads_used": cpu_threads(), "os_cpu_count": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """--gpus N > 1 without a torch.distributed environment: start N ranks
    through torch.distributed.run as a CHILD process (nothing in this process
    has touched the GPU or imported torch yet) and exit with its code.  The
    JSON line is printed by the child's rank 0 on the inherited stdout."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def load_valu_counters(workload, avg_ms):
    """Integer-VALU roofline of k_accumulate from rocprofv3 SQ counters of the
    same kernel on the same workload (profiles/pmc_valu.json, written by
    tools/pmc_valu.py from the committed CSV): v_mad_u64_u32-class (INT64)
    lane-ops per second against the measured 64-bit multiply-add issue peak,
    and the fraction of SIMD issue cycles the counted VALU mix occupies."""
    p = os.path.join(ROOT, "profiles", "pmc_valu.json")
    if not os.path.exists(p):
        return None
    d = json.load(open(p)).get(workload)
    if not d:
        return None
    s = avg_ms * 1e-3
    mad_rate = d["int64_insts_per_launch"] * 64 / s / 1e12
    return {"achieved": round(mad_rate, 3), "peak": d["int64_peak_Tops"], "unit": "T lane-mad64/s",
            "frac": round(mad_rate / d["int64_peak_Tops"], 4),
            "issue_frac": d.get("issue_frac"), "valu_insts_per_launch": d["valu_insts_per_launch"],
            "int64_insts_per_launch": d["int64_insts_per_launch"], "source": d["source"]}


def load_pmc_traffic(workload, launches_per_msm):
    """HBM bytes per k_accumulate launch from the committed PMC passes, if they
    were taken on this workload with the same launch structure."""
    p = os.path.join(ROOT, "profiles", "pmc_accumulate.json")
    if os.path.exists(p):
        d = json.load(open(p)).get("workloads", {}).get(workload)
        if d and d.get("launches_per_msm", 1) == launches_per_msm:
            return d.get("hbm_bytes_per_launch")
    return None


def load_ntt_valu(workload):
    """Integer-VALU fractions of the NTT passes from the committed SQ counters
    (profiles/pmc_ntt.json "valu", tools/ntt_valu.py)."""
    p = os.path.join(ROOT, "profiles", "pmc_ntt.json")
    if os.path.exists(p):
        return json.load(open(p)).get("workloads", {}).get(workload, {}).get("valu")
    return None


def load_ntt_traffic(workload):
    """HBM bytes per NTT (all passes) from the committed PMC passes
    (profiles/pmc_ntt.json: one entry per workload)."""
    p = os.path.join(ROOT, "profiles", "pmc_ntt.json")
    if os.path.exists(p):
        d = json.load(open(p))
        if d.get("workload") == workload:  # single-workload layout
            return d.get("hbm_bytes_per_ntt")
        return d.get("workloads", {}).get(workload, {}).get("hbm_bytes_per_ntt")
    return None


class HostCollectives:
    """PM_BENCH_SHARE_GPU=1: a rehearsal of the N-rank flow on a one-GPU box
    (every leg's collectives, barriers and rank-0 output with world > 1).  All
    ranks run on device 0 -- RCCL refuses two ranks on one device -- and the
    collectives go through gloo on host copies of the device tensors.  The
    numbers of such a run say nothing about scaling; only the driver's
    multi-GPU runs (RCCL over xGMI) do."""

    def __init__(self, d, torch):
        self.d, self.torch, self.ReduceOp = d, torch, d.ReduceOp

    class _Done:
        def wait(self):
            return None

    def barrier(self):
        self.d.barrier()

    def all_reduce(self, t, op=None):
        c = t.cpu()
        self.d.all_reduce(c, op=self.d.ReduceOp.SUM if op is None else op)
        t.copy_(c)

    def all_gather(self, out_list, t):
        parts = [self.torch.empty_like(t, device="cpu") for _ in out_list]
        self.d.all_gather(parts, t.cpu())
        for dst, src in zip(out_list, parts):
            dst.copy_(src)

    def all_gather_into_tensor(self, out, t, async_op=False):
        parts = [self.torch.empty_like(t, device="cpu") for _ in range(self.d.get_world_size())]
        self.d.all_gather(parts, t.cpu())
        out.copy_(self.torch.cat(parts).to(out.device))
        return self._Done() if async_op else None

    def destroy_process_group(self):
        self.d.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        return dry_run(args, rank, world)
    import numpy as np
    import torch

    import halo2_amd as H
    from sharded import combine_partials, points_fold, shard_range, split_range

    share = world > 1 and os.environ.get("PM_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0  # rehearsal: every rank on device 0 (see HostCollectives)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if share:
            dist.init_process_group("gloo")
            dist = HostCollectives(dist, torch)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    n = 1 << args.logn
    curve = H.PALLAS
    ctx = H.Context(local)
    if args.window:
        ctx.set_window(args.window)
    dev = torch.device("cuda", local)
    i0, _ = shard_range(rank, world, n)
    leg = run_msm_leg(args, ctx, dist, dev, world, curve, n, i0, roofline=True, breakdown=True,
                      host_leg=(world == 1))
    d_s, d_b, result = leg.pop("_d_s"), leg.pop("_d_b"), leg.pop("_result")
    gathered = torch.zeros(world * 8, dtype=torch.int64, device=dev)  # one all-gather target

    padd = points_fold(curve)  # the partials' fold: one pm_points_sum call
    fixed = run_fixed_base(args, ctx, dist, dev, world, d_s, d_b, n, gathered, padd, result) if args.fixed else None
    cpu = cpu_baseline(d_s, d_b, n, result, args.cpu_seconds) if (rank == 0 and world == 1 and not args.no_cpu) \
        else None
    del d_s, d_b
    big = None
    if args.logn22:
        # the north-star size: a 2^22 Pallas MSM per GPU (weak scaling)
        n22 = 1 << 22
        big = run_msm_leg(args, ctx, dist, dev, world, curve, n22, shard_range(rank, world, n22)[0], roofline=True,
                          breakdown=True, check_port=(rank == 0 and world == 1 and not args.no_cpu))
        for k in ("_d_s", "_d_b", "_result"):
            big.pop(k)
    strong = None
    if args.strong_logn:
        # SURVEY config 4: ONE fixed 2^k Vesta MSM split over the ranks
        # (strong scaling; sharded.split_range), partials all-gathered + folded
        nt = 1 << args.strong_logn
        lo, cnt = split_range(rank, world, nt)
        strong = run_msm_leg(args, ctx, dist, dev, world, H.VESTA, cnt, lo, roofline=False, breakdown=False,
                             n_total=nt, check_port=(rank == 0 and world == 1 and not args.no_cpu))
        for k in ("_d_s", "_d_b", "_result"):
            strong.pop(k)
    fixed23 = None
    if args.fixed and args.fixed23:
        # the outer prover's commit size (k = 23, examples/simple-example.rs:663,702):
        # 2^23 Pallas pairs per GPU against a 2^23 table (auto c = 20, ~7 GB)
        n23 = 1 << 23
        i23 = shard_range(rank, world, n23)[0]
        s23 = torch.empty((n23, 4), dtype=torch.int64, device=dev)
        b23 = torch.empty((n23, 8), dtype=torch.int64, device=dev)
        ctx.synth_scalars(curve, SEED_SCALARS, i23, n23, s23.data_ptr())
        ctx.synth_bases(curve, SEED_BASES, i23, n23, b23.data_ptr())
        torch.cuda.synchronize()
        want23 = combine_partials(ctx.msm_device(curve, s23.data_ptr(), b23.data_ptr(), n23), dist, dev, padd,
                                  world, gathered)
        fixed23 = run_fixed_base(args, ctx, dist, dev, world, s23, b23, n23, gathered, padd, want23, lg=23)
        del s23, b23
    torch.cuda.empty_cache()
    ntt = run_ntt(args, ctx, dist, dev, world) if args.ntt_logn > 0 else None
    # the extended-domain size of create_proof at k = 23 (three passes); its
    # parity is tests/test_ntt_gpu.py (three-pass form vs the oracle, 2^25
    # properties), no CPU leg
    ntt_big = run_ntt(args, ctx, dist, dev, world, k=args.ntt_large_logn, keep_state=False) \
        if args.ntt_large_logn > 0 else None
    torch.cuda.empty_cache()
    accum = run_accumulator(args, ctx, dist, dev, rank, world) if args.accum_batch > 0 else None
    # BASELINE config 3: 16 simple-example proofs at k = 14 per GPU
    accum16 = run_accumulator(args, ctx, dist, dev, rank, world, B=16, logn=14) if args.accum_b16 else None
    # BASELINE config 5 on 8 GPUs: 256 proofs = 32 per rank (the per-rank slice)
    accum32 = run_accumulator(args, ctx, dist, dev, rank, world, B=32, logn=17, light=True) \
        if args.accum_b32 else None
    inst = run_instance_commitments(args, ctx, dist, dev, rank, world) if args.inst_batch > 0 else None
    # many proofs in one pm_accum_batch_proofs_device call (the stream of a
    # busy aggregator): the batch fills the GPU instead of a latency chain
    accum_large = run_accumulator(args, ctx, dist, dev, rank, world, B=args.accum_large, logn=17, light=True,
                                  two=True) if args.accum_large else None

    if rank == 0:
        out = {
            "metric": METRIC, "value": leg["value"], "unit": "Mscalar/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": leg["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (SplitMix64 scalars in [0,r), bases [a_i]G generated on device)",
            "config": leg["config"],
            "kernels_ms": leg["kernels_ms"],
            "roofline": leg.get("roofline"),  # absent only when --logn puts the leg on the small-MSM path
        }
        for k in ("variable_base", "host_scalars", "dropin_pm_msm", "small_n"):
            if k in leg:
                out[k] = leg[k]
        if cpu is not None:
            out["cpu_baseline"] = cpu
        if big is not None:
            out["logn22"] = big
        if strong is not None:
            out["strong_vesta"] = strong
        if fixed is not None:
            out["fixed_base"] = fixed
        if fixed23 is not None:
            out["fixed_base_2^23"] = fixed23
        if ntt is not None:
            if world == 1 and not args.no_cpu:
                ntt["cpu_baseline"] = ntt_cpu_baseline(*ntt.pop("_state"), budget_s=6.0)
            else:
                ntt.pop("_state", None)
            out["ntt"] = ntt
        if ntt_big is not None:
            out[f"ntt_2^{args.ntt_large_logn}"] = ntt_big
        if accum is not None:
            if world == 1 and not args.no_cpu:
                accum["cpu_baseline"] = accum_cpu_baseline(*accum.pop("_state"), budget_s=8.0)
            else:
                accum.pop("_state", None)
            out["accumulator"] = accum
        if accum16 is not None:
            if world == 1 and not args.no_cpu:
                accum16["cpu_baseline"] = accum_cpu_baseline(*accum16.pop("_state"), budget_s=4.0)
            else:
                accum16.pop("_state", None)
            out["accumulator_b16_k14"] = accum16
        if accum32 is not None:
            accum32.pop("_state", None)
            out["accumulator_b32_k17"] = accum32
        if inst is not None:
            out["instance_commitments"] = inst
        if accum_large is not None:
            accum_large.pop("_state", None)
            out[f"accumulator_b{args.accum_large}"] = accum_large
        emit(out, args.detail)
    if dist:
        dist.destroy_process_group()


def settle(step, seconds=0.3):
    """Untimed local work (never a collective: ranks loop for different
    counts) for `seconds` before a leg's warmup: right after the
    setup (input synthesis, base upload) the first ~0.1 s of MSMs ran ~5 %
    slower than later ones in the same process (the GPU's clocks ramping up;
    tools/bench_vs_loop.py), which three warmup steps do not cover."""
    import torch

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        step()
    torch.cuda.synchronize()


def timed_steps(step, steps, warmup, dist, dev, drain=None):
    """W untimed steps, then K steps between barrier + synchronize on both
    sides; returns (max-over-ranks seconds, last step's result).  drain: a
    pipelined step (sharded.PartialPipe) returns step k - 1's result; drain()
    completes the last one, after the warmup (untimed) and inside the timed
    region."""
    import torch

    for _ in range(warmup):
        step()
    if drain:
        drain()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    result = None
    for _ in range(steps):
        result = step()
    if drain:
        last = drain()
        result = last if last is not None else result
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, result


MSM_KERNELS = ["bases_r261", "sort_hist", "scan", "sort_coarse", "sort_fine", "accumulate", "bucket_seg",
               "bucket_bits", "host_tail"]


def run_msm_leg(args, ctx, dist, dev, world, curve, n, i0, roofline, breakdown, n_total=None, check_port=False,
                host_leg=False):
    """One MSM leg: this rank's n pairs [i0, i0 + n) generated on the device,
    one step = pm_msm_resident_device against the rank's resident bases
    (pm_bases_upload_device: the SRS bases are uploaded and converted to the
    pipeline form once, untimed, like params.g in halo2) + all-gather of the
    partials + host fold.  n_total None: weak scaling (world * n pairs); else
    strong (n_total split over the ranks)."""
    import numpy as np
    import torch

    import halo2_amd as H
    from sharded import PartialPipe, points_fold

    d_s = torch.empty((max(n, 1), 4), dtype=torch.int64, device=dev)
    d_b = torch.empty((max(n, 1), 8), dtype=torch.int64, device=dev)
    ctx.synth_scalars(curve, SEED_SCALARS, i0, n, d_s.data_ptr())
    ctx.synth_bases(curve, SEED_BASES, i0, n, d_b.data_ptr())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rb = ctx.upload_bases(curve, d_bases=d_b.data_ptr(), n=n) if n else None
    upload_ms = (time.perf_counter() - t0) * 1e3
    gathered = torch.zeros(world * 8, dtype=torch.int64, device=dev)  # one all-gather target

    padd = points_fold(curve)

    # the exchange of MSM k (all-gather of the partials + fold) runs behind
    # MSM k + 1's kernels; every partial is still gathered and folded inside
    # the timed region (sharded.PartialPipe, drained at the end)
    pipe = PartialPipe(dist, dev, padd, world)

    def step():
        part = ctx.msm_resident_device(rb, 0, d_s.data_ptr(), n) if n else np.zeros(8, np.uint64)
        return pipe.step(part)

    # timed region: HIP events only around the roofline kernel (every event
    # pair costs ~10 us of stream time on MI355X)
    if roofline:
        # local MSMs only: no collective, so ranks may settle for different counts
        settle(lambda: ctx.msm_resident_device(rb, 0, d_s.data_ptr(), n) if n else None)
        for _ in range(args.warmup):
            step()
        ctx.set_timing(True, only="accumulate")
        ctx.reset_stats()
    elapsed, result = timed_steps(step, args.steps, 0 if roofline else args.warmup, dist, dev, drain=pipe.drain)
    launches, acc_ms = ctx.kernel_stats("accumulate") if roofline else (0, 0.0)
    ctx.set_timing(False)
    lg = (n_total or n).bit_length() - 1
    name = ("pallas", "vesta", "bn254")[curve]
    total = n_total if n_total is not None else world * n
    out = {"value": round(total / (elapsed / args.steps) / 1e6, 3), "unit": "Mscalar/s",
           "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
           "scaling": "strong" if n_total is not None else "weak",
           "config": {"workload": f"{name}_msm_2^{lg}" + ("_total" if n_total is not None else "_per_gpu"),
                      "curve": name, "n_per_gpu": n, "n_total": total, "scalars": "montgomery, HBM-resident",
                      "bases": "affine, HBM-resident SRS (pm_bases_upload_device: converted once at upload"
                               + (f" and kept as {rb.rows} rows [2^(256 j/{rb.rows})] P, "
                                  f"{rb.device_bytes / 2**20:.0f} MiB -- the row-table path; see "
                                  f"variable_base for non-SRS bases" if rb is not None and rb.rows > 1 else "")
                               + f"; {upload_ms:.1f} ms, untimed)",
                      "parallelism": f"point-slice x{world} + RCCL all-gather of partial points"}}
    if breakdown:
        # per-MSM kernel breakdown from a separate, untimed diagnostic run with
        # events around every launch
        out["kernels_ms"] = kernel_breakdown(ctx, step, MSM_KERNELS)
        pipe.drain()
    if roofline and launches:
        # one k_accumulate launch consumes all n (scalar, base) pairs of the MSM
        out["roofline"] = roofline_of(n, acc_ms / launches, launches / args.steps, f"{name}_msm_2^{lg}_per_gpu")
    if roofline:
        out["variable_base"] = run_variable_base(args, ctx, dist, dev, world, curve, d_s, d_b, n, result, name, lg)
    if host_leg and n:
        out["host_scalars"] = run_host_scalars(args, ctx, rb, d_s, n, dist, dev, world, result)
        S = d_s.cpu().numpy().view(np.uint64).copy()
        B = d_b.cpu().numpy().view(np.uint64).copy()
        out["dropin_pm_msm"] = run_dropin(args, curve, S, B, n, result)
        del S, B
        if args.small_n:
            out["small_n"] = run_small_n(curve)
    if check_port and n:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import msm_ref

        out["matches_c_port"] = bool(np.array_equal(
            np.asarray(result), msm_ref.best_multiexp(curve, d_s.cpu().numpy().view(np.uint64),
                                                      d_b.cpu().numpy().view(np.uint64), threads=cpu_threads())))
    if rb is not None:
        rb.release()
    out.update(_d_s=d_s, _d_b=d_b, _result=result)
    return out


def roofline_of(n, avg_ms, launches_per_msm, workload):
    """HBM roofline of k_accumulate: algorithmic bytes 96 B x n
    per MSM over the live HIP-event launch time."""
    alg_bytes = BYTES_PER_PAIR * n / launches_per_msm
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": load_pmc_traffic(workload, launches_per_msm),
            "kernel": "k_accumulate", "avg_launch_ms": round(avg_ms, 4),
            "launches_per_msm": launches_per_msm, "alg_bytes_per_launch": int(alg_bytes)}
    valu = load_valu_counters(workload, avg_ms)
    if valu:
        roof["valu_int"] = valu
    return roof


def run_variable_base(args, ctx, dist, dev, world, curve, d_s, d_b, n, want, name, lg):
    """The plain variable-base MSM on the same inputs, from raw device bases
    (Rust R = 2^256 layout, converted on every call; no row table):
    pm_msm_device.  This is the number for best_multiexp over bases that are
    not a resident SRS -- e.g. verify_proof's MSMs over proof commitments
    (examples/simple-example.rs:620,722) -- with its own roofline and kernel
    breakdown."""
    import numpy as np
    import torch

    import halo2_amd as H
    from sharded import combine_partials, points_fold

    gathered = torch.zeros(world * 8, dtype=torch.int64, device=dev)  # one all-gather target
    fold = points_fold(curve)

    def raw():
        part = ctx.msm_device(curve, d_s.data_ptr(), d_b.data_ptr(), n)
        return combine_partials(part, dist, dev, fold, world, gathered)

    steps = max(5, args.steps // 2)
    for _ in range(args.warmup):
        raw()
    ctx.set_timing(True, only="accumulate")
    ctx.reset_stats()
    el, got = timed_steps(raw, steps, 0, dist, dev)
    launches, acc_ms = ctx.kernel_stats("accumulate")
    ctx.set_timing(False)
    out = {"metric": f"{name} variable-base MSM Mscalar/s at 2^{lg} (raw bases, no table)",
           "value": round(world * n / (el / steps) / 1e6, 3), "unit": "Mscalar/s",
           "ms_per_step": round(el * 1e3 / steps, 4),
           "bases": "raw device bases, R = 2^256 Rust layout, converted per call (pm_msm_device)",
           "kernels_ms": kernel_breakdown(ctx, raw, MSM_KERNELS)}
    if launches:
        out["roofline"] = roofline_of(n, acc_ms / launches, launches / steps, f"{name}_msm_2^{lg}_raw")
    if world == 1:
        out["matches_row_table_path"] = bool(np.array_equal(np.asarray(got), np.asarray(want)))
    return out


def run_dropin(args, curve, S, B, n, want):
    """The literal drop-in call of INTEGRATION.md §2: pm_msm_ctx with host
    scalars AND host bases on a fresh context.  The first call with a base
    set runs the plain pipeline on uploaded bases (first_ms; the set is only
    remembered), the second admits it (admit_ms: upload + row-table build),
    later calls with the same base bytes hit the drop-in cache (warm: the
    scalars' PCIe copy, the keyed digest of the bases on host threads beside
    it, and the resident MSM, started speculatively behind the copy for the
    set the first and last 8 points predict, kept once the digest confirms
    it: speculation = pm_ctx_dropin_spec_stats)."""
    import numpy as np

    import halo2_amd as H

    ctx = H.Context(0)
    try:
        t0 = time.perf_counter()
        first = ctx.msm(curve, S, B)
        first_ms = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        second = ctx.msm(curve, S, B)
        admit_ms = (time.perf_counter() - t0) * 1e3
        k = max(5, args.steps // 2)
        for _ in range(2):
            ctx.msm(curve, S, B)
        t0 = time.perf_counter()
        for _ in range(k):
            got = ctx.msm(curve, S, B)
        warm = (time.perf_counter() - t0) * 1e3 / k
        # the same warm calls with one scalar copy (no split: MSM_OPT_SPLIT_COPY = 0)
        ctx.set_msm_option(H.MSM_OPT_SPLIT_COPY, 0)
        ctx.msm(curve, S, B)
        t0 = time.perf_counter()
        for _ in range(k):
            got1 = ctx.msm(curve, S, B)
        warm1 = (time.perf_counter() - t0) * 1e3 / k
        ctx.set_msm_option(H.MSM_OPT_SPLIT_COPY, -1)
        # host-side phases of a warm call (separate, untimed calls): the keyed
        # digest on the pool (start to join) and the scalar copy call beside it
        ctx.set_timing(True, only="")
        ctx.reset_stats()
        for _ in range(3):
            ctx.msm(curve, S, B)
        ctx.set_timing(False)
        phases = {k2: round(ctx.kernel_stats(k2)[1] / 3, 4) for k2 in ("dropin_digest", "dropin_copy_call", "h2d",
                                                                          "accumulate")}
        st = ctx.dropin_stats()
        kept, drained = ctx.dropin_spec_stats()
        return {"call": "pm_msm_ctx(curve, host scalars, host bases, n)", "first_ms": round(first_ms, 3),
                "admit_ms": round(admit_ms, 3), "warm_ms_per_msm": round(warm, 4),
                "warm_ms_one_copy": round(warm1, 4),
                "warm_Mscalar_s": round(n / (warm * 1e-3) / 1e6, 3), "warm_phases_ms": phases, "cache": st,
                "speculation": {"kept": kept, "drained": drained},
                "matches": bool(np.array_equal(first, want) and np.array_equal(second, want)
                                and np.array_equal(got, want) and np.array_equal(got1, want))}
    finally:
        ctx.close()


def run_small_n(curve, budget_s=4.0):
    """Latency of the drop-in call at n = 2^0 .. 2^16 (pm_msm_ctx, host
    inputs, fresh data each size) against the C port of best_multiexp on the
    host's threads: where the GPU call starts to win (the shim's threshold,
    halo2_amd.MSM_GPU_MIN_N).  Round 6: every GPU loop first runs ~20 ms of
    untimed calls of its own kind, and the C port is timed after all GPU
    loops (its 16 busy host threads, and the idle GPU's clocks dropping
    meanwhile, had added ~20-40 us to the next size's first GPU loop)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import halo2_amd as H
    import msm_ref

    ctx = H.Context(0)
    threads = cpu_threads()
    rows = []

    def settle(fn):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.02:
            fn()

    try:
        S = msm_ref.synth_scalars(curve, SEED_SCALARS, 0, 1 << 16, threads=threads)
        B = msm_ref.synth_bases(curve, SEED_BASES, 0, 1 << 16, threads=threads)
        for lg in range(0, 17):
            n = 1 << lg
            s, b = np.ascontiguousarray(S[:n]), np.ascontiguousarray(B[:n])
            reps = 20 if lg <= 12 else 8
            # fresh bases every call (the verifier's MSMs over proof points):
            # the small-MSM path; distinct windows of the base array
            fresh = [np.ascontiguousarray(B[k + 1:k + 1 + n]) for k in range(reps)] if 2 * n <= len(B) else []
            fresh_us = None
            if fresh:
                # (its own base sets: a set seen twice is kept by the drop-in cache)
                warm = [np.ascontiguousarray(B[len(B) - n - 1 - k:len(B) - 1 - k]) for k in range(2)]
                settle(lambda: [ctx.msm(curve, s, bf) for bf in warm])
                t0 = time.perf_counter()
                for bf in fresh:
                    ctx.msm(curve, s, bf)
                fresh_us = (time.perf_counter() - t0) * 1e6 / reps
            # the same bases every call (commit_lagrange against params.g_lagrange):
            # two untimed calls admit the set to the drop-in cache
            g = ctx.msm(curve, s, b)
            settle(lambda: ctx.msm(curve, s, b))
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.msm(curve, s, b)
            gpu_us = (time.perf_counter() - t0) * 1e6 / reps
            rows.append({"n": n, "gpu_us": round(gpu_us, 1), "gpu_us_fresh_bases": None if fresh_us is None
                         else round(fresh_us, 1), "_g": g, "_s": s, "_b": b, "_reps": reps})
    finally:
        ctx.close()
    for r in rows:
        s, b, reps = r.pop("_s"), r.pop("_b"), r.pop("_reps")
        g = r.pop("_g")
        c = msm_ref.best_multiexp(curve, s, b, threads=threads)
        t0 = time.perf_counter()
        for _ in range(reps):
            msm_ref.best_multiexp(curve, s, b, threads=threads)
        r["cpu_us"] = round((time.perf_counter() - t0) * 1e6 / reps, 1)
        r["match"] = bool(np.array_equal(g, c))
    cross = next((r["n"] for r in rows if r["gpu_us"] < r["cpu_us"]), None)
    return {"call": "pm_msm_ctx vs oracle/msm_ref.c best_multiexp; gpu_us: the same bases every call (kept by "
                    "the drop-in cache: n <= 64 on the many-MSM path after two sightings, n >= 4096 as a resident "
                    "set), gpu_us_fresh_bases: new bases every call (the small-MSM path)", "cpu_threads": threads,
            "curve": rows, "gpu_faster_from_n": cross, "shim_threshold": H.MSM_GPU_MIN_N}


def run_host_scalars(args, ctx, rb, d_s, n, dist, dev, world, want):
    """The drop-in path a Rust best_multiexp shim takes:
    scalars in (pageable) host memory, bases resident -> pm_msm_resident.
    Reports the PCIe-inclusive rate and the scalar H2D time on its own
    (HIP events around the copy, one pageable hipMemcpyAsync or the split
    copy's two parts)."""
    import numpy as np

    import halo2_amd as H

    S = d_s.cpu().numpy().view(np.uint64).copy()
    res = {}
    # "pageable": the automatic schedule (the split scalar copy from
    # PM_SPLIT_COPY_MIN_N points: the first 3/8's sort and accumulation beside
    # the rest's copy); "pageable_one_copy": MSM_OPT_SPLIT_COPY = 0
    for label, split in (("pageable", -1), ("pageable_one_copy", 0)):
        ctx.set_msm_option(H.MSM_OPT_SPLIT_COPY, split)
        k = max(3, args.steps // 2)
        el, got = timed_steps(lambda: ctx.msm_resident(rb, 0, S), k, 1, None, dev)
        ctx.set_timing(True, only="h2d")
        ctx.reset_stats()
        for _ in range(3):
            ctx.msm_resident(rb, 0, S)
        ctx.set_timing(False)
        cnt, h2d_ms = ctx.kernel_stats("h2d")
        h2d = h2d_ms / 3  # per MSM: the copy's span, or the two halves' spans summed
        res[label] = {"ms_per_msm": round(el * 1e3 / k, 4), "Mscalar_s": round(n / (el / k) / 1e6, 3),
                      "scalar_h2d_ms": round(h2d, 4), "copies_per_msm": round(cnt / 3, 2),
                      # no h2d events on the small-MSM path (its kernel reads pinned host memory)
                      "scalar_h2d_GBps": round(32 * n / (h2d * 1e-3) / 1e9, 2) if h2d > 0 else None,
                      "matches": bool(np.array_equal(np.asarray(got), np.asarray(want)))}
    ctx.set_msm_option(H.MSM_OPT_SPLIT_COPY, -1)
    # the prover's commit of many polynomials: K MSMs per call
    # (pm_msm_resident_batch), the scalar copy of MSM j+1 and the host tail of
    # MSM j-1 overlapping MSM j's kernels
    K = 8
    lists = [S] + [np.roll(S, 1 + j, axis=0) for j in range(K - 1)]
    el, got = timed_steps(lambda: ctx.msm_resident_batch(rb, 0, lists), max(2, args.steps // 8), 1, None, dev)
    steps = max(2, args.steps // 8)
    res["batch_8_pipelined"] = {"ms_per_msm": round(el * 1e3 / steps / K, 4),
                                "Mscalar_s": round(K * n / (el / steps) / 1e6, 3),
                                "matches": bool(np.array_equal(np.asarray(got[0]), np.asarray(want)))}
    return res


def dry_run(args, rank, world):
    """Launcher check without a GPU: gloo rendezvous, the same barrier /
    max-over-ranks timing as the real legs, and the JSON skeleton."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        print(compact_line({"metric": METRIC, "value": None, "unit": "Mscalar/s", "n_gpus": world,
                            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3, 4),
                            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
                            "data": "dry run (no GPU work)",
                            "config": {"workload": f"pallas_msm_2^{args.logn}_per_gpu"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def kernel_breakdown(ctx, step, names, reps=5):
    """Per-step kernel times from `reps` extra (untimed) steps with HIP events
    around every launch; every rank runs the same steps (collectives inside)."""
    ctx.set_timing(True)
    ctx.reset_stats()
    for _ in range(reps):
        step()
    ctx.set_timing(False)
    return {k: round(ctx.kernel_stats(k)[1] / reps, 4) for k in names}


def run_fixed_base(args, ctx, dist, dev, world, d_s, d_b, n, gathered, padd, want, lg=None):
    """Fixed-base MSM over the same scalars and bases: the
    SRS table [2^{o_w}] P_i is built once (untimed, reported as build_ms),
    then each step is pm_msm_fixed_device + the same all-gather / fold."""
    import numpy as np
    import torch

    from sharded import combine_partials

    t0 = time.perf_counter()
    fb = ctx.fixed_bases(0, d_bases=d_b.data_ptr(), n=n)
    build_ms = (time.perf_counter() - t0) * 1e3

    def step():
        part = fb.msm_device(d_s.data_ptr(), n)
        return combine_partials(part, dist, dev, padd, world, gathered)

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        got = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernels = kernel_breakdown(ctx, step, MSM_KERNELS[1:])
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    lg = lg or args.logn
    out = {"metric": f"Pallas fixed-base MSM Mscalar/s at 2^{lg} (precomputed SRS table)",
           "value": round(world * n / (elapsed / args.steps) / 1e6, 3), "unit": "Mscalar/s",
           "ms_per_step": round(elapsed * 1e3 / args.steps, 4), "c": fb.c, "windows": fb.windows,
           "table_GiB_per_gpu": round(fb.table_bytes / 2**30, 3), "build_ms": round(build_ms, 2),
           "matches_variable_base": bool(np.array_equal(np.asarray(got), np.asarray(want))),
           "kernels_ms": kernels}
    fb.release()
    return out


def run_ntt(args, ctx, dist, dev, world, k=None, keep_state=True):
    """NTT over the BN254 scalar field (halo2 best_fft): one step
    = one in-place pm_fft_device of 2^k HBM-resident elements per rank
    (independent transforms, weak scaling; the omega table is built in the
    warmup)."""
    import numpy as np
    import torch

    import halo2_amd as H
    import workloads as Wk

    curve, k = H.BN254, (k or args.ntt_logn)
    n = 1 << k
    r = H.SCALAR_MODULUS[curve]
    wv = Wk.domain_omega(curve, k) * (1 << 256) % r
    w = np.array([(wv >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)
    a = torch.empty((n, 4), dtype=torch.int64, device=dev)
    ctx.synth_scalars(curve, 0x77, 0, n, a.data_ptr())
    torch.cuda.synchronize()
    src = a.cpu().numpy().view(np.uint64).copy() if keep_state and (args.gpus == 1 or world == 1) else None
    ctx.fft_device(curve, a.data_ptr(), k, w)
    first = a.cpu().numpy().view(np.uint64).copy() if src is not None else None
    def step():
        ctx.fft_device(curve, a.data_ptr(), k, w)

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernels = kernel_breakdown(ctx, step, ("ntt_cols", "ntt_mid", "ntt_rows"))
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed * 1e3 / args.steps
    gpu_ms = kernels["ntt_cols"] + kernels["ntt_mid"] + kernels["ntt_rows"]
    passes = 3 if kernels["ntt_mid"] else 2
    # algorithmic bytes: read + write every 32-B element once; the four-step
    # form moves each element once per pass (2 x 32 B per pass) through HBM
    alg = 2 * 32 * n
    out = {"metric": f"NTT 2^{k} over the BN254 scalar field (halo2 best_fft)", "value": round(world * n / (ms * 1e-3) / 1e6, 1),
           "unit": "Melem/s", "ms_per_ntt": round(ms, 4), "higher_is_better": True, "scaling": "weak",
           "passes": passes, "kernels_ms": kernels,
           "roofline": {"bound": "hbm", "achieved": round(alg / (gpu_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / (gpu_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": load_ntt_traffic(f"ntt_bn254_2^{k}"),
                        "note": "achieved = 64 B/element (read + write once) over all passes' kernel time; "
                                "traffic = PMC FETCH+WRITE of all passes (profiles/pmc_ntt.json); the NTT is "
                                "VALU-bound (n/2 log n Montgomery products): valu_int"}}
    valu = load_ntt_valu(f"ntt_bn254_2^{k}")
    if valu:
        out["roofline"]["valu_int"] = valu
    if src is not None:
        out["_state"] = (curve, k, src, w, first)
    return out


def ntt_cpu_baseline(curve, k, src, w, first, budget_s):
    """C restatement of halo2 best_fft (oracle/msm_ref.c, halo2's own
    parallel_fft split over 16 threads) on the same input; bit-exact check of
    the GPU's first transform."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import msm_ref

    threads = cpu_threads()
    reps, t0 = 0, time.perf_counter()
    match = None
    while True:
        got = msm_ref.best_fft(curve, src, k, w, threads)
        if match is None:
            match = bool(np.array_equal(got, first))
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = (time.perf_counter() - t0) / reps
    return {"value": round((1 << k) / dt / 1e6, 3), "unit": "Melem/s", "cores": threads, "kind": "port",
            "host": cpu_info(),
            "sample": f"{reps} x best_fft(2^{k}) in oracle/msm_ref.c ({dt * 1e3:.1f} ms each)",
            "matches_gpu": match}


def run_accumulator(args, ctx, dist, dev, rank, world, B=None, logn=None, light=False, two=None):
    """Batch multiopen accumulator: B proofs per rank, timed like the MSM leg.
    One step starts from the proofs' BYTES, resident in HBM as halo2's
    Blake2bWrite serialized them: device decode (read_point decompression /
    read_scalar checks), transcript replay, scalar block and accumulator quad
    (pm_accum_batch_proofs_device), then the all-gather of the quads.
    `from_decoded` times the same batch from already-decoded points (the
    round-3 boundary, pm_accum_batch_transcript_device) for comparison."""
    import numpy as np
    import torch

    import halo2_amd as H
    import workloads as Wk

    curve, B, logn = H.BN254, B or args.accum_batch, logn or args.accum_logn
    shape = Wk.simple_example_shape(ctx, curve, logn)
    batch = Wk.SyntheticBatch(ctx, shape, B, i0=rank * B)
    batch.to_proof_bytes(shape)
    from sharded import gather_batches

    gathered = [torch.zeros_like(batch.quads) for _ in range(world)] if dist else None

    def step():
        batch.run_bytes(ctx, shape)
        gather_batches(batch.quads, dist, world, gathered)

    def step_decoded():
        batch.run(ctx, shape)
        gather_batches(batch.quads, dist, world, gathered)

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el * 1e3 / args.steps

    ms_dec = timed(step_decoded)
    quads_dec = batch.quads.clone()
    ms = timed(step)
    kernels = kernel_breakdown(ctx, step, ("proof_decode", "transcript", "acc_ladder", "acc_scalars",
                                            "acc_termmul", "acc_sum"))
    npts, nsc, nsets = shape.layout()
    # MSM terms per proof (accum_engine.hpp): the distinct commitments of f (every
    # proof point but the W_j, the fixed and sigma commitments: all queried in
    # the simple-example shape) with the h_i, then W_j for w and zw, and g1 for e
    nslots = (npts - nsets) + shape.c.num_fixed_columns + shape.c.n_perm_columns
    T = nslots + 2 * nsets + 1
    out = {"metric": "aggregated proofs verified/s", "value": round(world * B / (ms * 1e-3), 1), "unit": "proofs/s",
           "ms_per_batch": round(ms, 4), "higher_is_better": True, "scaling": "weak",
           "config": {"workload": f"multiopen_accumulator_simple_example_k{logn}", "curve": "bn254",
                      "proofs_per_gpu": B, "proofs_total": world * B, "proof_bytes": batch.psize,
                      "input": "serialized proofs in HBM (halo2 Blake2bWrite byte layout) + instance commitments",
                      "challenges": "Blake2b transcript replayed on the device (pm_accum_batch_proofs_device)",
                      "per_proof_work": "point decompression (square roots) + canonical checks, transcript replay, "
                                        "scalar block, multiopen accumulator quad (w, zw, f, e) and h_eval, status "
                                        "checked; the pairing / decider check on the quads is not part of the "
                                        "reference's verifier circuit either (verifier.rs:739-754 exposes the quad "
                                        "as instances)",
                      "parallelism": f"proof-batch x{world} + RCCL all-gather of B x 4 points"},
           "kernels_ms": kernels,
           "roofline": accum_latency_roofline(B, T, nslots, ms, kernels, shape=shape, psize=batch.psize),
           "status_nonzero": int((batch.status != 0).sum().item()),
           "from_decoded": {"ms_per_batch": round(ms_dec, 4), "value": round(world * B / (ms_dec * 1e-3), 1),
                            "entry": "pm_accum_batch_transcript_device (decoded points / scalars in HBM)",
                            "quads_match_bytes_path": bool(torch.equal(quads_dec, batch.quads))}}
    if world == 1 and (not light if two is None else two):
        out["two_in_flight"] = accum_two_in_flight(args, ctx, shape, batch, B)
    if B > 256:  # its first 256 proofs as a batch of their own: the same quads
        sub = 256
        q = torch.empty((sub, 4, 8), dtype=torch.int64, device=dev)
        hh = torch.empty((sub, 4), dtype=torch.int64, device=dev)
        cc = torch.empty((sub, 7, 4), dtype=torch.int64, device=dev)
        ss = torch.empty((sub,), dtype=torch.int32, device=dev)
        ctx.accum_batch_proofs_device(shape, sub, batch.vk_repr, batch.proofs.data_ptr(), batch.psize,
                                      batch.inst.data_ptr(), cc.data_ptr(), q.data_ptr(), hh.data_ptr(), ss.data_ptr())
        torch.cuda.synchronize()
        out["matches_b256_subbatch"] = bool(torch.equal(q, batch.quads[:sub]) and torch.equal(hh, batch.h_eval[:sub]))
    if rank == 0 and not light:
        host = {k: getattr(batch, k).cpu().numpy().view(np.uint64)
                for k in ("points", "scalars", "challenges", "quads", "h_eval")}
        host["vk_repr"] = np.asarray(batch.vk_repr, dtype=np.uint64)
        host["proofs"] = batch.proofs.cpu().numpy()
        host["inst"] = batch.inst.cpu().numpy().view(np.uint64)
        out["_state"] = (curve, shape, host, B)
    return out


def run_instance_commitments(args, ctx, dist, dev, rank, world, logn=17):
    """Per-proof instance commitments (examples/simple-example.rs:632-641:
    params_verifier.commit_lagrange(public_inputs), the instance column the
    verifier reads, src/verifier.rs:200-225, 312-316) for B proofs per rank
    with `--inst-npub` public inputs each, against a resident g_lagrange of
    2^logn synthetic bases (BN254, the reference's curve): ONE
    pm_msm_resident_many_device call per step.  Beside it: the same B MSMs
    as B pm_msm_resident_device calls (the per-proof loop it replaces, timed
    once, bit-exact check), and `with_accumulator`: the instance commitments
    then the accumulator batch from proof bytes fed with them (aggregated
    proofs verified/s counting the commitments)."""
    import numpy as np
    import torch

    import halo2_amd as H
    import workloads as Wk

    curve, B, npub = H.BN254, args.inst_batch, args.inst_npub
    nb = 1 << logn
    d_b = torch.empty((nb, 8), dtype=torch.int64, device=dev)
    ctx.synth_bases(curve, SEED_BASES ^ 0x1A6, 0, nb, d_b.data_ptr())
    d_s = torch.empty((B * npub, 4), dtype=torch.int64, device=dev)
    ctx.synth_scalars(curve, SEED_SCALARS ^ 0x1A6, rank * B * npub, B * npub, d_s.data_ptr())
    torch.cuda.synchronize()
    bases = ctx.upload_bases(curve, d_bases=d_b.data_ptr(), n=nb)
    n = [npub] * B
    t0 = time.perf_counter()
    res = ctx.msm_resident_many_device(bases, n, d_s.data_ptr())
    build_ms = (time.perf_counter() - t0) * 1e3
    pre, c, tbytes = bases.many_info()

    def step():
        ctx.msm_resident_many_device(bases, n, d_s.data_ptr())

    ms = timed_steps(step, args.steps, args.warmup, dist, dev)[0] * 1e3 / args.steps
    # the loop it replaces: one resident MSM per proof
    loop = []
    t0 = time.perf_counter()
    for i in range(B):
        loop.append(ctx.msm_resident_device(bases, 0, d_s.data_ptr() + 32 * npub * i, npub))
    ms_loop = (time.perf_counter() - t0) * 1e3
    match_loop = bool(np.array_equal(np.array(loop), res))
    out = {"value": round(world * B / (ms * 1e-3), 1), "unit": "instance commitments/s", "ms_per_batch": round(ms, 4),
           "higher_is_better": True, "scaling": "weak",
           "config": {"workload": f"commit_lagrange_b{B}_npub{npub}", "curve": "bn254", "proofs_per_gpu": B,
                      "public_inputs_per_proof": npub, "g_lagrange": nb, "entry": "pm_msm_resident_many_device",
                      "table": {"prefix": pre, "window_bits": c, "device_bytes": tbytes,
                                "first_call_ms_with_build": round(build_ms, 3)}},
           "per_proof_loop": {"ms_per_batch": round(ms_loop, 4), "entry": "B x pm_msm_resident_device",
                              "matches": match_loop},
           "speedup_vs_loop": round(ms_loop / ms, 1)}
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import msm_ref

        hb = d_b[:npub].cpu().numpy().view(np.uint64)
        hs = d_s.cpu().numpy().view(np.uint64)
        threads = cpu_threads()
        t0 = time.perf_counter()
        ok, k = True, 0
        while k < B and time.perf_counter() - t0 < 3.0:
            ok &= bool(np.array_equal(msm_ref.best_multiexp(curve, hs[k * npub:(k + 1) * npub], hb, threads=1),
                                      res[k]))
            k += 1
        el = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(k / el, 1), "unit": "instance commitments/s", "cores": 1,
                               "kind": "port", "sample": f"{k} of the {B} MSMs, oracle/msm_ref.c best_multiexp, "
                                                         "one thread each (independent MSMs: x cores for a pool)",
                               "matches": ok}
    # the batch accumulator fed with these commitments (proof bytes in HBM)
    shape = Wk.simple_example_shape(ctx, curve, logn)
    batch = Wk.SyntheticBatch(ctx, shape, B, i0=rank * B, seed=0x1A7)
    batch.to_proof_bytes(shape)

    def step_acc():
        q = ctx.msm_resident_many_device(bases, n, d_s.data_ptr())
        batch.inst.copy_(torch.from_numpy(q.view(np.int64)).reshape(B, 1, 8), non_blocking=False)
        batch.run_bytes(ctx, shape)

    ms_acc = timed_steps(step_acc, args.steps, args.warmup, dist, dev)[0] * 1e3 / args.steps
    out["with_accumulator"] = {"value": round(world * B / (ms_acc * 1e-3), 1), "unit": "proofs/s",
                               "ms_per_batch": round(ms_acc, 4),
                               "how": "pm_msm_resident_many_device -> H2D of the B commitments -> "
                                      "pm_accum_batch_proofs_device from proof bytes",
                               "status_nonzero": int((batch.status != 0).sum().item())}
    bases.release()
    return out


def accum_two_in_flight(args, ctx, shape, batch, B):
    """Two batches in flight: a second context (its own HIP streams and
    workspace) runs another B proofs from bytes on a second host thread
    while `ctx` runs `batch`.  One batch is a set of latency-bound chains
    that leave most SIMDs idle; the pair's combined rate
    is the throughput of a stream of batches.  Reported beside the
    one-batch `value`, which stays the headline."""
    import threading

    import torch

    import halo2_amd as H
    import workloads as Wk

    ctx2 = H.Context(0)
    b2 = Wk.SyntheticBatch(ctx2, shape, B, seed=0xACD)
    b2.to_proof_bytes(shape)
    b2.run_bytes(ctx2, shape)
    torch.cuda.synchronize()
    refs = [batch.quads.clone(), b2.quads.clone()]
    errs = []

    def loop(c, b):
        try:
            for _ in range(args.warmup + args.steps):
                b.run_bytes(c, shape)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=loop, args=cb) for cb in ((ctx, batch), (ctx2, b2))]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n = 2 * (args.warmup + args.steps)
    ok = not errs and all(torch.equal(r, b.quads) for r, b in zip(refs, (batch, b2)))
    ok = ok and int((batch.status != 0).sum().item()) == 0 and int((b2.status != 0).sum().item()) == 0
    del ctx2
    return {"value": round(n * B / el, 1), "unit": "proofs/s", "ms_per_batch": round(el * 1e3 / n, 4),
            "batches": n, "how": "2 contexts x 2 host threads, each looping pm_accum_batch_proofs_device on its "
                                 "own batch of B proofs from bytes (warmup included in the timed loop)",
            "quads_match_single_runs": ok, "errors": errs}


def _jsonl(path):
    if os.path.exists(path):
        for line in open(path):
            if line.strip().startswith("{"):
                yield json.loads(line)


def accum_step_costs():
    """The step costs of the accumulator's algorithmic floor, all from
    committed measurements: the best dependent field product (the row-sliced
    BN254 product, profiles/r05/microbench_slice.jsonl, the minimum over its
    occupancies), the best inversion (quad-cooperative safegcd, same file) and
    one Blake2b compression (profiles/r05/chain_latency.jsonl)."""
    P = INV = None
    for d in _jsonl(os.path.join(ROOT, "profiles", "r05", "microbench_slice.jsonl")):
        if d.get("field") != "bn254_fq":
            continue
        if "sliced_us_per_mul" in d:
            P = d["sliced_us_per_mul"] if P is None else min(P, d["sliced_us_per_mul"])
        if "inv_quad_safegcd_us" in d:
            INV = d["inv_quad_safegcd_us"]
    B2 = next((d["us_per_step"] for d in _jsonl(os.path.join(ROOT, "profiles", "r05", "chain_latency.jsonl"))
               if d.get("step") == "b2_compress_q"), None)
    if None in (P, INV, B2):
        return None
    return {"product_us": P, "inverse_us": INV, "blake2b_compress_us": B2,
            "source": "profiles/r05/microbench_slice.jsonl (min sliced BN254 product, quad safegcd inverse), "
                      "profiles/r05/chain_latency.jsonl (b2_compress_q)"}


def accum_valu_roofline(B, ms_batch):
    """Throughput legs (the one-lane form, B >= 2048): integer-VALU roofline of
    the whole batch from committed SQ counters of the same workload
    (profiles/pmc_acc_valu.json, tools/acc_valu.py over tools/gpu_r06_acc.sh):
    the issue time the batch's VALU instructions need at the measured peaks
    (INT64 class at the v_mad_u64_u32 peak, the rest at the simple-op peak,
    profiles/valu_peak.json) over the batch time."""
    p = os.path.join(ROOT, "profiles", "pmc_acc_valu.json")
    if not os.path.exists(p):
        return None
    d = json.load(open(p)).get("batches", {}).get(str(B))
    if not d:
        return None
    issue_s = d["issue_seconds_per_batch"]
    lane_ops = d["valu_lane_insts_per_batch"]
    return {"bound": "valu", "achieved": round(lane_ops / (ms_batch * 1e-3) / 1e12, 3),
            "peak": d["int64_peak_Tops"], "unit": "T lane-ops/s", "frac": round(issue_s / (ms_batch * 1e-3), 4),
            "traffic": None, "kernel_frac": {k: round(v["issue_frac"], 4) for k, v in d["kernels"].items()},
            "note": "frac = VALU issue time at the measured peaks (INT64 class 33.944 T/s, other 61.164 T/s) over "
                    "the batch time; kernel_frac = the same per kernel over its own duration",
            "source": d["source"]}


def accum_latency_roofline(B, T, nslots, ms_batch, kernels, shape=None, psize=0, from_bytes=True):
    """Latency roofline of the accumulator batch: every
    kernel on the critical path is a chain of dependent steps, and its floor
    is ALGORITHMIC -- the dependent field products the computation needs (not
    this code's instruction count) x the best product latency measured on
    MI355X, plus the best measured inversion and Blake2b compression
    (accum_step_costs):

      decode      the BN254 square root a^((p+1)/4): 251 dependent squarings
      transcript  ceil(stream bytes / 128) sequential Blake2b compressions
      scalars     x^n (log n squarings), 1 product into the batched
                  denominator, 1 inversion, 4 products (l_i, the fold, h_eval,
                  the e coefficient)
      ladder      127 doublings x 3 product levels
      term adds   ceil(85.3 / S) + log2 S additions x 4 product levels (S lanes
                  share a term's ~85.3 NAF digits)
      sums        ceil(nslots / (NL/4)) + log2(NL/4) additions x 4 levels, 1
                  inversion, 2 products (affine x, y)

    critical = max(ladder (after the decode unless twisted), decode +
    transcript + scalars) + term adds + sums.  Large batches (the one-lane
    form) are throughput work: their roofline is accum_valu_roofline."""
    if B >= 2048:
        v = accum_valu_roofline(B, ms_batch)
        if v:
            return v
    cost = accum_step_costs()
    if cost is None:
        return None
    P, INV, B2 = cost["product_us"], cost["inverse_us"], cost["blake2b_compress_us"]
    budget = 1024 * 2 * 64
    nterm = B * T
    lg = 0
    while lg < 3 and (nterm << (lg + 1)) <= budget:
        lg += 1
    if lg == 3:
        while lg < 5 and (nterm << (lg + 1)) <= budget // 2:
            lg += 1
    S = 1 << lg
    lgL = 0
    while lgL < 5 and ((B * 4) << (lgL + 1)) <= 16384:
        lgL += 1
    while lgL < 3 and ((B * 4) << (lgL + 1)) <= budget // 2:  # quads at large B (accum_engine.hpp)
        lgL += 1
    nq = max(1, (1 << lgL) // 4)
    c = shape.c if shape is not None else None
    npts = shape.layout()[0] if shape is not None else T
    nsc = shape.layout()[1] if shape is not None else 0
    log_n = c.log_n if c is not None else 17
    comps = -(-(npts * 65 + nsc * 33 + 33) // 128)
    nprf = B * npts
    # round 6: from bytes the ladder always runs beside the decode while the
    # powers tables are built (accum_engine.hpp proofs_device_impl)
    twist = from_bytes and 4 * (nprf << 2) <= 3 * budget
    f = {"proof_decode": 251 * P, "transcript": comps * B2, "acc_scalars": (log_n + 1 + 4) * P + INV,
         "acc_ladder": 127 * 3 * P, "acc_termmul": (-(-85.3 // S) + lg) * 4 * P,
         "acc_sum": ((-(-nslots // nq) + (nq.bit_length() - 1)) * 4 + 2) * P + INV}
    if not from_bytes:
        f.pop("proof_decode")
    d = f.get("proof_decode", 0.0)
    lad = f["acc_ladder"] if twist else d + f["acc_ladder"]
    crit = max(lad, d + f["transcript"] + f["acc_scalars"]) + f["acc_termmul"] + f["acc_sum"]
    out = {"bound": "latency", "achieved": round(ms_batch, 4), "unit": "ms per batch (critical path)",
           "peak": round(crit / 1e3, 4), "frac": round(crit / 1e3 / ms_batch, 4), "traffic": None,
           "alg_floor_ms": {k: round(v / 1e3, 4) for k, v in f.items()},
           "kernel_frac": {k: round(f[k] / 1e3 / kernels[k], 4) for k in f if kernels.get(k)},
           "lanes": {"term_additions_S": S, "sum_lanes_NL": 1 << lgL, "twisted_ladder": twist},
           "step_costs": cost}
    return out


def accum_cpu_baseline(curve, shape, host, B, budget_s):
    """C restatement of the same work from the same bytes (oracle/accum_ref.c:
    proof decoding with square roots, transcript replay, accumulator; all host
    threads) on the GPU's own batch: bit-exact check of every proof's
    challenges, quads and h_eval, and throughput over repeated passes of the
    batch within the budget."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import accum_ref

    threads = cpu_threads()
    reps, t0 = 0, time.perf_counter()
    match = None
    while True:
        o = accum_ref.batch_proofs(curve, shape.c, host["proofs"], host["inst"], vk_repr=host["vk_repr"],
                                   threads=threads)
        if match is None:
            match = bool(np.array_equal(o["challenges"].reshape(host["challenges"].shape), host["challenges"])
                         and np.array_equal(o["quads"].reshape(host["quads"].shape), host["quads"])
                         and np.array_equal(o["h_eval"].reshape(host["h_eval"].shape), host["h_eval"])
                         and not o["status"].any())
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(reps * B / dt, 2), "unit": "proofs/s", "cores": threads, "kind": "port",
            "host": cpu_info(),
            "sample": f"{reps} x the GPU's batch of {B} serialized proofs through oracle/accum_ref.c (decode + "
                      f"Blake2b replay + accumulator in C, {threads} threads, {dt:.1f} s)",
            "matches_gpu": match}


def cpu_baseline(d_s, d_b, n, gpu_result, budget_s):
    """C restatement of halo2 best_multiexp on the host, same inputs."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import msm_ref

    S = d_s.cpu().numpy().view(np.uint64)
    B = d_b.cpu().numpy().view(np.uint64)
    threads = cpu_threads()
    reps, t0 = 0, time.perf_counter()
    match = None
    while True:
        out = msm_ref.best_multiexp(0, S, B, threads=threads)
        reps += 1
        if match is None:
            match = bool(np.array_equal(out, gpu_result))
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(reps * n / dt / 1e6, 4), "unit": "Mscalar/s", "cores": threads, "kind": "port",
            "host": cpu_info(),
            "sample": f"{reps} x Pallas best_multiexp of the same 2^{n.bit_length() - 1} inputs "
                      f"({dt:.1f} s, oracle/msm_ref.c, {threads} threads)",
            "matches_gpu": match}


if __name__ == "__main__":
    main()
