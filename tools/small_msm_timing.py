"""Latency of pm_msm_ctx on the small-MSM path against the sorting pipeline
(threshold 0) for n = 2^0 .. 2^16, plus the small path's kernel and host-tail
split (HIP events, separate untimed pass).  One JSON line per n.
Usage (GPU box): python tools/small_msm_timing.py [max_log] [threshold]
         python tools/small_msm_timing.py only N [reps]   (N repeated: for rocprofv3)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import halo2_amd as H  # noqa: E402
import msm_ref  # noqa: E402
import pasta as P  # noqa: E402


def lat(ctx, curve, s, b, reps):
    ctx.msm(curve, s, b)
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.msm(curve, s, b)
        best = min(best, (time.perf_counter() - t0) / reps)
    return best * 1e6


def only(n, reps):
    ctx = H.Context(0)
    S = msm_ref.synth_scalars(0, P.SEED_SCALARS, 0, n, threads=16)
    B = msm_ref.synth_bases(0, P.SEED_BASES, 0, n, threads=16)
    us = lat(ctx, 0, S, B, reps)
    print(json.dumps({"n": n, "small_us": round(us, 1)}), flush=True)
    ctx.close()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "only":
        return only(int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 200)
    max_log = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    thr = int(sys.argv[2]) if len(sys.argv) > 2 else H.SMALL_MSM_LIMIT
    curve = 0
    ctx = H.Context(0)
    N = 1 << max_log
    S = msm_ref.synth_scalars(curve, P.SEED_SCALARS, 0, N, threads=16)
    B = msm_ref.synth_bases(curve, P.SEED_BASES, 0, N, threads=16)
    for lg in range(0, max_log + 1):
        n = 1 << lg
        s, b = np.ascontiguousarray(S[:n]), np.ascontiguousarray(B[:n])
        reps = 50 if lg <= 12 else 10
        ctx.set_small_msm(thr)
        small_us = lat(ctx, curve, s, b, reps)
        got = ctx.msm(curve, s, b)
        ctx.set_timing(True)
        ctx.reset_stats()
        for _ in range(5):
            ctx.msm(curve, s, b)
        split = {k: round(ctx.kernel_stats(k)[1] / 5 * 1e3, 1) for k in ("small_stage", "small_fused", "small_table", "small_sum", "host_tail")}
        ctx.set_timing(False)
        ctx.set_small_msm(0)
        pipe_us = lat(ctx, curve, s, b, reps)
        want = ctx.msm(curve, s, b)
        ctx.set_small_msm(H.SMALL_MSM_DEFAULT)
        print(json.dumps({"n": n, "small_us": round(small_us, 1), "pipeline_us": round(pipe_us, 1),
                          "small_split_us": split, "match": bool(np.array_equal(got, want))}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
