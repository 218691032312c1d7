"""Diagnostic: bench.py's MSM leg vs a bare loop of the same resident MSM in
one process (same inputs), to locate per-step overhead outside the library."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "halo2-aggregation_amd")]
sys.argv = ["bench.py", "--no-cpu", "--steps", "30"]
import torch  # noqa: E402

import bench  # noqa: E402
import halo2_amd as H  # noqa: E402


def loop(ctx, rb, s, n, reps=30):
    for _ in range(3):
        ctx.msm_resident_device(rb, 0, s.data_ptr(), n)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        ctx.msm_resident_device(rb, 0, s.data_ptr(), n)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3 / reps


def main():
    args = bench.parse()
    n = 1 << 20
    ctx = H.Context(0)
    dev = torch.device("cuda", 0)
    for rep in range(2):
        leg = bench.run_msm_leg(args, ctx, None, dev, 1, H.PALLAS, n, 0, roofline=True, breakdown=False)
        s = leg["_d_s"]
        b = leg["_d_b"]
        rb = ctx.upload_bases(H.PALLAS, d_bases=b.data_ptr(), n=n)
        ctx.set_timing(False)
        ms_loop = loop(ctx, rb, s, n)
        ctx.set_timing(True, only="accumulate")
        ms_loop_t = loop(ctx, rb, s, n)
        ctx.set_timing(False)
        rb.release()
        print(json.dumps({"bench_ms_per_step": leg["ms_per_step"], "loop_ms": round(ms_loop, 4),
                          "loop_timed_ms": round(ms_loop_t, 4)}), flush=True)


if __name__ == "__main__":
    main()
