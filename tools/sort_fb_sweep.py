"""Sweep the sort's fine-bit split (PM_SORT_FB) for the variable-base MSM at
2^20 / 2^22 and the fixed-base MSM at 2^23: per-kernel times (diagnostic).
Each FB value gets its own context (the knob is read at context creation).
Usage (through gpurun): python tools/sort_fb_sweep.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "halo2-aggregation_amd"))
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402

KS = ["sort_hist", "scan", "sort_coarse", "sort_fine", "accumulate", "fixup", "bucket_seg", "bucket_bits"]


def timed(ctx, fn, reps=5):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    wall = (time.perf_counter() - t) / reps
    ctx.set_timing(True)
    ctx.reset_stats()
    for _ in range(reps):
        fn()
    ctx.set_timing(False)
    return wall, {k: round(ctx.kernel_stats(k)[1] / reps, 4) for k in KS}


def main():
    nmax = 1 << 23
    s = torch.empty((nmax, 4), dtype=torch.int64, device="cuda")
    b = torch.empty((nmax, 8), dtype=torch.int64, device="cuda")
    c0 = H.Context(0)
    c0.synth_scalars(0, 0x5EED, 0, nmax, s.data_ptr())
    c0.synth_bases(0, 0xA11CE, 0, nmax, b.data_ptr())
    torch.cuda.synchronize()
    ref = {lg: c0.msm_device(0, s.data_ptr(), b.data_ptr(), 1 << lg) for lg in (20, 22, 23)}
    c0.close()
    combos = [tuple(int(y) for y in x.split(":")) for x in os.environ.get("COMBOS", "7:0,7:4096,7:6144,6:4096,6:6144,6:8192").split(",")]
    for fb, fc in combos:
        os.environ["PM_SORT_FB"] = str(fb)
        os.environ["PM_FINE_CACHE"] = str(fc)
        ctx = H.Context(0)
        for lg in (20, 22):
            n = 1 << lg
            wall, ks = timed(ctx, lambda: ctx.msm_device(0, s.data_ptr(), b.data_ptr(), n))
            ok = bool((ctx.msm_device(0, s.data_ptr(), b.data_ptr(), n) == ref[lg]).all())
            print(json.dumps({"fb": fb, "fine_cache": fc, "logn": lg, "fixed": False, "wall_ms": round(wall * 1e3, 3), "ok": ok,
                              "kernels_ms": ks}), flush=True)
        ctx.close()
    for fb, fc in [tuple(int(y) for y in x.split(":")) for x in os.environ.get("COMBOS_FIXED", "9:4096,9:8192,10:4096,10:8192,11:4096").split(",")]:
        os.environ["PM_SORT_FB"] = str(fb)
        os.environ["PM_FINE_CACHE"] = str(fc)
        ctx = H.Context(0)
        fbt = ctx.fixed_bases(0, d_bases=b.data_ptr(), n=nmax)
        wall, ks = timed(ctx, lambda: fbt.msm_device(s.data_ptr(), nmax))
        ok = bool((fbt.msm_device(s.data_ptr(), nmax) == ref[23]).all())
        print(json.dumps({"fb": fb, "fine_cache": fc, "logn": 23, "fixed": True, "c": fbt.c, "wall_ms": round(wall * 1e3, 3), "ok": ok,
                          "kernels_ms": ks}), flush=True)
        fbt.release()
        ctx.close()


if __name__ == "__main__":
    main()
