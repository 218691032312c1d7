"""Per-kernel timing of the MSM pipeline at several sizes (diagnostic)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "halo2-aggregation_amd"))
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402

KERNELS = ["bases_r261", "sort_hist", "scan", "sort_coarse", "sort_fine", "accumulate", "fixup", "bucket_seg", "bucket_bits", "bits_combine", "host_tail"]  # round-2 names kept for A/B against older builds


def main():
    curve = int(os.environ.get("CURVE", "0"))
    sizes = [int(x) for x in os.environ.get("LOGN", "16,18,20,22").split(",")]
    cs = [int(x) for x in os.environ.get("WINDOWS", "0").split(",")]
    mcs = [int(x) for x in os.environ.get("PM_SWEEP_MINCHUNK", "0").split(",")]
    ctx = H.Context(0)
    nmax = 1 << max(sizes)
    s = torch.empty((nmax, 4), dtype=torch.int64, device="cuda")
    b = torch.empty((nmax, 8), dtype=torch.int64, device="cuda")
    ctx.synth_scalars(curve, 0x5EED, 0, nmax, s.data_ptr())
    t = time.time()
    ctx.synth_bases(curve, 0xA11CE, 0, nmax, b.data_ptr())
    print(json.dumps({"synth_bases_s": time.time() - t, "n": nmax}), flush=True)
    resident = os.environ.get("RESIDENT", "0") == "1"  # the bench's path: pm_msm_resident_device
    for lg in sizes:
        n = 1 << lg
        rb = ctx.upload_bases(curve, d_bases=b.data_ptr(), n=n) if resident else None

        def run(n=n, rb=rb):
            if rb is not None:
                return ctx.msm_resident_device(rb, 0, s.data_ptr(), n)
            return ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n)

        for c, mc in [(c, mc) for c in cs for mc in mcs]:
            ctx.set_window(c)
            ctx.set_pipeline(0, mc)  # one window group (groups > 1 retired)
            ctx.set_timing(False)
            run()
            reps = int(os.environ.get("REPS", "5"))
            t = time.time()
            for _ in range(reps):
                run()
            wall = (time.time() - t) / reps
            ctx.set_timing(True)
            ctx.reset_stats()
            for _ in range(reps):
                run()
            ks = {k: round(ctx.kernel_stats(k)[1] / reps, 4) for k in KERNELS}  # per MSM (sum over groups)
            print(json.dumps({"logn": lg, "c": c, "min_chunk": mc, "resident_rows": rb.rows if rb else 0,
                              "wall_ms": round(wall * 1e3, 3), "Mscalar_s": round(n / wall / 1e6, 2),
                              "kernels_ms": ks}), flush=True)
        if rb is not None:
            rb.release()
    ctx.set_timing(False)
    # fixed-base MSM: table build once per (size, c), then timed MSMs
    fcs = [int(x) for x in os.environ.get("FIXED_C", "").split(",") if x]
    rows = int(os.environ.get("FIXED_ROWS", "0"))  # table rows (0 = one per window)
    for lg in sizes:
        n = 1 << lg
        for c in fcs:
            t = time.time()
            fb = ctx.fixed_bases(curve, d_bases=b.data_ptr(), n=n, c=c, rows=rows)
            build = time.time() - t
            fb.msm_device(s.data_ptr(), n)
            reps = 5
            t = time.time()
            for _ in range(reps):
                fb.msm_device(s.data_ptr(), n)
            wall = (time.time() - t) / reps
            ctx.set_timing(True)
            ctx.reset_stats()
            for _ in range(reps):
                fb.msm_device(s.data_ptr(), n)
            ctx.set_timing(False)
            ks = {k: round(ctx.kernel_stats(k)[1] / reps, 4) for k in KERNELS}
            print(json.dumps({"fixed": True, "logn": lg, "c": fb.c, "windows": fb.windows, "rows": rows,
                              "table_GiB": round(fb.table_bytes / 2**30, 3), "build_s": round(build, 3),
                              "wall_ms": round(wall * 1e3, 3), "Mscalar_s": round(n / wall / 1e6, 2),
                              "kernels_ms": ks}), flush=True)
            fb.release()


if __name__ == "__main__":
    main()
