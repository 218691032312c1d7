"""Split scalar copy A/B (round 6): row-table MSMs with scalars in host
memory -- pm_msm_resident (bases resident) and the drop-in pm_msm (host
scalars + host bases, cache warm) -- with one scalar copy
(pm_ctx_set_msm_option MSM_OPT_SPLIT_COPY = 0) against the split copy
(-1, auto), interleaved.  One JSON line per (path, log n, mode, round).
Usage: python tools/split_copy_ab.py > out.jsonl"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "halo2-aggregation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402


def timed(fn, reps):
    fn()
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        got = fn()
    return (time.perf_counter() - t0) * 1e3 / reps, got


def main():
    curve = H.PALLAS
    reps = int(os.environ.get("REPS", "20"))
    for lg in [int(x) for x in os.environ.get("LOGN", "20").split(",")]:
        n = 1 << lg
        ctx = H.Context(0)
        s = torch.empty((n, 4), dtype=torch.int64, device="cuda")
        b = torch.empty((n, 8), dtype=torch.int64, device="cuda")
        ctx.synth_scalars(curve, 0x5EED, 0, n, s.data_ptr())
        ctx.synth_bases(curve, 0xA11CE, 0, n, b.data_ptr())
        torch.cuda.synchronize()
        S = s.cpu().numpy().view(np.uint64).copy()
        B = b.cpu().numpy().view(np.uint64).copy()
        rb = ctx.upload_bases(curve, d_bases=b.data_ptr(), n=n)
        want = ctx.msm_resident_device(rb, 0, s.data_ptr(), n)
        dctx = H.Context(0)
        for _ in range(3):
            dctx.msm(curve, S, B)  # admit the set to the drop-in cache
        for rnd in range(int(os.environ.get("ROUNDS", "3"))):
            for mode in (0, -1):
                ctx.set_msm_option(H.MSM_OPT_SPLIT_COPY, mode)
                dctx.set_msm_option(H.MSM_OPT_SPLIT_COPY, mode)
                ms, got = timed(lambda: ctx.msm_resident(rb, 0, S), reps)
                dms, dgot = timed(lambda: dctx.msm(curve, S, B), reps)
                ctx.set_timing(True, only="bucket_seg")
                ctx.reset_stats()
                for _ in range(5):
                    ctx.msm_resident(rb, 0, S)
                ctx.set_timing(False)
                seg = ctx.kernel_stats("bucket_seg")[1] / 5
                print(json.dumps({"logn": lg, "round": rnd, "split_copy": "auto" if mode < 0 else "off",
                                  "bucket_seg_ms": round(seg, 4),
                                  "pm_msm_resident_ms": round(ms, 4), "dropin_pm_msm_ms": round(dms, 4),
                                  "matches": bool(np.array_equal(got, want) and np.array_equal(dgot, want))}),
                      flush=True)
        st = dctx.dropin_stats()
        print(json.dumps({"logn": lg, "dropin_stats": st, "spec": dctx.dropin_spec_stats()}), flush=True)
        rb.release()
        ctx.close()
        dctx.close()


if __name__ == "__main__":
    main()
