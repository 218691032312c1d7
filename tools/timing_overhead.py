"""Cost of the bench's live HIP-event timing of k_accumulate (diagnostic):
per-step wall of the resident 2^LOGN MSM with timing off, with events around
k_accumulate only, and with events around every launch."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "halo2-aggregation_amd"))
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402


def main():
    lg = int(os.environ.get("LOGN", "20"))
    n = 1 << lg
    ctx = H.Context(0)
    s = torch.empty((n, 4), dtype=torch.int64, device="cuda")
    b = torch.empty((n, 8), dtype=torch.int64, device="cuda")
    ctx.synth_scalars(0, 0x5EED, 0, n, s.data_ptr())
    ctx.synth_bases(0, 0xA11CE, 0, n, b.data_ptr())
    rb = ctx.upload_bases(0, d_bases=b.data_ptr(), n=n)
    for mode in ("off", "accumulate", "all", "off", "accumulate"):
        if mode == "off":
            ctx.set_timing(False)
        elif mode == "all":
            ctx.set_timing(True)
        else:
            ctx.set_timing(True, only=mode)
        for _ in range(3):
            ctx.msm_resident_device(rb, 0, s.data_ptr(), n)
        torch.cuda.synchronize()
        reps = 30
        t = time.perf_counter()
        for _ in range(reps):
            ctx.msm_resident_device(rb, 0, s.data_ptr(), n)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3 / reps
        print(json.dumps({"logn": lg, "timing": mode, "ms_per_msm": round(ms, 4)}), flush=True)
    ctx.set_timing(False)
    rb.release()


if __name__ == "__main__":
    main()
