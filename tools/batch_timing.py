"""Timing of pm_msm_resident_batch (K MSMs of 2^LOGN host scalars against
resident bases) against K single pm_msm_resident calls; every batch result is
checked against its single call.  PM_BATCH_SPLIT=0 runs each reduction on the
context stream (no overlap with the next MSM's kernels), for A/B."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "halo2-aggregation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402


def main():
    lg = int(os.environ.get("LOGN", "20"))
    K = int(os.environ.get("K", "8"))
    n = 1 << lg
    ctx = H.Context(0)
    b = torch.empty((n, 8), dtype=torch.int64, device="cuda")
    ctx.synth_bases(0, 0xA11CE, 0, n, b.data_ptr())
    rb = ctx.upload_bases(0, d_bases=b.data_ptr(), n=n)
    lists = []
    for j in range(K):
        s = torch.empty((n, 4), dtype=torch.int64, device="cuda")
        ctx.synth_scalars(0, 0x5EED + 17 * j, 0, n, s.data_ptr())
        torch.cuda.synchronize()
        lists.append(s.cpu().numpy().view(np.uint64).copy())
    want = [ctx.msm_resident(rb, 0, L) for L in lists]
    reps = 5
    t = time.time()
    for _ in range(reps):
        for L in lists:
            ctx.msm_resident(rb, 0, L)
    single = (time.time() - t) / reps / K
    got = ctx.msm_resident_batch(rb, 0, lists)
    t = time.time()
    for _ in range(reps):
        got = ctx.msm_resident_batch(rb, 0, lists)
    batch = (time.time() - t) / reps / K
    ok = all(np.array_equal(np.asarray(g), np.asarray(w)) for g, w in zip(got, want))
    print(json.dumps({"logn": lg, "K": K, "split": os.environ.get("PM_BATCH_SPLIT", "1"),
                      "single_ms": round(single * 1e3, 4), "batch_ms_per_msm": round(batch * 1e3, 4),
                      "batch_Mscalar_s": round(n / batch / 1e6, 2), "matches": ok}), flush=True)
    rb.release()


if __name__ == "__main__":
    main()
