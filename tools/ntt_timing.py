"""Per-kernel timing of the NTT (pm_fft_device) at several sizes (diagnostic;
PM_NTT_PASSES=2/3 forces the pass count)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402
import workloads as Wk  # noqa: E402

KERNELS = ["ntt_twiddles", "ntt_cols", "ntt_mid", "ntt_rows"]


def mont(r, v):
    v = v * (1 << 256) % r
    return np.array([(v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)], dtype=np.uint64)


def main():
    curve = int(os.environ.get("CURVE", "2"))
    sizes = [int(x) for x in os.environ.get("LOGN", "12,14,16,18,20,22,24").split(",")]
    ctx = H.Context(0)
    r = H.SCALAR_MODULUS[curve]
    for k in sizes:
        n = 1 << k
        a = torch.empty((n, 4), dtype=torch.int64, device="cuda")
        ctx.synth_scalars(curve, 0x77, 0, n, a.data_ptr())
        w = mont(r, Wk.domain_omega(curve, k))
        ctx.fft_device(curve, a.data_ptr(), k, w)  # builds the twiddle table
        reps = 10
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(reps):
            ctx.fft_device(curve, a.data_ptr(), k, w)
        wall = (time.time() - t) / reps
        ctx.set_timing(True)
        ctx.reset_stats()
        for _ in range(reps):
            ctx.fft_device(curve, a.data_ptr(), k, w)
        ctx.set_timing(False)
        ks = {kk: round(ctx.kernel_stats(kk)[1] / reps, 4) for kk in KERNELS}
        gpu_ms = ks["ntt_cols"] + ks["ntt_mid"] + ks["ntt_rows"]
        passes = 3 if ks["ntt_mid"] else 2
        print(json.dumps({"curve": curve, "log_n": k, "passes": passes, "wall_ms": round(wall * 1e3, 4),
                          "Melem_s": round(n / wall / 1e6, 1), "kernels_ms": ks,
                          "hbm_GBs": round(2 * passes * 32 * n / (gpu_ms * 1e-3) / 1e9, 1) if gpu_ms else None}),
              flush=True)


if __name__ == "__main__":
    main()
