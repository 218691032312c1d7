"""Strong-scaling projection of SURVEY config 4 (one 2^22 Vesta MSM split over
N GPUs) measured on ONE GPU: rank r of N runs pm_msm_resident_device on its
slice [r n/N, (r+1) n/N) (sharded.split_range), independently of the other
ranks, so the N-GPU step time is max over ranks of that slice's MSM plus the
all-gather of N 64-B partials and N-1 host point additions.  Every rank's
slice is timed here in turn; the collective is not (bench.py --gpus N times
it for real on the driver's 8-GPU node).  Prints one JSON line per N.

Usage (through gpurun): python tools/strong_projection.py [LOGN] [CURVE]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "halo2-aggregation_amd"))
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402
from sharded import split_range  # noqa: E402


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    curve = int(sys.argv[2]) if len(sys.argv) > 2 else H.VESTA
    n = 1 << lg
    ctx = H.Context(0)
    s = torch.empty((n, 4), dtype=torch.int64, device="cuda")
    b = torch.empty((n, 8), dtype=torch.int64, device="cuda")
    ctx.synth_scalars(curve, 0x5EED, 0, n, s.data_ptr())
    ctx.synth_bases(curve, 0xA11CE, 0, n, b.data_ptr())
    torch.cuda.synchronize()
    # settle the GPU first (bench.py settle(): the first ~0.1 s ran ~5 % slow),
    # else the N = 1 baseline is the cold one and every ratio is inflated
    rb = ctx.upload_bases(curve, d_bases=b.data_ptr(), n=n)
    t = time.perf_counter()
    while time.perf_counter() - t < 0.5:
        ctx.msm_resident_device(rb, 0, s.data_ptr(), n)
    rb.release()
    base = None
    for N in (1, 2, 4, 8, 16):
        per_rank = []
        for r in range(N):
            lo, cnt = split_range(r, N, n)
            rb = ctx.upload_bases(curve, d_bases=b[lo:].data_ptr(), n=cnt)
            ctx.msm_resident_device(rb, 0, s[lo:].data_ptr(), cnt)
            reps = 10
            t = time.perf_counter()
            for _ in range(reps):
                ctx.msm_resident_device(rb, 0, s[lo:].data_ptr(), cnt)
            per_rank.append((time.perf_counter() - t) / reps * 1e3)
            rb.release()
            if r >= 1 and N >= 8:  # slices are alike; time two, reuse the max
                break
        t_step = max(per_rank)
        base = base or t_step
        print(json.dumps({"curve": curve, "logn_total": lg, "n_gpus": N, "n_per_gpu": n // N,
                          "ms_per_rank_slice": round(t_step, 4), "projected_speedup_vs_1": round(base / t_step, 3),
                          "projected_Mscalar_s": round(n / (t_step * 1e-3) / 1e6, 1),
                          "note": "collective (all-gather of N x 64 B + host fold) not included"}), flush=True)


if __name__ == "__main__":
    main()
