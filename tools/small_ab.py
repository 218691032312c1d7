"""A/B of the small-MSM sum kernel's shape (quads vs lanes, slices per
window) on the GPU box: latency of pm_msm_ctx per setting.  Development
sweep: PM_SMALL_LANES / PM_SMALL_SLICES are read by msm_small_impl."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from small_msm_timing import H, P, lat, msm_ref  # noqa: E402


def main():
    ctx = H.Context(0)
    ctx.set_small_msm(H.SMALL_MSM_LIMIT)
    N = 8192
    S = msm_ref.synth_scalars(0, P.SEED_SCALARS, 0, N, threads=16)
    B = msm_ref.synth_bases(0, P.SEED_BASES, 0, N, threads=16)
    for n in (256, 1024, 2048, 4096, 8192):
        s, b = S[:n], B[:n]
        want = None
        for lanes in (0, 1):
            for slices in (4, 8, 16, 32):
                os.environ["PM_SMALL_LANES"] = str(lanes)
                os.environ["PM_SMALL_SLICES"] = str(slices)
                got = ctx.msm(0, s, b)
                want = got if want is None else want
                us = lat(ctx, 0, s, b, 30)
                print(json.dumps({"n": n, "lanes": lanes, "slices": slices, "us": round(us, 1),
                                  "same": bool((got == want).all())}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
