"""Host-input MSM paths at 2^20 (diagnostic): the pageable copy alone, the
resident MSM with device scalars / host scalars (chunked copy behind the
histogram pass), and the drop-in pm_msm_ctx (bases digest on host threads).
Env knobs of the library: PM_H2D_CHUNKS, PM_POOL_THREADS."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "halo2-aggregation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402


def t_ms(f, k=10):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        f()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) * 1e3 / k, 4)


def main():
    n = 1 << int(os.environ.get("LOGN", "20"))
    ctx = H.Context(0)
    s = torch.empty((n, 4), dtype=torch.int64, device="cuda")
    b = torch.empty((n, 8), dtype=torch.int64, device="cuda")
    ctx.synth_scalars(0, 0x5EED, 0, n, s.data_ptr())
    ctx.synth_bases(0, 0xA11CE, 0, n, b.data_ptr())
    torch.cuda.synchronize()
    S = s.cpu().numpy().view(np.uint64).copy()
    B = b.cpu().numpy().view(np.uint64).copy()
    St = torch.from_numpy(S.view(np.int64))
    rb = ctx.upload_bases(0, d_bases=b.data_ptr(), n=n)
    out = {"n": n, "h2d_chunks": os.environ.get("PM_H2D_CHUNKS"), "pool": os.environ.get("PM_POOL_THREADS"),
           "copy_pageable_ms": t_ms(lambda: s.copy_(St)),
           "resident_device_ms": t_ms(lambda: ctx.msm_resident_device(rb, 0, s.data_ptr(), n)),
           "resident_host_ms": t_ms(lambda: ctx.msm_resident(rb, 0, S)),
           "dropin_ms": t_ms(lambda: ctx.msm(0, S, B))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
