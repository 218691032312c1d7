"""Diagnostic: variable-base MSM with GLV mode on vs off on synthetic inputs
at several sizes (and the C oracle at the small ones)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402
import msm_ref  # noqa: E402

ctx = H.Context(0)
for curve in (0, 2):
    for lg in (12, 13, 14, 16, 17, 18, 19, 20):
        n = 1 << lg
        s = torch.empty((n, 4), dtype=torch.int64, device="cuda")
        b = torch.empty((n, 8), dtype=torch.int64, device="cuda")
        ctx.synth_scalars(curve, 0x5EED, 0, n, s.data_ptr())
        ctx.synth_bases(curve, 0xA11CE, 0, n, b.data_ptr())
        torch.cuda.synchronize()
        ctx.set_glv(True)
        a = ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n)
        ctx.set_glv(False)
        c = ctx.msm_device(curve, s.data_ptr(), b.data_ptr(), n)
        ref = None
        if lg <= 14:
            ref = msm_ref.best_multiexp(curve, s.cpu().numpy().view(np.uint64), b.cpu().numpy().view(np.uint64))
        print(curve, lg, "glv==plain", np.array_equal(a, c),
              "plain==ref" if ref is not None else "", np.array_equal(c, ref) if ref is not None else "",
              "glv==ref" if ref is not None else "", np.array_equal(a, ref) if ref is not None else "", flush=True)
ctx.set_glv(True)
