"""Step-by-step diagnostic of the C-ABI on a GPU box (prints before each call)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "halo2-aggregation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import halo2_amd as H  # noqa: E402


def step(msg):
    print(msg, flush=True)


step("devices=%d" % H.device_count())
ctx = H.Context(0)
step("ctx ok")
npz = np.load(os.path.join(ROOT, "tests/golden/msm_vectors.npz"))
for name in ["pallas_n1", "pallas_n33", "pallas_n1024", "bn254_n1"]:
    S, B, E = npz[name + ".scalars"], npz[name + ".bases"], npz[name + ".expected"]
    step("calling %s" % name)
    got = ctx.msm(int(npz[name + ".curve"]), S, B)
    step("%s ok=%s" % (name, np.array_equal(got, E)))
