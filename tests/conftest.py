import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    d = os.path.join(ROOT, "tests", "golden")
    npz = np.load(os.path.join(d, "msm_vectors.npz"), allow_pickle=False)
    idx = json.load(open(os.path.join(d, "msm_vectors.json")))
    cases = {}
    for name in idx:
        cases[name] = dict(curve=int(npz[f"{name}.curve"]), scalars=npz[f"{name}.scalars"],
                           bases=npz[f"{name}.bases"], expected=npz[f"{name}.expected"])
    return cases


@pytest.fixture(scope="session")
def gpu_ctx():
    import halo2_amd as H

    if H.device_count() < 1:
        pytest.fail("GPU test requested but no HIP device is visible")
    return H.Context(0)
