"""CPU tests of the C-ABI boundary: the library builds, loads and exports
every symbol include/pasta_msm.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

import halo2_amd as H
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exists_and_loads():
    assert os.path.exists(H.LIB_PATH)
    assert H.lib().pm_version().decode().startswith("pasta_msm")


def test_exports_every_header_symbol():
    syms = H.header_symbols()
    assert len(syms) >= 20
    L = ctypes.CDLL(H.LIB_PATH)
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_header_is_plain_c():
    txt = open(H.HEADER_PATH).read()
    assert 'extern "C"' in txt
    code = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)  # declarations only, no comments
    assert not re.search(r"\b(torch|at::|std::|hip[A-Z])", code)


def test_abi_version_matches_header():
    """pm_abi_version() == PM_ABI_VERSION: what a binding asserts at load."""
    m = re.search(r"#define PM_ABI_VERSION (\d+)", open(H.HEADER_PATH).read())
    assert m and H.abi_version() == int(m.group(1))


def test_crossover_threshold_is_one_number():
    """The GPU/CPU crossover of the drop-in: the header's PM_MSM_GPU_MIN_N,
    the Rust shim's constant in INTEGRATION.md and halo2_amd.MSM_GPU_MIN_N are
    the same measured number (bench.py small_n)."""
    h = re.search(r"#define PM_MSM_GPU_MIN_N (\d+)", open(H.HEADER_PATH).read())
    doc = re.search(r"pub const PM_MSM_GPU_MIN_N: usize = (\d+);", open(os.path.join(ROOT, "INTEGRATION.md")).read())
    assert h and doc
    assert int(h.group(1)) == int(doc.group(1)) == H.MSM_GPU_MIN_N


def test_small_msm_constants():
    """The small-MSM path's default threshold and limit: header == Python."""
    src = open(H.HEADER_PATH).read()
    d = re.search(r"#define PM_SMALL_MSM_DEFAULT (\d+)", src)
    lim = re.search(r"#define PM_SMALL_MSM_LIMIT (\d+)", src)
    assert d and lim
    assert (int(d.group(1)), int(lim.group(1))) == (H.SMALL_MSM_DEFAULT, H.SMALL_MSM_LIMIT)


def test_last_error_is_thread_local_string():
    assert isinstance(H.lib().pm_last_error(), bytes)


def test_gfx950_code_object_embedded():
    blob = open(H.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_device_code_has_every_launched_kernel():
    """Each kernel the host driver launches has a gfx950 kernel descriptor
    (.kd) in the embedded code objects (a missing device instantiation aborts
    at launch with 'Cannot find Symbol')."""
    blob = open(H.LIB_PATH, "rb").read()
    kds = set(re.findall(rb"(_ZN2pm[A-Za-z0-9_]+)\.kd", blob))
    names = [k.decode() for k in kds]

    def count(stem):
        return sum(1 for n in names if stem in n)

    assert count("11k_sort_hist") == 3 * 16 * 2  # 3 scalar fields x 16 window counts x {2-B, 4-B digits}
    assert count("14k_bucket_seg_q") == 3 * 3  # one sorted list / the split scalar copy's two or three (round 6)
    for stem in ("12k_accumulate", "13k_bucket_bits", "15k_bases_to_r261",
                 "16k_selftest_field", "9k_acc_sum", "13k_acc_scalars", "12k_acc_powers",
                 "15k_synth_scalars", "13k_synth_bases", "14k_transcript_s", "12k_transcriptI", "14k_acc_powers_s"):
        assert count(stem) == 3, stem
    assert count("13k_acc_termadd") == 3 * 2  # lane groups / quad-cooperative form
    assert count("13k_acc_termmul") == 3 * 2  # windows: one / two terms per lane (joint form retired, round 6)
    # the retired A/B kernels are gone (GLV mode, separate fixups, bit-sum fold pass)
    for stem in ("15k_sort_hist_glv", "11k_bases_glv", "7k_fixupI", "12k_fixup_long", "13k_fixup_short",
                 "12k_bucket_segI", "14k_bits_combine"):
        assert count(stem) == 0, stem
    assert count("13k_sort_coarse") == 4 * 4  # {2-B, 4-B digits} x {4-B, 8-B entries} x points per thread 1..8
    assert count("11k_sort_fine") == 2
    for stem in ("13k_scan_reduce", "11k_scan_down"):
        assert count(stem) == 1, stem


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_host_tail_adx_product(curve):
    """CPU: the host Horner tail's mulx/adcx/adox Montgomery product (and the
    doubling / addition chain built on it) equals the portable product, the
    Jacobian chain the XYZZ chain, and the split tail (sets claimed by pool
    threads, 1 / 3 / 16 of them) the single Horner on random terms."""
    got = H.selftest_host(curve, seed=0xC0FFEE + curve, n=20000)
    if got is None:
        pytest.skip("CPU without BMI2/ADX")
    assert got == 0


def test_missing_library_fails_loudly():
    """The product path has no CPU fallback: without the HIP library every
    entry point raises instead of computing (here: best_multiexp, the drop-in MSM)."""
    import subprocess
    import sys

    code = ("import numpy as np, halo2_amd as H\n"
            "try:\n"
            "    H.best_multiexp(H.PALLAS, np.zeros((1, 4), np.uint64), np.zeros((1, 8), np.uint64))\n"
            "except ImportError as e:\n"
            "    print('ImportError:', e)\n"
            "else:\n"
            "    print('computed without the library')\n")
    env = dict(os.environ, PM_LIB="/nonexistent/libpasta_msm.so",
               PYTHONPATH=os.path.join(ROOT, "halo2-aggregation_amd"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert "ImportError: libpasta_msm.so not built at /nonexistent" in r.stdout, r.stdout + r.stderr
