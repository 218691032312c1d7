"""Host-side sanitizers, CPU only: ``make -C
halo2-aggregation_amd asan`` builds

* the C-ABI library's host code (capi.hip + the per-curve engine objects,
  host-only: plans, argument checks, shape validation, the MSM's host Horner,
  Blake2b) with clang ASan + UBSan -> lib_asan/libpasta_msm.so,
* tests/native/host_asan.cpp (host_ec, inv_bgcd, blake2b, accum_plan) with
  g++ ASan + UBSan, which it runs,
* the C oracle with g++ ASan + UBSan -> oracle/_asan/libmsm_ref.so,

and the CPU tests that drive those libraries run again against the
sanitized builds, each in a child process with its sanitizer runtime
preloaded (any report aborts the child: -fno-sanitize-recover=all,
halt_on_error=1).  No GPU: the entry points that need a device only have
their argument handling exercised (they fail with PM_ERR_NODEV / PM_ERR_ARG).
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "halo2-aggregation_amd")
ASAN_OPTS = "detect_leaks=0:halt_on_error=1:abort_on_error=0:allocator_may_return_null=1"


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-j8", "-C", PKG, "asan"], capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "host_asan: all checks passed" in r.stdout, r.stdout[-2000:]
    return True


def _run(env_extra, args, timeout=900):
    env = dict(os.environ, ASAN_OPTIONS=ASAN_OPTS, UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               PYTHONPATH=os.pathsep.join([PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]),
               **env_extra)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "not gpu"] + args,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    return out


def test_host_harness(built):
    """tests/native/host_asan.cpp ran clean under g++ ASan + UBSan (make asan)."""
    assert os.path.exists(os.path.join(PKG, "build", "host_asan"))


def test_capi_host_paths_under_asan(built):
    """The C-ABI library (host code, clang ASan + UBSan) through the CPU tests
    that call it: symbol exports, argument checks, the host tail's field
    products, vk_repr (Blake2b), shape validation / layout."""
    rt = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so")
    if not rt:
        pytest.skip("clang ASan runtime not found")
    out = _run({"LD_PRELOAD": rt[0], "PM_LIB": os.path.join(PKG, "lib_asan", "libpasta_msm.so"),
                "PM_NO_TORCH": "1"},
               ["tests/test_capi.py", "tests/test_transcript_oracle.py", "tests/test_accum_oracle.py",
                "tests/test_asan_capi_args.py", "-k", "not device_code and not gfx950 and not missing_library"])
    assert " passed" in out


def test_c_oracle_under_asan(built):
    """The C oracle (g++ ASan + UBSan) through its CPU tests: best_multiexp on
    the golden vectors and thread counts, best_fft, the accumulator and
    transcript replay against the Python restatement."""
    rt = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(rt):
        pytest.skip("gcc libasan not found")
    out = _run({"LD_PRELOAD": rt, "PM_REF_LIB": os.path.join(ROOT, "oracle", "_asan", "libmsm_ref.so"),
                "PM_NO_TORCH": "1"},
               ["tests/test_oracle.py", "tests/test_ntt_oracle.py", "tests/test_accum_oracle.py", "-k",
                "c_oracle or c_best_fft or c_accumulator or c_transcript or c_layout or c_shape"])
    assert " passed" in out
