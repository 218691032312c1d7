"""TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/libmsm_ref.so (the C
restatement of halo2 best_multiexp).  Used by tests/ and bench.py's
cpu_baseline leg; never by the product path."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PM_REF_LIB: an alternative build of the same sources (the ASan / UBSan one,
# oracle/_asan/libmsm_ref.so, in tests/test_asan.py)
_LIB_PATH = os.environ.get("PM_REF_LIB") or os.path.join(_HERE, "libmsm_ref.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.msm_ref_best_multiexp.argtypes = [ctypes.c_int, u64p, u64p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_int, u64p]
        L.msm_ref_best_multiexp.restype = ctypes.c_int
        L.ntt_ref_best_fft.argtypes = [ctypes.c_int, u64p, ctypes.c_uint, u64p, ctypes.c_int]
        L.ntt_ref_best_fft.restype = ctypes.c_int
        for f in (L.msm_ref_synth_scalars, L.msm_ref_synth_bases):
            f.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int, u64p]
            f.restype = ctypes.c_int
        _lib = L
    return _lib


def default_threads():
    """CPUs this process may use (affinity mask), capped by OMP_NUM_THREADS:
    on the GPU pool os.cpu_count() reports the whole machine, not the job's share."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(cap)) if cap.isdigit() and int(cap) > 0 else n)


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def best_multiexp(curve: int, scalars: np.ndarray, bases: np.ndarray, canonical=False, threads=None):
    scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
    bases = np.ascontiguousarray(bases, dtype=np.uint64).reshape(-1, 8)
    assert scalars.shape[0] == bases.shape[0]
    out = np.zeros(8, dtype=np.uint64)
    threads = threads or default_threads()
    rc = lib().msm_ref_best_multiexp(curve, _p(scalars), _p(bases), scalars.shape[0], int(bool(canonical)),
                                     int(threads), _p(out))
    assert rc == 0
    return out


def synth_scalars(curve: int, seed: int, i0: int, n: int, threads=None):
    out = np.zeros((n, 4), dtype=np.uint64)
    rc = lib().msm_ref_synth_scalars(curve, seed, i0, n, int(threads or default_threads()), _p(out))
    assert rc == 0
    return out


def synth_bases(curve: int, seed: int, i0: int, n: int, threads=None):
    out = np.zeros((n, 8), dtype=np.uint64)
    rc = lib().msm_ref_synth_bases(curve, seed, i0, n, int(threads or default_threads()), _p(out))
    assert rc == 0
    return out


def best_fft(curve, values, log_n, omega, threads=1):
    """C restatement of halo2 best_fft (in a copy); values (2^log_n, 4) u64
    Montgomery scalars of `curve`'s scalar field, omega (4,) Montgomery."""
    a = np.ascontiguousarray(values, dtype=np.uint64).reshape(-1, 4).copy()
    w = np.ascontiguousarray(omega, dtype=np.uint64).reshape(4)
    if lib().ntt_ref_best_fft(curve, _p(a), log_n, _p(w), threads) != 0:
        raise ValueError("ntt_ref_best_fft failed")
    return a
