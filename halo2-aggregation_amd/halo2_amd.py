"""ctypes binding of libpasta_msm.so -- the host-side mirror of the reference
interface for the MSM / multiopen hot path.

The reference is Rust; its FFI for this path would bind the same C-ABI
(include/pasta_msm.h; Rust stub in INTEGRATION.md).  This module exposes the
same entry points to Python so tests and bench.py read like halo2's own call
sites:

    best_multiexp(curve, coeffs, bases)  ->  halo2 arithmetic::best_multiexp
    Context.msm_device(...)              ->  same, inputs resident in HBM

Fails loudly (ImportError) when the HIP library is missing -- there is no CPU
fallback on the product path.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libpasta_msm.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "pasta_msm.h")

PALLAS, VESTA, BN254 = 0, 1, 2
SCALARS_CANONICAL = 1
ACCUM_CURVES = (PALLAS, VESTA, BN254)

_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p


class PmError(RuntimeError):
    pass


def _load():
    # torch wheels bundle their own libamdhip64.so.7.  Loading torch first makes
    # the dynamic loader resolve our DT_NEEDED libamdhip64.so.7 to that same
    # copy, so the process runs ONE HIP runtime whether or not torch is used
    # (two runtimes in one process fail with "No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libpasta_msm.so not built at {LIB_PATH} (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "pm_version": ([], ctypes.c_char_p),
        "pm_last_error": ([], ctypes.c_char_p),
        "pm_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "pm_ctx_create": ([ctypes.c_int, ctypes.POINTER(_vp)], ctypes.c_int),
        "pm_ctx_destroy": ([_vp], ctypes.c_int),
        "pm_ctx_set_stream": ([_vp, _vp], ctypes.c_int),
        "pm_ctx_set_window": ([_vp, ctypes.c_int], ctypes.c_int),
        "pm_ctx_set_timing": ([_vp, ctypes.c_int], ctypes.c_int),
        "pm_ctx_kernel_stats": ([_vp, ctypes.c_char_p, _u64p, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "pm_ctx_reset_stats": ([_vp], ctypes.c_int),
        "pm_msm": ([ctypes.c_int, _u64p, _u64p, ctypes.c_size_t, ctypes.c_uint32, _u64p], ctypes.c_int),
        "pm_msm_ctx": ([_vp, ctypes.c_int, _u64p, _u64p, ctypes.c_size_t, ctypes.c_uint32, _u64p], ctypes.c_int),
        "pm_msm_device": ([_vp, ctypes.c_int, _vp, _vp, ctypes.c_size_t, ctypes.c_uint32, _u64p], ctypes.c_int),
        "pm_msm_multi": ([ctypes.c_int, _u64p, _u64p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int, _u64p],
                         ctypes.c_int),
        "pm_bases_upload": ([_vp, ctypes.c_int, _u64p, ctypes.c_size_t, ctypes.POINTER(_vp)], ctypes.c_int),
        "pm_bases_release": ([_vp], ctypes.c_int),
        "pm_msm_resident": ([_vp, _vp, ctypes.c_size_t, _u64p, ctypes.c_size_t, ctypes.c_uint32, _u64p],
                            ctypes.c_int),
        "pm_point_add": ([ctypes.c_int, _u64p, _u64p, _u64p], ctypes.c_int),
        "pm_synth_scalars": ([_vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32,
                              _vp], ctypes.c_int),
        "pm_synth_bases": ([_vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, _vp],
                           ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return L


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def header_symbols(path=HEADER_PATH):
    """Every `pm_*` function declared in include/pasta_msm.h."""
    txt = open(path).read()
    return sorted(set(re.findall(r"\b(pm_[a-z0-9_]+)\s*\(", txt)))


def _check(rc):
    if rc != 0:
        raise PmError(f"pm error {rc}: {lib().pm_last_error().decode()}")


def _p(a):
    return a.ctypes.data_as(_u64p)


def _as_u64(a, cols):
    return np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, cols)


def best_multiexp(curve, coeffs, bases, canonical=False):
    """sum_i coeffs[i] * bases[i]; coeffs (n,4) u64, bases (n,8) u64 affine
    Montgomery; returns (8,) u64 affine Montgomery, zeros = identity."""
    s, b = _as_u64(coeffs, 4), _as_u64(bases, 8)
    if s.shape[0] != b.shape[0]:
        raise ValueError("coeffs and bases differ in length")
    out = np.zeros(8, dtype=np.uint64)
    _check(lib().pm_msm(curve, _p(s), _p(b), s.shape[0], SCALARS_CANONICAL if canonical else 0, _p(out)))
    return out


def msm_multi(curve, coeffs, bases, ngpu, canonical=False):
    s, b = _as_u64(coeffs, 4), _as_u64(bases, 8)
    out = np.zeros(8, dtype=np.uint64)
    _check(lib().pm_msm_multi(curve, _p(s), _p(b), s.shape[0], SCALARS_CANONICAL if canonical else 0, ngpu,
                              _p(out)))
    return out


def point_add(curve, a, b):
    a, b = _as_u64(a, 8)[0].copy(), _as_u64(b, 8)[0].copy()
    out = np.zeros(8, dtype=np.uint64)
    _check(lib().pm_point_add(curve, _p(a), _p(b), _p(out)))
    return out


def device_count():
    c = ctypes.c_int(0)
    rc = lib().pm_device_count(ctypes.byref(c))
    return c.value if rc == 0 else 0


class Bases:
    def __init__(self, ctx, curve, bases):
        b = _as_u64(bases, 8)
        self.ctx, self.n = ctx, b.shape[0]
        h = _vp()
        _check(lib().pm_bases_upload(ctx.h, curve, _p(b), self.n, ctypes.byref(h)))
        self.h = h

    def release(self):
        if self.h:
            lib().pm_bases_release(self.h)
            self.h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class Context:
    """One device + HIP stream + workspace (pm_ctx)."""

    def __init__(self, device=0):
        h = _vp()
        _check(lib().pm_ctx_create(device, ctypes.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            lib().pm_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle):
        _check(lib().pm_ctx_set_stream(self.h, _vp(stream_handle or 0)))

    def set_window(self, c):
        _check(lib().pm_ctx_set_window(self.h, c))

    def set_timing(self, on=True):
        _check(lib().pm_ctx_set_timing(self.h, 1 if on else 0))

    def reset_stats(self):
        _check(lib().pm_ctx_reset_stats(self.h))

    def kernel_stats(self, name):
        n = ctypes.c_uint64(0)
        ms = ctypes.c_double(0)
        _check(lib().pm_ctx_kernel_stats(self.h, name.encode(), ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value

    def msm(self, curve, coeffs, bases, canonical=False):
        s, b = _as_u64(coeffs, 4), _as_u64(bases, 8)
        out = np.zeros(8, dtype=np.uint64)
        _check(lib().pm_msm_ctx(self.h, curve, _p(s), _p(b), s.shape[0], SCALARS_CANONICAL if canonical else 0,
                                _p(out)))
        return out

    def msm_device(self, curve, d_scalars, d_bases, n, canonical=False):
        out = np.zeros(8, dtype=np.uint64)
        _check(lib().pm_msm_device(self.h, curve, _vp(d_scalars), _vp(d_bases), n,
                                   SCALARS_CANONICAL if canonical else 0, _p(out)))
        return out

    def upload_bases(self, curve, bases):
        return Bases(self, curve, bases)

    def msm_resident(self, bases: Bases, offset, coeffs, canonical=False):
        s = _as_u64(coeffs, 4)
        out = np.zeros(8, dtype=np.uint64)
        _check(lib().pm_msm_resident(self.h, bases.h, offset, _p(s), s.shape[0],
                                     SCALARS_CANONICAL if canonical else 0, _p(out)))
        return out

    def synth_scalars(self, curve, seed, i0, n, d_out, canonical=False):
        _check(lib().pm_synth_scalars(self.h, curve, seed, i0, n, SCALARS_CANONICAL if canonical else 0,
                                      _vp(d_out)))

    def synth_bases(self, curve, seed, i0, n, d_out):
        _check(lib().pm_synth_bases(self.h, curve, seed, i0, n, _vp(d_out)))
