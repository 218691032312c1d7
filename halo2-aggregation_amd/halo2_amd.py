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
LIB_PATH = os.environ.get("PM_LIB") or os.path.join(_HERE, "lib", "libpasta_msm.so")  # PM_LIB: A/B builds
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "pasta_msm.h")

PALLAS, VESTA, BN254 = 0, 1, 2
ACC_OPT_TWIST, ACC_OPT_TAIL_STREAM, ACC_OPT_TERMS_PER_LANE, ACC_OPT_TRANSCRIPT = 1, 2, 3, 4  # pm_ctx_set_accum_option
MSM_OPT_SPLIT_COPY = 1  # pm_ctx_set_msm_option
SPLIT_COPY_MIN_N = 262144  # PM_SPLIT_COPY_MIN_N
SCALARS_CANONICAL = 1
LEGACY_STREAM = 1  # PM_STREAM_LEGACY: the HIP legacy null stream
# PM_MSM_GPU_MIN_N: below this many terms the Rust shim would keep halo2's CPU
# multiexp; with the small-MSM path the GPU wins from one
# term.  best_multiexp below runs every n on the GPU: there is no CPU path here.
MSM_GPU_MIN_N = 1
# PM_SMALL_MSM_DEFAULT / PM_SMALL_MSM_LIMIT: the small-MSM path's default and
# largest threshold (pm_ctx_set_small_msm)
SMALL_MSM_DEFAULT = 16384
SMALL_MSM_LIMIT = 65536
ACCUM_CURVES = (PALLAS, VESTA, BN254)
# per-proof status bits of the proof-byte entries (pm_*_proofs*)
PROOF_BAD_POINT = 8
PROOF_BAD_SCALAR = 16

_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_szp = ctypes.POINTER(ctypes.c_size_t)


class PmError(RuntimeError):
    pass


# ------------------------------------------------ accumulator shape (C mirror)
class PmQuery(ctypes.Structure):
    _fields_ = [("column", ctypes.c_uint32), ("rotation", ctypes.c_int32)]


class PmPermColumn(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("query_index", ctypes.c_uint32)]


_u32p = ctypes.POINTER(ctypes.c_uint32)


class PmProofShape(ctypes.Structure):
    _fields_ = [
        ("log_n", ctypes.c_uint32), ("blinding_factors", ctypes.c_uint32),
        ("num_instance_columns", ctypes.c_uint32), ("num_advice_columns", ctypes.c_uint32),
        ("num_fixed_columns", ctypes.c_uint32), ("num_lookups", ctypes.c_uint32),
        ("perm_chunk_len", ctypes.c_uint32), ("quotient_degree", ctypes.c_uint32),
        ("n_instance_queries", ctypes.c_uint32), ("n_advice_queries", ctypes.c_uint32),
        ("n_fixed_queries", ctypes.c_uint32), ("n_perm_columns", ctypes.c_uint32),
        ("instance_queries", ctypes.POINTER(PmQuery)), ("advice_queries", ctypes.POINTER(PmQuery)),
        ("fixed_queries", ctypes.POINTER(PmQuery)), ("perm_columns", ctypes.POINTER(PmPermColumn)),
        ("gate_code", _u32p), ("gate_code_len", ctypes.c_uint32),
        ("lookup_input_code", _u32p), ("lookup_input_code_len", ctypes.c_uint32),
        ("lookup_table_code", _u32p), ("lookup_table_code_len", ctypes.c_uint32),
        ("constants", _u64p), ("n_constants", ctypes.c_uint32),
        ("omega", ctypes.c_uint64 * 4), ("delta", ctypes.c_uint64 * 4), ("g1", ctypes.c_uint64 * 8),
        ("fixed_commitments", _u64p), ("sigma_commitments", _u64p),
    ]


# scalar-field moduli (pasta_msm.h curve ids): the field of the accumulator's scalars
SCALAR_MODULUS = {
    0: 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001,  # Pallas -> Fq
    1: 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001,  # Vesta -> Fp
    2: 21888242871839275222246405745257275088548364400416034343698204186575808495617,  # BN254 Fr
}
EXPR_OPS = {"const": 1, "fixed": 2, "advice": 3, "instance": 4, "neg": 5, "sum": 6, "prod": 7, "scaled": 8}


def _mont_limbs(v, r):
    v = v * (1 << 256) % r
    return [(v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)]


def compile_expressions(exprs, constants):
    """halo2 Expression trees (tuples: ("const", c) ("fixed", q) ("advice", q)
    ("instance", q) ("neg", e) ("sum", a, b) ("prod", a, b) ("scaled", e, c))
    -> postfix pm_expr_op words; constants are appended to ``constants``."""
    code = []

    def cidx(c):
        constants.append(c)
        return len(constants) - 1

    def walk(e):
        op = e[0]
        if op == "const":
            code.append(EXPR_OPS[op] | cidx(e[1]) << 8)
        elif op in ("fixed", "advice", "instance"):
            code.append(EXPR_OPS[op] | e[1] << 8)
        elif op == "neg":
            walk(e[1])
            code.append(EXPR_OPS[op])
        elif op in ("sum", "prod"):
            walk(e[1])
            walk(e[2])
            code.append(EXPR_OPS[op])
        elif op == "scaled":
            walk(e[1])
            code.append(EXPR_OPS[op] | cidx(e[2]) << 8)
        else:
            raise ValueError(f"unknown expression node {op!r}")

    for e in exprs:
        walk(e)
        code.append(0)  # PM_EXPR_END
    return code


class ProofShape:
    """Owns the arrays behind one pm_proof_shape (the VerifyingKey view of
    /root/reference/src/verifier.rs:227-285).  omega / delta / constants are
    canonical integers of the curve's scalar field; g1 and the VK commitments
    are (8,) / (n, 8) u64 affine Montgomery limbs."""

    def __init__(self, curve, *, log_n, blinding_factors, num_instance_columns, num_advice_columns,
                 num_fixed_columns, num_lookups, perm_chunk_len, quotient_degree, instance_queries,
                 advice_queries, fixed_queries, perm_columns, gates, lookup_inputs, lookup_tables, omega, delta,
                 g1, fixed_commitments, sigma_commitments):
        r = SCALAR_MODULUS[curve]
        self.curve = curve
        consts = []
        gate_code = compile_expressions(gates, consts)
        lkin = compile_expressions(lookup_inputs, consts)
        lktab = compile_expressions(lookup_tables, consts)

        def qarr(qs):
            a = (PmQuery * max(1, len(qs)))()
            for i, (c, rot) in enumerate(qs):
                a[i] = PmQuery(c, rot)
            return a

        self._keep = []

        def u32(xs):
            a = np.ascontiguousarray(np.array(xs if xs else [0], dtype=np.uint32))
            self._keep.append(a)
            return a.ctypes.data_as(_u32p)

        def u64(a):
            a = np.ascontiguousarray(np.array(a, dtype=np.uint64).reshape(-1))
            if a.size == 0:
                a = np.zeros(8, dtype=np.uint64)
            self._keep.append(a)
            return a.ctypes.data_as(_u64p)

        iq, aq, fq = qarr(instance_queries), qarr(advice_queries), qarr(fixed_queries)
        pc = (PmPermColumn * max(1, len(perm_columns)))()
        for i, (k, q) in enumerate(perm_columns):
            pc[i] = PmPermColumn(k, q)
        self._keep += [iq, aq, fq, pc]
        cl = [_mont_limbs(c % r, r) for c in consts]
        s = PmProofShape()
        s.log_n, s.blinding_factors = log_n, blinding_factors
        s.num_instance_columns, s.num_advice_columns = num_instance_columns, num_advice_columns
        s.num_fixed_columns, s.num_lookups = num_fixed_columns, num_lookups
        s.perm_chunk_len, s.quotient_degree = perm_chunk_len, quotient_degree
        s.n_instance_queries, s.n_advice_queries = len(instance_queries), len(advice_queries)
        s.n_fixed_queries, s.n_perm_columns = len(fixed_queries), len(perm_columns)
        s.instance_queries, s.advice_queries, s.fixed_queries, s.perm_columns = iq, aq, fq, pc
        s.gate_code, s.gate_code_len = u32(gate_code), len(gate_code)
        s.lookup_input_code, s.lookup_input_code_len = u32(lkin), len(lkin)
        s.lookup_table_code, s.lookup_table_code_len = u32(lktab), len(lktab)
        s.constants, s.n_constants = u64(cl), len(cl)
        s.omega[:] = _mont_limbs(omega % r, r)
        s.delta[:] = _mont_limbs(delta % r, r)
        s.g1[:] = [int(x) for x in np.asarray(g1, dtype=np.uint64).reshape(8)]
        s.fixed_commitments = u64(fixed_commitments)
        s.sigma_commitments = u64(sigma_commitments)
        self.c = s

    def layout(self):
        """(points_per_proof, scalars_per_proof, num_sets)"""
        a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().pm_shape_layout(ctypes.byref(self.c), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value


def _load():
    # torch wheels bundle their own libamdhip64.so.7.  Loading torch first makes
    # the dynamic loader resolve our DT_NEEDED libamdhip64.so.7 to that same
    # copy, so the process runs ONE HIP runtime whether or not torch is used
    # (two runtimes in one process fail with "No HIP GPUs are available").
    if not os.environ.get("PM_NO_TORCH"):  # PM_NO_TORCH: host-only checks (tests/test_asan.py)
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libpasta_msm.so not built at {LIB_PATH} (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "pm_version": ([], ctypes.c_char_p),
        "pm_abi_version": ([], ctypes.c_int),
        "pm_last_error": ([], ctypes.c_char_p),
        "pm_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "pm_ctx_create": ([ctypes.c_int, ctypes.POINTER(_vp)], ctypes.c_int),
        "pm_ctx_destroy": ([_vp], ctypes.c_int),
        "pm_ctx_set_stream": ([_vp, _vp], ctypes.c_int),
        "pm_ctx_use_own_stream": ([_vp], ctypes.c_int),
        "pm_ctx_set_window": ([_vp, ctypes.c_int], ctypes.c_int),
        "pm_ctx_set_small_msm": ([_vp, ctypes.c_size_t], ctypes.c_int),
        "pm_ctx_set_pipeline": ([_vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "pm_ctx_set_accum_split": ([_vp, ctypes.c_int], ctypes.c_int),
        "pm_ctx_set_accum_ladder": ([_vp, ctypes.c_int], ctypes.c_int),
        "pm_ctx_set_accum_option": ([_vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "pm_ctx_set_msm_option": ([_vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "pm_ctx_set_glv": ([_vp, ctypes.c_int], ctypes.c_int),
        "pm_ctx_set_timing": ([_vp, ctypes.c_int], ctypes.c_int),
        "pm_ctx_set_timing_filter": ([_vp, ctypes.c_char_p], ctypes.c_int),
        "pm_ctx_kernel_stats": ([_vp, ctypes.c_char_p, _u64p, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "pm_ctx_reset_stats": ([_vp], ctypes.c_int),
        "pm_ctx_dropin_stats": ([_vp, _u64p, _u64p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_size_t)],
                                ctypes.c_int),
        "pm_ctx_dropin_spec_stats": ([_vp, _u64p, _u64p], ctypes.c_int),
        "pm_ctx_dropin_oom_stats": ([_vp, _u64p, _u64p], ctypes.c_int),
        "pm_ctx_dropin_small_stats": ([_vp, _u64p, _u64p, ctypes.POINTER(ctypes.c_int), _szp], ctypes.c_int),
        "pm_ctx_dropin_clear": ([_vp], ctypes.c_int),
        "pm_ctx_dropin_key_id": ([_vp, _u64p], ctypes.c_int),
        "pm_msm": ([ctypes.c_int, _u64p, _u64p, ctypes.c_size_t, ctypes.c_uint32, _u64p], ctypes.c_int),
        # plain addresses (ints) for the drop-in call: a.ctypes.data_as() costs
        # ~1.5 us per pointer, a third of a short MSM call's binding overhead
        "pm_msm_ctx": ([_vp, ctypes.c_int, _vp, _vp, ctypes.c_size_t, ctypes.c_uint32, _vp], ctypes.c_int),
        "pm_msm_device": ([_vp, ctypes.c_int, _vp, _vp, ctypes.c_size_t, ctypes.c_uint32, _u64p], ctypes.c_int),
        "pm_msm_multi": ([ctypes.c_int, _u64p, _u64p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int, _u64p],
                         ctypes.c_int),
        "pm_bases_upload": ([_vp, ctypes.c_int, _u64p, ctypes.c_size_t, ctypes.POINTER(_vp)], ctypes.c_int),
        "pm_bases_upload_device": ([_vp, ctypes.c_int, _vp, ctypes.c_size_t, ctypes.POINTER(_vp)], ctypes.c_int),
        "pm_bases_release": ([_vp], ctypes.c_int),
        "pm_bases_info": ([_vp, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int),
                           ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "pm_msm_resident_device": ([_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_size_t, ctypes.c_uint32, _u64p],
                                   ctypes.c_int),
        "pm_ctx_set_h2d_threads": ([_vp, ctypes.c_int], ctypes.c_int),
        "pm_msm_resident_batch": ([_vp, _vp, ctypes.c_size_t, ctypes.POINTER(_u64p), ctypes.c_size_t,
                                   ctypes.c_size_t, ctypes.c_uint32, _u64p], ctypes.c_int),
        "pm_msm_resident": ([_vp, _vp, ctypes.c_size_t, _u64p, ctypes.c_size_t, ctypes.c_uint32, _u64p],
                            ctypes.c_int),
        "pm_msm_resident_many": ([_vp, _vp, ctypes.c_size_t, _szp, _szp, _u64p, ctypes.c_uint32, _u64p],
                                 ctypes.c_int),
        "pm_msm_resident_many_device": ([_vp, _vp, ctypes.c_size_t, _szp, _szp, _vp, ctypes.c_uint32, _u64p],
                                        ctypes.c_int),
        "pm_bases_many_prepare": ([_vp, _vp, ctypes.c_size_t], ctypes.c_int),
        "pm_bases_many_info": ([_vp, _szp, ctypes.POINTER(ctypes.c_int), _szp], ctypes.c_int),
        "pm_point_add": ([ctypes.c_int, _u64p, _u64p, _u64p], ctypes.c_int),
        "pm_points_sum": ([ctypes.c_int, _u64p, ctypes.c_size_t, _u64p], ctypes.c_int),
        "pm_selftest_field": ([_vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t, _u64p], ctypes.c_int),
        "pm_selftest_host": ([ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t, _u64p], ctypes.c_int),
        "pm_synth_scalars": ([_vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32,
                              _vp], ctypes.c_int),
        "pm_synth_bases": ([_vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, _vp],
                           ctypes.c_int),
        "pm_shape_layout": ([ctypes.POINTER(PmProofShape), ctypes.POINTER(ctypes.c_uint32),
                             ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
        "pm_accum_batch": ([_vp, ctypes.c_int, ctypes.POINTER(PmProofShape), ctypes.c_size_t, _u64p, _u64p, _u64p,
                            _u64p, _u64p, _u32p], ctypes.c_int),
        "pm_accum_batch_device": ([_vp, ctypes.c_int, ctypes.POINTER(PmProofShape), ctypes.c_size_t, _vp, _vp, _vp,
                                   _vp, _vp, _vp], ctypes.c_int),
        "pm_accum_batch_multi": ([ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_int, ctypes.POINTER(PmProofShape),
                                  ctypes.c_size_t, _u64p, _u64p, _u64p, _u64p, _u64p, _u64p, _u64p, _u32p],
                                 ctypes.c_int),
        "pm_fixed_bases_create": ([_vp, ctypes.c_int, _u64p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(_vp)],
                                  ctypes.c_int),
        "pm_fixed_bases_create_rows": ([_vp, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_int, ctypes.POINTER(_vp)], ctypes.c_int),
        "pm_fixed_bases_create_device": ([_vp, ctypes.c_int, _vp, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.POINTER(_vp)], ctypes.c_int),
        "pm_fixed_bases_info": ([_vp, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "pm_fixed_bases_release": ([_vp], ctypes.c_int),
        "pm_msm_fixed": ([_vp, _vp, _u64p, ctypes.c_size_t, ctypes.c_uint32, _u64p], ctypes.c_int),
        "pm_msm_fixed_device": ([_vp, _vp, _vp, ctypes.c_size_t, ctypes.c_uint32, _u64p], ctypes.c_int),
        "pm_fft": ([_vp, ctypes.c_int, _u64p, ctypes.c_uint32, _u64p, _u64p], ctypes.c_int),
        "pm_fft_device": ([_vp, ctypes.c_int, _vp, ctypes.c_uint32, _u64p, _u64p], ctypes.c_int),
        "pm_vk_transcript_repr": ([ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, _u64p], ctypes.c_int),
        "pm_transcript_batch": ([_vp, ctypes.c_int, ctypes.POINTER(PmProofShape), ctypes.c_size_t, _u64p, _u64p,
                                 _u64p, _u64p, _u32p], ctypes.c_int),
        "pm_transcript_batch_device": ([_vp, ctypes.c_int, ctypes.POINTER(PmProofShape), ctypes.c_size_t, _u64p,
                                        _vp, _vp, _vp, _vp], ctypes.c_int),
        "pm_accum_batch_transcript": ([_vp, ctypes.c_int, ctypes.POINTER(PmProofShape), ctypes.c_size_t, _u64p,
                                       _u64p, _u64p, _u64p, _u64p, _u64p, _u32p], ctypes.c_int),
        "pm_accum_batch_transcript_device": ([_vp, ctypes.c_int, ctypes.POINTER(PmProofShape), ctypes.c_size_t,
                                              _u64p, _vp, _vp, _vp, _vp, _vp, _vp], ctypes.c_int),
        "pm_proof_size": ([ctypes.POINTER(PmProofShape), ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "pm_decode_proofs": ([_vp, ctypes.c_int, ctypes.POINTER(PmProofShape), ctypes.c_size_t, ctypes.c_char_p,
                              ctypes.c_size_t, _u64p, _u64p, _u64p, _u32p], ctypes.c_int),
        "pm_decode_proofs_device": ([_vp, ctypes.c_int, ctypes.POINTER(PmProofShape), ctypes.c_size_t, _vp,
                                     ctypes.c_size_t, _vp, _vp, _vp, _vp], ctypes.c_int),
        "pm_accum_batch_proofs": ([_vp, ctypes.c_int, ctypes.POINTER(PmProofShape), ctypes.c_size_t, _u64p,
                                   ctypes.c_char_p, ctypes.c_size_t, _u64p, _u64p, _u64p, _u64p, _u32p],
                                  ctypes.c_int),
        "pm_accum_batch_proofs_device": ([_vp, ctypes.c_int, ctypes.POINTER(PmProofShape), ctypes.c_size_t, _u64p,
                                          _vp, ctypes.c_size_t, _vp, _vp, _vp, _vp, _vp], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        if not hasattr(L, name) and os.environ.get("PM_LIB"):
            continue  # an older A/B build (PM_LIB) without this entry point
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


def abi_version():
    """pm_abi_version(): bumped on every C-ABI signature / meaning change."""
    return int(lib().pm_abi_version())


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


def points_sum(curve, points):
    """pm_points_sum: the sum of n affine points ((n, 8) u64, (0,0) =
    identity) in one call -- the fold of a sharded MSM's partials."""
    pts = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1, 8)
    out = np.zeros(8, dtype=np.uint64)
    _check(lib().pm_points_sum(curve, _p(pts), pts.shape[0], _p(out)))
    return out


def accum_batch_multi(contexts, shape, points, scalars, challenges=None, vk_repr=None):
    """pm_accum_batch_multi: the proof batch sharded over `contexts` (one per
    device).  challenges None -> replay the transcript from vk_repr.
    Returns (challenges (B,7,4), quads (B,4,8), h_eval (B,4), status (B,))."""
    npts, nsc, _ = shape.layout()
    p = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1, npts, 8)
    B = p.shape[0]
    s = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(B, nsc, 4)
    ch_in = None if challenges is None else np.ascontiguousarray(challenges, dtype=np.uint64).reshape(B, 7, 4)
    vk = None if vk_repr is None else np.ascontiguousarray(vk_repr, dtype=np.uint64).reshape(4)
    ch = np.zeros((B, 7, 4), dtype=np.uint64)
    quads = np.zeros((B, 4, 8), dtype=np.uint64)
    hev = np.zeros((B, 4), dtype=np.uint64)
    st = np.zeros(B, dtype=np.uint32)
    arr = (_vp * len(contexts))(*[c.h for c in contexts])
    _check(lib().pm_accum_batch_multi(arr, len(contexts), shape.curve, ctypes.byref(shape.c), B, _p(p), _p(s),
                                      _p(ch_in) if ch_in is not None else None, _p(vk) if vk is not None else None,
                                      _p(ch), _p(quads), _p(hev), st.ctypes.data_as(_u32p)))
    return ch, quads, hev, st


def selftest_host(curve, seed=1, n=4096):
    """pm_selftest_host: the host tail's BMI2/ADX Montgomery product and its
    doubling / addition chain against the portable code (CPU only).  None when
    the CPU lacks BMI2/ADX."""
    m = ctypes.c_uint64(0)
    rc = lib().pm_selftest_host(curve, seed, n, ctypes.byref(m))
    if rc == -4:  # PM_ERR_UNSUPPORTED
        return None
    _check(rc)
    return m.value


def vk_transcript_repr(curve, pinned: bytes):
    """pm_vk_transcript_repr: the scalar the verifier absorbs first
    (src/verifier.rs:341-358), Montgomery limbs (4,) u64.  Host only."""
    out = np.zeros(4, dtype=np.uint64)
    _check(lib().pm_vk_transcript_repr(curve, pinned, len(pinned), _p(out)))
    return out


def proof_size(shape: ProofShape):
    """pm_proof_size: bytes of one serialized proof of this shape."""
    n = ctypes.c_size_t(0)
    _check(lib().pm_proof_size(ctypes.byref(shape.c), ctypes.byref(n)))
    return n.value


def device_count():
    c = ctypes.c_int(0)
    rc = lib().pm_device_count(ctypes.byref(c))
    return c.value if rc == 0 else 0


class Bases:
    """Device-resident SRS bases (pm_bases_upload / pm_bases_upload_device):
    host `bases` (n x 8 u64), or `d_bases` (device pointer) with `n`."""

    def __init__(self, ctx, curve, bases=None, d_bases=None, n=None):
        self.ctx, self.curve = ctx, curve
        h = _vp()
        if d_bases is not None:
            self.n = int(n)
            _check(lib().pm_bases_upload_device(ctx.h, curve, _vp(d_bases), self.n, ctypes.byref(h)))
        else:
            b = _as_u64(bases, 8)
            self.n = b.shape[0]
            _check(lib().pm_bases_upload(ctx.h, curve, _p(b), self.n, ctypes.byref(h)))
        self.h = h
        nn, rr, bb = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_size_t()
        _check(lib().pm_bases_info(h, ctypes.byref(nn), ctypes.byref(rr), ctypes.byref(bb)))
        self.rows, self.device_bytes = rr.value, bb.value  # rows of [2^{256 j / rows}] P kept at upload

    def many_info(self):
        """pm_bases_many_info -> (prefix n, window c, device bytes) of the
        multiples table (zeros before the first pm_msm_resident_many)."""
        nn, cc, bb = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_size_t()
        _check(lib().pm_bases_many_info(self.h, ctypes.byref(nn), ctypes.byref(cc), ctypes.byref(bb)))
        return nn.value, cc.value, bb.value

    def release(self):
        if self.h:
            lib().pm_bases_release(self.h)
            self.h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class FixedBases:
    """Fixed-base table (pm_fixed_bases_create*): [2^{o_w}] P_i for every
    window offset (rows = 0), or for every (W / rows)-th one
    (pm_fixed_bases_create_rows), resident on ctx's device.  ``bases`` is a
    host (n, 8) u64 array, or a device pointer with ``n`` given."""

    def __init__(self, ctx, curve, bases=None, c=0, d_bases=None, n=None, rows=0):
        self.ctx, self.curve, self.rows = ctx, curve, rows
        h = _vp()
        if rows:
            if d_bases is not None:
                _check(lib().pm_fixed_bases_create_rows(ctx.h, curve, _vp(d_bases), 1, n, c, rows, ctypes.byref(h)))
            else:
                b = _as_u64(bases, 8)
                _check(lib().pm_fixed_bases_create_rows(ctx.h, curve, _vp(b.ctypes.data), 0, b.shape[0], c, rows,
                                                        ctypes.byref(h)))
        elif d_bases is not None:
            _check(lib().pm_fixed_bases_create_device(ctx.h, curve, _vp(d_bases), n, c, ctypes.byref(h)))
        else:
            b = _as_u64(bases, 8)
            _check(lib().pm_fixed_bases_create(ctx.h, curve, _p(b), b.shape[0], c, ctypes.byref(h)))
        self.h = h
        nn, cc, ww, tb = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_int(), ctypes.c_size_t()
        _check(lib().pm_fixed_bases_info(h, ctypes.byref(nn), ctypes.byref(cc), ctypes.byref(ww), ctypes.byref(tb)))
        self.n, self.c, self.windows, self.table_bytes = nn.value, cc.value, ww.value, tb.value

    def msm(self, coeffs, canonical=False):
        s = _as_u64(coeffs, 4)
        out = np.zeros(8, dtype=np.uint64)
        _check(lib().pm_msm_fixed(self.ctx.h, self.h, _p(s), s.shape[0], SCALARS_CANONICAL if canonical else 0,
                                  _p(out)))
        return out

    def msm_device(self, d_scalars, n, canonical=False):
        out = np.zeros(8, dtype=np.uint64)
        _check(lib().pm_msm_fixed_device(self.ctx.h, self.h, _vp(d_scalars), n,
                                         SCALARS_CANONICAL if canonical else 0, _p(out)))
        return out

    def release(self):
        if self.h:
            lib().pm_fixed_bases_release(self.h)
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
        """Run on the caller's HIP stream; 0 / None = the context's own
        (blocking) stream again, LEGACY_STREAM = the legacy null stream."""
        _check(lib().pm_ctx_set_stream(self.h, _vp(stream_handle or None)))

    def use_own_stream(self):
        _check(lib().pm_ctx_use_own_stream(self.h))

    def set_window(self, c):
        _check(lib().pm_ctx_set_window(self.h, c))

    def set_small_msm(self, max_n):
        """MSMs of at most max_n terms (automatic window) take the small-MSM
        path (table + window-sum kernels, 33-window host Horner); 0 = never."""
        _check(lib().pm_ctx_set_small_msm(self.h, max_n))

    def set_pipeline(self, groups=0, min_chunk=0):
        """Minimum accumulate slice per lane (0 = automatic); groups must be
        0 or 1 (window groups are retired)."""
        _check(lib().pm_ctx_set_pipeline(self.h, groups, min_chunk))

    def set_glv(self, enable=True):
        """Retired GLV mode: only enable=False is accepted."""
        _check(lib().pm_ctx_set_glv(self.h, 1 if enable else 0))

    def set_accum_ladder(self, mode=-1):
        """pm_ctx_set_accum_ladder: 0 quads, 1 row-sliced waves, -1 auto."""
        _check(lib().pm_ctx_set_accum_ladder(self.h, mode))

    def set_accum_option(self, option, value=-1):
        """pm_ctx_set_accum_option: ACC_OPT_TWIST / _TAIL_STREAM / _TRANSCRIPT
        (0 off, -1 auto), ACC_OPT_TERMS_PER_LANE (1, 2, -1 auto)."""
        _check(lib().pm_ctx_set_accum_option(self.h, option, value))

    def set_msm_option(self, option, value=-1):
        """pm_ctx_set_msm_option: MSM_OPT_SPLIT_COPY (0 one scalar copy, -1 auto)."""
        _check(lib().pm_ctx_set_msm_option(self.h, option, value))

    def set_accum_split(self, lg_lanes=-1):
        """Accumulator: 2^lg_lanes lanes (bit segments) per MSM term, 0..5 (-1 = automatic)."""
        _check(lib().pm_ctx_set_accum_split(self.h, lg_lanes))

    def set_timing(self, on=True, only=None):
        """HIP-event timing; `only` restricts events to one kernel name (each
        event pair adds ~10 us of stream time)."""
        _check(lib().pm_ctx_set_timing_filter(self.h, (only or "").encode()))
        _check(lib().pm_ctx_set_timing(self.h, 1 if on else 0))

    def reset_stats(self):
        _check(lib().pm_ctx_reset_stats(self.h))

    def kernel_stats(self, name):
        n = ctypes.c_uint64(0)
        ms = ctypes.c_double(0)
        _check(lib().pm_ctx_kernel_stats(self.h, name.encode(), ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value

    def dropin_stats(self):
        """pm_ctx_dropin_stats -> dict(hits, misses, entries, device_bytes) of
        pm_msm_ctx's resident base cache."""
        hi, mi, en, by = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int(), ctypes.c_size_t()
        _check(lib().pm_ctx_dropin_stats(self.h, ctypes.byref(hi), ctypes.byref(mi), ctypes.byref(en),
                                         ctypes.byref(by)))
        return {"hits": hi.value, "misses": mi.value, "entries": en.value, "device_bytes": by.value}

    def dropin_spec_stats(self):
        """pm_ctx_dropin_spec_stats -> (kept, drained) speculative starts."""
        k, d = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().pm_ctx_dropin_spec_stats(self.h, ctypes.byref(k), ctypes.byref(d)))
        return k.value, d.value

    def dropin_oom_stats(self):
        """pm_ctx_dropin_oom_stats -> (flushes, failed_builds): out-of-memory
        events of the drop-in cache."""
        f, b = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().pm_ctx_dropin_oom_stats(self.h, ctypes.byref(f), ctypes.byref(b)))
        return f.value, b.value

    def dropin_small_stats(self):
        """pm_ctx_dropin_small_stats -> dict(hits, admitted, entries, device_bytes)."""
        h, a, e, b = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int(), ctypes.c_size_t()
        _check(lib().pm_ctx_dropin_small_stats(self.h, ctypes.byref(h), ctypes.byref(a), ctypes.byref(e),
                                               ctypes.byref(b)))
        return {"hits": h.value, "admitted": a.value, "entries": e.value, "device_bytes": b.value}

    def dropin_clear(self):
        _check(lib().pm_ctx_dropin_clear(self.h))

    def dropin_key_id(self):
        """pm_ctx_dropin_key_id: a fingerprint (2 x u64) of this context's
        secret digest key; distinct contexts hold distinct keys."""
        out = np.zeros(2, dtype=np.uint64)
        _check(lib().pm_ctx_dropin_key_id(self.h, out.ctypes.data_as(_u64p)))
        return (int(out[0]), int(out[1]))

    def msm(self, curve, coeffs, bases, canonical=False):
        """pm_msm_ctx: host scalars and host bases (the transparent
        best_multiexp drop-in, with the resident base cache)."""
        s, b = _as_u64(coeffs, 4), _as_u64(bases, 8)
        if s.shape[0] != b.shape[0]:
            raise ValueError("scalars and bases differ in length")
        out = np.zeros(8, dtype=np.uint64)
        _check(lib().pm_msm_ctx(self.h, curve, s.ctypes.data, b.ctypes.data, s.shape[0],
                                SCALARS_CANONICAL if canonical else 0, out.ctypes.data))
        return out

    def msm_device(self, curve, d_scalars, d_bases, n, canonical=False):
        out = np.zeros(8, dtype=np.uint64)
        _check(lib().pm_msm_device(self.h, curve, _vp(d_scalars), _vp(d_bases), n,
                                   SCALARS_CANONICAL if canonical else 0, _p(out)))
        return out

    def upload_bases(self, curve, bases=None, d_bases=None, n=None):
        return Bases(self, curve, bases, d_bases, n)

    def msm_resident_device(self, bases: Bases, offset, d_scalars, n, canonical=False):
        out = np.zeros(8, dtype=np.uint64)
        _check(lib().pm_msm_resident_device(self.h, bases.h, offset, _vp(d_scalars), n,
                                            SCALARS_CANONICAL if canonical else 0, _p(out)))
        return out

    def msm_resident_batch(self, bases: Bases, offset, coeff_list, canonical=False):
        """pm_msm_resident_batch: one MSM per host scalar array (all of the
        same length) against resident bases; returns (k, 8) u64."""
        arrs = [_as_u64(c, 4) for c in coeff_list]
        n = arrs[0].shape[0] if arrs else 0
        if any(a.shape[0] != n for a in arrs):
            raise ValueError("all scalar arrays of a batch must have the same length")
        ptrs = (_u64p * len(arrs))(*[_p(a) for a in arrs])
        out = np.zeros((len(arrs), 8), dtype=np.uint64)
        _check(lib().pm_msm_resident_batch(self.h, bases.h, offset, ptrs, len(arrs), n,
                                           SCALARS_CANONICAL if canonical else 0, _p(out)))
        return out

    def _many_args(self, n, offsets):
        nn = np.ascontiguousarray(np.asarray(n, dtype=np.uint64).reshape(-1))
        oo = None if offsets is None else np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64).reshape(-1))
        if oo is not None and oo.shape != nn.shape:
            raise ValueError("offsets and n differ in length")
        szp = lambda a: None if a is None else a.ctypes.data_as(_szp)  # noqa: E731
        return nn, oo, szp(nn), szp(oo)

    def msm_resident_many(self, bases: Bases, n, scalars, offsets=None, canonical=False):
        """pm_msm_resident_many: B = len(n) short MSMs against resident bases,
        MSM i over the next n[i] rows of `scalars` (sum(n) x 4 u64) and bases
        [offsets[i], offsets[i] + n[i]) (offsets None: 0); returns (B, 8) u64."""
        nn, oo, pn, po = self._many_args(n, offsets)
        s = _as_u64(scalars, 4) if int(nn.sum()) else np.zeros((1, 4), dtype=np.uint64)
        if int(nn.sum()) and s.shape[0] != int(nn.sum()):
            raise ValueError("scalars must hold sum(n) rows")
        out = np.zeros((nn.shape[0], 8), dtype=np.uint64)
        _check(lib().pm_msm_resident_many(self.h, bases.h, nn.shape[0], pn, po, _p(s),
                                          SCALARS_CANONICAL if canonical else 0, _p(out)))
        return out

    def msm_resident_many_device(self, bases: Bases, n, d_scalars, offsets=None, canonical=False):
        nn, oo, pn, po = self._many_args(n, offsets)
        out = np.zeros((nn.shape[0], 8), dtype=np.uint64)
        _check(lib().pm_msm_resident_many_device(self.h, bases.h, nn.shape[0], pn, po, _vp(d_scalars),
                                                 SCALARS_CANONICAL if canonical else 0, _p(out)))
        return out

    def bases_many_prepare(self, bases: Bases, max_n):
        _check(lib().pm_bases_many_prepare(self.h, bases.h, max_n))

    def set_h2d_threads(self, threads):
        """Retired pinned staging: only threads=0 is accepted."""
        _check(lib().pm_ctx_set_h2d_threads(self.h, threads))

    def fixed_bases(self, curve, bases=None, c=0, d_bases=None, n=None, rows=0):
        return FixedBases(self, curve, bases, c, d_bases, n, rows)

    def msm_resident(self, bases: Bases, offset, coeffs, canonical=False):
        s = _as_u64(coeffs, 4)
        out = np.zeros(8, dtype=np.uint64)
        _check(lib().pm_msm_resident(self.h, bases.h, offset, _p(s), s.shape[0],
                                     SCALARS_CANONICAL if canonical else 0, _p(out)))
        return out

    def synth_scalars(self, curve, seed, i0, n, d_out, canonical=False):
        _check(lib().pm_synth_scalars(self.h, curve, seed, i0, n, SCALARS_CANONICAL if canonical else 0,
                                      _vp(d_out)))

    def accum_batch(self, shape: ProofShape, points, scalars, challenges):
        """Batch multiopen accumulator (pm_accum_batch): points (B, npts, 8),
        scalars (B, nsc, 4), challenges (B, 7, 4) u64 Montgomery ->
        (quads (B, 4, 8): w, zw, f, e affine; h_eval (B, 4))."""
        npts, nsc, _ = shape.layout()
        p = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1, npts, 8)
        B = p.shape[0]
        s = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(B, nsc, 4)
        c = np.ascontiguousarray(challenges, dtype=np.uint64).reshape(B, 7, 4)
        quads = np.zeros((B, 4, 8), dtype=np.uint64)
        hev = np.zeros((B, 4), dtype=np.uint64)
        st = np.zeros(B, dtype=np.uint32)
        _check(lib().pm_accum_batch(self.h, shape.curve, ctypes.byref(shape.c), B, _p(p), _p(s), _p(c), _p(quads),
                                    _p(hev), st.ctypes.data_as(_u32p)))
        self.last_status = st
        return quads, hev

    def accum_batch_status(self, shape: ProofShape, points, scalars, challenges):
        """pm_accum_batch -> (quads, h_eval, status (B,) u32: PM_ACCUM_DENOM_ZERO)."""
        q, h = self.accum_batch(shape, points, scalars, challenges)
        return q, h, self.last_status

    def accum_batch_device(self, shape: ProofShape, B, d_points, d_scalars, d_challenges, d_quads, d_h=0,
                           d_status=0):
        _check(lib().pm_accum_batch_device(self.h, shape.curve, ctypes.byref(shape.c), B, _vp(d_points),
                                           _vp(d_scalars), _vp(d_challenges), _vp(d_quads), _vp(d_h or None),
                                           _vp(d_status or None)))

    def _proof_buffers(self, shape, points, scalars):
        npts, nsc, _ = shape.layout()
        p = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1, npts, 8)
        s = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(p.shape[0], nsc, 4)
        return p, s

    def transcript_batch(self, shape: ProofShape, points, scalars, vk_repr):
        """Blake2b transcript replay (pm_transcript_batch) -> (challenges
        (B, 7, 4) Montgomery, status (B,) u32)."""
        p, s = self._proof_buffers(shape, points, scalars)
        B = p.shape[0]
        vk = np.ascontiguousarray(vk_repr, dtype=np.uint64).reshape(4)
        ch = np.zeros((B, 7, 4), dtype=np.uint64)
        st = np.zeros(B, dtype=np.uint32)
        _check(lib().pm_transcript_batch(self.h, shape.curve, ctypes.byref(shape.c), B, _p(vk), _p(p), _p(s),
                                         _p(ch), st.ctypes.data_as(_u32p)))
        return ch, st

    def accum_batch_transcript(self, shape: ProofShape, points, scalars, vk_repr):
        """Transcript replay + accumulator (pm_accum_batch_transcript) ->
        (quads (B, 4, 8), h_eval (B, 4), challenges (B, 7, 4), status (B,))."""
        p, s = self._proof_buffers(shape, points, scalars)
        B = p.shape[0]
        vk = np.ascontiguousarray(vk_repr, dtype=np.uint64).reshape(4)
        ch = np.zeros((B, 7, 4), dtype=np.uint64)
        quads = np.zeros((B, 4, 8), dtype=np.uint64)
        hev = np.zeros((B, 4), dtype=np.uint64)
        st = np.zeros(B, dtype=np.uint32)
        _check(lib().pm_accum_batch_transcript(self.h, shape.curve, ctypes.byref(shape.c), B, _p(vk), _p(p), _p(s),
                                               _p(ch), _p(quads), _p(hev), st.ctypes.data_as(_u32p)))
        return quads, hev, ch, st

    def transcript_batch_device(self, shape: ProofShape, B, vk_repr, d_points, d_scalars, d_challenges, d_status=0):
        vk = np.ascontiguousarray(vk_repr, dtype=np.uint64).reshape(4)
        _check(lib().pm_transcript_batch_device(self.h, shape.curve, ctypes.byref(shape.c), B, _p(vk),
                                                _vp(d_points), _vp(d_scalars), _vp(d_challenges),
                                                _vp(d_status or None)))

    def accum_batch_transcript_device(self, shape: ProofShape, B, vk_repr, d_points, d_scalars, d_challenges,
                                      d_quads, d_h=0, d_status=0):
        vk = np.ascontiguousarray(vk_repr, dtype=np.uint64).reshape(4)
        _check(lib().pm_accum_batch_transcript_device(self.h, shape.curve, ctypes.byref(shape.c), B, _p(vk),
                                                      _vp(d_points), _vp(d_scalars), _vp(d_challenges),
                                                      _vp(d_quads), _vp(d_h or None), _vp(d_status or None)))

    # ---- proof bytes (pm_*_proofs*): the reference's read_point / read_scalar
    def _proof_bytes(self, shape: ProofShape, proofs, instance_points):
        """proofs: (B, stride) u8 (or a list of bytes of equal length);
        instance_points: (B, num_instance_columns, 8) u64 Montgomery affine."""
        if isinstance(proofs, (list, tuple)):
            proofs = np.frombuffer(b"".join(proofs), dtype=np.uint8).reshape(len(proofs), -1)
        pf = np.ascontiguousarray(proofs, dtype=np.uint8)
        B = pf.shape[0]
        ni = shape.c.num_instance_columns
        inst = np.ascontiguousarray(instance_points if instance_points is not None else np.zeros((B, ni, 8)),
                                    dtype=np.uint64).reshape(B, ni, 8)
        return pf, inst, B

    def proof_size(self, shape: ProofShape):
        return proof_size(shape)

    def decode_proofs(self, shape: ProofShape, proofs, instance_points=None):
        """pm_decode_proofs -> (points (B, npts, 8), scalars (B, nsc, 4), status (B,))."""
        pf, inst, B = self._proof_bytes(shape, proofs, instance_points)
        npts, nsc, _ = shape.layout()
        pts = np.zeros((B, npts, 8), dtype=np.uint64)
        scs = np.zeros((B, nsc, 4), dtype=np.uint64)
        st = np.zeros(B, dtype=np.uint32)
        _check(lib().pm_decode_proofs(self.h, shape.curve, ctypes.byref(shape.c), B,
                                      pf.ctypes.data_as(ctypes.c_char_p), pf.shape[1], _p(inst), _p(pts), _p(scs),
                                      st.ctypes.data_as(_u32p)))
        return pts, scs, st

    def accum_batch_proofs(self, shape: ProofShape, proofs, instance_points, vk_repr):
        """pm_accum_batch_proofs -> (quads (B, 4, 8), h_eval (B, 4), challenges (B, 7, 4), status (B,))."""
        pf, inst, B = self._proof_bytes(shape, proofs, instance_points)
        vk = np.ascontiguousarray(vk_repr, dtype=np.uint64).reshape(4)
        ch = np.zeros((B, 7, 4), dtype=np.uint64)
        quads = np.zeros((B, 4, 8), dtype=np.uint64)
        hev = np.zeros((B, 4), dtype=np.uint64)
        st = np.zeros(B, dtype=np.uint32)
        _check(lib().pm_accum_batch_proofs(self.h, shape.curve, ctypes.byref(shape.c), B, _p(vk),
                                           pf.ctypes.data_as(ctypes.c_char_p), pf.shape[1], _p(inst), _p(ch),
                                           _p(quads), _p(hev), st.ctypes.data_as(_u32p)))
        return quads, hev, ch, st

    def decode_proofs_device(self, shape: ProofShape, B, d_proofs, stride, d_inst, d_points, d_scalars, d_status):
        _check(lib().pm_decode_proofs_device(self.h, shape.curve, ctypes.byref(shape.c), B, _vp(d_proofs), stride,
                                             _vp(d_inst or None), _vp(d_points), _vp(d_scalars), _vp(d_status)))

    def accum_batch_proofs_device(self, shape: ProofShape, B, vk_repr, d_proofs, stride, d_inst, d_challenges,
                                  d_quads, d_h=0, d_status=0):
        vk = np.ascontiguousarray(vk_repr, dtype=np.uint64).reshape(4)
        _check(lib().pm_accum_batch_proofs_device(self.h, shape.curve, ctypes.byref(shape.c), B, _p(vk),
                                                  _vp(d_proofs), stride, _vp(d_inst or None), _vp(d_challenges),
                                                  _vp(d_quads), _vp(d_h or None), _vp(d_status or None)))

    def fft(self, curve, values, omega, scale=None):
        """pm_fft: natural-order NTT of values ((2^k, 4) u64 Montgomery) with
        root omega (4,) u64 Montgomery; returns a new array."""
        a = np.ascontiguousarray(values, dtype=np.uint64).reshape(-1, 4).copy()
        n = a.shape[0]
        k = n.bit_length() - 1
        if n != 1 << k:
            raise ValueError("length must be a power of two")
        w = np.ascontiguousarray(omega, dtype=np.uint64).reshape(4)
        sc = None if scale is None else np.ascontiguousarray(scale, dtype=np.uint64).reshape(4)
        _check(lib().pm_fft(self.h, curve, _p(a), k, _p(w), None if sc is None else _p(sc)))
        return a

    def fft_device(self, curve, d_data, log_n, omega, scale=None):
        w = np.ascontiguousarray(omega, dtype=np.uint64).reshape(4)
        sc = None if scale is None else np.ascontiguousarray(scale, dtype=np.uint64).reshape(4)
        _check(lib().pm_fft_device(self.h, curve, _vp(d_data), log_n, _p(w), None if sc is None else _p(sc)))

    def selftest_field(self, curve, seed, n):
        m = ctypes.c_uint64(0)
        _check(lib().pm_selftest_field(self.h, curve, seed, n, ctypes.byref(m)))
        return m.value

    def synth_bases(self, curve, seed, i0, n, d_out):
        _check(lib().pm_synth_bases(self.h, curve, seed, i0, n, _vp(d_out)))
