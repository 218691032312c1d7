"""TEST INFRASTRUCTURE ONLY: ctypes binding of accum_ref_batch in
oracle/libmsm_ref.so (oracle/accum_ref.c: the C restatement of the
multiopen accumulator + Blake2b transcript replay).  Used by tests/ (second
checker beside oracle/accum.py) and bench.py's accumulator cpu_baseline leg;
never by the product path.  The shape argument is a pm_proof_shape ctypes
structure (the C-ABI's VK view, include/pasta_msm.h), passed by reference."""
from __future__ import annotations

import ctypes

import numpy as np

import msm_ref


def _lib():
    L = msm_ref.lib()
    if not hasattr(L, "_accum_ref_ready"):
        u64p = ctypes.POINTER(ctypes.c_uint64)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.accum_ref_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, u64p, u64p, u64p, u64p,
                                      ctypes.c_int, u64p, u64p, u64p, u32p]
        L.accum_ref_batch.restype = ctypes.c_int
        L.accum_ref_batch_proofs.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p,
                                             ctypes.c_size_t, u64p, u64p, ctypes.c_int, u64p, u64p, u64p, u64p,
                                             u64p, u32p]
        L.accum_ref_batch_proofs.restype = ctypes.c_int
        L.accum_ref_layout.argtypes = [ctypes.c_void_p, u32p, u32p, u32p]
        L.accum_ref_layout.restype = ctypes.c_int
        L._accum_ref_ready = True
    return L


def layout(shape_struct):
    a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    rc = _lib().accum_ref_layout(ctypes.byref(shape_struct), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    assert rc == 0
    return a.value, b.value, c.value


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def accum_batch(curve, shape_struct, points, scalars, challenges=None, vk_repr=None, threads=None):
    """-> (challenges (B,7,4), quads (B,4,8), h_eval (B,4), status (B,)), all
    u64 Montgomery like the C-ABI; challenges None -> replayed from vk_repr."""
    npts, nsc, _ = layout(shape_struct)
    p = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1, npts, 8)
    B = p.shape[0]
    s = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(B, nsc, 4)
    c = None if challenges is None else np.ascontiguousarray(challenges, dtype=np.uint64).reshape(B, 7, 4)
    vk = None if vk_repr is None else np.ascontiguousarray(vk_repr, dtype=np.uint64).reshape(4)
    ch = np.zeros((B, 7, 4), dtype=np.uint64)
    q = np.zeros((B, 4, 8), dtype=np.uint64)
    h = np.zeros((B, 4), dtype=np.uint64)
    st = np.zeros(B, dtype=np.uint32)
    rc = _lib().accum_ref_batch(curve, ctypes.byref(shape_struct), B, _p(p), _p(s), _p(c), _p(vk),
                                int(threads or msm_ref.default_threads()), _p(ch), _p(q), _p(h),
                                st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    if rc != 0:
        raise ValueError("accum_ref_batch failed")
    return ch, q, h, st


def batch_proofs(curve, shape_struct, proofs, inst, vk_repr=None, threads=None, decode_only=False):
    """C decode (+ replay + accumulator) of serialized proofs ((B, stride) u8)
    -> dict(points, scalars, status[, challenges, quads, h_eval])."""
    npts, nsc, _ = layout(shape_struct)
    pf = np.ascontiguousarray(proofs, dtype=np.uint8)
    B = pf.shape[0]
    ni = shape_struct.num_instance_columns
    ins = np.ascontiguousarray(inst, dtype=np.uint64).reshape(B, ni, 8) if ni else np.zeros((B, 0, 8), np.uint64)
    out = {"points": np.zeros((B, npts, 8), dtype=np.uint64), "scalars": np.zeros((B, nsc, 4), dtype=np.uint64),
           "status": np.zeros(B, dtype=np.uint32)}
    acc = not decode_only
    if acc:
        out.update(challenges=np.zeros((B, 7, 4), dtype=np.uint64), quads=np.zeros((B, 4, 8), dtype=np.uint64),
                   h_eval=np.zeros((B, 4), dtype=np.uint64))
    vk = None if vk_repr is None else np.ascontiguousarray(vk_repr, dtype=np.uint64).reshape(4)
    rc = _lib().accum_ref_batch_proofs(curve, ctypes.byref(shape_struct), B, pf.ctypes.data_as(ctypes.c_char_p),
                                       pf.shape[1], _p(ins), _p(vk), int(threads or msm_ref.default_threads()),
                                       _p(out["points"]), _p(out["scalars"]), _p(out.get("challenges")),
                                       _p(out.get("quads")), _p(out.get("h_eval")),
                                       out["status"].ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    if rc != 0:
        raise ValueError("accum_ref_batch_proofs failed")
    return out
