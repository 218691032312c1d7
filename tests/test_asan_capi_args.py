"""C-ABI argument handling without a GPU (also run under ASan / UBSan by
tests/test_asan.py): every entry point rejects null / out-of-range
arguments with PM_ERR_ARG (or PM_ERR_NODEV when it would need a device)
instead of dereferencing them, and the host-only entries compute."""
import ctypes

import numpy as np
import pytest

import halo2_amd as H

ARG, NODEV, UNSUP = -1, -3, -4


def test_version_and_abi():
    assert H.lib().pm_version().decode().startswith("pasta_msm")
    assert H.abi_version() >= 3


def test_null_arguments_rejected():
    L = H.lib()
    z = ctypes.c_void_p(0)
    out = np.zeros(8, np.uint64)
    po = out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    one = np.zeros((1, 8), np.uint64)
    p1 = one.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    assert L.pm_device_count(None) == ARG
    assert L.pm_ctx_create(0, None) == ARG
    assert L.pm_ctx_set_stream(None, None) == ARG
    assert L.pm_ctx_set_window(None, 0) == ARG
    assert L.pm_msm_ctx(None, 0, p1, p1, 1, 0, po) == ARG
    assert L.pm_msm_device(None, 0, z, z, 1, 0, po) == ARG
    assert L.pm_msm_multi(0, None, None, 1, 0, 1, po) == ARG
    assert L.pm_point_add(0, None, p1, po) == ARG
    assert L.pm_point_add(9, p1, p1, po) == ARG
    assert L.pm_points_sum(0, None, 1, po) == ARG
    assert L.pm_points_sum(0, p1, 1, None) == ARG
    assert L.pm_points_sum(9, p1, 1, po) == ARG
    assert L.pm_ctx_set_accum_option(None, 1, 0) == ARG
    assert L.pm_ctx_set_msm_option(None, 1, 0) == ARG
    assert L.pm_bases_upload(None, 0, p1, 1, None) == ARG
    assert L.pm_msm_resident(None, None, 0, p1, 1, 0, po) == ARG
    assert L.pm_msm_resident_batch(None, None, 0, None, 1, 1, 0, po) == ARG
    assert L.pm_fixed_bases_create(None, 0, p1, 1, 0, None) == ARG
    assert L.pm_fft(None, 2, None, 4, None, None) == ARG
    assert L.pm_shape_layout(None, None, None, None) == ARG
    assert L.pm_vk_transcript_repr(0, None, 5, po) == ARG
    assert L.pm_selftest_host(0, 1, 1 << 30, po) == ARG
    assert L.pm_accum_batch(None, 0, None, 1, p1, p1, p1, po, None, None) == ARG
    assert L.pm_bases_release(None) == 0 and L.pm_fixed_bases_release(None) == 0
    assert H.lib().pm_last_error()


def test_no_device_is_reported():
    """Without a visible device pm_ctx_create fails cleanly (NODEV); with one
    (the GPU box) it succeeds."""
    h = ctypes.c_void_p()
    rc = H.lib().pm_ctx_create(0, ctypes.byref(h))
    if rc == 0:
        assert H.lib().pm_ctx_destroy(h) == 0
    else:
        assert rc == NODEV
    assert H.lib().pm_ctx_create(-1, ctypes.byref(h)) in (ARG, NODEV)


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_point_add_host(curve):
    """pm_point_add (host): identity + P = P, P + (-P) = identity."""
    import workloads as Wk

    g = Wk.generator_limbs(curve)
    assert np.array_equal(H.point_add(curve, np.zeros(8, np.uint64), g), g)
    p = Wk.BASE_MODULUS[curve]
    y = sum(int(g[4 + k]) << (64 * k) for k in range(4))
    ny = (p - y) % p
    neg = g.copy()
    neg[4:] = [(ny >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)]
    assert not H.point_add(curve, g, neg).any()
