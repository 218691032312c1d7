"""CPU tests of the C-ABI boundary: the library builds, loads and exports
every symbol include/pasta_msm.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

import halo2_amd as H

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


def test_last_error_is_thread_local_string():
    assert isinstance(H.lib().pm_last_error(), bytes)


def test_gfx950_code_object_embedded():
    blob = open(H.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
