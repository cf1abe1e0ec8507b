"""CPU tests of the product's host side: the C-ABI library loads and exports every symbol include/kfec.h
declares, the Python mirror keeps fec_code's error behaviour without touching a GPU, and the product
path fails loudly (no CPU fallback) when no GPU is present."""
from __future__ import annotations

import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from kcptube_amd.build import LIB, build_lib
    if not os.path.exists(LIB):
        build_lib()
    from kcptube_amd import load_library
    return load_library()


def test_header_symbols_exported(lib):
    from kcptube_amd.fec import header_functions
    names = header_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    # and the dynamic symbol table agrees (extern "C", unmangled)
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "kcptube_amd", "libkfec.so")],
                         capture_output=True, text=True).stdout
    for n in names:
        assert f" T {n}\n" in out, n


def test_library_is_gfx950_code(lib):
    """The code object inside libkfec.so targets gfx950 only (no dual paths)."""
    so = os.path.join(ROOT, "kcptube_amd", "libkfec.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"sm_"):
        assert b"amdgcn-amd-amdhsa--" + other not in data


def test_version_string(lib):
    from kcptube_amd import version
    assert "gfx950" in version()


def test_invalid_kn_is_value_error_without_gpu(lib):
    """fec_code(K, N) throws std::invalid_argument on a violation before any device work (fecpp.cpp:431)."""
    from kcptube_amd import FecCode
    for K, N in [(0, 0), (0, 5), (6, 5), (257, 257), (1, 257)]:
        with pytest.raises(ValueError):
            FecCode(K, N)
    c = FecCode()
    assert (c.get_K(), c.get_N()) == (0, 0)
    with pytest.raises(ValueError):
        c.reset_martix(3, 2)


def test_c_abi_argument_checks(lib):
    vp = ctypes.c_void_p()
    assert lib.kfec_create(0, 0, ctypes.byref(vp)) == -1
    assert lib.kfec_create(5, 4, ctypes.byref(vp)) == -1
    assert lib.kfec_create(1, 257, ctypes.byref(vp)) == -1
    assert lib.kfec_get_K(None) == 0 and lib.kfec_get_N(None) == 0
    assert lib.kfec_decode_workspace_size(None, 10) == 0
    lib.kfec_destroy(None)  # no-op


def test_no_cpu_fallback_without_gpu(lib):
    """On a host without a gfx950 GPU the coder refuses (ENODEV / KfecUnavailable) instead of computing."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from kcptube_amd import FecCode, KfecUnavailable
    vp = ctypes.c_void_p()
    assert lib.kfec_create(20, 23, ctypes.byref(vp)) == -2
    with pytest.raises(KfecUnavailable):
        FecCode(20, 23)


def test_product_does_not_import_oracle():
    """The product package never references the test-only oracle."""
    pkg = os.path.join(ROOT, "kcptube_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt, f
                assert "liboracle" not in txt and "libfecpp_ref" not in txt, f
