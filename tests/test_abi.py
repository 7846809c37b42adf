"""CPU checks of the C-ABI boundary: the library loads and exports every symbol the
public header declares (no compute calls: there is no GPU here)."""

import ctypes
import os
import re

from conftest import REPO

HEADER = os.path.join(REPO, "include", "sfm_amd.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(sr_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("sr_gemm", "sr_attention", "sr_layernorm", "sr_last_error", "sr_version"):
        assert s in syms


def test_library_exports_all_declared_symbols():
    from sailrecon_amd import _lib
    lib = _lib.load()
    for s in declared_symbols():
        assert hasattr(lib, s), f"{s} declared in sfm_amd.h but not exported"
    assert set(_lib.EXPORTED) == set(declared_symbols())
    assert lib.sr_version() >= 1
    assert lib.sr_last_error() == b""


def test_library_has_gfx950_code_object():
    from sailrecon_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_abi_validation_errors_without_gpu():
    """argument validation runs on the host before any launch: a bad shape is rejected."""
    from sailrecon_amd import _lib
    lib = _lib.load()
    ep = _lib.GemmEpi()
    rc = lib.sr_gemm(None, _lib.SR_BF16, _lib.SR_EPI_BIAS, ctypes.c_void_p(16), 64, ctypes.c_void_p(16), 64,
                     ctypes.c_void_p(16), 104, 10, 102, 64, ctypes.byref(ep))
    assert rc == -3 and b"multiple of 4" in lib.sr_last_error()
    d = _lib.AttnDesc()
    assert lib.sr_attention(None, _lib.SR_BF16, ctypes.byref(d)) == -1
