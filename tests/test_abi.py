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
    # key box: 33 heads, an unaligned k, and an instance stride below the rows are rejected
    for args in ((64, 10, 0, 1, 33), (64, 10, 0, 1, 1), (1024, 10, 5, 2, 16)):
        k = ctypes.c_void_p(18 if args == (64, 10, 0, 1, 1) else 16)
        assert lib.sr_attention_key_box(None, k, *args[:4], args[4], ctypes.c_void_p(16), None,
                                        ctypes.c_void_p(16)) == -1, args
        assert b"sr_attention_key_box" in lib.sr_last_error()
    assert lib.sr_attention_key_box_scratch(43968, 1, 16) > 0 and lib.sr_attention_key_box_scratch(10, 1, 33) == 0


def test_tuning_switches_without_gpu():
    """sr_set_tuning / sr_get_tuning / sr_tuning_name: every A/B switch the
    kernels read is one documented entry of sfm_amd.h's sr_tuning_key, starting from its
    environment variable; set returns the old value, unknown keys fail with SR_EINVAL."""
    from sailrecon_amd import _lib, ops
    lib = _lib.load()
    src = open(HEADER).read()
    keys = re.findall(r"^\s*(SR_TUNE_\w+)\s*=\s*(\d+)", src, flags=re.M)
    count = dict(keys).pop("SR_TUNE_COUNT")
    assert len(keys) - 1 == int(count) == len(ops.tuning_names())
    for name, k in keys:
        if name == "SR_TUNE_COUNT":
            assert lib.sr_tuning_name(int(k)) is None
            continue
        env = lib.sr_tuning_name(int(k)).decode()
        assert name.replace("SR_TUNE_", "SR_") == env
    assert ops.get_tuning("SR_ATTN_PIPE") == int(os.environ.get("SR_ATTN_PIPE", "1"))
    with ops.tuning(SR_ATTN_PIPE_SEG=1, SR_GEMM_GROUP_M=2):
        assert ops.get_tuning("SR_ATTN_PIPE_SEG") == 1 and ops.get_tuning("SR_GEMM_GROUP_M") == 2
    assert ops.get_tuning("SR_ATTN_PIPE_SEG") == int(os.environ.get("SR_ATTN_PIPE_SEG", "0"))
    assert lib.sr_set_tuning(99, 1) == -1 and b"unknown key" in lib.sr_last_error()
    assert lib.sr_get_tuning(-1) == -1
    assert lib.sr_last_kernel() == b""  # nothing launched on this thread


def test_no_getenv_outside_the_tuning_table():
    """The kernels' switches live in one table (sr_api.hip); no other translation unit reads the
    environment."""
    csrc = os.path.join(REPO, "self-supervise-sfm_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h", ".inc")) and f != "sr_api.hip":
            assert "getenv" not in open(os.path.join(csrc, f)).read(), f


def test_generated_asm_sweep_matches_generator(tmp_path):
    """csrc/sr_attn_pipe.inc is what tools/gen_attn_pipe.py emits with its default
    knobs (no stale or hand-edited variant ships)."""
    import subprocess
    import sys
    out = tmp_path / "pipe.inc"
    env = {k: v for k, v in os.environ.items() if not k.startswith("SR_PIPE_")}
    env["SR_PIPE_OUT"] = str(out)
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "gen_attn_pipe.py")], env=env, check=True,
                   capture_output=True)
    shipped = open(os.path.join(REPO, "self-supervise-sfm_amd", "csrc", "sr_attn_pipe.inc")).read()
    assert out.read_text() == shipped


def test_generated_bwd_asm_sweeps_match_generator(tmp_path):
    """csrc/sr_attn_bwd_pipe.inc (the dK/dV, concatenated-items dK/dV and dQ asm sweeps)
    is what tools/gen_attn_bwd_pipe.py emits with its default knobs."""
    import subprocess
    import sys
    out = tmp_path / "bwd_pipe.inc"
    env = {k: v for k, v in os.environ.items() if not k.startswith("SR_BWD_PIPE_")}
    env["SR_BWD_PIPE_OUT"] = str(out)
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "gen_attn_bwd_pipe.py")], env=env, check=True,
                   capture_output=True)
    shipped = open(os.path.join(REPO, "self-supervise-sfm_amd", "csrc", "sr_attn_bwd_pipe.inc")).read()
    assert out.read_text() == shipped
