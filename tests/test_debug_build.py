"""SURVEY §5 "race detection / sanitizers" (VERDICT r3 item 8): the ASan + UBSan host build of the
library (``make debug``: -Xarch_host -fsanitize=address,undefined on every translation unit) and
abi_host_check, which drives every entry point's argument validation and dispatch planning on the
CPU (no GPU: a call that passes validation fails at its launch with SR_ELAUNCH).  Also checks that
the ctypes mirror of every ABI struct (sailrecon_amd/_lib.py) has the C layout."""

import ctypes
import json
import os
import subprocess

import pytest

from conftest import REPO

CSRC = os.path.join(REPO, "self-supervise-sfm_amd", "csrc")
EXE = os.path.join(REPO, "self-supervise-sfm_amd", "build", "debug", "abi_host_check")


@pytest.fixture(scope="module")
def debug_build():
    r = subprocess.run(["make", "-C", CSRC, "-j", str(min(8, os.cpu_count() or 8)), "debug-build"],
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return EXE


def _run(exe, mode):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    return subprocess.run([exe, mode], capture_output=True, text=True, timeout=300, env=env)


def test_asan_ubsan_abi_sweep(debug_build):
    r = _run(debug_build, "check")
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "OK: 0 unexpected" in out, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out


def test_ctypes_struct_layout_matches_c(debug_build):
    from sailrecon_amd import _lib
    r = _run(debug_build, "layout")
    assert r.returncode == 0, r.stderr
    lay = json.loads(r.stdout)
    mirror = {"sr_gemm_epi": _lib.GemmEpi, "sr_gemm_problem": _lib.GemmProblem, "sr_wgrad_problem": _lib.WgradProblem,
              "sr_attn_desc": _lib.AttnDesc,
              "sr_attn_bwd_desc": _lib.AttnBwdDesc, "sr_imc_loss_desc": _lib.ImcLossDesc,
              "sr_weight_item": _lib.WeightItem}
    assert set(lay) == set(mirror)
    for name, cls in mirror.items():
        assert ctypes.sizeof(cls) == lay[name]["size"], name
        fields = {f[0] for f in cls._fields_}
        assert fields == set(lay[name]["fields"]), (name, fields ^ set(lay[name]["fields"]))
        for f, off in lay[name]["fields"].items():
            assert getattr(cls, f).offset == off, (name, f)
