"""bench.py's multi-GPU launcher (the driver's `python bench.py --gpus N` form).

CPU: `--gpus N --launch-only` starts N worker processes, each joins a gloo process group, and
rank 0's line reports n_gpus = N with N distinct ranks in ranks_seen (the launcher and the
report, without the model).  A worker that fails ends the others and the parent's exit code is
non-zero.  GPU: one rank through the RCCL ("nccl") process group on the box's GPU, a short
N=2 @518 bench step, and its ranks_seen entry names the device."""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _json_line(out: str):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _cpu_env():
    env = dict(os.environ)
    env["HIP_VISIBLE_DEVICES"] = ""  # keep the CPU test on gloo even where a GPU exists
    env["CUDA_VISIBLE_DEVICES"] = ""
    env.pop("WORLD_SIZE", None)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-only"], capture_output=True, text=True,
                       timeout=300, env=_cpu_env(), cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == n and line["backend"] == "gloo"
    assert sorted(s["rank"] for s in line["ranks_seen"]) == list(range(n))
    assert sorted(s["local_rank"] for s in line["ranks_seen"]) == list(range(n))


def test_launcher_single_process_default():
    r = subprocess.run([sys.executable, BENCH, "--launch-only"], capture_output=True, text=True, timeout=300,
                       env=_cpu_env(), cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 1 and line["backend"] is None


def test_launcher_propagates_failure():
    """Without a GPU and without --launch-only every worker must refuse (no CPU fallback of the HIP
    path); the parent returns non-zero and prints no bench line."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"], capture_output=True,
                       text=True, timeout=300, env=_cpu_env(), cwd=REPO)
    assert r.returncode != 0
    assert "no ROCm GPU" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.gpu
def test_bench_rccl_world1():
    """The RCCL process-group path of bench.py (init, ranks_seen all_gather_object, max-over-ranks
    all_reduce) at world 1 on the box's GPU, on a 2-view @518 step."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(29500 + os.getpid() % 1000))
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--steps", "1", "--warmup", "1", "--views", "2",
                        "--no-cpu-baseline", "--extras", "n64"], capture_output=True, text=True, timeout=600, env=env,
                       cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 1 and line["backend"] == "nccl"
    assert line["value"] > 0
    (x,) = line["extra_configs"]  # the 64-view extra workload rides inside the one line
    assert x["name"] == "n64" and "error" not in x and x["value"] > 0
    (seen,) = line["ranks_seen"]
    assert seen["rank"] == 0 and seen["device"].startswith("cuda") and "pci_bus" in seen
