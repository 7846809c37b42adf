#!/usr/bin/env python
"""Benchmark: aggregator fwd views/sec, N=32 @ 518px (BASELINE.json metric).

One step = SailRecon.forward on a synthetic 32-view scene in the
demo_imc_forward.py convention (the N images duplicated to 2N frames: anchors =
first half, queries = second half, fix_rank=300), i.e. Aggregator.forward under
bf16 autocast + CameraHead.forward (fp32) + pose decode — the north-star hot path.
Inputs are resident in HBM before the timed region.  Weights: the seeded synthetic
rule (pretrained weights are not available offline).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Multi-GPU: one process per GPU; the ONE 32-view scene is sharded by frame across the
ranks (Aggregator.set_frame_sharding: local DINO / frame / MLP work, RCCL all-gathers
of anchor K/V for the global block and of the anchor-subsample K/V for the reloc
block, replicated camera head).  value = the scene's views / max-over-ranks time,
scaling "strong" (total work fixed as N grows).

Prints ONE JSON line on rank 0 (contract in the task statement) with a
``roofline`` object for the dominant kernel class (live HIP-event timing inside
the timed region) and a ``cpu_baseline`` object (the CPU oracle on a bounded
sample, rank 0 at N=1 only).  A per-kernel-class breakdown goes to stderr.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip table); see gpu_peak()
PEAK_F32_TFLOPS = 157.3    # f32 MFMA
PEAK_HBM_GBS = 8000.0


def gpu_peak(device_index: int = 0):
    """Dense bf16 MFMA peak from rocminfo: CUs x max engine clock x 4096 bf16
    FLOP/clk/CU (32x32x16 bf16 = 32768 FLOP per 32 cycles per SIMD, 4 SIMDs).  Returns
    (TFLOP/s, description) or (None, reason) when rocminfo is unavailable."""
    import subprocess
    try:
        out = subprocess.run(["rocminfo"], capture_output=True, text=True, timeout=60).stdout
    except (OSError, subprocess.SubprocessError) as e:
        return None, f"rocminfo unavailable ({e})"
    agents, cur = [], {}
    for line in out.splitlines():
        line = line.strip()
        if line.startswith("Agent ") and cur:
            agents.append(cur)
            cur = {}
        if ":" in line:
            k, v = line.split(":", 1)
            cur.setdefault(k.strip(), v.strip())
    if cur:
        agents.append(cur)
    gpus = [a for a in agents if a.get("Device Type") == "GPU" and a.get("Name", "").startswith("gfx")]
    if not gpus:
        return None, "no GPU agent in rocminfo"
    a = gpus[min(device_index, len(gpus) - 1)]
    cus, mhz = int(a["Compute Unit"]), int(a["Max Clock Freq. (MHz)"].split()[0])
    tf = cus * mhz * 1e6 * 4096 / 1e12
    return tf, f"rocminfo {a['Name']}: {cus} CU x {mhz} MHz x 4096 bf16 FLOP/clk/CU = {tf:.1f} TFLOP/s"


def host_cpu():
    """(model name, physical cores, logical CPUs os.cpu_count()) of this host."""
    model, cores = "unknown", set()
    try:
        phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model == "unknown":
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
            elif not k and phys is not None:
                cores.add((phys, core))
                phys = core = None
    except OSError:
        pass
    return model, len(cores) or (os.cpu_count() or 1), os.cpu_count()

# timer class -> the kernel instantiation it launches at the N=32@518 workload
# (rocprofv3 row names; see DESIGN.md "Kernels").
KERNEL_OF_TAG = {
    "attn_global": "attn_bf16_kernel<4, 2, 2, false>", "attn_reloc": "attn_bf16_kernel<4, 2, 1, false>",
    "attn_frame": "attn_bf16_kernel<4, 2, 0, false>", "gemm_bias": "gemm256_kernel<0>", "gemm_gelu": "gemm256_kernel<1>",
    "gemm_resid": "gemm256_kernel<2>", "gemm_qkv": "gemm256_kernel<3>", "gemm_patch": "gemm256_kernel<4>",
}
# GEMM output width per timer class: the 256x256 kernel runs only when it yields >= 512 tiles
# (sr_gemm.hip dispatch); smaller row counts (C2) run the 128x128 gemm_kernel
_GEMM_N = {"gemm_bias": 3072, "gemm_gelu": 4096, "gemm_resid": 1024, "gemm_qkv": 3072, "gemm_patch": 1024}
_GEMM_EPI = {"gemm_bias": 0, "gemm_gelu": 1, "gemm_resid": 2, "gemm_qkv": 3, "gemm_patch": 4}


def kernel_of_tag(tag: str, views: int, img: int):
    """rocprofv3 row name of the kernel a timer class launches at this workload."""
    if tag in _GEMM_N:
        rows = 2 * views * ((img // 14) ** 2 + 5)
        if tag == "gemm_patch":
            rows = 2 * views * (img // 14) ** 2
        if (_GEMM_N[tag] // 256) * ((rows + 255) // 256) < 512:
            return f"gemm_kernel<__bf16, {_GEMM_EPI[tag]}, false>"
    return KERNEL_OF_TAG.get(tag)


TRAFFIC_FILES = [os.path.join(REPO, "profiles", f) for f in
                 ("r02_pmc_traffic.json", "r02_pmc_traffic_c5_fp8qkv.json")]


def pmc_traffic(kernel: str, views: int, img: int, fp8: str = "off"):
    """(HBM bytes per launch of ``kernel``, source file) from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.py: 2 x FETCH_SIZE + WRITE_SIZE), or (None, None).  Each file holds the
    passes of one workload (its ``workload``: views, img, fp8 mode); other workloads get None."""
    for path in TRAFFIC_FILES:
        try:
            with open(path) as f:
                d = json.load(f)
            wl = d.get("workload", {"views": 32, "img": 518})
            if (wl.get("views"), wl.get("img"), wl.get("fp8_global", "off")) != (views, img, fp8):
                continue
            k = d["kernels"].get(kernel)
        except (OSError, ValueError, KeyError):
            continue
        if k is not None:
            return k["traffic_bytes"], path
    return None, None


def algorithmic_tflop(n_views: int, img: int, C: int = 1024) -> float:
    """Required work per forward, SURVEY §8(d) closed form (TFLOP)."""
    S = 2 * n_views
    npatch = (img // 14) ** 2
    P, Pp = npatch + 5, min(300, npatch) + 5
    Lg = n_views * P
    f_stack = 24 * S * (P * 24 * C * C + 4 * P * P * C)
    f_global = 24 * (Lg * 24 * C * C + 4 * Lg * Lg * C)
    f_reloc = 24 * (n_views * Pp * 4 * C * C + n_views * P * 24 * C * C + 4 * n_views * P * (n_views * Pp + P) * C)
    f_patch = 2 * S * npatch * 588 * C
    C2 = 2 * C
    f_cam = 4 * (4 * S * 24 * C2 * C2 + 4 * 4 * S * S * C2 + S * (2 * 9 * C2 + 2 * C2 * 3 * C2 + 2 * C2 * C + 2 * C * 9))
    return (2 * f_stack + f_global + f_reloc + f_patch + f_cam) / 1e12


def build_model(device, seed_rule=True):
    from sailrecon_amd.models.sail_recon import SailRecon
    from sailrecon_amd.utils.synth_weights import synth_state_dict_like
    torch.manual_seed(0)
    model = SailRecon(enable_point=False, enable_depth=False).eval()
    sd = synth_state_dict_like(model) if seed_rule else None
    if sd is not None:
        model.load_state_dict(sd)
    return model.to(device), sd


def cpu_baseline(sd, img: int, n_views: int):
    """The CPU oracle (oracle/sfm_oracle.py, a port of the reference path: dense reloc mask,
    scatter reassembly, fp32) on a bounded sample: one full forward of an n_views scene
    (2*n_views frames, the headline's per-view structure at a size that runs in ~10-30 s).
    Threads = the physical cores of this process's CPU share (OMP_NUM_THREADS caps it on the
    GPU box, whose os.cpu_count() is the whole machine)."""
    from oracle import sfm_oracle as O
    model, phys, logical = host_cpu()
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(phys, cap) if cap > 0 else phys
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(n_views)
    x = torch.rand(n_views, 3, img, img, generator=g)
    images = torch.cat([x, x])[None]
    npatch = (img // 14) ** 2
    sub = O.draw_subsample_indices(torch.Generator().manual_seed(0), 24, 1, n_views, npatch, min(300, npatch))
    t0 = time.perf_counter()
    O.hot_path_forward(sd, O.AggCfg(), images, list(range(n_views)), list(range(n_views, 2 * n_views)), 300, sub)
    dt = time.perf_counter() - t0
    return {"value": n_views / dt, "unit": "views/s", "cores": threads, "kind": "port",
            "cpu_model": model, "physical_cores": phys, "os_cpu_count": logical,
            "threads_note": (f"min(physical cores {phys}, OMP_NUM_THREADS {cap}): the GPU box allots this "
                             "process a share of the host's CPUs per GPU, and os.cpu_count() counts the whole "
                             "machine") if cap > 0 else "physical cores",
            "sample": f"1 full fp32 forward of a {n_views}-view scene @{img}px ({2 * n_views} frames; "
                      f"aggregator+camera head+pose decode, the oracle port of the reference path) on the host "
                      f"CPU, {threads} threads, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--views", type=int, default=32)
    ap.add_argument("--img", type=int, default=518)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-views", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--fp8-global", choices=["off", "qk", "qkv"], default="off",
                    help="BASELINE C5: the global blocks' q.k^T (qk) or q.k^T and P.V (qkv) in block-scaled fp8 "
                         "e4m3; everything else bf16")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    device = torch.device("cuda", local if world > 1 else 0)

    from sailrecon_amd import ops

    model, sd = build_model(device)
    if world > 1:
        model.aggregator.set_frame_sharding(dist.group.WORLD)
    n = args.views
    g = torch.Generator().manual_seed(n)
    x = torch.rand(n, 3, args.img, args.img, generator=g)
    images = torch.cat([x, x])[None].to(device)  # demo_imc_forward.py:76-82
    no_reloc, reloc = list(range(n)), list(range(n, 2 * n))
    use_bf16 = args.dtype == "bf16"
    fp8 = args.fp8_global != "off" and use_bf16
    if fp8:
        model.aggregator.set_fp8_global(True, fp8_v=args.fp8_global == "qkv")

    def step():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=use_bf16):
            return model(images, no_reloc_list=no_reloc, reloc_list=reloc, fix_rank=300)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    if not args.no_kernel_timing:
        ops.TIMER = ops.KernelTimer()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    timer, ops.TIMER = ops.TIMER, None
    dt_t = torch.tensor([dt], device=device)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    total_views = n * args.steps  # one scene, sharded across the ranks

    roofline = None
    breakdown = {}
    peak_src = None
    if timer is not None:
        breakdown = timer.summary()
        bf16_peak = PEAK_BF16_TFLOPS
        tf, peak_src = gpu_peak(device.index or 0)
        if tf:
            bf16_peak = tf
        peak = bf16_peak if use_bf16 else PEAK_F32_TFLOPS
        dom = max(breakdown, key=lambda k: breakdown[k]["total_ms"])
        b = breakdown[dom]
        achieved = b["tflops"]
        kern = kernel_of_tag(dom, n, args.img) if use_bf16 else None
        if fp8 and dom == "attn_global":
            # half the attention flops (q.k^T) at the fp8 rate (2x bf16), half (P.V) at the bf16 rate
            if args.fp8_global == "qkv":  # every attention flop at the fp8 rate
                kern, peak = "attn_qk8_kernel<2, true>", 2 * bf16_peak
            else:
                kern, peak = "attn_qk8_kernel<2, false>", 1.0 / (0.5 / (2 * bf16_peak) + 0.5 / bf16_peak)
        traffic, tsrc = pmc_traffic(kern, n, args.img, args.fp8_global if fp8 else "off") if kern else (None, None)
        roofline = {"bound": "mfma", "kernel": kern or dom, "timer_class": dom, "achieved": round(achieved, 2),
                    "peak": round(peak, 1), "peak_source": peak_src, "unit": "TFLOP/s",
                    "frac": round(achieved / peak, 4),
                    "traffic": None if traffic is None else round(traffic),
                    "traffic_unit": "bytes/launch (HBM, PMC 2xFETCH_SIZE+WRITE_SIZE)",
                    "traffic_source": os.path.relpath(tsrc, REPO) if traffic is not None else None,
                    "algorithmic_bytes": round(b["bytes_per_launch"]),
                    "avg_launch_ms": round(b["avg_ms"], 4), "flop_per_launch": b["flops_per_launch"]}
        gems = [v for k, v in breakdown.items() if k.startswith("gemm_")]
        if gems:
            flop = sum(v["flops_per_launch"] * v["launches"] for v in gems)
            ms = sum(v["total_ms"] for v in gems)
            roofline["gemm_all_tflops"] = round(flop / (ms * 1e-3) / 1e12, 1)
            gpeak = bf16_peak if use_bf16 else PEAK_F32_TFLOPS  # GEMMs stay bf16 in the fp8 modes
            roofline["gemm_mfma_util"] = round(flop / (ms * 1e-3) / 1e12 / gpeak, 4)
        print(json.dumps({"kernel_breakdown": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv)
                                                   for kk, vv in v.items()} for k, v in breakdown.items()},
                          "step_ms": dt / args.steps * 1e3}), file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline({k: v for k, v in sd.items()}, args.img, args.cpu_views)

    if rank == 0:
        tflop = algorithmic_tflop(n, args.img)
        line = {
            "metric": f"aggregator fwd views/sec, N={n} @ {args.img}px",
            "value": total_views / dt,
            "unit": "views/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if world > 1 else "weak",
            "vs_baseline": None,
            "dtype": (f"bf16, global {'q.k^T' if args.fp8_global == 'qk' else 'q.k^T + P.V'} fp8-e4m3" if fp8
                      else args.dtype),
            "data": "synthetic (seeded U[0,1) images, seeded synthetic weights)",
            "config": {"workload": f"N={n} views @{args.img}px duplicated to {2 * n} frames (anchors+queries), "
                                   "fix_rank=300: Aggregator + CameraHead + pose decode",
                       "views": n, "img": args.img, "frames": 2 * n, "fix_rank": 300,
                       "parallelism": f"frame-sharded x{world} (RCCL K/V all-gather)" if world > 1 else "single GPU",
                       "algorithmic_tflop_per_step": round(tflop, 2),
                       "achieved_tflops_whole_step": round(tflop * args.steps / dt, 1)},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
