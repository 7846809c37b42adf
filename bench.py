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

Multi-GPU: one process per GPU.  Launched by torch.distributed.run (WORLD_SIZE set) the
ranks come from the environment; launched plainly with --gpus N > 1, bench.py starts N
worker processes itself (fresh interpreters, before anything touches the GPU — the
reference's mp.spawn(train_worker, nprocs=world_size), train/train_imc.py:555-576) with
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 set, and exits with the worst
worker exit code.  Each worker joins an RCCL ("nccl") process group; rank 0 reports
n_gpus = the group's world size and ``ranks_seen`` = the all-gathered (rank, device,
PCI bus) list, so the JSON line itself shows which devices took part.
The ONE 32-view scene is sharded by frame across the ranks
(Aggregator.set_frame_sharding: local DINO / frame / MLP work, RCCL all-gathers of
anchor K/V for the global block and of the anchor-subsample K/V for the reloc block,
replicated camera head).  value = the scene's views / max-over-ranks time, scaling
"strong" (total work fixed as N grows).  --launch-only runs the launcher, the process
group and the ranks_seen report without the model (gloo when no GPU is visible: the
CPU test of the launcher).

Prints ONE JSON line on rank 0 (contract in the task statement) with a
``roofline`` object for the dominant kernel class (live HIP-event timing inside
the timed region) and a ``cpu_baseline`` object (the CPU oracle on a bounded
sample, rank 0 at N=1 only).  A per-kernel-class breakdown goes to stderr.
After the headline's timed region the same model also times the ``extra_configs`` (--extras):
N=64 @518 (the north star's 64-view scaling workload, sharded like the headline), on one GPU
BASELINE C5 (N=128 @518 with fp8 global attention), and the headline workload at qk-norm gain 4
(``g4``: trained-like q_norm / k_norm weights); they ride inside the one line and are never its
``value``.
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

# the aggregator's bf16 GEMM timer classes (patch embed, QKV, proj / fc2, fc1): the scope of the
# north-star "MFMA peak on aggregator GEMMs"; the camera head's fp32 GEMMs (*_f32) are reported apart
AGG_GEMM_TAGS = ("gemm_bias", "gemm_gelu", "gemm_resid", "gemm_qkv", "gemm_patch")


def kernel_of_class(entry):
    """rocprofv3 name of the kernel a timer class launched, as the library itself reported it
    (ops.KernelTimer records sr_last_kernel per launch: the C dispatch is the single source of
    truth); the most-launched one if a class ran several.  None if unreported."""
    ks = entry.get("kernels") or {}
    return max(ks, key=ks.get) if ks else None


TRAFFIC_FILES = [os.path.join(REPO, "profiles", f) for f in
                 ("r06_s3_pmc_traffic.json", "r06_s2_pmc_traffic.json", "r06_final_pmc_traffic.json", "r06_pmc_traffic.json", "r05_final2_pmc_traffic.json",
                  "r05_pmc_traffic.json", "r04_pmc_traffic.json", "r03b_pmc_traffic.json", "r03_pmc_traffic.json", "r02_pmc_traffic.json", "r02_pmc_traffic_c5_fp8qkv.json")]


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


def scale_qk_gain(model, g: float) -> int:
    """Multiply every q_norm / k_norm weight (attention.py:78, qk_norm=True blocks) by g and drop
    the blocks' packed-weight caches; returns the number of norms scaled."""
    n = 0
    with torch.no_grad():
        for m in model.modules():
            for name in ("q_norm", "k_norm"):
                ln = getattr(m, name, None)
                if ln is not None and getattr(ln, "weight", None) is not None:
                    ln.weight.mul_(g)
                    n += 1
        for m in model.modules():
            if hasattr(m, "invalidate_packed"):
                m.invalidate_packed()
    return n


def _cpu_threads():
    model, phys, logical = host_cpu()
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(phys, cap) if cap > 0 else phys
    note = (f"min(physical cores {phys}, OMP_NUM_THREADS {cap}): the GPU box allots this process a share of the "
            "host's CPUs per GPU, and os.cpu_count() counts the whole machine") if cap > 0 else "physical cores"
    return model, phys, logical, threads, note


def cpu_full_forward(sd, img: int, n_views: int) -> float:
    """Seconds for one full oracle forward (aggregator + camera head + pose decode) of an
    n_views scene: the cross-check of the per-layer estimate below at a size that runs whole."""
    from oracle import sfm_oracle as O
    g = torch.Generator().manual_seed(n_views)
    x = torch.rand(n_views, 3, img, img, generator=g)
    images = torch.cat([x, x])[None]
    npatch = (img // 14) ** 2
    sub = O.draw_subsample_indices(torch.Generator().manual_seed(0), 24, 1, n_views, npatch, min(300, npatch))
    t0 = time.perf_counter()
    O.hot_path_forward(sd, O.AggCfg(), images, list(range(n_views)), list(range(n_views, 2 * n_views)), 300, sub)
    return time.perf_counter() - t0


def cpu_forward_by_layer(sd, img: int, n_views: int, depth: int = 24):
    """Seconds for one oracle forward of the n_views headline scene, timed per stack: the
    aggregator's 24 layers all have the same shapes, so one layer of each stack is run on
    tensors of the headline shape and multiplied by 24 (aggregator.py:242-433 order):
      patch embed (conv + cls + pos-embed + registers) of 2N frames, once;
      DINO block [2N, P, C] (eps 1e-6, no RoPE), x24, and the final DINO LayerNorm;
      frame block [2N, P, C] (qk-norm + RoPE), x24;
      the dense reloc mask (aggregator.py:302-311), once per forward as the reference builds it;
      subsample gather + global_reloc block over [N*P' ; N*P] tokens with that mask, x24;
      global block over the N*P anchor tokens, x24;
      reassembly into a fresh ones() tensor with two scatters (aggregator.py:393-399), x24;
      camera head (4 iterations x 4 trunk blocks, fp32) + pose decode on the 2N camera tokens, once.
    Returns (total seconds, {part: seconds per application})."""
    from oracle import sfm_oracle as O
    pre = "aggregator."
    S, n = 2 * n_views, n_views
    hp = img // 14
    npatch, psi, C = hp * hp, 5, 1024
    P, rank = npatch + psi, min(300, npatch)
    Pp = rank + psi
    g = torch.Generator().manual_seed(n_views)
    parts = {}

    def timed(name, fn):
        t0 = time.perf_counter()
        r = fn()
        parts[name] = time.perf_counter() - t0
        return r

    with torch.no_grad():
        imgs = torch.rand(S, 3, img, img, generator=g)
        mean = torch.tensor(O.RESNET_MEAN).view(1, 3, 1, 1)
        std = torch.tensor(O.RESNET_STD).view(1, 3, 1, 1)
        x = timed("patch_embed", lambda: O.dino_embed(sd, pre + "patch_embed.", (imgs - mean) / std, 14))
        x = timed("dino_block", lambda: O.block(sd, pre + "patch_embed.blocks.0.", x, 16, 1e-6))
        timed("dino_norm", lambda: O.layer_norm(x, sd[pre + "patch_embed.norm.weight"],
                                                sd[pre + "patch_embed.norm.bias"], 1e-6))
        tokens = torch.randn(S, P, C, generator=g)
        yy, xx = torch.meshgrid(torch.arange(hp), torch.arange(hp), indexing="ij")
        grid = torch.stack([yy.reshape(-1), xx.reshape(-1)], dim=-1) + 1
        pos = torch.cat([torch.zeros(psi, 2, dtype=torch.long), grid], dim=0)[None].expand(S, P, 2).contiguous()
        tokens = timed("frame_block", lambda: O.block(sd, pre + "frame_blocks.0.", tokens, 16, 1e-5, pos=pos,
                                                      qk_norm=True, rope_base=100.0))
        mask = timed("reloc_mask", lambda: O.reloc_mask(S, n, n, P, psi, rank))
        sub_idx = O.draw_subsample_indices(torch.Generator().manual_seed(0), 1, 1, n, npatch, rank)[0]

        def reloc():
            fo = tokens.view(1, S, P, C)
            anc, anc_pos = fo[:, :n], pos.view(1, S, P, 2)[:, :n]
            sel = sub_idx[..., :rank] + psi
            gt = torch.gather(anc, 2, sel[..., None].expand(1, n, rank, C))
            gp = torch.gather(anc_pos, 2, sel[..., None].expand(1, n, rank, 2))
            sub = torch.cat([anc[:, :, :psi], gt], dim=2).reshape(1, n * Pp, C)
            sub_pos = torch.cat([anc_pos[:, :, :psi], gp], dim=2).reshape(1, n * Pp, 2)
            seq = torch.cat([sub, fo[:, n:].reshape(1, n * P, C)], dim=1)
            sp = torch.cat([sub_pos, pos.view(1, S, P, 2)[:, n:].reshape(1, n * P, 2)], dim=1)
            return O.block(sd, pre + "global_reloc_blocks.0.", seq, 16, 1e-5, pos=sp, mask=mask, qk_norm=True,
                           rope_base=100.0)[:, n * Pp:]

        reloc_out = timed("reloc_block", reloc)
        del mask
        glob = timed("global_block", lambda: O.block(
            sd, pre + "global_blocks.0.", tokens.view(1, S, P, C)[:, :n].reshape(1, n * P, C), 16, 1e-5,
            pos=pos.view(1, S, P, 2)[:, :n].reshape(1, n * P, 2), qk_norm=True, rope_base=100.0))

        def reassemble():
            new = torch.ones(1, S, P, C)
            new[:, :n] = glob.view(1, n, P, C)
            new[:, n:] = reloc_out.view(1, n, P, C)
            return new

        timed("reassembly", reassemble)
        feats_last = torch.randn(1, n, P, 2 * C, generator=g)
        cam_last = torch.randn(1, n, 2 * C, generator=g)

        def head():
            poses = O.camera_head_forward(sd, feats_last, cam_last)
            return O.pose_encoding_to_extri_intri(poses[-1], (img, img))

        timed("camera_head_pose", head)
    per_layer = ("dino_block", "frame_block", "reloc_block", "global_block", "reassembly")
    total = sum(parts[k] * (depth if k in per_layer else 1) for k in parts)
    return total, parts


def cpu_baseline(sd, img: int, n_views: int, cross_views: int = 4):
    """The CPU oracle (oracle/sfm_oracle.py, a port of the reference path: dense reloc mask,
    scatter reassembly, fp32 torch ops) on the headline scene, estimated per layer
    (cpu_forward_by_layer: one layer of each stack at the N-view shapes x 24 + the once-per-
    forward parts), with one full forward of a small scene as a cross-check.  Threads = the
    physical cores of this process's CPU share (OMP_NUM_THREADS caps it on the GPU box, whose
    os.cpu_count() is the whole machine)."""
    model, phys, logical, threads, note = _cpu_threads()
    torch.set_num_threads(threads)
    t0 = time.perf_counter()
    est, parts = cpu_forward_by_layer(sd, img, n_views)
    wall = time.perf_counter() - t0
    out = {"value": n_views / est, "unit": "views/s", "cores": threads, "kind": "port",
           "cpu_model": model, "physical_cores": phys, "os_cpu_count": logical, "threads_note": note,
           "sample": f"N={n_views} @{img}px ({2 * n_views} frames, fp32 oracle port of the reference path), one "
                     f"layer of each stack timed at the N={n_views} shapes x 24 layers + patch embed, dense reloc "
                     f"mask, camera head and pose decode once: {est:.1f} s per forward estimated from {wall:.1f} s "
                     f"of CPU work on {threads} threads",
           "seconds_per_part": {k: round(v, 3) for k, v in parts.items()}}
    # the full N-view oracle forward, timed whole once on a GPU box's host (tools/cpu_full.py; too long
    # for every bench run): the check of the per-layer estimate at the headline size
    full = os.path.join(REPO, "profiles", "r04_cpu_full.json")
    try:
        with open(full) as f:
            d = json.load(f)
        if (d.get("views"), d.get("img")) == (n_views, img):
            out["full_forward_check"] = {k: d[k] for k in ("full_forward_s", "per_layer_estimate_s", "estimate_over_full",
                                                           "views_per_s_full_forward", "cpu_model", "threads")}
            out["full_forward_check"]["source"] = os.path.relpath(full, REPO) + " (tools/cpu_full.py, a separate run)"
    except (OSError, ValueError, KeyError):
        pass
    if cross_views:
        dt = cpu_full_forward(sd, img, cross_views)
        est_small, _ = cpu_forward_by_layer(sd, img, cross_views)
        out["cross_check"] = {"views": cross_views, "full_forward_s": round(dt, 2),
                              "per_layer_estimate_s": round(est_small, 2),
                              "views_per_s_full_forward": round(cross_views / dt, 4)}
    return out


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_workers(n: int, argv) -> int:
    """Start n bench.py worker processes (one per GPU) and wait for them.  The parent never
    initialises the GPU: the world size comes from --gpus, not from a device query.  A worker
    that fails ends the others (their exact PIDs); the parent returns the worst exit code."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                for q in live:  # a failed rank would leave its peers waiting in a collective
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    return rc if rc >= 0 else 128 - rc


def ranks_report(device):
    """(rank, local device, PCI bus, host) of every rank, all-gathered over the process group."""
    import socket
    me = {"rank": dist.get_rank() if dist.is_initialized() else 0, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
          "device": str(device), "host": socket.gethostname()}
    if device.type == "cuda":
        p = torch.cuda.get_device_properties(device)
        me["pci_bus"] = f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:" \
                        f"{getattr(p, 'pci_device_id', 0):02x}"
        me["gpu"] = p.name
    if not dist.is_initialized():
        return [me]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, me)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--views", type=int, default=32)
    ap.add_argument("--img", type=int, default=518)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-views", type=int, default=4,
                    help="views of the full-forward cross-check of the per-layer CPU estimate (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--fp8-global", choices=["off", "qk", "qkv"], default="off",
                    help="BASELINE C5: the global blocks' q.k^T (qk) or q.k^T and P.V (qkv) in block-scaled fp8 "
                         "e4m3; everything else bf16")
    ap.add_argument("--breakdown-steps", type=int, default=2,
                    help="instrumented steps after the timed region for the per-class kernel breakdown")
    ap.add_argument("--extras", default="n64,c5,c5qk,g4",
                    help="comma list of extra workloads timed after the headline on the same model and reported "
                         "inside its line as extra_configs (not the metric): n64 = N=64 @518 bf16 (the north "
                         "star's 64-view scaling workload, sharded like the headline), c5 = BASELINE C5 as BASELINE "
                         "states it (N=128 @518, the global blocks' fp8 QKV path: q.k^T and P.V in block-scaled "
                         "e4m3), c5qk = the same with only q.k^T in fp8 (one GPU only, both); g4 = the headline at "
                         "qk-norm gain 4; '' or 'none' to skip")
    ap.add_argument("--c5-fp8", choices=["qk", "qkv"], default="qkv",
                    help="the c5 extra's fp8 mode: q.k^T and P.V (qkv, BASELINE C5's fp8 QKV path) or q.k^T "
                         "only (qk)")
    ap.add_argument("--qk-gain", type=float, default=1.0,
                    help="scale every q_norm / k_norm weight of the aggregator by this factor (trained models carry "
                         "gains of ~2-3; the synthetic weights ~1): the attention softmax's peakedness, for A/B of "
                         "the kernels' behaviour under trained-weight statistics; reported in config")
    ap.add_argument("--launch-only", action="store_true",
                    help="launcher / process-group / ranks_seen check without the model (gloo if no GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_workers(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; reporting the process group's size",
              file=sys.stderr)
    on_gpu = torch.cuda.is_available()
    if not on_gpu and not args.launch_only:
        raise SystemExit("bench.py: no ROCm GPU visible (the HIP path has no CPU fallback); "
                         "--launch-only checks the launcher alone")
    # SR_BENCH_REHEARSE=1 (rehearsal only, never a measurement): every rank on cuda:0 over gloo, so
    # the N-rank path (sharding plan, collectives, extras, the JSON line) runs end to end on a
    # one-GPU box; the driver's multi-GPU runs leave it unset (one GPU per rank, RCCL)
    rehearse = os.environ.get("SR_BENCH_REHEARSE", "0") == "1"
    device = torch.device("cuda", 0 if rehearse else local) if on_gpu else torch.device("cpu")
    if on_gpu:
        torch.cuda.set_device(device)
    use_pg = "WORLD_SIZE" in os.environ  # torchrun / the launcher, any world size
    if use_pg:
        dist.init_process_group("nccl" if on_gpu and not rehearse else "gloo")
    seen = ranks_report(device)
    if args.launch_only:
        if rank == 0:
            print(json.dumps({"launch_only": True, "n_gpus": dist.get_world_size() if use_pg else 1,
                              "backend": dist.get_backend() if use_pg else None, "ranks_seen": seen}))
        if use_pg:
            dist.barrier()
            dist.destroy_process_group()
        return

    from sailrecon_amd import ops

    model, sd = build_model(device)
    if args.qk_gain != 1.0:
        scale_qk_gain(model, args.qk_gain)
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
    # inside the timed region HIP events bracket the dominant class's launches only (DOMINANT_TAG,
    # the pair launch: 24 per step); events around every launch (~1,100 per step) cost the step host
    # and queue time, so the per-class breakdown comes from --breakdown-steps more steps after it
    if not args.no_kernel_timing:
        ops.TIMER = ops.KernelTimer(tags={DOMINANT_TAG})
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    timer_dom, ops.TIMER = ops.TIMER, None
    dt_t = torch.tensor([dt], device=device)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    total_views = n * args.steps  # one scene, sharded across the ranks
    timer = None
    if timer_dom is not None and args.breakdown_steps > 0:
        ops.TIMER = ops.KernelTimer()
        for _ in range(args.breakdown_steps):
            step()
        barrier()
        timer, ops.TIMER = ops.TIMER, None

    roofline = None
    breakdown = {}
    peak_src = None
    if timer is not None:
        breakdown = timer.summary()
        live = timer_dom.summary()  # the dominant class, measured inside the timed region
        bf16_peak = PEAK_BF16_TFLOPS
        tf, peak_src = gpu_peak(device.index or 0)
        if tf:
            bf16_peak = tf
        peak = bf16_peak if use_bf16 else PEAK_F32_TFLOPS
        dom = max(breakdown, key=lambda k: breakdown[k]["total_ms"])
        b = live[dom] if dom in live else breakdown[dom]
        achieved = b["tflops"]
        kern = kernel_of_class(b)
        if fp8 and dom == "attn_global":
            # half the attention flops (q.k^T) at the fp8 rate (2x bf16), half (P.V) at the bf16 rate
            if args.fp8_global == "qkv":  # every attention flop at the fp8 rate
                peak = 2 * bf16_peak
            else:
                peak = 1.0 / (0.5 / (2 * bf16_peak) + 0.5 / bf16_peak)
        traffic, tsrc = pmc_traffic(kern, n, args.img, args.fp8_global if fp8 else "off") if kern else (None, None)
        roofline = {"bound": "mfma", "kernel": kern or dom, "kernel_source": "sr_last_kernel" if kern else None,
                    "timer_class": dom, "achieved": round(achieved, 2),
                    "peak": round(peak, 1), "peak_source": peak_src, "unit": "TFLOP/s",
                    "frac": round(achieved / peak, 4),
                    "traffic": None if traffic is None else round(traffic),
                    "traffic_unit": "bytes/launch (HBM, PMC 2xFETCH_SIZE+WRITE_SIZE)",
                    "traffic_source": os.path.relpath(tsrc, REPO) if traffic is not None else None,
                    "algorithmic_bytes": round(b["bytes_per_launch"]),
                    "avg_launch_ms": round(b["avg_ms"], 4), "flop_per_launch": b["flops_per_launch"],
                    "timing": (f"HIP events around the {dom} launches inside the timed region ({b['launches']} "
                               f"launches); the other classes (gemm_mfma_util) from {args.breakdown_steps} "
                               "instrumented steps after it" if dom in live else
                               f"{args.breakdown_steps} instrumented steps after the timed region")}
        def gemm_rate(tags):
            sel = [breakdown[k] for k in tags if k in breakdown]
            if not sel:
                return None
            flop = sum(v["flops_per_launch"] * v["launches"] for v in sel)
            return flop / (sum(v["total_ms"] for v in sel) * 1e-3) / 1e12

        gpeak = bf16_peak if use_bf16 else PEAK_F32_TFLOPS  # GEMMs stay bf16 in the fp8 modes
        agg = gemm_rate(list(AGG_GEMM_TAGS))
        if agg is not None:
            roofline["gemm_agg_tflops"] = round(agg, 1)
            roofline["gemm_mfma_util"] = round(agg / gpeak, 4)
            roofline["gemm_mfma_util_scope"] = "aggregator GEMMs (" + ", ".join(k for k in AGG_GEMM_TAGS
                                                                                  if k in breakdown) + ")"
        allr = gemm_rate([k for k in breakdown if k.startswith("gemm_")])
        if allr is not None:
            roofline["gemm_all_tflops"] = round(allr, 1)
        print(json.dumps({"kernel_breakdown": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv)
                                                   for kk, vv in v.items()} for k, v in breakdown.items()},
                          "breakdown_steps": args.breakdown_steps, "step_ms": dt / args.steps * 1e3}),
              file=sys.stderr)

    extras = []
    if use_bf16 and not fp8:
        for name in [e for e in args.extras.split(",") if e and e != "none"]:
            if name in ("c5", "c5qk") and world > 1:
                continue
            if name not in ("n64", "c5", "c5qk", "g4"):
                raise SystemExit(f"bench.py: unknown extra workload {name!r}")
            if name == "g4" and args.qk_gain != 1.0:
                continue  # the headline already runs at a scaled gain
            extras.append(extra_config(model, device, args, world, name))

    calib = box_calibration(device) if use_bf16 else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline({k: v for k, v in sd.items()}, args.img, n, args.cpu_views)

    if rank == 0:
        tflop = algorithmic_tflop(n, args.img)
        line = {
            "metric": f"aggregator fwd views/sec, N={n} @ {args.img}px",
            "value": total_views / dt,
            "unit": "views/s",
            "n_gpus": dist.get_world_size() if use_pg else 1,
            "backend": dist.get_backend() if use_pg else None,
            "ranks_seen": seen,
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
                       "views": n, "img": args.img, "frames": 2 * n, "fix_rank": 300, "qk_gain": args.qk_gain,
                       "parallelism": f"frame-sharded x{world} (RCCL K/V all-gather)" if world > 1 else "single GPU",
                       "algorithmic_tflop_per_step": round(tflop, 2),
                       "achieved_tflops_whole_step": round(tflop * args.steps / dt, 1)},
            "roofline": roofline,
            "box_calibration": calib,
            "cpu_baseline": cpu,
            "extra_configs": extras,
        }
        if rehearse:
            line["rehearsal"] = "SR_BENCH_REHEARSE: every rank on cuda:0 over gloo (a code-path check, not a measurement)"
        if calib and calib.get("tflops"):
            # views/s as if on a box whose calibration GEMM runs CALIB_REF_TFLOPS (round-over-round
            # comparisons independent of the box the driver drew; the raw value stays `value`)
            calib["normalised_value"] = round(line["value"] * CALIB_REF_TFLOPS / calib["tflops"], 3)
            calib["normalised_to_tflops"] = CALIB_REF_TFLOPS
        print(json.dumps(line))
    if use_pg:
        dist.destroy_process_group()


# the timer class of the headline's dominant kernel (the global attention + reloc subsample pair
# launch; the fp8 global attention in C5): the one class timed inside the measured region
DOMINANT_TAG = "attn_global"

# the calibration GEMM's rate on a typical box of this pool (rounds 4-5: 1,143-1,206 TF/s)
CALIB_REF_TFLOPS = 1180.0


def box_calibration(device):
    """One fixed kernel timed after the measured region, so that lines from different MI355X boxes
    can be compared: MFMA-bound loops run 1-12 % apart across devices at the clock each holds under
    load (MI355X_MICROARCH.md 'DVFS give-back' item 5).  The library's 256x256 bf16 GEMM on seeded
    random 8192^3 operands (bias epilogue), 10 launches after 3 warm-up ones, HIP events."""
    from sailrecon_amd import _lib, ops
    n = 8192
    g = torch.Generator(device=device).manual_seed(7)
    a = torch.rand(n, n, device=device, generator=g, dtype=torch.float32).sub_(0.5).bfloat16()
    w = torch.rand(n, n, device=device, generator=g, dtype=torch.float32).sub_(0.5).bfloat16()
    out = torch.empty(n, n, device=device, dtype=torch.bfloat16)
    for _ in range(3):
        ops.gemm(a, w, out, _lib.SR_EPI_BIAS)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.gemm(a, w, out, _lib.SR_EPI_BIAS)
    e1.record()
    torch.cuda.synchronize(device)
    ms = e0.elapsed_time(e1) / 10
    kern = ops.last_kernel()
    del a, w, out
    return {"kernel": kern, "shape": "8192^3 bf16, seeded U[-0.5, 0.5)", "avg_launch_ms": round(ms, 4),
            "tflops": round(2.0 * n ** 3 / ms / 1e9, 1)}


def extra_config(model, device, args, world, name):
    """An extra workload timed on the same model after the headline (reported inside the headline
    line's ``extra_configs``, never as its value): ``n64`` = N=64 @518 bf16, the north star's
    64-view scaling workload (frame-sharded like the headline when world > 1); ``c5`` = BASELINE
    config 5 (N=128 @518, 256 frames, L_g = 175,872) with the global blocks' attention in fp8
    (Aggregator.set_fp8_global; --c5-fp8, default q.k^T and P.V: BASELINE's "fp8 MFMA QKV path"),
    ``c5qk`` the same with q.k^T alone in fp8, one GPU; ``g4`` = the headline workload with every q_norm / k_norm
weight x 4 (scale_qk_gain, undone after).  One untimed warmup, then a few steps between barriers +
    synchronize, max over ranks.  A Python error is reported in the object, not raised."""
    from sailrecon_amd import ops
    n = {"n64": 64, "c5": 128, "c5qk": 128}.get(name, args.views)
    fp8 = name in ("c5", "c5qk")
    fp8_mode = "qk" if name == "c5qk" else args.c5_fp8
    gain = 4.0 if name == "g4" else None
    steps = 2 if fp8 else 3
    g = torch.Generator().manual_seed(n)
    x = torch.rand(n, 3, args.img, args.img, generator=g)
    images = torch.cat([x, x])[None].to(device)
    no_reloc, reloc = list(range(n)), list(range(n, 2 * n))
    dtype = (f"bf16, global {'q.k^T' if fp8_mode == 'qk' else 'q.k^T + P.V'} fp8-e4m3" if fp8 else "bf16")
    what = {"n64": " (north-star 64-view workload)", "c5": f" (BASELINE C5, fp8 global attention: {fp8_mode})",
            "c5qk": " (BASELINE C5, fp8 global attention: q.k^T only)",
            "g4": " at qk-norm gain 4 (trained-like q_norm / k_norm weights: every one x 4)"}.get(name, "")
    out = {"name": name, "metric": f"aggregator fwd views/sec, N={n} @ {args.img}px" + what,
           "unit": "views/s", "dtype": dtype, "views": n, "frames": 2 * n, "steps": steps, "warmup": 1}
    if gain is not None:
        out["qk_gain"] = gain

    def step():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            return model(images, no_reloc_list=no_reloc, reloc_list=reloc, fix_rank=300)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    timer = None
    try:
        if fp8:
            model.aggregator.set_fp8_global(True, fp8_v=fp8_mode == "qkv")
        if gain is not None:
            scale_qk_gain(model, gain)
        step()
        barrier()
        ops.TIMER = ops.KernelTimer(tags={DOMINANT_TAG})
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        barrier()
        dt = time.perf_counter() - t0
        timer = ops.TIMER
    except Exception as e:  # noqa: BLE001  (reported, the headline stands)
        out["error"] = f"{type(e).__name__}: {e}"
        return out
    finally:
        ops.TIMER = None
        if fp8:
            model.aggregator.set_fp8_global(False)
        if gain is not None:
            scale_qk_gain(model, 1.0 / gain)  # a power of two: the weights come back exactly
    dt_t = torch.tensor([dt], device=device)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    att = timer.summary().get("attn_global") if timer is not None else None
    tflop = algorithmic_tflop(n, args.img)
    out.update({"value": n * steps / dt, "ms_per_step": dt / steps * 1e3,
                "algorithmic_tflop_per_step": round(tflop, 2),
                "achieved_tflops_whole_step": round(tflop * steps / dt, 1),
                "attn_global": None if att is None else {"avg_launch_ms": round(att["avg_ms"], 4),
                                                         "tflops": round(att["tflops"], 1),
                                                         "kernels": att.get("kernels")}})
    if fp8 and att is not None and gpu_peak()[0]:
        # the global attention against the MFMA peak of its operand mix: qkv runs both products on the
        # block-scaled fp8 MFMA (2x the bf16 rate); qk runs half the flops there and half at the bf16
        # rate, i.e. 4/3 of the bf16 peak (MI355X_MICROARCH.md, "Matrix cores")
        bf16_peak, _ = gpu_peak()
        peak = bf16_peak * (2.0 if fp8_mode == "qkv" else 4.0 / 3.0)
        out["roofline"] = {"bound": "mfma", "kernel": next(iter(att.get("kernels") or {}), None),
                           "achieved": round(att["tflops"], 1), "peak": round(peak, 1), "unit": "TFLOP/s",
                           "frac": round(att["tflops"] / peak, 4),
                           "peak_source": f"{'2' if fp8_mode == 'qkv' else '4/3'} x the bf16 peak {bf16_peak:.1f} "
                                          "(block-scaled e4m3 MFMA at 2x the bf16 rate)"}
    del images
    return out


if __name__ == "__main__":
    main()
