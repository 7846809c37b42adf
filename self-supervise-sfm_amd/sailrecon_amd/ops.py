"""Tensor-level wrappers over the C ABI (include/sfm_amd.h).

Every function takes device tensors (2-D row-strided views, unit column stride),
launches on the current torch stream and returns nothing (outputs are written in
place).  No function here computes anything on the host.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import AttnDesc, GemmEpi, check

Tensor = torch.Tensor


class KernelTimer:
    """Records HIP events around tagged launches on the launching (current torch) stream.

    Used by bench.py to measure the dominant kernel's average launch duration inside the
    timed region; ``work`` is the algorithmic FLOP count of the launch.
    """

    def __init__(self, tags=None):
        self.tags = None if tags is None else set(tags)
        self.records = {}
        self.kernels = {}  # tag -> {kernel name: launches}

    def wants(self, tag: Optional[str]) -> bool:
        return tag is not None and (self.tags is None or tag in self.tags)

    def start(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def stop(self, tag: str, ev0, work: float, nbytes: float = 0.0, kernel: Optional[str] = None):
        """``kernel``: the rocprof name of the launch's kernel, as the library reports it
        (last_kernel(), sr_last_kernel) -- the library's own dispatch decision."""
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self.records.setdefault(tag, []).append((ev0, ev1, work, nbytes))
        if kernel:
            k = self.kernels.setdefault(tag, {})
            k[kernel] = k.get(kernel, 0) + 1

    def summary(self):
        """tag -> dict(launches, total_ms, avg_ms, flops_per_launch, tflops, bytes_per_launch, gbs,
        kernels = {rocprof kernel name: launches} as the library reported them)

        ``bytes_per_launch`` is the algorithmic (compulsory) HBM traffic of a launch:
        every operand read once, every output written once."""
        torch.cuda.synchronize()
        out = {}
        for tag, recs in self.records.items():
            ms = [r[0].elapsed_time(r[1]) for r in recs]
            work = sum(r[2] for r in recs)
            nbytes = sum(r[3] for r in recs)
            tot = sum(ms)
            sec = tot * 1e-3
            out[tag] = dict(launches=len(recs), total_ms=tot, avg_ms=tot / len(recs),
                            flops_per_launch=work / len(recs), tflops=(work / sec / 1e12) if tot else 0.0,
                            bytes_per_launch=nbytes / len(recs), gbs=(nbytes / sec / 1e9) if tot else 0.0,
                            kernels=dict(self.kernels.get(tag, {})))
        return out


TIMER: Optional[KernelTimer] = None


# ---- the library's tuning switches (sfm_amd.h sr_tuning_key), by environment-variable name
_TUNE_KEYS: dict = {}


def _tune_key(name: str) -> int:
    if not _TUNE_KEYS:
        lib = _lib.load()
        k = 0
        while True:
            n = lib.sr_tuning_name(k)
            if n is None:
                break
            _TUNE_KEYS[n.decode()] = k
            k += 1
    if name not in _TUNE_KEYS:
        raise KeyError(f"unknown tuning switch {name!r} (known: {sorted(_TUNE_KEYS)})")
    return _TUNE_KEYS[name]


def tuning_names():
    """Every switch the library has (sr_tuning_name), e.g. 'SR_ATTN_PIPE'."""
    _tune_key("SR_ATTN_PIPE")
    return sorted(_TUNE_KEYS, key=_TUNE_KEYS.get)


def get_tuning(name: str) -> int:
    """Current value of a library tuning switch (sr_get_tuning); it starts from the environment."""
    return int(_lib.load().sr_get_tuning(_tune_key(name)))


def set_tuning(name: str, value: int) -> int:
    """Sets a library tuning switch (sr_set_tuning) for every later launch; returns the old value."""
    return int(_lib.load().sr_set_tuning(_tune_key(name), int(value)))


@contextlib.contextmanager
def tuning(**switches):
    """with ops.tuning(SR_ATTN_PIPE_SEG=1): ... -- switches set for the block, restored after."""
    old = {k: set_tuning(k, v) for k, v in switches.items()}
    try:
        yield
    finally:
        for k, v in old.items():
            set_tuning(k, v)


def last_kernel() -> str:
    """The main kernel the last library call on this thread launched (sr_last_kernel)."""
    return _lib.load().sr_last_kernel().decode()

_EPI_NAME = {_lib.SR_EPI_BIAS: "bias", _lib.SR_EPI_BIAS_GELU: "gelu", _lib.SR_EPI_BIAS_RESID: "resid",
             _lib.SR_EPI_QKV: "qkv", _lib.SR_EPI_PATCH: "patch", _lib.SR_EPI_F32: "f32",
             _lib.SR_EPI_GELU_BWD: "gelu_bwd"}


def _p(t: Optional[Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(t: Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.bfloat16:
        return _lib.SR_BF16
    if dt == torch.float32:
        return _lib.SR_F32
    raise TypeError(f"unsupported dtype {dt} (bf16 or fp32)")


def _rowmajor(t: Tensor, name: str) -> int:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name} must be a 2-D view with unit column stride, got shape {tuple(t.shape)} "
                         f"stride {t.stride()}")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    return t.stride(0)


_SPLITK_WS = {}  # (device, stream) -> fp32 workspace of sr_gemm_splitk


def _splitk_plan(M: int, N: int, K: int, epi: int, dtype: torch.dtype) -> int:
    """K slices for few-row GEMMs (the camera trunk, M = 2N views): enough 128x128-tile
    workgroups to spread the weight stream over the CUs; 1 = plain sr_gemm."""
    if M > 256 or epi not in (_lib.SR_EPI_BIAS, _lib.SR_EPI_BIAS_GELU, _lib.SR_EPI_BIAS_RESID, _lib.SR_EPI_F32):
        return 1
    ktiles = K // (64 if dtype == torch.bfloat16 else 32)
    # sr_gemm's tiles: 64 x 256 for M <= 64 (SR_GEMM_SMALLM), else 128 x 128
    wgs = -(-N // 256) if (M <= 64 and N > 128 and get_tuning("SR_GEMM_SMALLM")) else -(-M // 128) * (N // 128)
    # partial-tile traffic (2 * splits * M * N) <= the weight stream (N * K), at most one workgroup per
    # CU: measured best at the camera trunk's shapes (tools/kbench.py gemm_cam, M = 64, fp32: qkv 8,
    # proj 16, fc1 8, fc2 32 slices; profiles/r05_j2_kbench_gemm_cam.log)
    cap = max(1, K // (2 * M))
    splits = 1
    while (wgs * splits * 2 <= 256 and splits * 2 <= cap and ktiles % (splits * 2) == 0
           and ktiles // (splits * 2) >= 4):
        splits *= 2
    return splits


def _ws_stream_key(device):
    """Scratch buffers are keyed by (device, current stream): launches on different streams (the
    opt-in concurrent reloc stack, SR_CONCURRENT_STACKS) never share one."""
    d = torch.device(device)
    return (str(d), torch.cuda.current_stream(d).cuda_stream if d.type == "cuda" else 0)


def _splitk_workspace(device, numel: int) -> Tensor:
    key = _ws_stream_key(device)
    ws = _SPLITK_WS.get(key)
    if ws is None or ws.numel() < numel:
        ws = torch.empty(numel, device=device, dtype=torch.float32)
        _SPLITK_WS[key] = ws
    return ws


def _fill_qkv_epi(ep: GemmEpi, qkv: dict) -> None:
    """qk-norm / RoPE / position fields of sr_gemm_epi (runtime.qkv_params dict)."""
    ep.qn_w, ep.qn_b = _p(qkv.get("qn_w")), _p(qkv.get("qn_b"))
    ep.kn_w, ep.kn_b = _p(qkv.get("kn_w")), _p(qkv.get("kn_b"))
    ep.qk_eps = qkv.get("qk_eps", 1e-5)
    cos, sin = qkv.get("rope_cos"), qkv.get("rope_sin")
    ep.rope_cos, ep.rope_sin = _p(cos), _p(sin)
    ep.rope_npos = 0 if cos is None else cos.shape[0]
    ep.col_offset = qkv.get("col_offset", 0)
    ep.head_dim = qkv.get("head_dim", 64)
    ep.embed_dim = qkv["embed_dim"]
    ep.pos_yx = _p(qkv.get("pos_yx"))
    ep.pos_rowmap = _p(qkv.get("pos_rowmap"))
    ep.pos_row_base = qkv.get("pos_row_base", 0)
    ep.tokens_per_frame = qkv.get("tokens_per_frame", 1)
    ep.patch_start = qkv.get("patch_start", 0)
    ep.grid_w = qkv.get("grid_w", 1)
    # the Q block of a full q|k|v output leaves as c*q, rounded once (runtime.q_prescale)
    if qkv.get("q_scale") and ep.col_offset == 0:
        ep.q_scale, ep.q_cols = float(qkv["q_scale"]), ep.embed_dim


def gemm(a: Tensor, w: Tensor, out: Tensor, epi: int, *, bias: Optional[Tensor] = None,
         gamma: Optional[Tensor] = None, rows: Optional[int] = None, qkv: Optional[dict] = None,
         patch: Optional[dict] = None, tag: Optional[str] = None, splits: Optional[int] = None,
         aux: Optional[Tensor] = None, q_scale: float = 0.0, q_cols: int = 0,
         colsum: Optional[Tensor] = None) -> None:
    """out = epilogue(a[M,K] . w[N,K]^T).  ``rows`` overrides M (PATCH: out has more rows).
    ``splits`` K slices (sr_gemm_splitk); default: automatic for few rows.  ``aux`` (a's dtype,
    [M, N] view): BIAS_GELU / QKV store the pre-activation there; GELU_BWD reads it.
    ``colsum`` (GELU_BWD; fp32, contiguous, >= colsum_blocks(M) * N): the output's column sums per
    64-row block (sr_gemm_epi.colsum), so colsum(colsum_view) gives the bias gradient.
    ``q_scale`` / ``q_cols`` (BIAS / QKV): output columns [0, q_cols) leave multiplied by q_scale
    before their one rounding (sr_gemm_epi.q_scale; a QKV dict's "q_scale" key sets both)."""
    lda = _rowmajor(a, "a")
    ldw = _rowmajor(w, "w")
    ldo = _rowmajor(out, "out")
    M = a.shape[0] if rows is None else rows
    N, K = w.shape
    if a.shape[1] != K:
        raise ValueError(f"gemm: a has K={a.shape[1]}, w has K={K}")
    if a.dtype != w.dtype:
        raise TypeError("gemm: a and w dtypes differ")
    ep = GemmEpi()
    ep.bias = _p(bias)
    ep.gamma = _p(gamma)
    if qkv is not None:
        _fill_qkv_epi(ep, qkv)
    if q_scale:
        ep.q_scale, ep.q_cols = float(q_scale), int(q_cols)
    if aux is not None:
        if aux.dtype != a.dtype:
            raise TypeError("gemm: aux must have the operand dtype")
        ep.aux, ep.ld_aux = _p(aux), _rowmajor(aux, "aux")
    if colsum is not None:
        _check_colsum(colsum, M, N)
        ep.colsum = _p(colsum)
        splits = 1
    if patch is not None:
        ep.seg_rows = patch["seg_rows"]
        ep.seg_stride = patch["seg_stride"]
        ep.seg_offset = patch["seg_offset"]
        ep.row_add = _p(patch["row_add"])
    if tag == "gemm":  # one timer class per kernel instantiation (matches rocprof rows)
        tag = f"gemm_{_EPI_NAME.get(epi, epi)}" + ("" if a.dtype == torch.bfloat16 else "_f32")
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    if splits is None:  # the split-K reduction has no aux output: saved pre-activations need one pass
        splits = 1 if aux is not None else _splitk_plan(M, N, K, epi, a.dtype)
    elif splits > 1 and aux is not None:
        raise ValueError("gemm: aux outputs are not supported with split-K")
    if splits > 1:
        ws = _splitk_workspace(a.device, splits * M * N)
        rc = _lib.load().sr_gemm_splitk(_stream(a), dtype_code(a.dtype), epi, _p(a), lda, _p(w), ldw, _p(out), ldo,
                                        M, N, K, splits, _p(ws), ctypes.byref(ep))
        check(rc, "sr_gemm_splitk")
    else:
        rc = _lib.load().sr_gemm(_stream(a), dtype_code(a.dtype), epi, _p(a), lda, _p(w), ldw, _p(out), ldo,
                                 M, N, K, ctypes.byref(ep))
        check(rc, "sr_gemm")
    if timed:
        es, eo = a.element_size(), out.element_size()
        nb = (M * K + N * K) * es + M * N * eo * (2 if epi == _lib.SR_EPI_BIAS_RESID else 1)
        TIMER.stop(tag, ev0, 2.0 * M * N * K, nb, kernel=last_kernel())


def colsum_blocks(M: int) -> int:
    """Rows of a GELU_BWD colsum buffer (sr_gemm_epi.colsum): one per 64 output rows."""
    return (M + 63) // 64


def _check_colsum(t: Tensor, M: int, N: int) -> None:
    if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() < colsum_blocks(M) * N or t.data_ptr() % 16:
        raise ValueError(f"gemm: colsum must be a contiguous 16-B aligned fp32 buffer of >= {colsum_blocks(M) * N}")


GEMM_GROUP_MAX = 4
_GEMM_GROUP = os.environ.get("SR_GEMM_GROUP", "1") != "0"


def gemm_group_eligible(problems) -> bool:
    """Whether gemm_group can take these problems (bf16, N % 256 == 0, 1..4 of them; SR_GEMM_GROUP=0
    turns grouping off)."""
    return (_GEMM_GROUP and 1 <= len(problems) <= GEMM_GROUP_MAX and
            all(p["a"].dtype == torch.bfloat16 and p["w"].shape[0] % 256 == 0 for p in problems))


def gemm_group(problems, epi: int, tag: Optional[str] = None) -> None:
    """Several independent gemm() calls of one epilogue kind in ONE launch of the 256x256 kernel
    (sr_gemm_group): each problem a dict with a, w, out and gemm()'s bias / gamma / qkv / aux keywords;
    their last partial workgroup rounds merge."""
    if not gemm_group_eligible(problems):
        raise ValueError("gemm_group: bf16 problems with N % 256 == 0, at most 4")
    arr = (_lib.GemmProblem * len(problems))()
    flops = nbytes = 0.0
    for i, p in enumerate(problems):
        a, w, out = p["a"], p["w"], p["out"]
        N, K = w.shape
        if a.shape[1] != K or a.dtype != w.dtype:
            raise ValueError("gemm_group: a / w shapes or dtypes differ")
        q = arr[i]
        q.A, q.lda, q.W, q.ldw = _p(a), _rowmajor(a, "a"), _p(w), _rowmajor(w, "w")
        q.out, q.ldo = _p(out), _rowmajor(out, "out")
        q.M, q.N, q.K = a.shape[0], N, K
        q.ep.bias, q.ep.gamma = _p(p.get("bias")), _p(p.get("gamma"))
        if p.get("qkv") is not None:
            _fill_qkv_epi(q.ep, p["qkv"])
        if p.get("q_scale"):
            q.ep.q_scale, q.ep.q_cols = float(p["q_scale"]), int(p["q_cols"])
        if p.get("aux") is not None:  # GELU_BWD's saved pre-activation / the forward's aux output
            aux = p["aux"]
            if aux.dtype != a.dtype:
                raise TypeError("gemm_group: aux must have the operand dtype")
            q.ep.aux, q.ep.ld_aux = _p(aux), _rowmajor(aux, "aux")
        if p.get("colsum") is not None:  # GELU_BWD's per-64-row-block column sums
            _check_colsum(p["colsum"], a.shape[0], N)
            q.ep.colsum = _p(p["colsum"])
        flops += 2.0 * a.shape[0] * N * K
        nbytes += (a.shape[0] * K + N * K) * a.element_size() + a.shape[0] * N * out.element_size()
    if tag == "gemm":
        tag = f"gemm_{_EPI_NAME.get(epi, epi)}"
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    rc = _lib.load().sr_gemm_group(_stream(problems[0]["a"]), dtype_code(torch.bfloat16), epi, len(problems), arr)
    check(rc, "sr_gemm_group")
    if timed:
        TIMER.stop(tag, ev0, flops, nbytes, kernel=last_kernel())


# fixed-offset softmax sweep (sr_attn_desc.key_bound); SR_ATTN_BOUND=0 keeps the per-tile row max
_ATTN_BOUND = os.environ.get("SR_ATTN_BOUND", "1") != "0"
# key-split attention: SR_ATTN_KSPLIT=0 disables it, =S forces S chunks where they divide the keys
_KSPLIT_ENV = os.environ.get("SR_ATTN_KSPLIT")
_KSPLIT_WGS = 2560  # 256-row workgroups a split launch should reach (10 per CU)
_KSPLIT_MIN_KEYS = 2048  # shortest key chunk (32 tiles of 64 keys per workgroup)


def key_split_parts(*, dtype: torch.dtype, batch: int, lq: int, heads: int, l0: int, l1: int, mask_mode: int) -> int:
    """Key chunks one bf16 attention launch is split into (1 = no split).  A single query set too
    short to fill the chip (the per-rank query slice of a frame-sharded global block: G=8 at C3
    leaves 43 q-tiles x 16 heads = 688 workgroups for 256 CUs) runs as S items over key chunks
    of equal length, each writing a normalised partial output and its LSE, merged by
    sr_attn_merge_n.  The fp32 accumulation inside a chunk is unchanged; the partials round to
    bf16 once before the merge."""
    if dtype != torch.bfloat16 or batch != 1 or l1 != 0 or mask_mode != _lib.SR_MASK_NONE:
        return 1
    wgs = (lq + 255) // 256 * heads
    if _KSPLIT_ENV is not None:
        s = int(_KSPLIT_ENV)
        return s if s > 1 and l0 % s == 0 else 1
    if wgs >= 2048:  # the C3 global block (2752 workgroups) runs best unsplit
        return 1
    # powers of two first: measured at C3's per-rank slices (tools/kbench.py attn_rank), S = 3 / 6
    # trail S = 2 / 4 / 8 by 3-8 %
    for cands in ((2, 4, 8), (3, 6)):
        best = 1
        for s in cands:
            if l0 % s or l0 // s < _KSPLIT_MIN_KEYS:
                continue
            best = s
            if wgs * s >= _KSPLIT_WGS:
                break
        if best > 1:
            return best
    return 1


def attention(q: Tensor, k0: Tensor, v0: Tensor, o: Tensor, *, heads: int, head_dim: int, batch: int, lq: int,
              q_bstride: int, l0: int, k0_bstride: int, k1: Optional[Tensor] = None, v1: Optional[Tensor] = None,
              l1: int = 0, k1_bstride: int = 0, mask_mode: int = _lib.SR_MASK_NONE, n_anchor: int = 0,
              scale: Optional[float] = None, tag: Optional[str] = None, lse: Optional[Tensor] = None,
              key_norm_max: float = 0.0, mask: Optional[Tensor] = None, tail_readable: bool = False,
              merge_o: Optional[Tensor] = None, merge_lse: Optional[Tensor] = None,
              sweep_stats: Optional[Tensor] = None, query_norm_max: float = 0.0, q_scaled: bool = False) -> None:
    """softmax(scale q k^T) v over segment 0 (+ segment 1) keys; see sr_attn_desc.  ``mask``
    (mask_mode SR_MASK_DENSE: bool / uint8, nonzero = attend; SR_MASK_ADD: fp32 added to the
    scores) is a [batch, heads, lq, l0 + l1] view (broadcast dims may have stride 0, the last dim
    stride 1), fp32 q / k / v only.  ``lse``
    (fp32 [batch, heads, lq]) receives the rows' log2-domain LSE for attention_bwd.
    ``key_norm_max`` > 0: a static bound of every key's per-head 2-norm (runtime.key_norm_bound),
    which replaces the key scan of the fixed-offset sweep.  ``query_norm_max`` > 0: the same bound
    for the queries (runtime.query_norm_bound); where scale*log2(e)*|q|*|k| leaves the sweep's
    window the launch first computes the per-dimension key and value boxes (sr_attention_key_box,
    sr_attn_desc.key_box / value_box; SR_ATTN_KEY_BOX=1 always, =0 never).  A bf16 single query set too short to
    fill the chip runs key-split (key_split_parts, attention_partials + attn_merge_n).
    ``tail_readable``: at least 64 rows of finite values follow every key segment in memory
    (runtime.Workspace buffers: zero-initialised, 64 rows of padding), which lets the
    hand-scheduled sweep take ragged and two-segment launches (sr_attn_desc.tail_rows_readable).
    ``merge_o`` / ``merge_lse`` (bf16 only): a row-normalised result of the same query rows over a
    DISJOINT key set ([R, >= heads*head_dim] bf16, row item*q_bstride + i) and its log2-domain LSE
    (fp32 [heads, R]); o then receives the softmax over the union (sr_attn_desc.merge_o).
    ``sweep_stats`` (int32 [2], caller-zeroed, bf16): the launch adds its waves on the
    hand-scheduled sweep / on the compiled loop (sr_attn_desc.sweep_stats); it forces one launch.
    ``q_scaled`` (bf16): q holds c*q, c = scale*log2(e), rounded once by the QKV GEMM's epilogue
    (runtime.q_prescale, sr_attn_desc.q_scaled); False: the kernel forms c*q itself."""
    parts = key_split_parts(dtype=q.dtype, batch=batch, lq=lq, heads=heads, l0=l0, l1=l1, mask_mode=mask_mode)
    if sweep_stats is not None:
        parts = 1
    if merge_o is not None:
        if q.dtype != torch.bfloat16 or merge_o.dtype != torch.bfloat16 or merge_o.stride(1) != 1 or \
                merge_lse is None or merge_lse.dtype != torch.float32 or not merge_lse.is_contiguous() or \
                merge_lse.dim() != 2 or merge_lse.shape[0] != heads or merge_o.shape[1] < heads * head_dim or \
                merge_o.shape[0] < merge_lse.shape[1] or merge_lse.shape[1] < (batch - 1) * q_bstride + lq:
            raise ValueError("attention: merge_o must be bf16 [R, heads*head_dim] rows and merge_lse fp32 "
                             "[heads, R] covering every query row")
        parts = 1
    if parts > 1:
        if lse is not None and (lse.dtype != torch.float32 or not lse.is_contiguous() or lse.numel() != heads * lq):
            raise ValueError("attention: lse must be contiguous fp32 [batch, heads, lq]")
        o_parts, lse_parts = key_split_workspace(q.device, parts, lq, heads * head_dim, heads)
        attention_partials(q, k0, v0, o_parts, lse_parts, heads=heads, head_dim=head_dim, lq=lq, l0=l0, parts=parts,
                           scale=scale, tag=tag, key_norm_max=key_norm_max, tail_readable=tail_readable,
                           query_norm_max=query_norm_max, q_scaled=q_scaled)
        attn_merge_n(o_parts, lse_parts, o, parts=parts, rows=lq, heads=heads, head_dim=head_dim, lse_out=lse)
        return
    d = _attn_desc(q, k0, v0, o, heads=heads, head_dim=head_dim, batch=batch, lq=lq, q_bstride=q_bstride, l0=l0,
                   k0_bstride=k0_bstride, k1=k1, v1=v1, l1=l1, k1_bstride=k1_bstride, mask_mode=mask_mode,
                   n_anchor=n_anchor, scale=scale, lse=lse, q_scaled=q_scaled)
    if tail_readable:
        d.tail_rows_readable = 64
    _set_sweep_stats(d, sweep_stats)
    if merge_o is not None:
        d.merge_o, d.ld_merge_o = _p(merge_o), merge_o.stride(0)
        d.merge_lse, d.merge_rows = _p(merge_lse), merge_lse.shape[1]
    if mask_mode in (_lib.SR_MASK_DENSE, _lib.SR_MASK_ADD):
        want = torch.float32 if mask_mode == _lib.SR_MASK_ADD else (torch.bool, torch.uint8)
        if mask is None or mask.dim() != 4 or tuple(mask.shape) != (batch, heads, lq, l0 + l1) or \
                mask.device != q.device or (mask.dtype != want if mask_mode == _lib.SR_MASK_ADD else
                                            mask.dtype not in want) or mask.stride(3) != 1:
            raise ValueError(f"attention: mask must be a [{batch}, {heads}, {lq}, {l0 + l1}] "
                             f"{'fp32' if mask_mode == _lib.SR_MASK_ADD else 'bool'} view with unit key stride "
                             f"on {q.device}")
        if q.dtype != torch.float32:
            raise ValueError("attention: dense / additive masks run on the fp32 kernel")
        d.mask = _p(mask)
        d.mask_bstride, d.mask_hstride, d.mask_ld = mask.stride(0), mask.stride(1), mask.stride(2)
    _launch_attention(d, q, tag, key_norm_max, 4.0 * batch * heads * lq * (l0 + l1) * head_dim,
                      q.element_size() * heads * head_dim *
                      (2 * batch * lq + 2 * ((l0 if k0_bstride == 0 else batch * l0) + batch * l1)),
                      query_norm_max=query_norm_max)


def _set_sweep_stats(d: AttnDesc, stats: Optional[Tensor]) -> None:
    if stats is None:
        return
    if stats.dtype != torch.int32 or stats.numel() < 2 or not stats.is_cuda or not stats.is_contiguous():
        raise ValueError("sweep_stats must be a contiguous int32 device tensor of >= 2 elements")
    d.sweep_stats = _p(stats)


def pair_eligible(dtype: torch.dtype, l0: int, head_dim: int, key_norm_max: float) -> bool:
    """Whether a single-query-set attention may go into attention_pair (sr_attention_pair's
    conditions: bf16, head_dim 64, whole 64-key tiles (>= 4), a static key bound; SR_ATTN_PAIR=0
    turns pairing off)."""
    return (_ATTN_PAIR and dtype == torch.bfloat16 and head_dim == 64 and l0 >= 256 and l0 % 64 == 0 and
            key_norm_max > 0.0 and _ATTN_BOUND)


_ATTN_PAIR = os.environ.get("SR_ATTN_PAIR", "1") != "0"


def attention_pair(a: dict, b: dict, *, heads: int, head_dim: int, tag: Optional[str] = None) -> None:
    """Two single-query-set bf16 attentions in ONE launch (sr_attention_pair): ``a`` / ``b`` are
    dicts with q, k0, v0, o, lq, l0, key_norm_max and optionally lse, query_norm_max, q_scaled (keys
    as attention()'s, batch 1, one segment) and vt (v0 as vt_tiles(); both or neither:
    sr_attention_pair_vt, bit-identical).
    a's workgroups run first and b's fill the CUs a's last round leaves idle.  Both must pass
    pair_eligible (checked)."""
    descs = []
    flops = nbytes = 0.0
    for p in (a, b):
        if not pair_eligible(p["q"].dtype, p["l0"], head_dim, p["key_norm_max"]):
            raise ValueError("attention_pair: a problem does not qualify (see pair_eligible)")
        d = _attn_desc(p["q"], p["k0"], p["v0"], p["o"], heads=heads, head_dim=head_dim, batch=1, lq=p["lq"],
                       q_bstride=0, l0=p["l0"], k0_bstride=0, lse=p.get("lse"), q_scaled=p.get("q_scaled", False))
        d.key_norm_max = float(p["key_norm_max"])
        _set_sweep_stats(d, p.get("sweep_stats"))
        _attach_key_box(d, p["k0"].device, p.get("query_norm_max", 0.0), "attn_key_box" + str(len(descs)))
        descs.append(d)
        flops += 4.0 * heads * p["lq"] * p["l0"] * head_dim
        nbytes += p["q"].element_size() * heads * head_dim * (2 * p["lq"] + 2 * p["l0"])
    vts = [p.get("vt") for p in (a, b)]
    if (vts[0] is None) != (vts[1] is None):
        raise ValueError("attention_pair: V^T tiles for both problems or for neither")
    for p, vt in zip((a, b), vts):
        if vt is not None:
            _check_vt_tiles(vt, p["l0"], heads)
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    lib = _lib.load()
    if vts[0] is not None:
        rc = lib.sr_attention_pair_vt(_stream(a["q"]), dtype_code(a["q"].dtype), ctypes.byref(descs[0]),
                                      ctypes.byref(descs[1]), _p(vts[0]), _p(vts[1]))
    else:
        rc = lib.sr_attention_pair(_stream(a["q"]), dtype_code(a["q"].dtype), ctypes.byref(descs[0]),
                                   ctypes.byref(descs[1]))
    check(rc, "sr_attention_pair")
    if timed:
        TIMER.stop(tag, ev0, flops, nbytes, kernel=last_kernel())


# SR_ATTN_PAIR_VT=1: the forward's pair launch reads pre-transposed V^T tiles (sr_vt_tiles +
# sr_attention_pair_vt) instead of V with transposing LDS reads.  Bit-identical; measured level, off:
# the launch gains 18-21 us of 7.88 ms, the two sr_vt_tiles cost 38 us (profiles/r06_j5_kpair_vt.log)
PAIR_VT = os.environ.get("SR_ATTN_PAIR_VT", "0") == "1"


def vt_tile_shape(L: int, heads: int) -> tuple:
    """(rows, 64) of the bf16 V^T tile buffer sr_vt_tiles fills for L keys."""
    return (heads * ((L + 63) // 64) * 64, 64)


def _check_vt_tiles(vt: torch.Tensor, L: int, heads: int) -> None:
    if vt.dtype != torch.bfloat16 or not vt.is_contiguous() or vt.numel() < heads * ((L + 63) // 64) * 4096 \
            or vt.data_ptr() % 16:
        raise ValueError("V^T tiles: contiguous bf16, 16-B aligned, heads * ceil(L / 64) * 4096 elements")


def vt_tiles(v: torch.Tensor, L: int, heads: int, out: torch.Tensor, tag: Optional[str] = None) -> torch.Tensor:
    """V (bf16 [L][heads * 64], row stride v.stride(0)) -> V^T tiles (sr_vt_tiles) for attention_pair's
    ``vt``: [heads][ceil(L/64)][64 d][64 key slots], the bf16 P fragment's key order."""
    if v.dtype != torch.bfloat16 or v.stride(1) != 1 or v.shape[0] < L or v.shape[1] < heads * 64:
        raise ValueError("vt_tiles: v must be bf16 [L][>= heads * 64] with unit column stride")
    _check_vt_tiles(out, L, heads)
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    check(_lib.load().sr_vt_tiles(_stream(v), _p(v), v.stride(0), L, heads, _p(out)), "sr_vt_tiles")
    if timed:
        TIMER.stop(tag, ev0, 0.0, 4.0 * L * heads * 64, kernel=last_kernel())
    return out


_KEY_BOX = os.environ.get("SR_ATTN_KEY_BOX", "auto")  # auto | 1 (always) | 0 (never)
# sr_attn.hip's default window: P <= 2^FIX_HI, the row's max P >= 2^-FIX_LO.  With every score in
# [-qs, qs] and qs <= (FIX_HI + FIX_LO) / 2 = 87 the offset m = max(0, qs - FIX_HI) always fits it
# (the row max >= -qs >= m - FIX_LO), so the boxes only pay above that
_BOX_MIN_BOUND = (64.0 + 110.0) / 2


def _attach_key_box(d: AttnDesc, device, query_norm_max: float, name: str) -> None:
    """Set d.key_box, d.value_box and d.key_norm2 (the keys' actual max |k|^2, which tightens the
    static key_norm_max) when the 2-norm score bound scale*log2(e)*|q|*|k| exceeds 87, above which the
    default window can miss: sr_attention_key_box over each key and value segment into a
    per-stream workspace, instances as sr_attention_bound_floats' (k0's, then k1's)."""
    if _KEY_BOX == "0" or not (d.key_norm_max > 0.0) or d.head_dim != 64 or d.heads > 32:
        return
    if _KEY_BOX != "1" and not (query_norm_max > 0.0 and
                                d.scale * 1.4426950408889634 * query_norm_max * d.key_norm_max > _BOX_MIN_BOUND):
        return
    n0 = 1 if d.k0_bstride == 0 else d.batch
    n1 = (1 if d.k1_bstride == 0 else d.batch) if d.l1 > 0 else 0
    per = d.heads * 128
    ws = _train_ws(device, name, (2 * per + d.heads) * (n0 + n1))
    lib = _lib.load()
    stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    segs = [(d.k0, d.ldk0, d.v0, d.ldv0, d.l0, d.k0_bstride, n0, 0)]
    if n1:
        segs.append((d.k1, d.ldk1, d.v1, d.ldv1, d.l1, d.k1_bstride, n1, n0 * per))
    vb, nb = (n0 + n1) * per, 2 * (n0 + n1) * per
    sc = _train_ws(device, "attn_box_scratch",
                   max(lib.sr_attention_key_box_scratch(g[4], g[6], d.heads) for g in segs))
    for k, ldk, v, ldv, rows, bstride, n, off in segs:
        check(lib.sr_attention_key_box(stream, k, ldk, rows, bstride, n, d.heads, _p(ws[off:]),
                                       _p(ws[nb + off // 128:]), _p(sc)), "sr_attention_key_box")
        check(lib.sr_attention_key_box(stream, v, ldv, rows, bstride, n, d.heads, _p(ws[vb + off:]), None, _p(sc)),
              "sr_attention_key_box(values)")
    d.key_box, d.value_box, d.key_norm2 = _p(ws), _p(ws[vb:]), _p(ws[nb:])


def _attach_scan_boxes(d: AttnDesc, device) -> None:
    """Key-scan launches (no static key bound: the training forward, whose weights move every
    step) of one long query set -- the hand-scheduled sweep's launches: the key and value boxes as
    well (sr_attn_desc.key_box / value_box; the launch scans max |k| itself).  There is no static
    |q| |k| to decide by, and the two passes cost ~1 % of such a launch, so they always run
    (SR_ATTN_KEY_BOX=0: never)."""
    if _KEY_BOX == "0" or d.head_dim != 64 or d.heads > 32 or not (d.batch == 1 or d.q_bstride == 0) or \
            d.lq < 4096 or d.mask_mode != _lib.SR_MASK_NONE:
        return
    n0 = 1 if d.k0_bstride == 0 else d.batch
    n1 = (1 if d.k1_bstride == 0 else d.batch) if d.l1 > 0 else 0
    per = d.heads * 128
    ws = _train_ws(device, "attn_scan_box", 2 * (n0 + n1) * per)
    lib = _lib.load()
    stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    segs = [(d.k0, d.ldk0, d.v0, d.ldv0, d.l0, d.k0_bstride, n0, 0)]
    if n1:
        segs.append((d.k1, d.ldk1, d.v1, d.ldv1, d.l1, d.k1_bstride, n1, n0 * per))
    vb = (n0 + n1) * per
    sc = _train_ws(device, "attn_box_scratch", max(lib.sr_attention_key_box_scratch(g[4], g[6], d.heads) for g in segs))
    for k, ldk, v, ldv, rows, bstride, n, off in segs:
        check(lib.sr_attention_key_box(stream, k, ldk, rows, bstride, n, d.heads, _p(ws[off:]), None, _p(sc)),
              "sr_attention_key_box")
        check(lib.sr_attention_key_box(stream, v, ldv, rows, bstride, n, d.heads, _p(ws[vb + off:]), None, _p(sc)),
              "sr_attention_key_box(values)")
    d.key_box, d.value_box = _p(ws), _p(ws[vb:])


def _launch_attention(d: AttnDesc, q: Tensor, tag: Optional[str], key_norm_max: float, flops: float,
                      nbytes: float, query_norm_max: float = 0.0) -> None:
    if q.dtype == torch.bfloat16 and _ATTN_BOUND and key_norm_max > 0.0:
        d.key_norm_max = float(key_norm_max)
        _attach_key_box(d, q.device, query_norm_max, "attn_key_box")
    elif q.dtype == torch.bfloat16 and _ATTN_BOUND:
        nb = _lib.load().sr_attention_bound_floats(ctypes.byref(d))
        if nb > 0:
            d.key_bound = _p(_train_ws(q.device, "attn_key_bound", nb))
            _attach_scan_boxes(d, q.device)
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    rc = _lib.load().sr_attention(_stream(q), dtype_code(q.dtype), ctypes.byref(d))
    check(rc, "sr_attention")
    if timed:
        TIMER.stop(tag, ev0, flops, nbytes, kernel=last_kernel())


def key_split_workspace(device, parts: int, rows: int, cols: int, heads: int, name: str = "attn_ksplit"):
    """(o_parts bf16 [parts*rows, cols], lse_parts fp32 [parts, heads, rows]) in one reusable
    per-stream workspace."""
    n_o = (parts * rows * cols + 1) // 2  # bf16 pairs
    ws = _train_ws(device, name, n_o + parts * heads * rows)
    o_parts = ws[:n_o].view(torch.bfloat16)[:parts * rows * cols].view(parts * rows, cols)
    return o_parts, ws[n_o:n_o + parts * heads * rows].view(parts, heads, rows)


def attention_partials(q: Tensor, k0: Tensor, v0: Tensor, o_parts: Tensor, lse_parts: Tensor, *, heads: int,
                       head_dim: int, lq: int, l0: int, parts: int, scale: Optional[float] = None,
                       tag: Optional[str] = None, key_norm_max: float = 0.0, tail_readable: bool = False,
                       query_norm_max: float = 0.0, q_scaled: bool = False) -> None:
    """One bf16 launch of ``parts`` items over equal key chunks of k0/v0 (item s: keys
    [s*l0/parts, (s+1)*l0/parts)) against the same lq queries: item s writes its normalised
    partial output at rows s*lq of o_parts and its LSE to lse_parts[s] ([heads, lq]).  The parts
    of one or more such launches (stacked in one buffer) merge with attn_merge_n."""
    if l0 % parts:
        raise ValueError(f"attention_partials: {parts} parts do not divide {l0} keys")
    if o_parts.shape[0] < parts * lq or lse_parts.dtype != torch.float32 or not lse_parts.is_contiguous() or \
            lse_parts.numel() != parts * heads * lq:
        raise ValueError("attention_partials: o_parts [parts*lq, C] / lse_parts fp32 [parts, heads, lq]")
    chunk = l0 // parts
    d = _attn_desc(q, k0, v0, o_parts, heads=heads, head_dim=head_dim, batch=parts, lq=lq, q_bstride=0, l0=chunk,
                   k0_bstride=chunk, scale=scale, lse=lse_parts, q_scaled=q_scaled)
    d.o_bstride = lq
    if tail_readable:  # rows past k0/v0's end readable: each chunk's ragged tile may go to the asm sweep
        d.tail_rows_readable = 64
    _launch_attention(d, q, tag, key_norm_max, 4.0 * heads * lq * l0 * head_dim,
                      q.element_size() * heads * head_dim * (lq + 2 * parts * lq + 2 * l0),
                      query_norm_max=query_norm_max)


def attn_merge(o_a: Tensor, lse_a: Tensor, o_b: Tensor, lse_b: Tensor, out: Tensor, *, heads: int, head_dim: int,
               lse_out: Optional[Tensor] = None, tag: Optional[str] = None) -> None:
    """Softmax over the union of two disjoint key sets from the two passes' outputs (o [rows, C])
    and log2-domain LSEs (fp32 [heads, rows]); see sr_attn_merge.  out may alias o_a / o_b."""
    rows = out.shape[0]
    for t in (o_a, o_b):
        if t.dtype != out.dtype or t.shape[0] != rows:
            raise ValueError("attn_merge: o_a / o_b / out must share dtype and rows")
    for t in (lse_a, lse_b) + (() if lse_out is None else (lse_out,)):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != heads * rows:
            raise ValueError("attn_merge: lse must be contiguous fp32 [heads, rows]")
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    rc = _lib.load().sr_attn_merge(_stream(out), dtype_code(out.dtype), rows, heads, head_dim, _p(o_a),
                                   _rowmajor(o_a, "o_a"), _p(lse_a), _p(o_b), _rowmajor(o_b, "o_b"), _p(lse_b), _p(out),
                                   _rowmajor(out, "out"), _p(lse_out))
    check(rc, "sr_attn_merge")
    if timed:
        TIMER.stop(tag, ev0, 0.0, out.element_size() * rows * heads * head_dim * 3 + 12 * rows * heads)


def attn_merge_n(o_parts: Tensor, lse_parts: Tensor, out: Tensor, *, parts: int, rows: int, heads: int,
                 head_dim: int, lse_out: Optional[Tensor] = None, seg_rows=None) -> None:
    """attn_merge over ``parts`` partial results stacked in o_parts ([parts * rows, C], part p at
    rows p*rows) with LSEs lse_parts (fp32, heads*rows per part); ``seg_rows[p]`` = the rows of
    one LSE block of part p ([rows/g][heads][g]; default g = rows); see sr_attn_merge_n."""
    if o_parts.dtype != out.dtype or o_parts.shape[0] < parts * rows or out.shape[0] < rows:
        raise ValueError("attn_merge_n: o_parts must hold parts*rows rows of out's dtype")
    if lse_parts.dtype != torch.float32 or not lse_parts.is_contiguous() or lse_parts.numel() < parts * heads * rows:
        raise ValueError("attn_merge_n: lse_parts must be contiguous fp32 [parts, heads, rows]")
    if lse_out is not None and (lse_out.dtype != torch.float32 or not lse_out.is_contiguous()
                                or lse_out.numel() != heads * rows):
        raise ValueError("attn_merge_n: lse_out must be contiguous fp32 [heads, rows]")
    if parts > _lib.SR_ATTN_MERGE_MAX_PARTS:
        raise ValueError(f"attn_merge_n: at most {_lib.SR_ATTN_MERGE_MAX_PARTS} parts")
    sg = None
    if seg_rows is not None:
        if len(seg_rows) != parts:
            raise ValueError("attn_merge_n: one seg_rows entry per part")
        sg = (ctypes.c_int * parts)(*seg_rows)
    rc = _lib.load().sr_attn_merge_n(_stream(out), dtype_code(out.dtype), parts, rows, heads, head_dim, _p(o_parts),
                                     _rowmajor(o_parts, "o_parts"), rows, _p(lse_parts), sg, _p(out),
                                     _rowmajor(out, "out"), _p(lse_out))
    check(rc, "sr_attn_merge_n")


def quant_fp8(src: Tensor, mul: float, dst: Optional[Tensor] = None, exp_out: Optional[Tensor] = None):
    """e4m3 copy of ``mul * src`` (bf16 [rows, cols]) with one power-of-two scale (sr_quant_fp8):
    returns (dst uint8 [rows, cols], exp int32 device scalar) with mul * src ~= dst * 2^exp."""
    if src.dtype != torch.bfloat16 or src.dim() != 2:
        raise ValueError("quant_fp8: src must be 2-D bf16")
    rows, cols = src.shape
    if dst is None:
        dst = torch.empty(rows, cols, device=src.device, dtype=torch.uint8)
    if exp_out is None:
        exp_out = torch.empty(1, device=src.device, dtype=torch.int32)
    ws = _train_ws(src.device, "fp8_amax", 1)
    rc = _lib.load().sr_quant_fp8(_stream(src), _p(src), _rowmajor(src, "src"), rows, cols, float(mul), _p(dst),
                                  _rowmajor(dst, "dst"), _p(ws), _p(exp_out))
    check(rc, "sr_quant_fp8")
    return dst, exp_out


class Fp8Workspace:
    """Reusable fp8 buffers of one attention shape (q8, k8, the V8T tiles and the exponents)."""

    def __init__(self):
        self.bufs = {}

    def get(self, rows_q: int, rows_k: int, cols: int, device) -> tuple:
        key = (rows_q, rows_k, cols, str(device))
        if key not in self.bufs:
            self.bufs.clear()
            ntiles = (rows_k + 63) // 64
            self.bufs[key] = (torch.empty(rows_q, cols, device=device, dtype=torch.uint8),
                              torch.empty(rows_k, cols, device=device, dtype=torch.uint8),
                              torch.empty(3, device=device, dtype=torch.int32),
                              torch.empty(cols // 64 * ntiles * 4096, device=device, dtype=torch.uint8))
        return self.bufs[key][:3]

    def v8t(self):
        return next(iter(self.bufs.values()))[3]


def quant_fp8_vt(v: Tensor, heads: int, dst: Tensor, exp_out: Tensor) -> None:
    """V (bf16 [L, heads*64]) -> e4m3 tiles in the accumulator key order of the fp8 P.V
    (sr_quant_fp8_vt), exponent into exp_out."""
    ws = _train_ws(v.device, "fp8_amax", 1)
    rc = _lib.load().sr_quant_fp8_vt(_stream(v), _p(v), _rowmajor(v, "v"), v.shape[0], heads, _p(dst), _p(ws),
                                     _p(exp_out))
    check(rc, "sr_quant_fp8_vt")


def attention_qk8(q: Tensor, k0: Tensor, v0: Tensor, o: Tensor, *, heads: int, batch: int, lq: int, q_bstride: int,
                  l0: int, k0_bstride: int, scale: Optional[float] = None, tag: Optional[str] = None,
                  lse: Optional[Tensor] = None, ws: Optional[Fp8Workspace] = None, fp8_v: bool = False,
                  key_norm_max: float = 0.0, q_scaled: bool = False) -> None:
    """attention() with q.k^T in block-scaled fp8 (BASELINE C5): q and k (bf16, head_dim 64) are
    quantised to e4m3 with one power-of-two scale each (q with scale*log2(e) folded in); V / P.V
    stay bf16 unless ``fp8_v`` (then V is quantised too and P enters the MFMA as e4m3).  One key
    segment, no mask.  ``q_scaled``: q already holds c*q (see attention), so it is quantised as is."""
    head_dim = 64
    d = _attn_desc(q, k0, v0, o, heads=heads, head_dim=head_dim, batch=batch, lq=lq, q_bstride=q_bstride, l0=l0,
                   k0_bstride=k0_bstride, scale=scale, lse=lse)
    if _ATTN_BOUND and key_norm_max > 0.0:  # fixed-offset sweep (q.k^T-only mode; see sr_attn_desc)
        d.key_norm_max = float(key_norm_max)
    C = heads * head_dim
    ws = ws or Fp8Workspace()
    q8, k8, ex = ws.get(q.shape[0], k0.shape[0], C, q.device)
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    quant_fp8(q[:, :C], 1.0 if q_scaled else d.scale * 1.4426950408889634, q8, ex[0:1])
    quant_fp8(k0[:, :C], 1.0, k8, ex[1:2])
    if fp8_v:
        if batch != 1:
            raise ValueError("attention_qk8(fp8_v=True): one item (the global block) only")
        v8t = ws.v8t()
        quant_fp8_vt(v0[:, :C], heads, v8t, ex[2:3])
        rc = _lib.load().sr_attention_qkv8(_stream(q), ctypes.byref(d), _p(q8), C, _p(k8), C, _p(v8t), _p(ex))
        check(rc, "sr_attention_qkv8")
    else:
        rc = _lib.load().sr_attention_qk8(_stream(q), ctypes.byref(d), _p(q8), C, _p(k8), C, _p(ex))
        check(rc, "sr_attention_qk8")
    if timed:
        kv_rows = l0 if k0_bstride == 0 else batch * l0
        nb = heads * head_dim * (2 * batch * lq + kv_rows) + 2 * heads * head_dim * (batch * lq + kv_rows)
        TIMER.stop(tag, ev0, 4.0 * batch * heads * lq * l0 * head_dim, nb, kernel=last_kernel())


def _attn_desc(q, k0, v0, o, *, heads, head_dim, batch, lq, q_bstride, l0, k0_bstride, k1=None, v1=None, l1=0,
               k1_bstride=0, mask_mode=_lib.SR_MASK_NONE, n_anchor=0, scale=None, lse=None,
               q_scaled=False) -> AttnDesc:
    d = AttnDesc()
    d.q, d.ldq = _p(q), _rowmajor(q, "q")
    d.k0, d.ldk0 = _p(k0), _rowmajor(k0, "k0")
    d.v0, d.ldv0 = _p(v0), _rowmajor(v0, "v0")
    if l1 > 0:
        d.k1, d.ldk1 = _p(k1), _rowmajor(k1, "k1")
        d.v1, d.ldv1 = _p(v1), _rowmajor(v1, "v1")
    d.o, d.ldo = _p(o), _rowmajor(o, "o")
    d.batch, d.heads, d.head_dim = batch, heads, head_dim
    d.lq, d.q_bstride = lq, q_bstride
    d.l0, d.k0_bstride = l0, k0_bstride
    d.l1, d.k1_bstride = l1, k1_bstride
    d.mask_mode, d.n_anchor = mask_mode, n_anchor
    d.scale = head_dim ** -0.5 if scale is None else scale
    if q_scaled:
        if q.dtype != torch.bfloat16:
            raise ValueError("attention: q_scaled is a bf16-path convention")
        d.q_scaled = 1
    if lse is not None:
        if lse.dtype != torch.float32 or not lse.is_contiguous() or lse.numel() != batch * heads * lq:
            raise ValueError("attention: lse must be contiguous fp32 [batch, heads, lq]")
        d.lse = _p(lse)
    return d


def attention_bwd(q: Tensor, k0: Tensor, v0: Tensor, o: Tensor, lse: Tensor, dout: Tensor, dq: Tensor, dk0: Tensor,
                  dv0: Tensor, delta: Tensor, *, heads: int, batch: int, lq: int, q_bstride: int, l0: int,
                  k0_bstride: int, k1: Optional[Tensor] = None, v1: Optional[Tensor] = None,
                  dk1: Optional[Tensor] = None, dv1: Optional[Tensor] = None, l1: int = 0, k1_bstride: int = 0,
                  scale: Optional[float] = None, tag: Optional[str] = None) -> None:
    """Gradient of attention(): dq / dk* / dv* fp32 in q's / k's / v's layouts; ``delta`` fp32
    [batch, heads, lq] workspace.  bf16 operands (head_dim 64): sr_attention_bwd; fp32 operands
    (TrainGraph's fp32 mode, head_dim 64 | 128): the exact sr_attention_bwd_f32."""
    f32 = q.dtype == torch.float32
    for t, name in ((k0, "k0"), (v0, "v0"), (o, "o"), (dout, "dout")) + (((k1, "k1"), (v1, "v1")) if l1 > 0 else ()):
        if t.dtype != q.dtype:
            raise TypeError(f"attention_bwd: {name} must have q's dtype {q.dtype}")
    head_dim = q.shape[1] // heads if f32 else 64
    b = _lib.AttnBwdDesc()
    b.f = _attn_desc(q, k0, v0, o, heads=heads, head_dim=head_dim, batch=batch, lq=lq, q_bstride=q_bstride, l0=l0,
                     k0_bstride=k0_bstride, k1=k1, v1=v1, l1=l1, k1_bstride=k1_bstride, scale=scale, lse=lse)
    for t, name in ((dq, "dq"), (dk0, "dk0"), (dv0, "dv0"), (delta, "delta")) + \
            (((dk1, "dk1"), (dv1, "dv1")) if l1 > 0 else ()):
        if t is None or t.dtype != torch.float32 or not t.is_cuda:
            raise ValueError(f"attention_bwd: {name} must be an fp32 device tensor")
    if delta.numel() < batch * heads * lq:
        raise ValueError("attention_bwd: delta too small")
    b.dout, b.lddo = _p(dout), _rowmajor(dout, "dout")
    b.delta = _p(delta)
    b.dq, b.lddq = _p(dq), _rowmajor(dq, "dq")
    b.dk0, b.lddk0 = _p(dk0), _rowmajor(dk0, "dk0")
    b.dv0, b.lddv0 = _p(dv0), _rowmajor(dv0, "dv0")
    if l1 > 0:
        b.dk1, b.lddk1 = _p(dk1), _rowmajor(dk1, "dk1")
        b.dv1, b.lddv1 = _p(dv1), _rowmajor(dv1, "dv1")
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    fn = "sr_attention_bwd_f32" if f32 else "sr_attention_bwd"
    check(getattr(_lib.load(), fn)(_stream(q), ctypes.byref(b)), fn)
    if timed:
        kv = (l0 if k0_bstride == 0 else batch * l0) + batch * l1
        TIMER.stop(tag, ev0, 10.0 * batch * heads * lq * (l0 + l1) * 64, 2 * heads * 64 * (4 * batch * lq + 4 * kv))


def layernorm(x: Tensor, w: Optional[Tensor], b: Optional[Tensor], eps: float, out: Tensor,
              rowmap: Optional[Tensor] = None, rows: Optional[int] = None, x_copy: Optional[Tensor] = None) -> None:
    """out = LayerNorm(x rows) (sr_layernorm); ``x_copy`` (fp32, no rowmap): also the input rows
    copied there in the same pass (sr_layernorm_copy)."""
    ldx = _rowmajor(x, "x")
    ldo = _rowmajor(out, "out")
    if x.dtype != torch.float32:
        raise TypeError("layernorm input must be fp32")
    n = out.shape[0] if rows is None else rows
    if x_copy is not None:
        if rowmap is not None or x_copy.dtype != torch.float32 or x_copy.shape[0] < n or x_copy.shape[1] != x.shape[1]:
            raise ValueError("layernorm: x_copy must be fp32 [>= rows, cols] and takes no rowmap")
        rc = _lib.load().sr_layernorm_copy(_stream(x), dtype_code(out.dtype), _p(x), ldx, _p(w), _p(b), eps, _p(out),
                                           ldo, _p(x_copy), _rowmajor(x_copy, "x_copy"), n, x.shape[1])
        check(rc, "sr_layernorm_copy")
        return
    rc = _lib.load().sr_layernorm(_stream(x), dtype_code(out.dtype), _p(x), ldx, _p(rowmap), _p(w), _p(b),
                                  eps, _p(out), ldo, n, x.shape[1])
    check(rc, "sr_layernorm")


RESIDUAL_LN_COLS = (256, 512, 768, 1024, 1536, 2048)


def residual_layernorm(x: Tensor, y: Tensor, gamma: Optional[Tensor], w: Optional[Tensor], b: Optional[Tensor],
                       eps: float, out: Tensor) -> None:
    """x += gamma * y (fp32 x in place; y in the compute dtype), then out = LayerNorm(x) (block.py:86-89:
    the attention branch's residual update followed by norm2); see sr_residual_layernorm."""
    if x.dtype != torch.float32 or y.dtype != out.dtype or x.shape != y.shape or x.shape != out.shape:
        raise ValueError("residual_layernorm: x fp32 [rows, cols]; y and out [rows, cols] of one dtype")
    if x.shape[1] not in RESIDUAL_LN_COLS:
        raise ValueError(f"residual_layernorm: cols must be one of {RESIDUAL_LN_COLS}")
    rc = _lib.load().sr_residual_layernorm(_stream(x), dtype_code(out.dtype), _p(x), _rowmajor(x, "x"), _p(y),
                                           _rowmajor(y, "y"), _p(gamma), _p(w), _p(b), eps, _p(out),
                                           _rowmajor(out, "out"), x.shape[0], x.shape[1])
    check(rc, "sr_residual_layernorm")


_MEAN = (0.485, 0.456, 0.406)  # aggregator.py:31-32
_STD = (0.229, 0.224, 0.225)


def im2col_normalize(img: Tensor, patch: int, out: Tensor, kpad: int, normalize: bool = True) -> None:
    """out[f*gh*gw + p][k] = patch p's pixel k of frame f ((x - mean) / std when ``normalize``,
    aggregator.py:267; raw for a standalone PatchEmbed, patch_embed.py:78), K zero-padded."""
    if not img.is_contiguous() or img.dtype != torch.float32:
        raise ValueError("im2col: images must be contiguous fp32 [F,3,H,W]")
    F_, C_, H, W = img.shape
    mean = (ctypes.c_float * 3)(*(_MEAN if normalize else (0.0, 0.0, 0.0)))
    std = (ctypes.c_float * 3)(*(_STD if normalize else (1.0, 1.0, 1.0)))
    rc = _lib.load().sr_im2col_normalize(_stream(img), dtype_code(out.dtype), _p(img), F_, H, W, patch, mean, std,
                                         _p(out), kpad)
    check(rc, "sr_im2col_normalize")


def set_special_tokens(x: Tensor, frames: int, tokens_per_frame: int, table: Tensor, type_of_frame: Tensor) -> None:
    n_types, n_special, cols = table.shape
    rc = _lib.load().sr_set_special_tokens(_stream(x), _p(x), _rowmajor(x, "x"), frames, tokens_per_frame, n_special,
                                           _p(table), _p(type_of_frame), cols)
    check(rc, "sr_set_special_tokens")


def mul_cols(x: Tensor, gamma: Tensor, out: Tensor) -> None:
    """out = x * gamma (per column), x / out 2-D of one dtype, gamma fp32 [cols]."""
    if x.shape != out.shape or x.dtype != out.dtype or gamma.dtype != torch.float32 or gamma.numel() != x.shape[1]:
        raise ValueError("mul_cols: x / out [rows, cols] of one dtype, gamma fp32 [cols]")
    check(_lib.load().sr_mul_cols(_stream(x), dtype_code(x.dtype), _p(x), _rowmajor(x, "x"), _p(gamma), _p(out),
                                  _rowmajor(out, "out"), x.shape[0], x.shape[1]), "sr_mul_cols")


def copy_rows(dst: Tensor, src: Tensor, rows: int, rowmap: Optional[Tensor] = None) -> None:
    if dst.dtype != torch.float32 or src.dtype != torch.float32 or src.shape[-1] < dst.shape[1]:
        raise ValueError("copy_rows: fp32 rows, src at least as wide as dst")
    rc = _lib.load().sr_copy_rows_f32(_stream(dst), _p(dst), _rowmajor(dst, "dst"), _p(src), _rowmajor(src, "src"),
                                      _p(rowmap), rows, dst.shape[1])
    check(rc, "sr_copy_rows_f32")


def linear_small(a: Tensor, w: Tensor, bias: Optional[Tensor], out: Tensor, rows: int, act_in: int = 0,
                 lda: Optional[int] = None) -> None:
    N, K = w.shape
    lda = a.stride(0) if lda is None else lda
    rc = _lib.load().sr_linear_small_f32(_stream(out), _p(a), lda, _p(w), _p(bias), _p(out),
                                         _rowmajor(out, "out"), rows, N, K, act_in)
    check(rc, "sr_linear_small_f32")


def silu(x: Tensor, y: Tensor) -> None:
    check(_lib.load().sr_silu_f32(_stream(x), _p(x), _p(y), x.numel()), "sr_silu_f32")


def adaln_modulate(xn: Tensor, x: Tensor, mod: Tensor, out: Tensor) -> None:
    rows, cols = x.shape
    check(_lib.load().sr_adaln_modulate_f32(_stream(x), _p(xn), _p(x), _p(mod), _p(out), rows, cols),
          "sr_adaln_modulate_f32")


def pose_update(pred: Tensor, delta: Tensor, act: Tensor, first: bool) -> None:
    check(_lib.load().sr_pose_update_f32(_stream(pred), _p(pred), _p(delta), delta.stride(0), _p(act),
                                         pred.shape[0], int(first)), "sr_pose_update_f32")


def pose_decode(enc: Tensor, hw, ext: Tensor, intr: Tensor) -> None:
    H, W = hw
    check(_lib.load().sr_pose_decode_f32(_stream(enc), _p(enc), enc.stride(0), enc.shape[0], int(H), int(W),
                                         _p(ext), _p(intr)), "sr_pose_decode_f32")


# ---------------------------------------------------------------- DPT heads (NHWC fp32)
def _nhwc(x: Tensor, name: str):
    if x.dim() != 4 or not x.is_contiguous() or x.dtype != torch.float32 or not x.is_cuda:
        raise ValueError(f"{name} must be a contiguous fp32 NHWC device tensor, got {tuple(x.shape)} {x.dtype}")
    return x.shape


def im2col3x3(x: Tensor, stride: int, relu_in: bool, out: Tensor) -> None:
    """out[n*ho*wo, 9c] = im2col of a 3x3 / pad 1 conv (K order ky, kx, ci); ReLU on the input."""
    n, h, w, c = _nhwc(x, "im2col3x3 x")
    ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
    if not out.is_contiguous() or out.numel() < n * ho * wo * 9 * c:
        raise ValueError("im2col3x3: output buffer too small / not contiguous")
    check(_lib.load().sr_im2col3x3_f32(_stream(x), _p(x), n, h, w, c, stride, int(relu_in), _p(out)),
          "sr_im2col3x3_f32")


_ZERO128 = {}


def conv3x3(x: Tensor, w: Tensor, out: Tensor, *, stride: int = 1, relu_in: bool = False,
            bias: Optional[Tensor] = None, resid_gamma: Optional[Tensor] = None, tag: Optional[str] = None) -> None:
    """Implicit-GEMM 3x3 / pad 1 conv of NHWC fp32 x [n,h,w,c] with w [cout, 9c] (K order ky, kx,
    ci) into out [n,ho,wo,cout] (sr_conv3x3_f32): out = conv + bias, or out += gamma * (conv +
    bias) when ``resid_gamma`` is given."""
    n, h, wd, c = _nhwc(x, "conv3x3 x")
    cout = w.shape[0]
    ho, wo = (h - 1) // stride + 1, (wd - 1) // stride + 1
    if w.dtype != torch.float32 or not w.is_contiguous() or w.shape[1] != 9 * c:
        raise ValueError("conv3x3: w must be contiguous fp32 [cout, 9*c]")
    if out.dtype != torch.float32 or not out.is_contiguous() or tuple(out.shape) != (n, ho, wo, cout):
        raise ValueError(f"conv3x3: out must be contiguous fp32 [{n}, {ho}, {wo}, {cout}]")
    z = _ZERO128.get(x.device)
    if z is None:
        z = _ZERO128[x.device] = torch.zeros(32, device=x.device, dtype=torch.float32)
    ep = GemmEpi()
    ep.bias = _p(bias)
    ep.gamma = _p(resid_gamma)
    epi = _lib.SR_EPI_BIAS if resid_gamma is None else _lib.SR_EPI_BIAS_RESID
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    check(_lib.load().sr_conv3x3_f32(_stream(x), _p(x), n, h, wd, c, stride, int(relu_in), _p(w), cout, epi,
                                     ctypes.byref(ep), _p(out), cout, _p(z)), "sr_conv3x3_f32")
    if timed:
        TIMER.stop(tag, ev0, 2.0 * n * ho * wo * cout * 9 * c, 4.0 * (x.numel() + w.numel() + out.numel()))


def convt_scatter(g: Tensor, n: int, h: int, w: int, k: int, co: int, bias: Optional[Tensor], out: Tensor) -> None:
    _nhwc(out, "convt_scatter out")
    check(_lib.load().sr_convt_scatter_f32(_stream(g), _p(g), n, h, w, k, co, _p(bias), _p(out)),
          "sr_convt_scatter_f32")


def resize_bilinear(x: Tensor, out: Tensor, add: Optional[Tensor] = None) -> None:
    """out = interpolate(x, out's size, bilinear, align_corners=True) (+ add: one [ho, wo, c]
    table added to every frame)."""
    n, h, w, c = _nhwc(x, "resize x")
    _, ho, wo, _ = _nhwc(out, "resize out")
    if add is not None and (add.dtype != torch.float32 or not add.is_contiguous() or add.numel() != ho * wo * c):
        raise ValueError("resize_bilinear: add must be a contiguous fp32 [ho, wo, c] table")
    check(_lib.load().sr_resize_bilinear_f32(_stream(x), _p(x), n, h, w, c, ho, wo, _p(add), _p(out)),
          "sr_resize_bilinear_f32")


def add_(dst: Tensor, src: Tensor) -> None:
    if dst.shape != src.shape or not (dst.is_contiguous() and src.is_contiguous()):
        raise ValueError("add_: shapes differ / not contiguous")
    check(_lib.load().sr_add_f32(_stream(dst), _p(dst), _p(src), dst.numel()), "sr_add_f32")


def relu_(x: Tensor) -> None:
    if not x.is_contiguous() or x.dtype != torch.float32:
        raise ValueError("relu_: contiguous fp32 tensor required")
    check(_lib.load().sr_relu_f32(_stream(x), _p(x), x.numel()), "sr_relu_f32")


def dpt_pos_embed_(x: Tensor, aspect: float, ratio: float = 0.1) -> None:
    n, h, w, c = _nhwc(x, "pos_embed x")
    check(_lib.load().sr_dpt_pos_embed_f32(_stream(x), _p(x), n, h, w, c, aspect, ratio), "sr_dpt_pos_embed_f32")


DPT_ACT = {"inv_log": 0, "exp": 1, "linear": 2, "relu": 3}
DPT_CONF_ACT = {"expp1": 0, "expp0": 1, "sigmoid": 2}


def dpt_head_out(hidden: Tensor, w: Tensor, b: Optional[Tensor], activation: str, conf_activation: str,
                 preds: Tensor, conf: Tensor) -> None:
    if activation not in DPT_ACT or conf_activation not in DPT_CONF_ACT:
        raise ValueError(f"unsupported DPT activation {activation!r} / {conf_activation!r}")
    npix, cin = hidden.shape
    cout = w.shape[0]
    check(_lib.load().sr_dpt_head_out_f32(_stream(hidden), _p(hidden), _rowmajor(hidden, "hidden"), npix, cin, _p(w),
                                          _p(b), cout, DPT_ACT[activation], DPT_CONF_ACT[conf_activation], _p(preds),
                                          _p(conf)), "sr_dpt_head_out_f32")


def unproject_depth(depth: Tensor, extrinsic: Tensor, intrinsic: Tensor, out: Tensor) -> None:
    s, h, w = depth.shape[:3]
    for t, name in ((depth, "depth"), (extrinsic, "extrinsic"), (intrinsic, "intrinsic"), (out, "out")):
        if not t.is_contiguous() or t.dtype != torch.float32 or not t.is_cuda:
            raise ValueError(f"unproject_depth: {name} must be a contiguous fp32 device tensor")
    check(_lib.load().sr_unproject_depth_f32(_stream(depth), _p(depth), _p(extrinsic), _p(intrinsic), s, h, w,
                                             _p(out)), "sr_unproject_depth_f32")


# ---------------------------------------------------------------- input formation (io.py:75-153)
def pil_resample_h(mode: int, img: Tensor, bounds: Tensor, coeffs: Tensor, tw: int, tmp: Tensor) -> None:
    """img [n, h, w, c] uint8 (mode 0) / [n, h, w, 1] int16-viewed uint16 (mode 1) -> planar tmp
    [n, c, h, ldt], ldt = tw rounded up to 4 (see pil_tmp); quad-major image-space table."""
    n, h, w, c = img.shape
    if not img.is_contiguous() or not tmp.is_contiguous() or tmp.shape != (n, c, h, (tw + 3) // 4 * 4) \
            or tmp.dtype != img.dtype:
        raise ValueError(f"pil_resample_h: img {tuple(img.shape)} / tmp {tuple(tmp.shape)} mismatch")
    if bounds.dim() != 3 or coeffs.dim() != 3 or bounds.shape[0] != (tw + 3) // 4 or coeffs.shape[0] != bounds.shape[0]:
        raise ValueError("pil_resample_h: needs the quad-major table for the output width (pil_table(quads=True))")
    check(_lib.load().sr_pil_resample_h(_stream(img), mode, _p(img), n, h, w, c, _p(bounds), _p(coeffs),
                                        coeffs.shape[1], tw, _p(tmp)), "sr_pil_resample_h")


def pil_resample_v(mode: int, tmp: Tensor, bounds: Tensor, coeffs: Tensor, divisor: float, out: Tensor) -> None:
    """planar tmp [n, c, rows, ldt] -> out [n, c, th, tw] fp32 (any strides with unit column stride);
    the table rows [0, th) are the output rows (slice the table for a crop)."""
    n, c, rows, ldt = tmp.shape
    tw = out.shape[3]
    if out.dim() != 4 or out.shape[0] != n or out.shape[1] != c or ldt != (tw + 3) // 4 * 4 or out.stride(3) != 1 \
            or out.dtype != torch.float32 or not tmp.is_contiguous():
        raise ValueError(f"pil_resample_v: out {tuple(out.shape)} does not match tmp {tuple(tmp.shape)}")
    th = out.shape[2]
    if bounds.shape[0] < th or coeffs.shape[0] < th:
        raise ValueError("pil_resample_v: table shorter than the output height")
    check(_lib.load().sr_pil_resample_v_f32(_stream(tmp), mode, _p(tmp), n, rows, tw, c, _p(bounds), _p(coeffs),
                                            coeffs.shape[1], th, float(divisor), _p(out), out.stride(0),
                                            out.stride(1), out.stride(2)), "sr_pil_resample_v_f32")



def pil_tmp(n: int, c: int, rows: int, tw: int, dtype: torch.dtype, device) -> Tensor:
    """Planar intermediate of the two resample passes: [n, c, rows, tw rounded up to 4]."""
    return torch.empty(n, c, rows, (tw + 3) // 4 * 4, dtype=dtype, device=device)


def resize_crop_chw(x: Tensor, size: int, top: int, left: int, out: Tensor, bicubic: bool) -> None:
    """out[c, i, j] = F.interpolate(x[None], (size, size), bicubic | bilinear, align_corners=False)[0, c,
    top + i, left + j] for x fp32 [C, h, w] and out fp32 [C, ho, wo] (contiguous, on device), in one
    launch (sr_resize_crop_chw_f32): ImagePreprocessor.reverse_transform_tensor's resize + crop."""
    if x.dtype != torch.float32 or out.dtype != torch.float32 or x.dim() != 3 or out.dim() != 3 or \
            not x.is_contiguous() or not out.is_contiguous() or x.shape[0] != out.shape[0]:
        raise ValueError("resize_crop_chw: x [C, h, w] and out [C, ho, wo] contiguous fp32")
    C, h, w = x.shape
    ho, wo = out.shape[1], out.shape[2]
    rc = _lib.load().sr_resize_crop_chw_f32(_stream(x), _p(x), C, h, w, size, size, top, left, ho, wo,
                                            1 if bicubic else 0, _p(out))
    check(rc, "sr_resize_crop_chw_f32")


# ---------------------------------------------------------------- training step
_TRAIN_WS = {}  # ((device, stream), name) -> fp32 workspace


def _train_ws(device, name: str, numel: int) -> Tensor:
    key = (_ws_stream_key(device), name)
    ws = _TRAIN_WS.get(key)
    if ws is None or ws.numel() < numel:
        ws = torch.empty(max(numel, 1), device=device, dtype=torch.float32)
        _TRAIN_WS[key] = ws
    return ws


def _wgrad_splits(M: int, N: int, K: int) -> int:
    """Reduction slices.  256x256 tiles (sr_gemm_wgrad's one-workgroup-per-CU kernel when N and K
    are multiples of 256): the most slices that still fit one round of 256 workgroups, each slice
    >= 8 m-tiles of 64 rows, at most 16.  128x128 tiles: >= 512 workgroups (2 per CU), powers of 2;
    the fp32 partials stay <= 16x the output."""
    mt = -(-M // 64)
    if get_tuning("SR_WGRAD256") and N % 256 == 0 and K % 256 == 0:
        tiles = (N // 256) * (K // 256)
        return max(1, min(256 // tiles, 16, mt // 8))
    tiles = (N // 128) * (K // 128)
    s = 1
    while tiles * s < 512 and mt // (2 * s) >= 8 and 2 * s <= 16:
        s *= 2
    return s


def gemm_wgrad(dy: Tensor, x: Tensor, dw: Tensor, *, accumulate: bool = False, rowscale: Optional[Tensor] = None,
               wdot: Optional[Tensor] = None, rowdot: Optional[Tensor] = None, splits: Optional[int] = None,
               tag: Optional[str] = None) -> None:
    """dw[N,K] (fp32) (+)= rowscale[n] * dy[M,N]^T x[M,K] (bf16); rowdot[n] += <wdot[n], G[n]>."""
    M, N = dy.shape
    K = x.shape[1]
    if x.shape[0] != M or dw.shape != (N, K) or dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 \
            or dw.dtype != torch.float32:
        raise ValueError(f"gemm_wgrad: dy {tuple(dy.shape)} x {tuple(x.shape)} dw {tuple(dw.shape)} mismatch")
    if splits is None:
        splits = _wgrad_splits(M, N, K)
    ws = _train_ws(dy.device, "wgrad", splits * N * K)
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    rc = _lib.load().sr_gemm_wgrad(_stream(dy), _p(dy), _rowmajor(dy, "dy"), _p(x), _rowmajor(x, "x"), _p(dw),
                                   _rowmajor(dw, "dw"), M, N, K, int(accumulate), _p(rowscale), _p(wdot),
                                   0 if wdot is None else _rowmajor(wdot, "wdot"), _p(rowdot), splits, _p(ws))
    check(rc, "sr_gemm_wgrad")
    if timed:
        TIMER.stop(tag, ev0, 2.0 * M * N * K, 2 * M * (N + K) + 4 * N * K * (3 if accumulate else 2))


def wgrad_pair_splits(M0: int, M1: int, N: int, K: int) -> Optional[Tuple[int, int]]:
    """Slices per problem when two gemm_wgrad problems of equal N, K share one launch
    (gemm_wgrad_pair), or None where that does not pay: both problems' slices must fill one round
    of 256 workgroups exactly as one problem alone would (256 / tiles even: proj / fc1 / fc2 at
    C = 1,024, not qkv's 48 tiles), so each slice walks twice the m-tiles and the two launches'
    fixed costs and half the fp32 partials go."""
    if not get_tuning("SR_WGRAD256") or N % 256 or K % 256:
        return None
    tiles = (N // 256) * (K // 256)
    per = 256 // tiles
    if per < 2 or per % 2:
        return None
    s = min(per // 2, 16)
    return max(1, min(s, -(-M0 // 64) // 8)), max(1, min(s, -(-M1 // 64) // 8))


def gemm_wgrad_pair(probs, splits: Tuple[int, int], tag: Optional[str] = None) -> None:
    """Two gemm_wgrad problems (dicts: dy, x, dw and gemm_wgrad's accumulate / rowscale / wdot /
    rowdot keywords) of equal N, K in one launch (sr_gemm_wgrad_pair), ``splits`` slices each."""
    if len(probs) != 2:
        raise ValueError("gemm_wgrad_pair: exactly two problems")
    arr = (_lib.WgradProblem * 2)()
    flops = nbytes = 0.0
    for i, p in enumerate(probs):
        dy, x, dw = p["dy"], p["x"], p["dw"]
        M, N = dy.shape
        K = x.shape[1]
        if x.shape[0] != M or dw.shape != (N, K) or dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 \
                or dw.dtype != torch.float32:
            raise ValueError(f"gemm_wgrad_pair: dy {tuple(dy.shape)} x {tuple(x.shape)} dw {tuple(dw.shape)} mismatch")
        q = arr[i]
        q.A, q.lda, q.B, q.ldb = _p(dy), _rowmajor(dy, "dy"), _p(x), _rowmajor(x, "x")
        q.dW, q.lddw = _p(dw), _rowmajor(dw, "dw")
        q.M, q.N, q.K, q.accumulate = M, N, K, int(p.get("accumulate", False))
        q.rowscale, q.wdot, q.rowdot = _p(p.get("rowscale")), _p(p.get("wdot")), _p(p.get("rowdot"))
        q.ldwd = 0 if p.get("wdot") is None else _rowmajor(p["wdot"], "wdot")
        q.splits = int(splits[i])
        q.workspace = _p(_train_ws(dy.device, f"wgrad{i}", splits[i] * N * K))
        flops += 2.0 * M * N * K
        nbytes += 2 * M * (N + K) + 4 * N * K * (3 if q.accumulate else 2)
    timed = TIMER is not None and TIMER.wants(tag)
    ev0 = TIMER.start() if timed else None
    check(_lib.load().sr_gemm_wgrad_pair(_stream(probs[0]["dy"]), arr), "sr_gemm_wgrad_pair")
    if timed:
        TIMER.stop(tag, ev0, flops, nbytes)


def colsum(x: Tensor, out: Tensor, *, rows: Optional[int] = None, cols: Optional[int] = None,
           accumulate: bool = False, scale: float = 1.0) -> None:
    """out[c] (+)= scale * sum_r x[r, c] over a row-strided 2-D view (bf16 or fp32)."""
    ldx = _rowmajor(x, "x")
    M = x.shape[0] if rows is None else rows
    N = x.shape[1] if cols is None else cols
    if out.dtype != torch.float32 or out.numel() < N:
        raise ValueError("colsum: out must be fp32 with >= cols elements")
    lib = _lib.load()
    nws = lib.sr_colsum_workspace_floats(M, N)
    ws = _train_ws(x.device, "colsum", max(1, nws))
    rc = lib.sr_colsum(_stream(x), dtype_code(x.dtype), _p(x), ldx, M, N, _p(out), int(accumulate),
                       float(scale), _p(ws), ws.numel())
    check(rc, "sr_colsum")


def colsum_fma(x: Tensor, pairs) -> None:
    """out[c] += mul[c] * sum_r x[r, c] for each (out, mul) of ``pairs`` (one or two; fp32 [cols]),
    in the launches of one column sum (sr_colsum_fma; the same bits as colsum + vec_fma)."""
    ldx = _rowmajor(x, "x")
    M, N = x.shape
    if not 1 <= len(pairs) <= 2 or any(o.dtype != torch.float32 or o.numel() < N or m.numel() < N for o, m in pairs):
        raise ValueError("colsum_fma: one or two (out, mul) fp32 pairs of >= cols elements")
    (o1, m1), (o2, m2) = pairs[0], (pairs[1] if len(pairs) == 2 else (None, None))
    lib = _lib.load()
    nws = lib.sr_colsum_workspace_floats(M, N)
    ws = _train_ws(x.device, "colsum", max(1, nws))
    rc = lib.sr_colsum_fma(_stream(x), dtype_code(x.dtype), _p(x), ldx, M, N, _p(o1), _p(m1), _p(o2), _p(m2), _p(ws),
                           ws.numel())
    check(rc, "sr_colsum_fma")


def layernorm_bwd(x: Tensor, dy: Tensor, w: Optional[Tensor], eps: float, dx: Tensor, *,
                  dxb: Optional[Tensor] = None, dw: Optional[Tensor] = None, db: Optional[Tensor] = None,
                  rowmap: Optional[Tensor] = None, rows: Optional[int] = None,
                  dx_sum: Optional[Tensor] = None) -> None:
    """dx[rows] += LayerNorm backward (see sr_layernorm_bwd); dxb = bf16 copy of the updated rows;
    dx_sum (fp32 [cols], with dw / db, cols <= 2048) = the column sum of the updated rows."""
    n = dy.shape[0] if rows is None else rows
    cols = x.shape[1]
    if dx_sum is not None and (dw is None or dx_sum.dtype != torch.float32 or dx_sum.numel() < cols or
                               not dx_sum.is_contiguous()):
        raise ValueError("layernorm_bwd: dx_sum needs dw / db and a contiguous fp32 [cols] output")
    ws = _train_ws(x.device, "lnbwd", 4 * 1024 * cols) if dw is not None else None
    rc = _lib.load().sr_layernorm_bwd(_stream(x), dtype_code(dy.dtype), _p(x), _rowmajor(x, "x"), _p(rowmap), _p(dy),
                                      _rowmajor(dy, "dy"), _p(w), eps, _p(dx), _rowmajor(dx, "dx"), _p(dxb),
                                      0 if dxb is None else _rowmajor(dxb, "dxb"), _p(dw), _p(db), n, cols, _p(ws),
                                      _p(dx_sum))
    check(rc, "sr_layernorm_bwd")


def qk_bwd(raw: Optional[Tensor], dsrc: Tensor, out: Tensor, qkv: dict, *, grads: Optional[Tensor] = None,
           ncols: Optional[int] = None, bias_grad: Optional[Tensor] = None) -> None:
    """d(pre-norm q|k|v) (out: bf16, or fp32 for fp32 blocks with raw fp32) from fp32 d(q|k|v)
    through RoPE^T and the qk-norm backward; grads fp32 [4, 64] += (dqn_w, dqn_b, dkn_w, dkn_b).
    ``bias_grad`` (fp32 [ncols]): += the column sums of out (the qkv bias gradient) from the same
    pass (sr_gemm_epi.colsum of sr_qk_bwd), no re-read of out."""
    ep = GemmEpi()
    _fill_qkv_epi(ep, qkv)
    rows = dsrc.shape[0]
    nc = out.shape[1] if ncols is None else ncols
    if raw is not None and raw.dtype != out.dtype:
        raise TypeError("qk_bwd: raw and out must share a dtype")
    if bias_grad is not None:
        if bias_grad.dtype != torch.float32 or not bias_grad.is_contiguous() or bias_grad.numel() < nc:
            raise ValueError("qk_bwd: bias_grad must be contiguous fp32 [ncols]")
        ep.colsum = _p(bias_grad)
    ws = _train_ws(dsrc.device, "qkbwd", max(4352 * 256, int(_lib.load().sr_qk_bwd_workspace_floats(rows, nc))))
    fn = "sr_qk_bwd_f32" if out.dtype == torch.float32 else "sr_qk_bwd"
    rc = getattr(_lib.load(), fn)(_stream(dsrc), _p(raw), 0 if raw is None else _rowmajor(raw, "raw"), _p(dsrc),
                                  _rowmajor(dsrc, "dsrc"), _p(out), _rowmajor(out, "out"), rows, nc, ctypes.byref(ep),
                                  _p(grads), _p(ws))
    check(rc, fn)


def cast_bf16(src: Tensor, dst: Tensor, scale: float = 1.0) -> None:
    rows, cols = src.shape
    check(_lib.load().sr_cast_bf16(_stream(src), _p(src), _rowmajor(src, "src"), _p(dst), _rowmajor(dst, "dst"),
                                   rows, cols, float(scale)), "sr_cast_bf16")


def nonfinite_check(g: Tensor, found: Tensor, scale: Optional[Tensor] = None) -> None:
    check(_lib.load().sr_nonfinite_check(_stream(g), _p(g), g.numel(), _p(scale), _p(found)), "sr_nonfinite_check")


def adam(p: Tensor, g: Tensor, m: Tensor, v: Tensor, *, lr: float, beta1: float, beta2: float, eps: float,
         weight_decay: float, step: int, scale: Optional[Tensor] = None, found_inf: Optional[Tensor] = None) -> None:
    for t in (p, g, m, v):
        if not t.is_contiguous() or t.dtype != torch.float32 or t.numel() != p.numel():
            raise ValueError("adam: p / g / m / v must be contiguous fp32 of one size")
    check(_lib.load().sr_adam_f32(_stream(p), _p(p), _p(g), _p(m), _p(v), p.numel(), lr, beta1, beta2, eps,
                                  weight_decay, step, _p(scale), _p(found_inf)), "sr_adam_f32")


def _weight_items(items):
    arr = (_lib.WeightItem * len(items))()
    for it, (src, cast, trans, rowscale) in zip(arr, items):
        R, C = src.shape
        if src.dtype != torch.float32 or (cast is None and trans is None):
            raise ValueError("weight_refresh: fp32 src and a cast and / or trans output")
        for t, shape in ((cast, (R, C)), (trans, (C, R))):
            if t is not None and (t.dtype != torch.bfloat16 or tuple(t.shape) != shape):
                raise ValueError(f"weight_refresh: bf16 outputs {(R, C)} / {(C, R)}")
        it.src, it.lds, it.rows, it.cols = src.data_ptr(), _rowmajor(src, "src"), R, C
        it.rowscale = None if rowscale is None else rowscale.data_ptr()
        it.cast, it.ldc = (None, 0) if cast is None else (cast.data_ptr(), _rowmajor(cast, "cast"))
        it.trans, it.ldt = (None, 0) if trans is None else (trans.data_ptr(), _rowmajor(trans, "trans"))
    return arr


def weight_refresh(items) -> None:
    """Up to 4 fp32 weights in one launch (sr_weight_refresh_bf16): ``items`` = (src fp32 [R, C],
    cast bf16 [R, C] or None, trans bf16 [C, R] or None, rowscale fp32 [R] or None) -- the bf16
    forward operand and the rowscaled transposed dgrad operand from one read of each weight."""
    if not 0 < len(items) <= _lib.SR_WEIGHT_REFRESH_MAX:
        raise ValueError("weight_refresh: 1..4 items")
    arr = _weight_items(items)
    check(_lib.load().sr_weight_refresh_bf16(_stream(items[0][0]), len(items), arr), "sr_weight_refresh_bf16")


def weight_refresh_table(items, device) -> dict:
    """The device-resident table of sr_weight_refresh_list_bf16 for any number of weight_refresh
    items (validated by sr_weight_refresh_plan); the tensors' addresses must stay put while it is used."""
    if not items:
        raise ValueError("weight_refresh_table: no items")
    arr = _weight_items(items)
    start = (ctypes.c_int * (len(items) + 1))()
    check(_lib.load().sr_weight_refresh_plan(len(items), arr, start), "sr_weight_refresh_plan")
    raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return dict(n=len(items), tiles=int(start[len(items)]), items=raw.to(device),
                start=torch.tensor(list(start), dtype=torch.int32).to(device))


def weight_refresh_list(table: dict) -> None:
    """Every item of a weight_refresh_table in ONE launch (sr_weight_refresh_list_bf16)."""
    check(_lib.load().sr_weight_refresh_list_bf16(_stream(table["items"]), table["n"], _p(table["items"]),
                                                  _p(table["start"]), table["tiles"]), "sr_weight_refresh_list_bf16")


def transpose(src: Tensor, dst: Tensor, rowscale: Optional[Tensor] = None) -> None:
    """dst[c, r] = dst.dtype(rowscale[r] * src[r, c]) (fp32 src)."""
    R, C = src.shape
    if src.dtype != torch.float32 or dst.shape != (C, R):
        raise ValueError(f"transpose: src {tuple(src.shape)} {src.dtype} -> dst {tuple(dst.shape)}")
    check(_lib.load().sr_transpose_f32(_stream(src), dtype_code(dst.dtype), _p(src), _rowmajor(src, "src"), R, C,
                                       _p(rowscale), _p(dst), _rowmajor(dst, "dst")), "sr_transpose_f32")


def wgrad_small(dy: Tensor, x: Tensor, dw: Tensor, *, db: Optional[Tensor] = None, accumulate: bool = False,
                rowscale: Optional[Tensor] = None, wdot: Optional[Tensor] = None,
                rowdot: Optional[Tensor] = None) -> None:
    """fp32 dw[N,K] (+)= rowscale[n] * dy[M,N]^T x[M,K]; db[N] (+)= colsum(dy); rowdot += <wdot, G>."""
    M, N = dy.shape
    K = x.shape[1]
    if dw.shape != (N, K) or x.shape[0] != M:
        raise ValueError("wgrad_small: shape mismatch")
    ws = _train_ws(dy.device, "wgrad", N * K) if (rowscale is not None or wdot is not None) else None
    check(_lib.load().sr_wgrad_small_f32(_stream(dy), _p(dy), _rowmajor(dy, "dy"), _p(x), _rowmajor(x, "x"), _p(dw),
                                         _rowmajor(dw, "dw"), M, N, K, int(accumulate), _p(db), _p(rowscale),
                                         _p(wdot), 0 if wdot is None else _rowmajor(wdot, "wdot"), _p(rowdot),
                                         _p(ws)), "sr_wgrad_small_f32")


def attention_bwd_small(q: Tensor, k: Tensor, v: Tensor, dout: Tensor, dq: Tensor, dk: Tensor, dv: Tensor, *,
                        heads: int, head_dim: int, mask_mode: int = _lib.SR_MASK_NONE, n_anchor: int = 0,
                        scale: Optional[float] = None) -> None:
    L = q.shape[0]
    ld = _rowmajor(q, "q")
    if _rowmajor(k, "k") != ld or _rowmajor(v, "v") != ld:
        raise ValueError("attention_bwd_small: q / k / v must share a row stride")
    ldg = _rowmajor(dq, "dq")
    if _rowmajor(dk, "dk") != ldg or _rowmajor(dv, "dv") != ldg:
        raise ValueError("attention_bwd_small: dq / dk / dv must share a row stride")
    ws = _train_ws(q.device, "attn_small", 2 * heads * L * L)
    check(_lib.load().sr_attention_bwd_small_f32(_stream(q), _p(q), _p(k), _p(v), ld, _p(dout),
                                                 _rowmajor(dout, "dout"), _p(dq), _p(dk), _p(dv), ldg, L, heads,
                                                 head_dim, head_dim ** -0.5 if scale is None else scale, mask_mode,
                                                 n_anchor, _p(ws)), "sr_attention_bwd_small_f32")


def adaln_bwd(xn: Tensor, mod: Tensor, dxm: Tensor, dxn: Tensor, dmod: Tensor) -> None:
    rows, cols = xn.shape
    check(_lib.load().sr_adaln_bwd_f32(_stream(xn), _p(xn), _p(mod), _p(dxm), _p(dxn), _p(dmod), rows, cols),
          "sr_adaln_bwd_f32")


ACT_SILU, ACT_GELU = 0, 1


def act_bwd(mode: int, x: Tensor, dy: Tensor, dx: Tensor) -> None:
    for t in (x, dy, dx):
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise ValueError("act_bwd: contiguous fp32 tensors required")
    check(_lib.load().sr_act_bwd_f32(_stream(x), mode, _p(x), _p(dy), _p(dx), x.numel()), "sr_act_bwd_f32")


def vec_fma(out: Tensor, a: Tensor, b: Tensor, out2: Optional[Tensor] = None, a2: Optional[Tensor] = None) -> None:
    """out += a * b (and out2 += a2 * b in the same launch), fp32, one fused multiply-add each."""
    if out2 is None:
        check(_lib.load().sr_vec_fma_f32(_stream(out), _p(out), _p(a), _p(b), out.numel()), "sr_vec_fma_f32")
        return
    if a2 is None or out2.numel() != out.numel():
        raise ValueError("vec_fma: out2 needs a2 and out's length")
    check(_lib.load().sr_vec_fma2_f32(_stream(out), _p(out), _p(a), _p(out2), _p(a2), _p(b), out.numel()),
          "sr_vec_fma2_f32")


def scatter_rows(dst: Tensor, rowmap: Tensor, src: Tensor, *, accumulate: bool = True, rows: Optional[int] = None) -> None:
    """dst[rowmap[r]] (+)= src[r] (src with row stride 0 = one broadcast row)."""
    n = rowmap.numel() if rows is None else rows
    lds = 0 if src.dim() == 1 else _rowmajor(src, "src")
    check(_lib.load().sr_scatter_rows_f32(_stream(dst), _p(dst), _rowmajor(dst, "dst"), _p(rowmap), _p(src), lds, n,
                                          dst.shape[1], int(accumulate)), "sr_scatter_rows_f32")


def copy2d(dst: Tensor, src: Tensor, *, accumulate: bool = False) -> None:
    """dst (+)= src for 2-D fp32 row-strided views of one shape (any column count)."""
    if dst.shape != src.shape or dst.dtype != torch.float32 or src.dtype != torch.float32:
        raise ValueError(f"copy2d: {tuple(dst.shape)} vs {tuple(src.shape)}")
    check(_lib.load().sr_copy2d_f32(_stream(dst), _p(dst), _rowmajor(dst, "dst"), _p(src), _rowmajor(src, "src"),
                                    dst.shape[0], dst.shape[1], int(accumulate)), "sr_copy2d_f32")


def pose_act_bwd(dd: Tensor, d_act: Tensor, act: Tensor, n_anchor: int) -> None:
    for t in (dd, d_act, act):
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise ValueError("pose_act_bwd: contiguous fp32 tensors required")
    check(_lib.load().sr_pose_act_bwd_f32(_stream(dd), _p(dd), _p(d_act), _p(act), dd.shape[0], n_anchor),
          "sr_pose_act_bwd_f32")
