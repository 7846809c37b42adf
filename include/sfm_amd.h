/*
 * sfm_amd.h — C ABI of the MI355X-native SailRecon hot path (libsfm_amd.so).
 *
 * The reference (ShngJZ/self-supervise-sfm) has no FFI: its boundary is the
 * Python nn.Module API.  These entry points are what that API's
 * torch ops bottom out in on the hot path; each names the reference call site
 * it replaces.  The framework's Python mirror (sailrecon_amd.*) is the only
 * caller and owns every buffer.
 *
 * Conventions
 *   - every pointer is a borrowed DEVICE pointer (except where noted);
 *   - leading dimensions / strides are in ELEMENTS of the pointed-to type;
 *   - launches are asynchronous on the caller's stream (hipStream_t, NULL = default);
 *   - return 0 (SR_OK) or a negative sr_status; sr_last_error() explains it;
 *   - no allocation, no synchronisation inside a call (safe to capture into a hipGraph);
 *     the only process-wide mutable state is the tuning switches (sr_set_tuning), whose
 *     SR_TUNE_SYNC_CHECK debug mode is the one exception to "no synchronisation".
 */
#ifndef SFM_AMD_H
#define SFM_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* sr_stream_t; /* hipStream_t */

enum sr_dtype { SR_F32 = 0, SR_BF16 = 1 };

enum sr_status {
  SR_OK = 0,
  SR_EINVAL = -1,       /* bad shape / pointer / enum */
  SR_ELAUNCH = -2,      /* hipLaunch / runtime error */
  SR_EUNSUPPORTED = -3  /* valid but not implemented shape */
};

/* Message for the most recent failing call on this thread ("" if none). */
const char* sr_last_error(void);
/* ABI version: (major << 16) | minor. */
int sr_version(void);

/* The main device kernel (the one its time goes to) of the most recent launching call on this
 * thread, named as rocprofv3 names it (e.g. "attn_bf16_pair_kernel<2>", "gemm256_kernel<2>"): the library's
 * own dispatch decision, for profilers and benchmarks that attribute time to kernels ("" if
 * none yet).  Per thread, like sr_last_error. */
const char* sr_last_kernel(void);

/* ------------------------------------------------------------------------
 * Tuning switches: the library's one piece of process-wide mutable state (besides the
 * per-thread strings above).  Each switch selects between kernels or schedules that compute
 * the same function (A/B experiments; the defaults are the measured best).  Values
 * start from the environment variable sr_tuning_name(key) (read once, at the first use), and
 * are read at every launch, so sr_set_tuning takes effect for the next call on any thread.
 * Not synchronised with launches in flight on other threads.
 * ---------------------------------------------------------------------- */
enum sr_tuning_key {  /* renumbered in ABI 1.3: switches that measured level or slower were removed */
  SR_TUNE_ATTN_MZERO = 0,   /* 1: a fixed softmax offset of 0 drops the -m fold MFMAs, and the
                               hand-scheduled sweep may run (0: neither)               default 1 */
  SR_TUNE_ATTN_CFG = 1,     /* -1 auto; 0 | 1 | 2: force the bf16 attention workgroup shape
                               (4x2 | 8x1 | 2x2 waves x q-blocks)                      default -1 */
  SR_TUNE_ATTN_PIPE = 2,    /* 1: the hand-scheduled (asm) sweep where it applies    default 1 */
  SR_TUNE_ATTN_PIPE_SEG = 3,/* 1: its two-segment / ragged variant for every launch with
                               readable tails (0: only for one long query set)         default 0 */
  SR_TUNE_ATTN_NO_SHORT = 4,/* 1: no short-sequence fp32 attention kernel             default 0 */
  SR_TUNE_GEMM_GROUP_M = 5, /* -1 auto (4 for N >= 3072, else row-major); g: tile order in groups
                               of g row tiles for sr_gemm's and sr_gemm_group's 256x256 tiles */
  SR_TUNE_GEMM_SMALLM = 6,  /* 1: 64x256 tiles for M <= 64                             default 1 */
  SR_TUNE_GEMM_NO256 = 7,   /* 1: never the 256x256 GEMM kernel                        default 0 */
  SR_TUNE_GEMM_REG_EPI = 8, /* 1: register (not LDS-staged) bf16 epilogue              default 0 */
  SR_TUNE_CONV_NO_NARROW = 9,/* 1: no narrow (Cout <= 32) conv kernel                  default 0 */
  SR_TUNE_WGRAD256 = 10,    /* 1: 256x256 weight-gradient tiles where they fit         default 1 */
  SR_TUNE_SYNC_CHECK = 11,  /* 1: debug mode -- every launching call synchronises the device and
                               returns SR_ELAUNCH with the runtime's message if a kernel faulted
                               (HIP_LAUNCH_BLOCKING-style attribution; not graph-capturable) */
  SR_TUNE_RLN_WIDE = 12,    /* sr_residual_layernorm variant bits: 1 16-B lanes, 2 two rows per wave, 4 nt x stores (0) */
  SR_TUNE_GEMM_TAIL = 13,   /* 1: a 256x256 GEMM whose last workgroup round would run few tiles computes
                               the rows past its last whole round on the 128x128 kernel (second launch)  (1) */
  SR_TUNE_GEMM_RESID_LDS = 14,/* 1: the 256x256 RESID GEMM's epilogue stages the x tile through LDS by
                               LDS-DMA (64-row quarters, two in flight; whole-row stores)  default 1 */
  SR_TUNE_GEMM_ROPE_LDS = 15,/* 1: the 256x256 QKV epilogue reads its RoPE tables from LDS (staged by DMA
                               under the first k-tile; 0: from global memory)           default 1 */
  SR_TUNE_ATTN_BWD_PIPE = 16,/* 1: the dK/dV sweep as the hand-scheduled asm pipeline (one wave per SIMD,
                               64 keys; one item per workgroup, >= 4 full query tiles;
                               bit-identical)                                           default 1 */
  SR_TUNE_ATTN_BWD_DQ_PIPE = 17,/* 1: the attention backward's dQ sweep as the hand-scheduled asm pipeline
                               (one wave per SIMD, 64 queries; one key segment of >= 4 full
                               tiles, query padding within 2 % of the compiled sweep's or
                               >= 4,096 keys; 2: always; bit-identical)                default 1 */
  SR_TUNE_ATTN_BWD_CAT = 18,/* 1: keys shared by a batch > 1 whose items' queries are consecutive rows:
                               the dK/dV asm sweep over the concatenated queries (one sequence of
                               batch * lq rows; same sum, other tile grouping)          default 1 */
  SR_TUNE_COUNT = 19
};
/* Sets a switch; returns its previous value (SR_EINVAL for an unknown key). */
int sr_set_tuning(int key, int value);
/* Current value of a switch (SR_EINVAL for an unknown key). */
int sr_get_tuning(int key);
/* The environment variable a switch starts from (e.g. "SR_ATTN_PIPE"); NULL for an unknown key. */
const char* sr_tuning_name(int key);

/* ------------------------------------------------------------------------
 * GEMM with fused epilogue:  out = epilogue(A[M,K] . W[N,K]^T)
 * Replaces nn.Linear -> addmm for qkv / proj / fc1 / fc2
 * (attention.py:48,73,120; mlp.py:34-40) and the 14x14/s14 patch conv
 * (patch_embed.py:62-64,78) as an im2col GEMM.
 * A, W, out (except RESID / PATCH outputs, which are fp32) use `dtype`.
 * Requires N % 128 == 0 and K % (64 bf16 | 32 f32) == 0; M arbitrary.
 * ---------------------------------------------------------------------- */
enum sr_epilogue {
  SR_EPI_BIAS = 0,       /* out = acc + bias                                   */
  SR_EPI_BIAS_GELU = 1,  /* out = gelu_erf(acc + bias)           (mlp.py:36)   */
  SR_EPI_BIAS_RESID = 2, /* out(f32) += gamma * (acc + bias)  (block.py:110-111,
                            layer_scale.py:22-23)                              */
  SR_EPI_QKV = 3,        /* out = rope(qk_norm(acc + bias)) on Q,K columns
                            (attention.py:72-82, rope.py:165-207)               */
  SR_EPI_PATCH = 4,      /* out(f32)[remap(row)] = acc + bias + row_add[row % seg_rows]
                            (vision_transformer.py:242-259)                     */
  /* training step: backward epilogues of the same GEMM,
     with W^T packed as the "W" operand (dX = dY . W) */
  SR_EPI_F32 = 5,        /* out(f32) = acc + bias   (dgrad into LayerNorm backward) */
  SR_EPI_GELU_BWD = 6    /* out = acc * gelu_erf'(aux[row, col])  (fc2 dgrad fused with
                            the GELU backward, mlp.py:36; aux = saved fc1 pre-activation) */
};

typedef struct sr_gemm_epi {
  const float* bias;  /* [N] or NULL */
  const float* gamma; /* [N] LayerScale gamma (RESID) */
  /* QKV: per-head LayerNorm(head_dim) over Q and K columns + 2-D RoPE */
  const float* qn_w;
  const float* qn_b;
  const float* kn_w;
  const float* kn_b;       /* [head_dim] each, or all NULL (no qk-norm)    */
  float qk_eps;            /* 1e-5 (attention.py:49-50)                    */
  const float* rope_cos;   /* [rope_npos][head_dim/4] or NULL (no RoPE)    */
  const float* rope_sin;
  int rope_npos;
  int col_offset;          /* column of out-col 0 inside [Q|K|V] (K/V-only GEMM: embed_dim) */
  int head_dim;
  int embed_dim;
  const int32_t* pos_yx;     /* explicit int32 (y, x) per GEMM row, or NULL: derive from the token row */
  const int32_t* pos_rowmap; /* token row of GEMM row r (NULL: pos_row_base + r) */
  int64_t pos_row_base;
  int tokens_per_frame;    /* P = patch_start + grid_h*grid_w */
  int patch_start;         /* 5 (aggregator.py:176) */
  int grid_w;              /* W / patch */
  /* PATCH */
  int seg_rows;
  int seg_stride;
  int seg_offset;
  const float* row_add;    /* [seg_rows][N] */
  /* training: BIAS_GELU / QKV also store the pre-activation (acc + bias, before GELU /
     qk-norm / RoPE) to aux (dtype, row stride ld_aux) for the backward; GELU_BWD reads it */
  void* aux;
  int64_t ld_aux;
  /* BIAS / QKV (bf16 outputs): output columns [0, q_cols) -- the Q block -- are multiplied by
     q_scale in fp32 before the one rounding to the output type (0 = off).  With q_scale =
     scale * log2(e) the attention reads c*q rounded once (sr_attn_desc.q_scaled) instead of
     re-rounding c * bf16(q) (ABI 1.0).  q_cols a multiple of 64. */
  float q_scale;
  int q_cols;
  /* GELU_BWD (training): per-64-row-block column sums of the bf16 output dH, i.e. the fc1 bias
     gradient's partials without re-reading dH (ABI 1.4): colsum[(r / 64) * N + c] = sum over the
     block's rows r < M of bf16(dH[r][c]), written (not accumulated) for every block the call
     covers; ceil(M / 64) * N floats, 16-B aligned.  NULL = off.  sr_colsum over the ceil(M / 64)
     rows then gives the full column sum. */
  float* colsum;
} sr_gemm_epi;

/* bf16 kernels: 256x256 tiles (one workgroup per CU) for >= 512 such tiles, else 128x128; with
 * SR_TUNE_GEMM_TAIL the rows past the 256x256 kernel's last whole workgroup round run on the 128x128
 * kernel in a second launch.  Both run the same MFMA over the same k order per output element, so
 * the accumulators agree and only the epilogue's fp32 contraction may differ (rel <= 1e-6,
 * test_kernels_gpu.py::test_gemm_tail_split over every epilogue, aux and row-map form); the
 * split-K path (sr_gemm_splitk) sums in another order. */
int sr_gemm(sr_stream_t stream, int dtype, int epilogue, const void* A, int64_t lda, const void* W,
            int64_t ldw, void* out, int64_t ldo, int M, int N, int K, const sr_gemm_epi* ep);

/* One problem of sr_gemm_group: the arguments of sr_gemm. */
typedef struct sr_gemm_problem {
  const void* A;
  int64_t lda;
  const void* W;
  int64_t ldw;
  void* out;
  int64_t ldo;
  int M, N, K;
  sr_gemm_epi ep;
} sr_gemm_problem;

/* 1..4 independent bf16 GEMMs of one epilogue kind (BIAS, QKV, BIAS_GELU, BIAS_RESID, and the training
 * dgrads' F32 / GELU_BWD; N % 256 == 0)
 * in ONE launch of the 256x256 kernel, so that their last partial workgroup rounds merge (the
 * layer's query, anchor and anchor-subsample QKV projections after a frame block).  Every problem
 * runs on the 256x256 kernel with sr_gemm's tile order, so it is bit-identical to sr_gemm only
 * where sr_gemm also picks that kernel (>= 512 tiles of 256x256); a smaller problem (the C3
 * anchor-subsample K/V projection: ~312 tiles) differs from sr_gemm's 128x128 kernel by
 * accumulation order (fp32 accumulate, rel ~1e-6).  Replaces the qkv nn.Linear calls of one layer's
 * global_reloc and global blocks (attention.py:73; aggregator.py:672-769). */
int sr_gemm_group(sr_stream_t stream, int dtype, int epi, int n, const sr_gemm_problem* problems);

/* Split-K form of sr_gemm for few rows and long K (the camera trunk: M = 2N views against
 * 2048 x 8192 weights, camera_head.py:163-168).  `splits` workgroup slices of K write fp32
 * partial tiles to `workspace` (>= splits * M * N floats, 16-B aligned, caller-owned; no
 * allocation inside), then one reduction applies the epilogue.  Epilogues BIAS, BIAS_GELU,
 * BIAS_RESID and F32 (the camera trunk's dgrad); deterministic (fixed summation order).  K/splits must be a multiple of
 * the k-tile (64 bf16 | 32 f32). */
int sr_gemm_splitk(sr_stream_t stream, int dtype, int epilogue, const void* A, int64_t lda, const void* W,
                   int64_t ldw, void* out, int64_t ldo, int M, int N, int K, int splits, float* workspace,
                   const sr_gemm_epi* ep);

/* ------------------------------------------------------------------------
 * Fused multi-head attention  O = softmax(scale * Q K^T + mask) V
 * Replaces F.scaled_dot_product_attention (attention.py:103-109) for the
 * frame, global, global_reloc (implicit block mask, aggregator.py:302-311,
 * 832-851) and camera-trunk (camera_head.py:165, 197-228) calls.
 *
 * Batch item b, head h: query rows  q + (b*q_bstride + i)*ldq + h*head_dim, i < lq
 * keys: segment 0 rows k0 + (b*k0_bstride + j)*ldk0 (+h*head_dim), j < l0
 *       segment 1 rows k1 + (b*k1_bstride + j)*ldk1,                j < l1
 * Every query row attends to all l0 + l1 keys of its item (the reloc mask:
 * anchor subsample shared via k0_bstride = 0, own frame via segment 1).
 * mask_mode SR_MASK_CAMERA (l1 == 0): row i sees key j iff j < n_anchor or j == i.
 * dtype SR_BF16: MFMA kernel, head_dim 64.  SR_F32: exact-f32 kernel, head_dim 64|128.
 * ---------------------------------------------------------------------- */
enum sr_mask_mode { SR_MASK_NONE = 0, SR_MASK_CAMERA = 1, SR_MASK_DENSE = 2, SR_MASK_ADD = 3 };

typedef struct sr_attn_desc {
  const void* q;
  int64_t ldq;
  const void* k0;
  const void* v0;
  int64_t ldk0, ldv0;
  const void* k1;
  const void* v1;
  int64_t ldk1, ldv1;
  void* o;
  int64_t ldo;
  int batch, heads, head_dim;
  int lq;
  int64_t q_bstride;
  int l0;
  int64_t k0_bstride;
  int l1;
  int64_t k1_bstride;
  int mask_mode, n_anchor;
  float scale;
  float* lse;  /* optional: [batch][heads][lq] row log-sum-exp of scale*log2(e)*q.k (log2
                  domain), saved for sr_attention_bwd and for sr_attn_merge */
  float* key_bound; /* optional scratch (bf16 path, >= sr_attention_bound_floats(d) floats, 4-B
                  aligned): per key-segment instance and head, max |k|^2 over the keys, scanned by the
                  launch itself.  With it a query row whose Cauchy-Schwarz bound c|q| max|k| lies
                  within 2^174 of its first tile's max runs the sweep with a FIXED softmax offset
                  m = max(tile max, bound - 64) (m = 0 for a bound <= 64): no per-tile row max, no
                  rescale; every P <= 2^64 and the row's largest P >= 2^-110, so no overflow and the
                  same precision.  The hand-scheduled sweep (bf16, 256-row workgroups) fixes
                  m = max(0, bound - 64) for every row whose bound is within 2^174 of its max over the
                  first three key tiles; other waves run the compiled loop; NULL (and no key_norm_max,
                  no key_norm2) = per-tile max.  IGNORED when key_norm_max > 0 (no scan). */
  float key_norm_max; /* optional (bf16 path): > 0 = a static upper bound of |k| (2-norm per head)
                  for every key, used INSTEAD of key_bound (no key scan).  For keys that come out of
                  the qk LayerNorm (attention.py:49-50,78) and RoPE (a rotation), |k| <=
                  sqrt(head_dim) max|w| + |b| of the k_norm affine; 0 = unset */
  int64_t o_bstride; /* output rows per item (o and its rows); 0 = q_bstride.  With q_bstride = 0
                  and k0_bstride = l0 the items split ONE query set's keys into chunks whose
                  normalised partial outputs (o_bstride apart) and LSEs merge with sr_attn_merge_n
                  (key-split attention: more workgroups when the queries alone cannot fill the chip) */
  /* SR_MASK_DENSE / SR_MASK_ADD (f32 path): Attention.forward's general attn_mask
     (attention.py:70,103-109 — F.scaled_dot_product_attention(q, k, v, attn_mask)).  Element
     (item b, head h, query row i, key j; j the logical key index: segment 0 then segment 1) at
     mask + b*mask_bstride + h*mask_hstride + i*mask_ld + j (element strides; 0 = broadcast).
     DENSE: uint8, nonzero = attend (SDPA's bool mask); ADD: fp32 added to scale*q.k before the
     softmax (SDPA's float mask; -inf = masked).  A row with no attended key yields zeros (and
     LSE -inf), as torch's SDPA does since 2.5 (safe softmax). */
  const void* mask;
  int64_t mask_bstride, mask_hstride, mask_ld;
  int32_t tail_rows_readable; /* optional (bf16 path): >= 64 = the caller guarantees at least 64
                  readable rows of finite values past the end of every key segment (K and V; e.g.
                  the next frame's rows or zeroed workspace padding), so the hand-scheduled sweep
                  may stage a ragged last tile whole and mask its extra keys; 0 = unset */
  /* optional merge-in (sr_attention, bf16 path): merge_o holds a result of the SAME query rows over
     a DISJOINT key set, row-normalised bf16 (row r at merge_o + r*ld_merge_o, the head's columns at
     head*head_dim), and merge_lse its log2-domain LSE ([heads][merge_rows]); the row of (item,
     query row i) is item*q_bstride + i.  o then receives the softmax over the union of the key
     sets (sr_attn_merge's formula) and lse, if set, the union's LSE.  NULL = off */
  const void* merge_o;
  int64_t ld_merge_o;
  const float* merge_lse;
  int64_t merge_rows;
  int32_t* sweep_stats; /* optional (bf16 path, diagnostics): two int32 counters the launch ADDS to
                  (atomically, caller zeroes): [0] waves with query rows that ran the hand-scheduled
                  sweep, [1] such waves that ran the compiled loop (a row whose fixed softmax offset
                  falls outside the sweep's 2^174 window, or a launch the sweep does not cover).
                  NULL = off (no extra work) */
  const float* key_box; /* optional (bf16 path, with key_bound or key_norm_max): per key-segment
                  instance and head the per-dimension max and min of the keys, [inst][heads][2][64]
                  fp32 (sr_attention_key_box; instances as key_bound's).  Each row's bound then becomes
                  min(c|q| max|k|, sum_d max(cq_d kmax_d, cq_d kmin_d)) -- far tighter when the keys
                  share a direction (all scores of a row well below the 2-norm bound, which otherwise
                  sends the row outside the fixed-offset window).  NULL = the 2-norm bound alone */
  const float* value_box; /* optional (same path and layout as key_box, sr_attention_key_box run on
                  the values): with max|v| known the fixed-offset window's upper side widens from 2^64
                  to what the launch's fp32 sums allow, 125 - ceil(log2(l0 + l1)) -
                  ceil(log2 max|v|) (at most 100), so rows with a larger gap between their bound and
                  their true score max stay on the hand-scheduled sweep.  NULL = the 2^64 side */
  /* ABI 1.0 */
  const float* key_norm2; /* optional (bf16 path), CALLER-FILLED: per key-segment instance and head
                  (layout as key_bound), max |k|^2 over the keys (sr_attention_key_box's norm2_out).
                  The bound uses sqrt of it, or the smaller of it and key_norm_max when both are set.
                  NULL = unset.  (Before ABI 1.0 this was key_bound's meaning when key_norm_max > 0.) */
  int32_t q_scaled; /* bf16 path: 1 = q already holds c*q, c = scale*log2(e), rounded once to bf16
                  (sr_gemm_epi.q_scale in the QKV / bias epilogue that wrote it), so the kernel uses
                  it as is; 0 = q is plain and the kernel forms c*q itself (a second rounding of
                  q).  sr_attention_qk8 / qkv8 take their q from sr_quant_fp8 and ignore it; the f32
                  kernel and sr_attention_bwd reject 1. */
} sr_attn_desc;

/* floats of key_bound scratch sr_attention needs for d (0 if d does not use it) */
int sr_attention_bound_floats(const sr_attn_desc* d);

/* out[inst][h][0][d] / out[inst][h][1][d] = max / min over rows r < rows of k[inst*inst_stride + r]
 * [h*64 + d] (bf16 keys, head_dim 64; out fp32, n_inst*heads*128 floats): the key box of
 * sr_attn_desc.key_box for one key segment (inst_stride 0 with n_inst 1: keys shared by every item);
 * on the values, sr_attn_desc.value_box.  norm2_out (optional, n_inst*heads floats): max over the rows
 * of |k|^2 per instance and head (fp32 sums of the bf16 squares): sr_attn_desc.key_norm2.  out and
 * norm2_out 16-B aligned (the attention reads the boxes as 16-B vectors).  Two launches (per-workgroup partial boxes in scratch, then their reduction), no atomics.
 * Replaces nothing in the reference: a bound the fixed-offset softmax of attention.py:103-109's
 * replacement uses. */
int sr_attention_key_box(sr_stream_t stream, const void* k, int64_t ldk, int rows, int64_t inst_stride, int n_inst,
                         int heads, float* out, float* norm2_out, float* scratch);
/* floats of scratch (4-B aligned, stream-ordered reuse) sr_attention_key_box needs for the shape */
int sr_attention_key_box_scratch(int rows, int n_inst, int heads);

int sr_attention(sr_stream_t stream, int dtype, const sr_attn_desc* d);

/* Two independent single-query-set bf16 attentions in ONE launch of the hand-scheduled sweep:
 * d0's workgroups are dispatched first, d1's fill the CUs d0 leaves idle in its last round (the
 * C3 global block's anchors against themselves and the split reloc block's queries against the
 * anchor subsample, 10.75 workgroup rounds each).  Each desc as sr_attention's bf16 path with
 * batch 1, one key segment of whole 64-key tiles (>= 4), a static key_norm_max, no mask or
 * merge_o (lse optional), equal head counts; SR_EUNSUPPORTED otherwise (the caller then launches them apart).
 * Replaces the two F.scaled_dot_product_attention calls of one layer's global and global_reloc
 * blocks (attention.py:103-109; aggregator.py:672-769). */
int sr_attention_pair(sr_stream_t stream, int dtype, const sr_attn_desc* d0, const sr_attn_desc* d1);

/* sr_attention_pair with each problem's V given ALSO as pre-transposed tiles (ABI 1.5): vt0 / vt1 from
 * sr_vt_tiles over the desc's v0 (L = l0), 16-B aligned.  The sweep then stages V^T and reads each
 * P.V operand fragment with one ds_read_b128 instead of two transposing reads.  Bit-identical to
 * sr_attention_pair (same products in the same order); v0 is still required and validated. */
int sr_attention_pair_vt(sr_stream_t stream, int dtype, const sr_attn_desc* d0, const sr_attn_desc* d1,
                         const void* vt0, const void* vt1);

/* V bf16 [L][ldv] (heads * 64 columns used) -> V^T tiles [heads][ceil(L/64)][64 d][64 key slots] bf16
 * (ABI 1.5): slot 32kb + 16s2 + 8h + j of a tile holds key 32kb + 16s2 + 8(j >> 2) + 4h + (j & 3) --
 * the bf16 P fragment's k order -- and keys past L are zero.  dst: heads * ceil(L/64) * 8192 bytes.
 * ldv a multiple of 8, v / dst 16-B aligned. */
int sr_vt_tiles(sr_stream_t stream, const void* v, int64_t ldv, int L, int heads, void* dst);

/* Merge two attention results of the same query rows over DISJOINT key sets, given each one's
 * log2-domain LSE ([heads][rows] fp32, as sr_attention writes for batch 1):
 *   out = (2^(la-m) o_a + 2^(lb-m) o_b) / (2^(la-m) + 2^(lb-m)),  m = max(la, lb)
 * i.e. softmax over the union of the keys, exactly.  out may alias o_a or o_b; lse_out
 * (optional, may alias lse_a) receives the union's LSE.  Replaces nothing in the reference:
 * the frame-sharded global block starts on the local anchors' K/V while the
 * remote anchors' K/V are still being all-gathered, then merges (DESIGN.md "Multi-GPU"). */
int sr_attn_merge(sr_stream_t stream, int dtype, int rows, int heads, int head_dim, const void* o_a, int64_t lda,
                  const float* lse_a, const void* o_b, int64_t ldb, const float* lse_b, void* out, int64_t ldo,
                  float* lse_out);
/* The same merge over `parts` (<= SR_ATTN_MERGE_MAX_PARTS) partial results: part p's output rows
 * start at o_parts + p * part_rows * ld (row stride ld); its LSE block of heads * rows floats
 * starts at lse_parts + p * heads * rows, laid out [rows / g][heads][g] with g = lse_seg_rows[p]
 * (g = rows, i.e. [heads][rows], for every part when lse_seg_rows is null): g = rows for the parts
 * of a key-split launch over one query set, g = lq for a batch launch of rows / lq items.  out
 * must not alias o_parts; lse_out ([heads][rows]) optional. */
#define SR_ATTN_MERGE_MAX_PARTS 16
int sr_attn_merge_n(sr_stream_t stream, int dtype, int parts, int rows, int heads, int head_dim, const void* o_parts,
                    int64_t ld, int64_t part_rows, const float* lse_parts, const int* lse_seg_rows, void* out,
                    int64_t ldo, float* lse_out);

/* fp8 (OCP e4m3) quantisation with ONE power-of-two scale per tensor (BASELINE C5, "fp8 QKV";
 * e4m3 Q/K/V with per-tensor scales):
 *   e = ceil(log2(amax(|mul * src|) / 448))   (0 for an all-zero tensor)
 *   dst = e4m3(mul * src * 2^-e),  so  mul * src ~= dst * 2^e.
 * src bf16 [rows][cols] (ld elements), dst bytes [rows][cols] (ldd bytes); *exp_out <- e (device
 * int, read by sr_attention_qk8); workspace: 1 float.  cols, ld, ldd multiples of 8. */
int sr_quant_fp8(sr_stream_t stream, const void* src, int64_t ld, int rows, int cols, float mul, void* dst,
                 int64_t ldd, float* workspace, int* exp_out);

/* Attention (replaces the global block's F.scaled_dot_product_attention, attention.py:103-109) with
 * the score product q.k^T in block-scaled fp8 (v_mfma_scale_f32_32x32x64_f8f6f4, 2x the bf16 MFMA
 * rate): q8 = sr_quant_fp8(q, mul = d->scale * log2(e)) with exponent qk_exp[0], k8 =
 * sr_quant_fp8(k, mul = 1) with exponent qk_exp[1] (device ints).  V, O, lse and all sizes come
 * from d (d->q / d->ldq unused); one key segment, no mask, head_dim 64.  Softmax and P.V as
 * sr_attention's bf16 path. */
int sr_attention_qk8(sr_stream_t stream, const sr_attn_desc* d, const void* q8, int64_t ldq8, const void* k8,
                     int64_t ldk8, const int* qk_exp);

/* V for an fp8 P.V: e4m3 with one power-of-two scale (exponent -> *exp_out, as sr_quant_fp8),
 * transposed into per-(head, 64-key tile) 64 x 64-B tiles [heads][ceil(L/64)][64 d][64 key slots]
 * whose key slots follow the S accumulator's row order (slot 32h + 16kb + r holds key
 * 32kb + (r & 3) + 8 (r >> 2) + 4h), so P needs no lane movement.  v bf16 [L][heads*64];
 * dst heads * ceil(L/64) * 4096 bytes; workspace 1 float. */
int sr_quant_fp8_vt(sr_stream_t stream, const void* v, int64_t ldv, int L, int heads, void* dst, float* workspace,
                    int* exp_out);

/* sr_attention_qk8 with P.V in fp8 too (P in e4m3 unscaled, V from sr_quant_fp8_vt with exponent
 * qkv_exp[2]); one item (the global block: d->batch == 1). */
int sr_attention_qkv8(sr_stream_t stream, const sr_attn_desc* d, const void* q8, int64_t ldq8, const void* k8,
                      int64_t ldk8, const void* v8t, const int* qkv_exp);

/* ------------------------------------------------------------------------
 * Attention backward (training step; the gradient of
 * F.scaled_dot_product_attention in Attention.forward, attention.py:103-109), bf16 inputs,
 * head_dim 64, the same key segments as the forward (frame / global / global_reloc):
 *   delta = rowsum(dO * O);  P = exp2(scale*log2e*q.k - lse);  dS = P * (dO.v - delta)
 *   dQ = scale * dS K,  dK = scale * dS^T Q,  dV = P^T dO      (fp32 outputs)
 * A segment with batch stride 0 (the shared anchor subsample) gets the sum over every
 * item's queries.  delta is caller workspace [batch][heads][lq].
 * ---------------------------------------------------------------------- */
typedef struct sr_attn_bwd_desc {
  sr_attn_desc f;          /* the forward's description (q, k/v segments, o, sizes, scale, lse) */
  const void* dout;        /* dO, bf16, o's layout */
  int64_t lddo;
  float* delta;            /* [batch][heads][lq] workspace */
  float* dq;               /* fp32, q's layout */
  int64_t lddq;
  float* dk0;
  float* dv0;
  int64_t lddk0, lddv0;
  float* dk1;
  float* dv1;
  int64_t lddk1, lddv1;
} sr_attn_bwd_desc;

int sr_attention_bwd(sr_stream_t stream, const sr_attn_bwd_desc* d);

/* The same gradient for fp32 operands (q / k / v / o / dout fp32; head_dim 64 | 128, no mask),
 * exact fp32 on the VALU with the softmax recomputed from the forward's LSE (sr_attention with
 * dtype SR_F32 and lse set): TrainGraph's fp32 mode (ABI 1.2), whose whole-graph gradients are
 * checked against fp32 autograd.  Same outputs and batch-stride-0 summation as sr_attention_bwd. */
int sr_attention_bwd_f32(sr_stream_t stream, const sr_attn_bwd_desc* d);

/* ------------------------------------------------------------------------
 * Training step (train_imc.py:320-429, the backward of every
 * nn.Linear / LayerNorm / LayerScale / qk-norm + RoPE of the Blocks, and the Adam step).
 * ---------------------------------------------------------------------- */

/* Weight gradient of nn.Linear (the addmm backward's mat2 grad, attention.py:48,52 /
 * mlp.py:34-40):  G[N,K] = A[M,N]^T . B[M,K]  (A = dY, B = the layer input; bf16, fp32
 * accumulation), reduction over M split into `splits` slices of fp32 partials in
 * `workspace` (>= splits*N*K floats), then per output row n:
 *   dW[n,:] = (accumulate ? dW[n,:] : 0) + (rowscale ? rowscale[n] : 1) * G[n,:]
 *   rowdot[n] += sum_k wdot[n,k] * G[n,k]          (if rowdot: LayerScale gamma grads,
 *                                                  layer_scale.py:22-23, with G unscaled)
 * N % 128 == 0, K % 128 == 0, M > 0 arbitrary, 16-B aligned rows.  Deterministic. */
int sr_gemm_wgrad(sr_stream_t stream, const void* A, int64_t lda, const void* B, int64_t ldb, float* dW,
                  int64_t lddw, int M, int N, int K, int accumulate, const float* rowscale, const float* wdot,
                  int64_t ldwd, float* rowdot, int splits, float* workspace);

/* One problem of sr_gemm_wgrad_pair: the arguments of sr_gemm_wgrad. */
typedef struct sr_wgrad_problem {
  const void* A;
  int64_t lda;
  const void* B;
  int64_t ldb;
  float* dW;
  int64_t lddw;
  int M, N, K, accumulate;
  const float* rowscale;
  const float* wdot;
  int64_t ldwd;
  float* rowdot;
  int splits;
  float* workspace; /* its own: splits * N * K floats */
} sr_wgrad_problem;

/* Two sr_gemm_wgrad problems of equal N and K (multiples of 256; different rows and weights: the
 * layer's reloc and global blocks) with their M slices in ONE launch of the 256x256 kernel, so each
 * problem can take half the slices and the slices stay long; per problem the same m-tiles, k order
 * and reduction as sr_gemm_wgrad with the same `splits` (bit-identical to it).  Replaces the weight
 * grads of the two blocks' nn.Linear layers in loss.backward() (train_imc.py:404). */
int sr_gemm_wgrad_pair(sr_stream_t stream, const sr_wgrad_problem* problems);

/* Column sums (bias / token / positional-embedding grads):
 *   out[c] = (accumulate ? out[c] : 0) + scale * sum_{r<M} X[r*ldx + c],  c < N (N % 4 == 0).
 * X is `dtype`; two deterministic passes through `workspace` (16-B aligned, workspace_floats >=
 * sr_colsum_workspace_floats(M, N), checked: at most ceil(M / 16) * N and 1024 * N; ABI 1.0 adds the
 * size argument so that a caller sized to an older contract fails with SR_EINVAL, not an
 * out-of-bounds write). */
int64_t sr_colsum_workspace_floats(int M, int N);
int sr_colsum(sr_stream_t stream, int dtype, const void* X, int64_t ldx, int M, int N, float* out, int accumulate,
              float scale, float* workspace, int64_t workspace_floats);
/* The LayerScale residual's parameter grads from one column sum s = sum_r X[r][c] (ABI 1.5):
 *   out1[c] += mul1[c] * s[c],  out2[c] += mul2[c] * s[c]   (either pair may be NULL, not both)
 * -- sr_colsum into a scratch row followed by sr_vec_fma_f32 per pair, in the same two launches the
 * column sum alone takes (bit-identical to that sequence).  Workspace as sr_colsum. */
int sr_colsum_fma(sr_stream_t stream, int dtype, const void* X, int64_t ldx, int M, int N, float* out1,
                  const float* mul1, float* out2, const float* mul2, float* workspace, int64_t workspace_floats);

/* LayerNorm backward (block.py:50,70 norm1 / norm2; vision_transformer.py:300 norm):
 * for row r (x row / dx row = rowmap ? rowmap[r] : r):
 *   xhat = (x - mean) * rstd  (statistics recomputed as sr_layernorm does)
 *   dx  += rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w (w NULL: 1)
 *   dxb[r] = bf16(updated dx row)  (if dxb: the next GEMM operand)
 *   dw  += sum_r dy * xhat,  db += sum_r dy   (if dw / db; accumulate)
 *   dx_colsum[c] = sum_r updated dx[r][c]     (if dx_colsum: assigned; needs dw / db, cols <= 2048 --
 *                  the bias grad of the residual branch that wrote x, without a second pass over dx)
 * dy is `dtype` [rows][lddy].  `workspace` >= 4 * 1024 * cols floats (3 * without dx_colsum).
 * cols in {128,256,384,512,768,1024,1536,2048,4096}.  Rows of one call must map to distinct
 * dx rows. */
int sr_layernorm_bwd(sr_stream_t stream, int dtype, const float* x, int64_t ldx, const int32_t* rowmap,
                     const void* dy, int64_t lddy, const float* w, float eps, float* dx, int64_t lddx, void* dxb,
                     int64_t lddxb, float* dw, float* db, int rows, int cols, float* workspace, float* dx_colsum);

/* qk-norm + 2-D RoPE backward (attention.py:72-82, rope.py:165-207), the inverse of the
 * SR_EPI_QKV epilogue: raw = the saved pre-norm q|k|v (bf16, aux of the forward),
 * dsrc = dq|dk|dv (fp32, from sr_attention_bwd); columns [0, ncols) of each row, column c
 * in region (c + ep->col_offset) / embed_dim (0 = Q, 1 = K, 2 = V):
 *   Q/K: dy = RoPE^T(dsrc); draw = rstd (dy w - mean(dy w) - nhat mean(dy w nhat))
 *        dqn_w += dy nhat, dqn_b += dy (or dkn_*)     (norm params of ep; NULL = no norm)
 *   V:   draw = dsrc
 * out = bf16(draw) [rows][ldo].  ep supplies qn/kn weights, eps, rope tables and the row
 * positions exactly as for the forward GEMM.  grads = fp32 [4][head_dim] accumulators
 * (dqn_w, dqn_b, dkn_w, dkn_b; NULL if no norm).  workspace >= 4352 * 4 * head_dim floats.
 * head_dim 64, ncols % 64 == 0. */
int sr_qk_bwd(sr_stream_t stream, const void* raw, int64_t ldr, const float* dsrc, int64_t lds, void* out,
              int64_t ldo, int rows, int ncols, const sr_gemm_epi* ep, float* grads, float* workspace);

/* ep->colsum (ABI 1.4, optional): also colsum[c] += sum over the rows of out[r][c] (the qkv bias
 * gradient, summed from the values as stored, in a fixed order), ncols <= 3072; the workspace then
 * holds >= sr_qk_bwd_workspace_floats(rows, ncols) floats. */
int64_t sr_qk_bwd_workspace_floats(int rows, int ncols);

/* sr_qk_bwd for fp32 blocks (autocast off: the reference's fp32 Attention with qk_norm / RoPE):
 * raw and out fp32, otherwise identical.  out may alias dsrc (same ld). */
int sr_qk_bwd_f32(sr_stream_t stream, const float* raw, int64_t ldr, const float* dsrc, int64_t lds, float* out,
                  int64_t ldo, int rows, int ncols, const sr_gemm_epi* ep, float* grads, float* workspace);

/* out[r, c] = bf16(scale * src[r, c])  (fp32 -> bf16 GEMM operands), cols % 4 == 0 */
int sr_cast_bf16(sr_stream_t stream, const float* src, int64_t lds, void* dst, int64_t ldd, int rows, int cols,
                 float scale);

/* found_inf |= any(!isfinite(g[i] * inv_scale)) over n values; inv_scale = 1 / *scale
 * (scale NULL: 1).  GradScaler.unscale_'s check (torch.cuda.amp, train_imc.py:406-408). */
int sr_nonfinite_check(sr_stream_t stream, const float* g, int64_t n, const float* scale, int* found_inf);

/* torch.optim.Adam step (train_imc.py:480, betas / eps as given, amsgrad off) over one flat
 * fp32 parameter buffer, skipped entirely if *found_inf (GradScaler.step):
 *   g = grad * inv_scale (+ weight_decay * p);  m = lerp(m, g, 1 - beta1);
 *   v = beta2 v + (1 - beta2) g^2;  p -= (lr / (1 - beta1^t)) m / (sqrt(v) / sqrt(1 - beta2^t) + eps)
 * `step` = t (already incremented). */
int sr_adam_f32(sr_stream_t stream, float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                float beta2, float eps, float weight_decay, int step, const float* scale, const int* found_inf);

/* Per-optimizer-step weight refresh of one block (train/model.py refresh_packs): for each item the
 * fp32 weight src [rows][cols] is read once and written as (cast, if set) its bf16 copy [rows][cols]
 * and (trans, if set) its transposed bf16 copy [cols][rows] with rowscale[r] (if set) folded in --
 * the forward GEMM operand and the dgrad GEMM operand in one launch for up to
 * SR_WEIGHT_REFRESH_MAX weights. */
#define SR_WEIGHT_REFRESH_MAX 4
typedef struct sr_weight_item {
  const float* src;
  int64_t lds;
  int rows, cols;
  const float* rowscale;
  void* cast;
  int64_t ldc;
  void* trans;
  int64_t ldt;
} sr_weight_item;
int sr_weight_refresh_bf16(sr_stream_t stream, int n, const sr_weight_item* items);
/* The whole model's refresh in ONE launch (ABI 1.5): the caller keeps `n` items and their tile
 * prefix in DEVICE memory (static across steps: the flat parameter buffer and the packs do not
 * move).  sr_weight_refresh_plan validates a host copy of the items exactly as
 * sr_weight_refresh_bf16 does and fills start[0..n] (n + 1 ints; start[n] = the launch's tiles);
 * upload both, then sr_weight_refresh_list_bf16(stream, n, items_dev, start_dev, start[n]) per
 * step.  Per item the same tiles and values as sr_weight_refresh_bf16. */
int sr_weight_refresh_plan(int n, const sr_weight_item* items, int* start);
int sr_weight_refresh_list_bf16(sr_stream_t stream, int n, const sr_weight_item* items_dev, const int* start_dev,
                                int tiles);

/* dst[c][r] = out_dtype(rowscale[r] * src[r][c])  (fp32 src [rows][lds]; W^T packs of the dgrad
 * GEMMs with LayerScale gamma folded into W's rows; rowscale may be NULL) */
int sr_transpose_f32(sr_stream_t stream, int out_dtype, const float* src, int64_t lds, int rows, int cols,
                     const float* rowscale, void* dst, int64_t ldd);

/* Camera-head backward (fp32, few rows; camera_head.py:123-186 under autocast off):
 * G[n][k] = sum_m A[m][n] B[m][k];  db[n] (+)= sum_m A[m][n] (db may be NULL);
 * dW = (accumulate ? dW : 0) + (rowscale ? rowscale[n] : 1) G;  rowdot[n] += <wdot[n], G[n]>
 * (rowscale / wdot need workspace >= N*K floats and K % 4 == 0), any N, K otherwise. */
int sr_wgrad_small_f32(sr_stream_t stream, const float* A, int64_t lda, const float* B, int64_t ldb, float* dW,
                       int64_t lddw, int M, int N, int K, int accumulate, float* db, const float* rowscale,
                       const float* wdot, int64_t ldwd, float* rowdot, float* workspace);

/* fp32 attention backward of one item of L <= 1024 rows (q|k|v rows of stride ld, head h at
 * column h*head_dim), mask SR_MASK_NONE or SR_MASK_CAMERA (~build_lr_mask): dq, dk, dv fp32
 * [L][ldg] (written).  Softmax recomputed; workspace >= 2 * heads * L * L floats. */
int sr_attention_bwd_small_f32(sr_stream_t stream, const float* q, const float* k, const float* v, int64_t ld,
                               const float* dout, int64_t lddo, float* dq, float* dk, float* dv, int64_t ldg, int L,
                               int heads, int head_dim, float scale, int mask_mode, int n_anchor, float* workspace);

/* adaLN modulate backward (camera_head.py:156-161): dxn = dxm*gate*(1+scale); dmod [rows][3*cols]
 * = [dxm*gate | dxm*gate*xn | dxm*(xn*(1+scale)+shift)] (the residual dx += dxm is the caller's). */
int sr_adaln_bwd_f32(sr_stream_t stream, const float* xn, const float* mod, const float* dxm, float* dxn, float* dmod,
                     int rows, int cols);

/* dx = dy * act'(x): mode 0 SiLU, 1 erf-GELU (fp32, exact) */
int sr_act_bwd_f32(sr_stream_t stream, int mode, const float* x, const float* dy, float* dx, int64_t n);

/* dst[rowmap[r]] (+)= src[r] for r < rows (fp32 rows, cols % 4 == 0; lds 0 broadcasts one row):
 * the gradient of the aggregator's camera-token reads / special-token writes
 * (aggregator.py:287-299,414-423).  Rows of one call must be distinct. */
int sr_scatter_rows_f32(sr_stream_t stream, float* dst, int64_t ldd, const int32_t* rowmap, const float* src,
                        int64_t lds, int rows, int cols, int accumulate);

/* dst[r][c] (+)= src[r][c], any cols (lds 0 broadcasts one row) */
int sr_copy2d_f32(sr_stream_t stream, float* dst, int64_t ldd, const float* src, int64_t lds, int rows, int cols,
                  int accumulate);

/* activate_pose backward for the camera head's last iteration (head_act.py:12-60; T / quat
 * linear, FoV ReLU): dd [rows][9] = 0 on anchor rows r < n_anchor, else
 * d_act[r - n_anchor] * (c < 7 || act[r][c] > 0); act = the forward's activated encoding. */
int sr_pose_act_bwd_f32(sr_stream_t stream, float* dd, const float* d_act, const float* act, int rows, int n_anchor);

/* out[i] += a[i] * b[i]  (one fused multiply-add) */
int sr_vec_fma_f32(sr_stream_t stream, float* out, const float* a, const float* b, int n);
/* out1[i] += a1[i] * b[i] and out2[i] += a2[i] * b[i] in one launch (ABI 1.5; each as sr_vec_fma_f32) */
int sr_vec_fma2_f32(sr_stream_t stream, float* out1, const float* a1, float* out2, const float* a2, const float* b,
                    int n);

/* Self-supervised IMC loss (compute_loss, train/train_imc.py:141-246; CDFLossIndexPytorch,
 * train/losses/cdf_loss.py:19-242; geometry, train/utils/geometry.py:89-303): value and the
 * gradient with respect to the query views' pose encodings, in one call.
 *   enc      [n_views][9] activated pose encoding (absT_quaR_FoV), image H x W
 *   kp2k     [n_views][3][3] K' -> K recovery matrices; shared_focal averages the recovered K
 *   pairs    src_idx / dst_idx [n_pairs] (views), coords [n_pairs][n_points][2], depths
 *            [n_pairs][n_points]; node_src / node_dst [n_pairs] the CDF histogram of each side
 *            (the reference's module indices; train_epoch builds it on [0] / [0])
 *   CDF      [min_val, max_val) in num_bins bins; smooth_w [2*smooth_radius+1] Gaussian taps
 *   out      loss[0] (device fp32) and d_enc [n_views][9] = grad_scale * dloss/denc
 * workspace >= sr_imc_loss_workspace(...) floats.  n_views <= 64, num_bins <= 1024. */
typedef struct sr_imc_loss_desc {
  const float* enc;
  int n_views, H, W;
  const float* kp2k;
  int shared_focal;
  int n_pairs, n_points;
  const int32_t* src_idx;
  const int32_t* dst_idx;
  const float* src_coords;
  const float* dst_coords;
  const float* src_depth;
  const float* dst_depth;
  const int32_t* node_src;
  const int32_t* node_dst;
  int n_nodes;
  float min_val, max_val;
  int num_bins;
  const float* smooth_w;
  int smooth_radius;
  float grad_scale;
  float* loss;
  float* d_enc;
  float* workspace;
} sr_imc_loss_desc;

int64_t sr_imc_loss_workspace(int n_views, int n_pairs, int n_points, int n_nodes, int num_bins);
int sr_imc_loss(sr_stream_t stream, const sr_imc_loss_desc* desc);

/* ------------------------------------------------------------------------
 * LayerNorm over the last dim of fp32 rows (block.py:50,70; camera_head.py:64-77;
 * vision_transformer.py:192,300).  out_row r = LN(x[rowmap ? rowmap[r] : r]).
 * w/b may be NULL (no affine).  out dtype = out_dtype.  cols % 64 == 0, <= 4096.
 * ---------------------------------------------------------------------- */
int sr_layernorm(sr_stream_t stream, int out_dtype, const float* x, int64_t ldx, const int32_t* rowmap,
                 const float* w, const float* b, float eps, void* out, int64_t ldo, int rows, int cols);
/* sr_layernorm (no rowmap) that also writes each fp32 input row to x_copy (row stride ldc): the
 * training tape's saved block input (engine.run_block_train) without a separate copy pass. */
int sr_layernorm_copy(sr_stream_t stream, int out_dtype, const float* x, int64_t ldx, const float* w, const float* b,
                      float eps, void* out, int64_t ldo, float* x_copy, int64_t ldc, int rows, int cols);

/* ------------------------------------------------------------------------
 * Residual update + LayerNorm (block.py:86-89: x = x + ls1(attn(norm1(x))) then norm2(x)):
 *   x[r] += gamma * y[r]   (fp32 x updated in place; y in `dtype` = the compute dtype, the
 *                           projection GEMM's SR_EPI_BIAS output; gamma NULL = 1)
 *   out[r] = LN(x[r]) * w + b   (out in `dtype`; w/b may both be NULL)
 * cols in {256, 512, 768, 1024, 1536, 2048}; y / out must not alias x.
 * ---------------------------------------------------------------------- */
int sr_residual_layernorm(sr_stream_t stream, int dtype, float* x, int64_t ldx, const void* y, int64_t ldy,
                          const float* gamma, const float* w, const float* b, float eps, void* out, int64_t ldo,
                          int rows, int cols);

/* image normalisation (aggregator.py:267) + 14x14 patch im2col, K zero-padded
 * to kpad: out[(f*gh+py)*gw+px][c*ps*ps + ky*ps + kx]  (patch_embed.py:78) */
int sr_im2col_normalize(sr_stream_t stream, int dtype, const float* img, int frames, int H, int W,
                        int patch, const float* mean3, const float* std3, void* out, int kpad);

/* x[f*tokens_per_frame + t] = table[type_of_frame[f]][t] for t < n_special
 * (aggregator.py:287-299, vision_transformer.py:250-257) */
int sr_set_special_tokens(sr_stream_t stream, float* x, int64_t ldx, int frames, int tokens_per_frame,
                          int n_special, const float* table, const int32_t* type_of_frame, int cols);

/* dst[r] = src[rowmap ? rowmap[r] : r], fp32 rows (aggregator.py:403-423 intermediates) */
int sr_copy_rows_f32(sr_stream_t stream, float* dst, int64_t ldd, const float* src, int64_t lds,
                     const int32_t* rowmap, int rows, int cols);

/* out[r][c] = x[r][c] * gamma[c] (dtype in = out; gamma fp32): LayerScale.forward as a standalone
 * module call (layer_scale.py:22-23).  Inside a Block the scale is fused into the residual GEMM
 * epilogue (SR_EPI_BIAS_RESID). */
int sr_mul_cols(sr_stream_t stream, int dtype, const void* x, int64_t ldx, const float* gamma, void* out, int64_t ldo,
                int rows, int cols);

/* out[M,N] = act_in(A)[M,K] . W[N,K]^T + bias, fp32, any shape (small camera-head
 * linears: embed_pose 9->C, pose_branch.fc2 C/2->9).  act_in: 0 none, 1 SiLU. */
int sr_linear_small_f32(sr_stream_t stream, const float* A, int64_t lda, const float* W, const float* bias,
                        float* out, int64_t ldo, int M, int N, int K, int act_in);

/* elementwise SiLU, fp32 (camera_head.py:72-74) */
int sr_silu_f32(sr_stream_t stream, const float* x, float* y, int64_t n);

/* out = gate*(xn*(1+scale)+shift) + x, mod = [shift|scale|gate] rows of 3*cols
 * (camera_head.py:153-161, modulate :189-194) */
int sr_adaln_modulate_f32(sr_stream_t stream, const float* xn, const float* x, const float* mod,
                          float* out, int rows, int cols);

/* pred = first ? delta : pred + delta; act = activate_pose(pred) with
 * trans/quat linear, fov ReLU (camera_head.py:172-184, head_act.py:12-60) */
int sr_pose_update_f32(sr_stream_t stream, float* pred, const float* delta, int64_t ld_delta, float* act,
                       int rows, int first);

/* 9-d pose encoding -> extrinsic [n,3,4], intrinsic [n,3,3] (pose_enc.py:68-135) */
int sr_pose_decode_f32(sr_stream_t stream, const float* enc, int64_t ld_enc, int n, int H, int W,
                       float* extrinsic, float* intrinsic);

/* ------------------------------------------------------------------------
 * DPT point / depth heads (dpt_head.py:151-349) and depth unprojection (geometry.py:19-130),
 * SURVEY §8(f) rank 1.  Feature maps are NHWC fp32 [n][h][w][c] (c % 4 == 0); convolutions
 * run as sr_gemm (fp32): 1x1 conv = GEMM over pixels, 3x3 conv = sr_im2col3x3_f32 + GEMM with
 * K ordered (ky, kx, ci), ConvTranspose(k, stride k) = GEMM to (ky, kx, co) + scatter.
 * ---------------------------------------------------------------------- */
/* out[n*ho*wo][9c] im2col of a 3x3 / pad 1 / stride 1|2 conv; ReLU on the input when relu_in
 * (ResidualConvUnit, dpt_head.py:470-476).  ho = (h-1)/stride + 1. */
int sr_im2col3x3_f32(sr_stream_t stream, const float* x, int n, int h, int w, int c, int stride, int relu_in,
                     float* out);
/* Implicit-GEMM 3x3 / pad 1 / stride 1|2 conv, fp32 (every 3x3 conv of the DPT heads:
 * layer{1-4}_rn, resize_layers[3], the ResidualConvUnits, output_conv1, output_conv2[0];
 * dpt_head.py:79-108,470-565): out[n*ho*wo][cout] (row stride ldo) = epilogue(im2col(x) . wgt^T)
 * without materialising im2col — the GEMM's LDS-DMA gathers each 32-channel slice of a tap
 * straight from the NHWC input, out-of-image taps from `zero` (>= 128 zero bytes, 16-B aligned,
 * caller-owned).  wgt [cout][9c] with K ordered (ky, kx, ci); relu_in applies ReLU to the input
 * (ResidualConvUnit, dpt_head.py:470-476); epilogue SR_EPI_BIAS (out = acc + bias) or
 * SR_EPI_BIAS_RESID (out += gamma * (acc + bias)).  c % 32 == 0, cout % 4 == 0. */
int sr_conv3x3_f32(sr_stream_t stream, const float* x, int n, int h, int w, int c, int stride, int relu_in,
                   const float* wgt, int cout, int epilogue, const sr_gemm_epi* ep, float* out, int64_t ldo,
                   const float* zero);
/* ConvTranspose2d(kernel = stride = k, pad 0) scatter: g[n*h*w][(ky*k+kx)*co + c] (+ bias[c])
 * -> out[n][h*k][w*k][co]  (dpt_head.py:89-104). */
int sr_convt_scatter_f32(sr_stream_t stream, const float* g, int n, int h, int w, int k, int co, const float* bias,
                         float* out);
/* Bilinear resize, align_corners=True (custom_interpolate, dpt_head.py:568-598), plus an
 * optional `add` table [ho][wo][c] added to every frame (NULL = none): the DPT positional
 * embedding of the upsampled map (dpt_head.py:263-266) fused into the resize.  out must not
 * alias x. */
int sr_resize_bilinear_f32(sr_stream_t stream, const float* x, int n, int h, int w, int c, int ho, int wo,
                           const float* add, float* out);
/* dst += src over n floats (n % 4 == 0): skip_add of FeatureFusionBlock (dpt_head.py:540-545). */
int sr_add_f32(sr_stream_t stream, float* dst, const float* src, int64_t n);
/* x = max(x, 0) in place over n floats: the in-place nn.ReLU at the entry of each
 * ResidualConvUnit, whose skip connection therefore adds relu(x) (dpt_head.py:470-487). */
int sr_relu_f32(sr_stream_t stream, float* x, int64_t n);
/* x += ratio * sincos(uv grid) positional embedding (DPTHead._apply_pos_embed, dpt_head.py:300-315;
 * utils.py create_uv_grid / position_grid_to_embed); aspect = image W / H. */
int sr_dpt_pos_embed_f32(sr_stream_t stream, float* x, int n, int h, int w, int c, float aspect, float ratio);
/* output_conv2[1:] + activate_head (dpt_head.py:285-290, head_act.py:63-127): o = W relu(hidden) + b
 * (W [cout][cin]); preds[p][0..cout-2] = act(o), conf[p] = conf_act(o[cout-1]).
 * act: 0 inv_log, 1 exp, 2 linear, 3 relu;  conf_act: 0 expp1, 1 expp0, 2 sigmoid. */
int sr_dpt_head_out_f32(sr_stream_t stream, const float* hidden, int64_t ldh, int64_t npix, int cin, const float* w,
                        const float* b, int cout, int act, int conf_act, float* preds, float* conf);
/* Depth [s][h][w] -> world points [s][h][w][3] with extrinsic [s][3][4] (cam from world) and
 * intrinsic [s][3][3] (unproject_depth_map_to_point_map, geometry.py:19-130). */
int sr_unproject_depth_f32(sr_stream_t stream, const float* depth, const float* extrinsic, const float* intrinsic,
                           int s, int h, int w, float* out);

/* ------------------------------------------------------------------------------------------
 * Input formation (ImagePreprocessor.process_image_with_matrices, train/utils/io.py:75-153;
 * called per view by datasets/imc2021.py:264-280): zero-pad to a centred square of side
 * `side`, PIL Image.resize((t, t), BICUBIC), ToTensor (RGB / 255) or uint16 depth / 1000.
 * Bit-exact with Pillow's separable resampler.  Tables per axis (host-built, Pillow's filter):
 * bounds[o] = {first input index, tap count}, coeffs[o][ksize] = int32 22-bit fixed point
 * (mode 0, 8-bit) or double (mode 1, 'I;16'); the horizontal pass takes them quad-major.
 * ------------------------------------------------------------------------------------------ */
/* Horizontal pass: img [n][h][w][c] (uint8, mode 0, c <= 4; uint16, mode 1, c == 1) -> planar tmp
 * [n][c][h][ldt] of the same element type, ldt = tw rounded up to a multiple of 4 (columns >= tw
 * are 0).  bounds/coeffs: the w -> tw table in image coordinates (the canvas padding folded in:
 * taps on padding dropped) in quad-major layout, one entry per 4 output columns: bounds int32
 * [ldt/4][2][4] (first indices, tap counts), coeffs [ldt/4][ksize][4] (0 past a column's taps).
 * SR_EUNSUPPORTED for image rows over 64 KiB. */
int sr_pil_resample_h(sr_stream_t stream, int mode, const void* img, int n, int h, int w, int c, const int* bounds,
                      const void* coeffs, int ksize, int tw, void* tmp);
/* Vertical pass + ToTensor: tmp [n][c][rows][ldt] -> out[f * frame_stride + ch * chan_stride + y * ldo + x]
 * = stored value / divisor (255 for RGB, 1000 for depth), fp32, for th output rows (bounds/coeffs:
 * the image-row table [th][2] / [th][ksize], padding folded in like the horizontal one, offset
 * by the first output row for a centre crop). */
int sr_pil_resample_v_f32(sr_stream_t stream, int mode, const void* tmp, int n, int rows, int tw, int c,
                          const int* bounds, const void* coeffs, int ksize, int th, float divisor, float* out,
                          int64_t frame_stride, int64_t chan_stride, int64_t ldo);

/* ImagePreprocessor.reverse_transform_tensor (train/utils/io.py:197-259): a processed (C, h, w) fp32
 * tensor resized back to (hs, ws) with F.interpolate(mode = bicubic (1) | bilinear (0),
 * align_corners=False) and the padding cropped away, fused: out[ch][oy][ox] = resized[ch][oy + y0]
 * [ox + x0] for the (ho, wo) crop (the resized max_side^2 image is never materialised).  torch's
 * index / weight rules (scale in / out, cubic A = -0.75, border-clamped taps). */
int sr_resize_crop_chw_f32(sr_stream_t stream, const float* x, int c, int h, int w, int hs, int ws, int y0, int x0,
                           int ho, int wo, int mode, float* out);

#ifdef __cplusplus
}
#endif

#endif /* SFM_AMD_H */
