// Host-side check of the C ABI, built by `make debug` against an AddressSanitizer +
// UndefinedBehaviorSanitizer build of the library (host code only: -Xarch_host -fsanitize=...;
// SURVEY §5 "race detection / sanitizers").  Needs no GPU: it drives every entry point's argument
// validation and dispatch planning up to the launch (which fails without a device, SR_ELAUNCH),
// so ASan / UBSan see the host paths the Python mirror takes.
//
//   abi_host_check layout   JSON: size and field offsets of every ABI struct (tests/test_abi.py
//                           compares them with the ctypes mirror in sailrecon_amd/_lib.py)
//   abi_host_check check    the validation sweep; exit 0 iff every call returned what it should
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sfm_amd.h"

namespace {

int g_fail = 0;

void expect(const char* what, int rc, bool ok_launch_fail) {
  // rc < 0 always (no device: a call that passes validation fails at its launch, SR_ELAUNCH);
  // a validation failure must say why
  const char* msg = sr_last_error();
  bool good = rc < 0 && msg && *msg;
  if (!ok_launch_fail && rc == SR_ELAUNCH) good = false;  // should have been rejected before launching
  std::printf("%-44s rc=%d  %s%s\n", what, rc, good ? "" : "UNEXPECTED  ", msg ? msg : "(null)");
  if (!good) ++g_fail;
}

// fake, suitably aligned device addresses: validation never dereferences them
template <typename T = void>
T* fake(uintptr_t i) { return reinterpret_cast<T*>(0x7f0000000000ull + (i << 12)); }

#define FIELD(S, F) std::printf("%s\"%s\": %zu", first ? "" : ", ", #F, offsetof(S, F)), first = false
#define STRUCT(S, BODY)                                                 \
  do {                                                                  \
    bool first = true;                                                  \
    std::printf("%s\"%s\": {\"size\": %zu, \"fields\": {", sep, #S, sizeof(S)); \
    BODY;                                                               \
    std::printf("}}");                                                  \
    sep = ", ";                                                         \
  } while (0)

void layout() {
  const char* sep = "";
  std::printf("{");
  STRUCT(sr_gemm_epi, (FIELD(sr_gemm_epi, bias), FIELD(sr_gemm_epi, gamma), FIELD(sr_gemm_epi, qn_w),
                       FIELD(sr_gemm_epi, qn_b), FIELD(sr_gemm_epi, kn_w), FIELD(sr_gemm_epi, kn_b),
                       FIELD(sr_gemm_epi, qk_eps), FIELD(sr_gemm_epi, rope_cos), FIELD(sr_gemm_epi, rope_sin),
                       FIELD(sr_gemm_epi, rope_npos), FIELD(sr_gemm_epi, col_offset), FIELD(sr_gemm_epi, head_dim),
                       FIELD(sr_gemm_epi, embed_dim), FIELD(sr_gemm_epi, pos_yx), FIELD(sr_gemm_epi, pos_rowmap),
                       FIELD(sr_gemm_epi, pos_row_base), FIELD(sr_gemm_epi, tokens_per_frame),
                       FIELD(sr_gemm_epi, patch_start), FIELD(sr_gemm_epi, grid_w), FIELD(sr_gemm_epi, seg_rows),
                       FIELD(sr_gemm_epi, seg_stride), FIELD(sr_gemm_epi, seg_offset), FIELD(sr_gemm_epi, row_add),
                       FIELD(sr_gemm_epi, aux), FIELD(sr_gemm_epi, ld_aux), FIELD(sr_gemm_epi, q_scale),
                       FIELD(sr_gemm_epi, q_cols), FIELD(sr_gemm_epi, colsum)));
  STRUCT(sr_gemm_problem, (FIELD(sr_gemm_problem, A), FIELD(sr_gemm_problem, lda), FIELD(sr_gemm_problem, W),
                           FIELD(sr_gemm_problem, ldw), FIELD(sr_gemm_problem, out), FIELD(sr_gemm_problem, ldo),
                           FIELD(sr_gemm_problem, M), FIELD(sr_gemm_problem, N), FIELD(sr_gemm_problem, K),
                           FIELD(sr_gemm_problem, ep)));
  STRUCT(sr_wgrad_problem,
         (FIELD(sr_wgrad_problem, A), FIELD(sr_wgrad_problem, lda), FIELD(sr_wgrad_problem, B),
          FIELD(sr_wgrad_problem, ldb), FIELD(sr_wgrad_problem, dW), FIELD(sr_wgrad_problem, lddw),
          FIELD(sr_wgrad_problem, M), FIELD(sr_wgrad_problem, N), FIELD(sr_wgrad_problem, K),
          FIELD(sr_wgrad_problem, accumulate), FIELD(sr_wgrad_problem, rowscale), FIELD(sr_wgrad_problem, wdot),
          FIELD(sr_wgrad_problem, ldwd), FIELD(sr_wgrad_problem, rowdot), FIELD(sr_wgrad_problem, splits),
          FIELD(sr_wgrad_problem, workspace)));
  STRUCT(sr_attn_desc,
         (FIELD(sr_attn_desc, q), FIELD(sr_attn_desc, ldq), FIELD(sr_attn_desc, k0), FIELD(sr_attn_desc, v0),
          FIELD(sr_attn_desc, ldk0), FIELD(sr_attn_desc, ldv0), FIELD(sr_attn_desc, k1), FIELD(sr_attn_desc, v1),
          FIELD(sr_attn_desc, ldk1), FIELD(sr_attn_desc, ldv1), FIELD(sr_attn_desc, o), FIELD(sr_attn_desc, ldo),
          FIELD(sr_attn_desc, batch), FIELD(sr_attn_desc, heads), FIELD(sr_attn_desc, head_dim),
          FIELD(sr_attn_desc, lq), FIELD(sr_attn_desc, q_bstride), FIELD(sr_attn_desc, l0),
          FIELD(sr_attn_desc, k0_bstride), FIELD(sr_attn_desc, l1), FIELD(sr_attn_desc, k1_bstride),
          FIELD(sr_attn_desc, mask_mode), FIELD(sr_attn_desc, n_anchor), FIELD(sr_attn_desc, scale),
          FIELD(sr_attn_desc, lse), FIELD(sr_attn_desc, key_bound), FIELD(sr_attn_desc, key_norm_max),
          FIELD(sr_attn_desc, o_bstride), FIELD(sr_attn_desc, mask), FIELD(sr_attn_desc, mask_bstride),
          FIELD(sr_attn_desc, mask_hstride), FIELD(sr_attn_desc, mask_ld), FIELD(sr_attn_desc, tail_rows_readable),
          FIELD(sr_attn_desc, merge_o), FIELD(sr_attn_desc, ld_merge_o), FIELD(sr_attn_desc, merge_lse),
          FIELD(sr_attn_desc, merge_rows), FIELD(sr_attn_desc, sweep_stats),
          FIELD(sr_attn_desc, key_box), FIELD(sr_attn_desc, value_box), FIELD(sr_attn_desc, key_norm2),
          FIELD(sr_attn_desc, q_scaled)));
  STRUCT(sr_attn_bwd_desc,
         (FIELD(sr_attn_bwd_desc, f), FIELD(sr_attn_bwd_desc, dout), FIELD(sr_attn_bwd_desc, lddo),
          FIELD(sr_attn_bwd_desc, delta), FIELD(sr_attn_bwd_desc, dq), FIELD(sr_attn_bwd_desc, lddq),
          FIELD(sr_attn_bwd_desc, dk0), FIELD(sr_attn_bwd_desc, dv0), FIELD(sr_attn_bwd_desc, lddk0),
          FIELD(sr_attn_bwd_desc, lddv0), FIELD(sr_attn_bwd_desc, dk1), FIELD(sr_attn_bwd_desc, dv1),
          FIELD(sr_attn_bwd_desc, lddk1), FIELD(sr_attn_bwd_desc, lddv1)));
  STRUCT(sr_imc_loss_desc,
         (FIELD(sr_imc_loss_desc, enc), FIELD(sr_imc_loss_desc, n_views), FIELD(sr_imc_loss_desc, H),
          FIELD(sr_imc_loss_desc, W), FIELD(sr_imc_loss_desc, kp2k), FIELD(sr_imc_loss_desc, shared_focal),
          FIELD(sr_imc_loss_desc, n_pairs), FIELD(sr_imc_loss_desc, n_points), FIELD(sr_imc_loss_desc, src_idx),
          FIELD(sr_imc_loss_desc, dst_idx), FIELD(sr_imc_loss_desc, src_coords), FIELD(sr_imc_loss_desc, dst_coords),
          FIELD(sr_imc_loss_desc, src_depth), FIELD(sr_imc_loss_desc, dst_depth), FIELD(sr_imc_loss_desc, node_src),
          FIELD(sr_imc_loss_desc, node_dst), FIELD(sr_imc_loss_desc, n_nodes), FIELD(sr_imc_loss_desc, min_val),
          FIELD(sr_imc_loss_desc, max_val), FIELD(sr_imc_loss_desc, num_bins), FIELD(sr_imc_loss_desc, smooth_w),
          FIELD(sr_imc_loss_desc, smooth_radius), FIELD(sr_imc_loss_desc, grad_scale), FIELD(sr_imc_loss_desc, loss),
          FIELD(sr_imc_loss_desc, d_enc), FIELD(sr_imc_loss_desc, workspace)));
  STRUCT(sr_weight_item,
         (FIELD(sr_weight_item, src), FIELD(sr_weight_item, lds), FIELD(sr_weight_item, rows),
          FIELD(sr_weight_item, cols), FIELD(sr_weight_item, rowscale), FIELD(sr_weight_item, cast),
          FIELD(sr_weight_item, ldc), FIELD(sr_weight_item, trans), FIELD(sr_weight_item, ldt)));
  std::printf("}\n");
}

sr_attn_desc attn(int batch, int heads, int lq, int l0, int l1) {
  sr_attn_desc d;
  std::memset(&d, 0, sizeof(d));
  d.q = fake(1);
  d.k0 = fake(2);
  d.v0 = fake(3);
  d.o = fake(4);
  d.ldq = d.ldk0 = d.ldv0 = d.ldo = heads * 64 * 3;
  d.batch = batch;
  d.heads = heads;
  d.head_dim = 64;
  d.lq = lq;
  d.q_bstride = lq;
  d.l0 = l0;
  d.l1 = l1;
  if (l1) {
    d.k1 = fake(5);
    d.v1 = fake(6);
    d.ldk1 = d.ldv1 = d.ldk0;
    d.k1_bstride = l1;
  }
  d.scale = 0.125f;
  return d;
}

void check() {
  // ---- tuning table and strings
  if (sr_version() < (1 << 16)) ++g_fail;
  for (int k = 0; k < SR_TUNE_COUNT; ++k) {
    const char* n = sr_tuning_name(k);
    const int v = sr_get_tuning(k);
    if (!n || sr_set_tuning(k, v + 1) != v || sr_get_tuning(k) != v + 1 || sr_set_tuning(k, v) != v + 1) ++g_fail;
  }
  if (sr_tuning_name(SR_TUNE_COUNT) || sr_set_tuning(SR_TUNE_COUNT, 0) != SR_EINVAL || sr_get_tuning(-1) != SR_EINVAL)
    ++g_fail;
  std::printf("tuning table: %d switches\n", (int)SR_TUNE_COUNT);

  sr_gemm_epi ep;
  std::memset(&ep, 0, sizeof(ep));
  // ---- GEMM: rejected shapes, then the planned paths of every epilogue / size class
  expect("sr_gemm null A", sr_gemm(nullptr, SR_BF16, SR_EPI_BIAS, nullptr, 64, fake(1), 64, fake(2), 64, 8, 64, 64, &ep), false);
  expect("sr_gemm N % 4", sr_gemm(nullptr, SR_BF16, SR_EPI_BIAS, fake(0), 64, fake(1), 64, fake(2), 66, 8, 66, 64, &ep), false);
  expect("sr_gemm K % 64", sr_gemm(nullptr, SR_BF16, SR_EPI_BIAS, fake(0), 96, fake(1), 96, fake(2), 64, 8, 64, 96, &ep), false);
  expect("sr_gemm RESID without gamma", sr_gemm(nullptr, SR_BF16, SR_EPI_BIAS_RESID, fake(0), 64, fake(1), 64, fake(2), 64, 8, 64, 64, &ep), false);
  expect("sr_gemm bad epilogue", sr_gemm(nullptr, SR_BF16, 42, fake(0), 64, fake(1), 64, fake(2), 64, 8, 64, 64, &ep), true);
  ep.gamma = fake<float>(9);
  const int Ms[] = {1, 64, 300, 87936};
  const int Ns[] = {256, 1024, 3072, 4096};
  for (int M : Ms)
    for (int N : Ns)
      for (int epi : {SR_EPI_BIAS, SR_EPI_BIAS_GELU, SR_EPI_BIAS_RESID, SR_EPI_F32}) {
        char what[96];
        std::snprintf(what, sizeof(what), "sr_gemm bf16 epi %d M %d N %d", epi, M, N);
        expect(what, sr_gemm(nullptr, SR_BF16, epi, fake(0), 1024, fake(1), 1024, fake(2), N, M, N, 1024, &ep), true);
        std::snprintf(what, sizeof(what), "sr_gemm f32 epi %d M %d N %d", epi, M, N);
        expect(what, sr_gemm(nullptr, SR_F32, epi, fake(0), 1024, fake(1), 1024, fake(2), N, M, N, 1024, &ep), true);
      }
  ep.q_scale = 0.18f;  // ABI 1.0: the Q block of a BIAS / QKV output leaves scaled
  ep.q_cols = 1024;
  expect("sr_gemm BIAS q_scale", sr_gemm(nullptr, SR_BF16, SR_EPI_BIAS, fake(0), 1024, fake(1), 1024, fake(2), 3072, 87936, 3072, 1024, &ep), true);
  expect("sr_gemm RESID q_scale", sr_gemm(nullptr, SR_BF16, SR_EPI_BIAS_RESID, fake(0), 1024, fake(1), 1024, fake(2), 3072, 87936, 3072, 1024, &ep), false);
  ep.q_cols = 100;
  expect("sr_gemm q_cols not a multiple of 64", sr_gemm(nullptr, SR_BF16, SR_EPI_BIAS, fake(0), 1024, fake(1), 1024, fake(2), 3072, 87936, 3072, 1024, &ep), false);
  ep.q_scale = 0.f;
  ep.q_cols = 0;
  expect("sr_gemm_splitk 3 slices of 16 tiles", sr_gemm_splitk(nullptr, SR_BF16, SR_EPI_BIAS, fake(0), 1024, fake(1), 1024, fake(2), 1024, 64, 1024, 1024, 3, fake<float>(3), &ep), false);
  expect("sr_gemm_splitk 4 slices", sr_gemm_splitk(nullptr, SR_BF16, SR_EPI_BIAS, fake(0), 1024, fake(1), 1024, fake(2), 1024, 64, 1024, 1024, 4, fake<float>(3), &ep), true);
  std::vector<sr_gemm_problem> pr(5);
  for (auto& p : pr) {
    std::memset(&p, 0, sizeof(p));
    p.A = fake(0);
    p.W = fake(1);
    p.out = fake(2);
    p.lda = p.ldw = 1024;
    p.ldo = 3072;
    p.M = 43968;
    p.N = 3072;
    p.K = 1024;
    p.ep = ep;
  }
  expect("sr_gemm_group 5 problems", sr_gemm_group(nullptr, SR_BF16, SR_EPI_BIAS, 5, pr.data()), false);
  expect("sr_gemm_group 3 problems", sr_gemm_group(nullptr, SR_BF16, SR_EPI_BIAS, 3, pr.data()), true);
  pr[1].N = 1000;
  pr[1].ldo = 1000;
  expect("sr_gemm_group N % 256", sr_gemm_group(nullptr, SR_BF16, SR_EPI_BIAS, 3, pr.data()), false);

  // ---- attention: every dispatch class of the bf16 and f32 paths
  sr_attn_desc d = attn(1, 16, 43968, 43968, 0);
  expect("sr_attention null desc", sr_attention(nullptr, SR_BF16, nullptr), false);
  d.k0 = nullptr;
  expect("sr_attention null k0", sr_attention(nullptr, SR_BF16, &d), false);
  d = attn(1, 16, 43968, 43968, 0);
  d.head_dim = 128;
  expect("sr_attention bf16 head_dim 128", sr_attention(nullptr, SR_BF16, &d), false);
  d = attn(1, 16, 43968, 43968, 0);
  d.key_norm_max = 40.f;
  expect("sr_attention global (asm sweep)", sr_attention(nullptr, SR_BF16, &d), true);
  d.key_norm_max = 0.f;
  d.key_bound = fake<float>(7);
  expect("sr_attention global, key scan", sr_attention(nullptr, SR_BF16, &d), true);
  // ABI 1.0: the caller-filled norms have their own field; boxes need a bound and 16-B alignment
  d = attn(1, 16, 43968, 43968, 0);
  d.key_norm_max = 40.f;
  d.key_norm2 = fake<float>(10);
  d.key_box = fake<float>(11);
  d.value_box = fake<float>(12);
  d.q_scaled = 1;
  expect("sr_attention global, key_norm2 + boxes + q_scaled", sr_attention(nullptr, SR_BF16, &d), true);
  d.key_box = (const float*)((const char*)fake<float>(11) + 4);
  expect("sr_attention misaligned key_box", sr_attention(nullptr, SR_BF16, &d), false);
  d.key_box = fake<float>(11);
  d.key_norm_max = 0.f;
  d.key_norm2 = nullptr;
  expect("sr_attention boxes without a bound", sr_attention(nullptr, SR_BF16, &d), false);
  d = attn(4, 16, 300, 300, 0);
  d.q_scaled = 1;
  expect("sr_attention f32 q_scaled", sr_attention(nullptr, SR_F32, &d), false);
  d.q_scaled = 2;
  expect("sr_attention bf16 q_scaled 2", sr_attention(nullptr, SR_BF16, &d), false);
  d = attn(64, 16, 1374, 1374, 0);
  d.k0_bstride = 1374;
  expect("sr_attention frame", sr_attention(nullptr, SR_BF16, &d), true);
  d = attn(32, 16, 1374, 9760, 1374);
  d.tail_rows_readable = 64;
  expect("sr_attention reloc (two segments)", sr_attention(nullptr, SR_BF16, &d), true);
  d.merge_o = fake(8);
  d.merge_lse = fake<float>(9);
  d.merge_rows = 32 * 1374;
  d.ld_merge_o = 1024;
  expect("sr_attention reloc merge-in", sr_attention(nullptr, SR_BF16, &d), true);
  d.merge_rows = 0;
  expect("sr_attention merge-in without rows", sr_attention(nullptr, SR_BF16, &d), false);
  d = attn(4, 16, 300, 300, 0);
  expect("sr_attention f32 short", sr_attention(nullptr, SR_F32, &d), true);
  d = attn(1, 16, 64, 64, 0);
  d.head_dim = 128;
  d.mask_mode = SR_MASK_CAMERA;
  d.n_anchor = 32;
  expect("sr_attention f32 camera mask", sr_attention(nullptr, SR_F32, &d), true);
  d.mask_mode = SR_MASK_DENSE;
  expect("sr_attention dense mask without mask", sr_attention(nullptr, SR_F32, &d), false);
  d.mask_mode = 7;
  expect("sr_attention bad mask mode", sr_attention(nullptr, SR_F32, &d), false);
  sr_attn_desc a = attn(1, 16, 43968, 43968, 0), b = attn(1, 16, 43968, 9728, 0);
  a.key_norm_max = b.key_norm_max = 40.f;
  expect("sr_attention_pair", sr_attention_pair(nullptr, SR_BF16, &a, &b), true);
  expect("sr_attention_pair_vt null tiles", sr_attention_pair_vt(nullptr, SR_BF16, &a, &b, fake(0), nullptr), false);
  expect("sr_vt_tiles null", sr_vt_tiles(nullptr, nullptr, 3072, 64, 16, nullptr), false);
  b.l0 = 9760;
  expect("sr_attention_pair ragged keys", sr_attention_pair(nullptr, SR_BF16, &a, &b), false);
  b = attn(1, 8, 43968, 9728, 0);
  b.key_norm_max = 40.f;
  expect("sr_attention_pair head counts", sr_attention_pair(nullptr, SR_BF16, &a, &b), false);
  d = attn(1, 16, 43968, 43968, 0);
  std::printf("bound floats: %d\n", sr_attention_bound_floats(&d));
  std::printf("key box scratch floats: %d\n", sr_attention_key_box_scratch(43968, 1, 16));
  expect("sr_attention_key_box", sr_attention_key_box(nullptr, fake(0), 3072, 43968, 0, 1, 16, fake<float>(1),
                                                      fake<float>(2), fake<float>(3)), true);
  expect("sr_attention_key_box null scratch", sr_attention_key_box(nullptr, fake(0), 3072, 43968, 0, 1, 16,
                                                                   fake<float>(1), nullptr, nullptr), false);
  expect("sr_attention_key_box 33 heads", sr_attention_key_box(nullptr, fake(0), 3072, 100, 0, 1, 33, fake<float>(1),
                                                               nullptr, fake<float>(3)), false);
  expect("sr_attention_key_box overlapping instances", sr_attention_key_box(nullptr, fake(0), 1024, 1374, 1000, 64,
                                                                             16, fake<float>(1), nullptr,
                                                                             fake<float>(3)), false);

  // ---- merges
  const int seg[SR_ATTN_MERGE_MAX_PARTS] = {43968, 1374};
  expect("sr_attn_merge_n", sr_attn_merge_n(nullptr, SR_BF16, 2, 43968, 16, 64, fake(0), 1024, 43968, fake<float>(1), seg, fake(2), 1024, nullptr), true);
  expect("sr_attn_merge_n 17 parts", sr_attn_merge_n(nullptr, SR_BF16, 17, 43968, 16, 64, fake(0), 1024, 43968, fake<float>(1), nullptr, fake(2), 1024, nullptr), false);
  const int bad_seg[SR_ATTN_MERGE_MAX_PARTS] = {43968, 1000};
  expect("sr_attn_merge_n seg rows", sr_attn_merge_n(nullptr, SR_BF16, 2, 43968, 16, 64, fake(0), 1024, 43968, fake<float>(1), bad_seg, fake(2), 1024, nullptr), false);
  expect("sr_attn_merge", sr_attn_merge(nullptr, SR_BF16, 100, 16, 64, fake(0), 1024, fake<float>(1), fake(2), 1024, fake<float>(3), fake(4), 1024, nullptr), true);

  // ---- the rest of the ABI: null / empty arguments are rejected, never dereferenced
  expect("sr_layernorm null", sr_layernorm(nullptr, SR_BF16, nullptr, 1024, nullptr, nullptr, nullptr, 1e-5f, nullptr, 1024, 0, 1024), false);
  expect("sr_layernorm", sr_layernorm(nullptr, SR_BF16, fake<float>(0), 1024, nullptr, fake<float>(1), fake<float>(2), 1e-5f, fake(3), 1024, 87936, 1024), true);
  expect("sr_quant_fp8 null", sr_quant_fp8(nullptr, nullptr, 8, 8, 8, 1.f, nullptr, 8, nullptr, nullptr), false);
  expect("sr_attention_qk8 null", sr_attention_qk8(nullptr, nullptr, nullptr, 0, nullptr, 0, nullptr), false);
  expect("sr_attention_qkv8 null", sr_attention_qkv8(nullptr, nullptr, nullptr, 0, nullptr, 0, nullptr, nullptr), false);
  expect("sr_colsum_fma no pair", sr_colsum_fma(nullptr, SR_F32, fake(0), 8, 8, 8, nullptr, nullptr, nullptr, nullptr,
                                                   fake<float>(1), 1 << 20), false);
  expect("sr_vec_fma2_f32 null", sr_vec_fma2_f32(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 8), false);
  expect("sr_quant_fp8_vt null", sr_quant_fp8_vt(nullptr, nullptr, 8, 8, 1, nullptr, nullptr, nullptr), false);
  expect("sr_attention_bwd null", sr_attention_bwd(nullptr, nullptr), false);
  expect("sr_attention_bwd_f32 null", sr_attention_bwd_f32(nullptr, nullptr), false);
  if (sr_qk_bwd_workspace_floats(43968, 3072) < 1024LL * 3072 || sr_qk_bwd_workspace_floats(0, 3072) != 0) ++g_fail;
  expect("sr_gemm_wgrad null", sr_gemm_wgrad(nullptr, nullptr, 0, nullptr, 0, nullptr, 0, 0, 0, 0, 0, nullptr, nullptr, 0, nullptr, 0, nullptr), false);
  expect("sr_colsum null", sr_colsum(nullptr, SR_F32, nullptr, 0, 0, 0, nullptr, 0, 1.f, nullptr, 0), false);
  {  // ABI 1.0: the workspace size is checked against sr_colsum_workspace_floats
    const int64_t need = sr_colsum_workspace_floats(87936, 1024);
    if (need <= 0 || need > 1024LL * 1024) ++g_fail;
    expect("sr_colsum workspace one float short",
           sr_colsum(nullptr, SR_F32, fake(1), 1024, 87936, 1024, fake<float>(2), 0, 1.f, fake<float>(3), need - 1), false);
    expect("sr_colsum sized workspace",
           sr_colsum(nullptr, SR_F32, fake(1), 1024, 87936, 1024, fake<float>(2), 0, 1.f, fake<float>(3), need), true);
  }
  expect("sr_imc_loss null", sr_imc_loss(nullptr, nullptr), false);
  std::printf("imc workspace floats: %lld\n", (long long)sr_imc_loss_workspace(4, 3, 1024, 1, 100));
  expect("sr_pose_decode_f32 null", sr_pose_decode_f32(nullptr, nullptr, 9, 0, 518, 518, nullptr, nullptr), false);
  expect("sr_copy_rows_f32 null", sr_copy_rows_f32(nullptr, nullptr, 0, nullptr, 0, nullptr, 0, 0), false);
  expect("sr_conv3x3_f32 null", sr_conv3x3_f32(nullptr, nullptr, 1, 8, 8, 32, 1, 0, nullptr, 32, SR_EPI_BIAS, &ep, nullptr, 32, nullptr), false);
  sr_weight_item wi{};
  expect("sr_weight_refresh_bf16 0 items", sr_weight_refresh_bf16(nullptr, 0, &wi), false);
  expect("sr_weight_refresh_bf16 no outputs", sr_weight_refresh_bf16(nullptr, 1, &wi), false);
  wi.src = fake<float>(0);
  wi.lds = 1024;
  wi.rows = 3072;
  wi.cols = 1024;
  wi.cast = fake(1);
  wi.ldc = 1024;
  wi.trans = fake(2);
  wi.ldt = 3072;
  expect("sr_weight_refresh_bf16", sr_weight_refresh_bf16(nullptr, 1, &wi), true);
  {
    sr_weight_item two[2] = {wi, wi};
    int start[3] = {-1, -1, -1};
    const int rc = sr_weight_refresh_plan(2, two, start);  // host-only: SR_OK
    const bool ok = rc == SR_OK && start[0] == 0 && start[1] == 768 && start[2] == 1536;
    std::printf("%-44s rc=%d  %sprefix %d %d %d\n", "sr_weight_refresh_plan", rc, ok ? "" : "UNEXPECTED  ", start[0],
                start[1], start[2]);
    if (!ok) ++g_fail;
    two[1].trans = nullptr;
    two[1].cast = nullptr;
    expect("sr_weight_refresh_plan no outputs", sr_weight_refresh_plan(2, two, start), false);
    expect("sr_weight_refresh_list_bf16 empty", sr_weight_refresh_list_bf16(nullptr, 0, nullptr, nullptr, 0), false);
  }
  expect("sr_im2col_normalize null", sr_im2col_normalize(nullptr, SR_BF16, nullptr, 0, 518, 518, 14, nullptr, nullptr, nullptr, 0), false);
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "check";
  if (mode == "layout") {
    layout();
    return 0;
  }
  check();
  std::printf("%s: %d unexpected result(s)\n", g_fail ? "FAIL" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
