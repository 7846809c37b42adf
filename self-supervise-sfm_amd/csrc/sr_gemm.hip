// GEMM  out = epilogue(A[M,K] . W[N,K]^T)  for gfx950.
//
// Replaces nn.Linear (addmm) on the hot path: qkv / proj (attention.py:48,52,73,120),
// fc1 / fc2 (mlp.py:34-40) and the patch-embed conv as an im2col GEMM
// (patch_embed.py:62-64,78).  Both operands are K-contiguous ("NT"), which is the
// natural MFMA operand layout: every lane reads 16 contiguous bytes of one row.
//
// Structure (v1):
//   * 128x128 output tile per 256-thread workgroup, 4 waves as 2x2, 64x64 per wave;
//   * K staged 128 bytes per row per k-tile (64 bf16 / 32 f32) by LDS-DMA
//     (global_load_lds_dwordx4), double-buffered; the next tile's DMA stays in flight
//     across the raw s_barrier (counted vmcnt, cdna_hip_programming.md §5);
//   * LDS rows XOR-swizzled (16-B chunk ^= (row>>1)&7) on the DMA SOURCE address and on
//     the ds_read_b128 address, conflict-free for the MFMA fragment pattern;
//   * bf16: v_mfma_f32_16x16x32_bf16, one per 16-B chunk pair;
//     f32 (parity mode): four v_mfma_f32_16x16x4_f32 per chunk pair — exact fp32;
//   * bijective XCD-aware tile remap so tiles that share A rows share an L2;
//   * epilogues fused in registers: bias, erf-GELU, LayerScale+residual, patch remap +
//     positional add, and qk-LayerNorm + 2-D RoPE (each wave owns one 64-wide head).
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include <type_traits>

#include "sr_common.h"

namespace {

constexpr int BM = 128, BN = 128;
constexpr int ROWB = 128;                     // bytes per tile row per k-tile
constexpr int NTHREADS = 256;
constexpr int BIG = 256;                      // the 256x256 kernels' tile
constexpr int STAGE_BIG = 2 * BIG * ROWB;     // their K stage: 64 KiB

struct GemmArgs {
  const char* A;
  int64_t lda_b;
  const char* W;
  int64_t ldw_b;
  void* out;
  int64_t ldo;
  int M, N, K, ktiles;
  int lds_epi;  // 256x256 kernels: stage the epilogue through LDS (outputs 16-B aligned rows)
  int kt_per_split;  // split-K (gemm_kernel, gridDim.y slices): k-tiles per slice
  float* partial;    // split-K: [slices][M][N] fp32 partial tiles (epilogue runs in the reduction)
  int group_m;       // 256x256 kernels: tile order in groups of group_m row tiles (<= 1: row-major)
  int resid_lds;     // 256x256 RESID: the x tile staged through LDS by LDS-DMA (SR_TUNE_GEMM_RESID_LDS)
  int rope_lds;      // 256x256 QKV: RoPE tables staged in LDS (SR_TUNE_GEMM_ROPE_LDS)
  sr_gemm_epi ep;
  // implicit-GEMM 3x3 / pad-1 conv (gemm_kernel<float, EPI, true>): A row m = output pixel
  // (n, yo, xo) of the NHWC fp32 input x [n][H][W][C], A column k = (ky, kx, ci) — exactly
  // the im2col row, gathered by the LDS-DMA itself (out-of-image taps read `zero`)
  struct {
    const char* x;
    const char* zero;  // >= 128 bytes of zeros
    int H, W, C, Ho, Wo, stride, relu;
  } conv;
};

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static constexpr int KT = 64;
  __device__ __forceinline__ static void run(const uint4& a, const uint4& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                0, 0, 0);
  }
};
template <> struct Mma<float> {
  static constexpr int KT = 32;
  // lane group g holds k = 4*(chunk) + j; MFMA j consumes element j of every lane's chunk:
  // A and B use the same k permutation, so the sum over (g, j) covers the chunk exactly.
  __device__ __forceinline__ static void run(const uint4& a, const uint4& b, f32x4& c) {
    const f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[0], fb[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[1], fb[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[2], fb[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[3], fb[3], c, 0, 0, 0);
  }
};

// Element types the epilogues store: RESID / F32 / PATCH write fp32 whatever the operand type,
// the others the operand type; the saved pre-activation (sr_gemm_epi.aux) has the operand type.
template <typename T, int EPI>
using OutT = std::conditional_t<EPI == SR_EPI_BIAS_RESID || EPI == SR_EPI_F32 || EPI == SR_EPI_PATCH, float, T>;
template <typename T>
using AuxT = T;

// Fused epilogue on C^T accumulator tiles: acc[mi][ni] covers output rows
// rowbase + mi*16 + lr and the 4 consecutive columns colw + ni*16 + 4*lg + r.
// Final per-lane values of every epilogue but PATCH, handed to emit(row, col, v[4]):
//   BIAS acc + bias;  GELU gelu(acc + bias);  RESID gamma * (acc + bias) (the sink adds it to x);
//   QKV  rope(qk_norm(acc + bias)) on the Q / K column blocks, acc + bias on V.
// acc[mi][ni] holds the C^T 16x16 tile (W rows as the MFMA A operand): lane owns output
// row  rowbase + mi*16 + lr  and the 4 CONSECUTIVE columns  colw + ni*16 + 4*lg + r.
// Rows >= M are emitted too; the sink drops them.
// RoPE tables of the QKV epilogue staged into LDS by the 256x256 kernels (stage_rope): cos rows at
// offset 0, sin rows at ROPE_LDS / 2, 64 B per position (16 floats), up to ROPE_LDS_POS positions
constexpr int ROPE_LDS = 8192;
constexpr int ROPE_LDS_POS = ROPE_LDS / 2 / 64;

// GELU_BWD's column sums: per lane and 64-row block (4 accumulator rows mi), the 16 columns
// colw + 16 ni + 4 lg + r summed over its rows; the 16 lanes lr of a 16-lane DPP row share those
// columns, so four DPP adds (quad swaps, half-row and row mirrors) leave the block's sums in every
// lane and lane lr = 0 stores them: ep.colsum[(row block) * N + col].
template <int MT>
__device__ __forceinline__ void colsum_store(const GemmArgs& g, float (&cs)[MT / 4][4][4], int rowbase, int colw,
                                             int lr, int lg) {
#pragma unroll
  for (int i = 0; i < MT / 4; ++i) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[i][ni][r] = sr::dpp_sum16(cs[i][ni][r]);
    const int rb = rowbase + i * 64;
    if (lr == 0 && rb < g.M) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int col = colw + ni * 16 + 4 * lg;
        if (col < g.N)
          *(float4*)(g.ep.colsum + (int64_t)(rb >> 6) * g.N + col) =
              make_float4(cs[i][ni][0], cs[i][ni][1], cs[i][ni][2], cs[i][ni][3]);
      }
    }
  }
}

template <typename T, int EPI, int MT, typename Emit>
__device__ __forceinline__ void produce(const GemmArgs& g, f32x4 (&acc)[MT][4], int rowbase, int colw, int lr,
                                        int lg, Emit&& emit, const char* rope_lds = nullptr) {
  const sr_gemm_epi& ep = g.ep;
  float4 bias[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
    bias[ni] = ep.bias && colw + ni * 16 + 4 * lg < g.N ? *(const float4*)(ep.bias + colw + ni * 16 + 4 * lg)
                                                          : make_float4(0.f, 0.f, 0.f, 0.f);
  auto biased = [&](int mi, int ni, float (&v)[4]) {
    v[0] = acc[mi][ni][0] + bias[ni].x;
    v[1] = acc[mi][ni][1] + bias[ni].y;
    v[2] = acc[mi][ni][2] + bias[ni].z;
    v[3] = acc[mi][ni][3] + bias[ni].w;
  };
  // training forward: the pre-activation (acc + bias) for the backward (sr_gemm_epi.aux)
  auto save_aux = [&](int row, int col, const float (&v)[4]) {
    if (row >= g.M || col >= g.N) return;
    if constexpr (sr::is_bf16<T>::value) {
      const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      *(bf16x4*)((T*)ep.aux + (int64_t)row * ep.ld_aux + col) = o;
    } else {
      *(float4*)((T*)ep.aux + (int64_t)row * ep.ld_aux + col) = make_float4(v[0], v[1], v[2], v[3]);
    }
  };

  if constexpr (EPI == SR_EPI_GELU_BWD) {
    // dH = acc * gelu'(u), u = the saved fc1 pre-activation (aux, T) of the same element; with
    // ep.colsum also the column sums of the stored (T-rounded) dH per 64-row block (colsum_store)
    float cs[MT / 4][4][4];
#pragma unroll
    for (int i = 0; i < MT / 4; ++i)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[i][ni][r] = 0.f;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int row = rowbase + mi * 16 + lr;
      const T* urow = (const T*)ep.aux + (int64_t)min(row, g.M - 1) * ep.ld_aux;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int col = min(colw + ni * 16 + 4 * lg, g.N - 4);
        float u[4];
        if constexpr (sr::is_bf16<T>::value) {
          const bf16x4 t = *(const bf16x4*)(urow + col);
          u[0] = (float)t[0]; u[1] = (float)t[1]; u[2] = (float)t[2]; u[3] = (float)t[3];
        } else {
          const float4 t = *(const float4*)(urow + col);
          u[0] = t.x; u[1] = t.y; u[2] = t.z; u[3] = t.w;
        }
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[mi][ni][r] * sr::gelu_erf_grad<sr::is_bf16<T>::value>(u[r]);
        emit(row, colw + ni * 16 + 4 * lg, v);
        if (ep.colsum && row < g.M) {
#pragma unroll
          for (int r = 0; r < 4; ++r) cs[mi >> 2][ni][r] += sr::to_f32(sr::from_f32<T>(v[r]));
        }
      }
    }
    if (ep.colsum) colsum_store<MT>(g, cs, rowbase, colw, lr, lg);
  } else if constexpr (EPI == SR_EPI_BIAS || EPI == SR_EPI_BIAS_GELU || EPI == SR_EPI_F32) {
    // the Q block of a plain-bias QKV projection (DINO) leaves scaled by q_scale (wave-uniform:
    // the wave's 64 columns start at colw, q_cols is a multiple of 64)
    const float qs = EPI == SR_EPI_BIAS && ep.q_scale != 0.f && colw < ep.q_cols ? ep.q_scale : 1.f;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int row = rowbase + mi * 16 + lr;
      {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          float v[4];
          biased(mi, ni, v);
          if (qs != 1.f) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] *= qs;
          }
          if constexpr (EPI == SR_EPI_BIAS_GELU) {
            if (ep.aux) save_aux(row, colw + ni * 16 + 4 * lg, v);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if constexpr (sr::is_bf16<T>::value) v[r] = sr::gelu_erf_fast(v[r]);
              else v[r] = sr::gelu_erf(v[r]);  // fp32 parity mode: exact erff
            }
          }
          emit(row, colw + ni * 16 + 4 * lg, v);
        }
      }
    }
  } else if constexpr (EPI == SR_EPI_BIAS_RESID) {
    float4 gam[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      gam[ni] = colw + ni * 16 + 4 * lg < g.N ? *(const float4*)(ep.gamma + colw + ni * 16 + 4 * lg)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int row = rowbase + mi * 16 + lr;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        float v[4];
        biased(mi, ni, v);
        v[0] *= gam[ni].x;
        v[1] *= gam[ni].y;
        v[2] *= gam[ni].z;
        v[3] *= gam[ni].w;
        emit(row, colw + ni * 16 + 4 * lg, v);
      }
    }
  } else if constexpr (EPI == SR_EPI_QKV) {
    // the wave's 64 columns are exactly one head: for one output row the 64 values sit in
    // the 4 lanes lr, lr+16, lr+32, lr+48 (16 each: ni x r).  head dim d = 16 ni + 4 lg + r.
    const int region = (colw + ep.col_offset) / ep.embed_dim;  // 0 = Q, 1 = K, 2 = V
    const bool qk = region < 2;
    const float* nw = region == 0 ? ep.qn_w : ep.kn_w;
    const float* nb = region == 0 ? ep.qn_b : ep.kn_b;
    const bool do_norm = qk && nw != nullptr;
    const bool do_rope = qk && ep.rope_cos != nullptr;
    const float q_scale = ep.q_scale != 0.f && colw < ep.q_cols ? ep.q_scale : 1.f;  // wave-uniform
    float4 w4[4], b4[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      w4[ni] = do_norm ? *(const float4*)(nw + ni * 16 + 4 * lg) : make_float4(1.f, 1.f, 1.f, 1.f);
      b4[ni] = do_norm ? *(const float4*)(nb + ni * 16 + 4 * lg) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int row = rowbase + mi * 16 + lr;
      float v[4][4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) biased(mi, ni, v[ni]);
      if (ep.aux) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) save_aux(row, colw + ni * 16 + 4 * lg, v[ni]);
      }
      if (do_norm) {  // LayerNorm over the head's 64 values: 16 in-lane x 4 lanes (xor 16, 32)
        float sum = 0.f;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) sum += (v[ni][0] + v[ni][1]) + (v[ni][2] + v[ni][3]);
        sum = sr::sum_x32(sr::sum_x16(sum));
        const float mean = sum * (1.f / 64.f);
        float d2 = 0.f;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[ni][r] -= mean;
            d2 += v[ni][r] * v[ni][r];
          }
        d2 = sr::sum_x32(sr::sum_x16(d2));
        const float rstd = rsqrtf(d2 * (1.f / 64.f) + ep.qk_eps);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          v[ni][0] = v[ni][0] * rstd * w4[ni].x + b4[ni].x;
          v[ni][1] = v[ni][1] * rstd * w4[ni].y + b4[ni].y;
          v[ni][2] = v[ni][2] * rstd * w4[ni].z + b4[ni].z;
          v[ni][3] = v[ni][3] * rstd * w4[ni].w + b4[ni].w;
        }
      }
      if (do_rope) {  // pairs (d, d+16): y half ni 0|1, x half ni 2|3; same lane, same r
        int py, px;
        sr::rope_pos(ep, min(row, g.M - 1), py, px);
        float4 cy, sy, cx, sx;
        if (rope_lds) {  // the tables in LDS (no global-load latency per row)
          cy = *(const float4*)(rope_lds + py * 64 + 16 * lg);
          sy = *(const float4*)(rope_lds + ROPE_LDS / 2 + py * 64 + 16 * lg);
          cx = *(const float4*)(rope_lds + px * 64 + 16 * lg);
          sx = *(const float4*)(rope_lds + ROPE_LDS / 2 + px * 64 + 16 * lg);
        } else {
          cy = *(const float4*)(ep.rope_cos + py * 16 + 4 * lg);
          sy = *(const float4*)(ep.rope_sin + py * 16 + 4 * lg);
          cx = *(const float4*)(ep.rope_cos + px * 16 + 4 * lg);
          sx = *(const float4*)(ep.rope_sin + px * 16 + 4 * lg);
        }
        const float cyv[4] = {cy.x, cy.y, cy.z, cy.w}, syv[4] = {sy.x, sy.y, sy.z, sy.w};
        const float cxv[4] = {cx.x, cx.y, cx.z, cx.w}, sxv[4] = {sx.x, sx.y, sx.z, sx.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float y0 = v[0][r] * cyv[r] - v[1][r] * syv[r], y1 = v[1][r] * cyv[r] + v[0][r] * syv[r];
          const float x0 = v[2][r] * cxv[r] - v[3][r] * sxv[r], x1 = v[3][r] * cxv[r] + v[2][r] * sxv[r];
          v[0][r] = y0;
          v[1][r] = y1;
          v[2][r] = x0;
          v[3][r] = x1;
        }
      }
      if (q_scale != 1.f) {  // c*q for the attention, rounded once (sr_attn_desc.q_scaled)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[ni][r] *= q_scale;
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) emit(row, colw + ni * 16 + 4 * lg, v[ni]);
    }
  }
}

// Register epilogue: every lane stores its own 4-column vectors (8 B bf16 / 16 B fp32).
template <typename T, int EPI, int MT>
__device__ __forceinline__ void epilogue(const GemmArgs& g, f32x4 (&acc)[MT][4], int rowbase, int colw, int lr,
                                         int lg, const char* rope_lds = nullptr) {
  const sr_gemm_epi& ep = g.ep;
  if constexpr (EPI == SR_EPI_PATCH) {
    float4 bias[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      bias[ni] = ep.bias && colw + ni * 16 + 4 * lg < g.N ? *(const float4*)(ep.bias + colw + ni * 16 + 4 * lg)
                                                          : make_float4(0.f, 0.f, 0.f, 0.f);
    auto biased = [&](int mi, int ni, float (&v)[4]) {
      v[0] = acc[mi][ni][0] + bias[ni].x;
      v[1] = acc[mi][ni][1] + bias[ni].y;
      v[2] = acc[mi][ni][2] + bias[ni].z;
      v[3] = acc[mi][ni][3] + bias[ni].w;
    };
    float* x = (float*)g.out;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int row = rowbase + mi * 16 + lr;
      if (row < g.M) {
        const int f = row / ep.seg_rows, p = row - f * ep.seg_rows;
        const int64_t orow = (int64_t)f * ep.seg_stride + ep.seg_offset + p;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int col = colw + ni * 16 + 4 * lg;
          if (col >= g.N) continue;
          float v[4];
          biased(mi, ni, v);
          const float4 ra = *(const float4*)(ep.row_add + (int64_t)p * g.N + col);
          *(float4*)(x + orow * g.ldo + col) = make_float4(v[0] + ra.x, v[1] + ra.y, v[2] + ra.z, v[3] + ra.w);
        }
      }
    }
  } else {
    produce<T, EPI, MT>(g, acc, rowbase, colw, lr, lg, [&](int row, int col, const float (&v)[4]) {
      if (row >= g.M || col >= g.N) return;
      static_assert(sizeof(OutT<T, EPI>) == (EPI == SR_EPI_BIAS_RESID || EPI == SR_EPI_F32 ? 4 : sizeof(T)),
                    "row_slice's element sizes must match these stores");
      if constexpr (EPI == SR_EPI_BIAS_RESID) {
        float4* p = (float4*)((float*)g.out + (int64_t)row * g.ldo + col);
        float4 xv = *p;
        xv.x += v[0];
        xv.y += v[1];
        xv.z += v[2];
        xv.w += v[3];
        *p = xv;
      } else if constexpr (EPI == SR_EPI_F32 || !sr::is_bf16<T>::value) {
        *(float4*)((float*)g.out + (int64_t)row * g.ldo + col) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        *(bf16x4*)((T*)g.out + (int64_t)row * g.ldo + col) = o;
      }
    }, rope_lds);
  }
}

// x += gamma * (acc + bias) for a full 256x256 tile (every row < M; N % 256 == 0 here), without
// per-vector guards: the guarded form compiles to an exec branch per vector with a vmcnt(0)
// before every store.  Here the loads of the next quarter of the wave's rows are in flight
// while the current quarter is updated and stored (kbench proj +3.5 %, fc2 +1 %).  An LDS-staged
// variant with 16 rows per wave in flight was 11 % slower, and staggering the first-round
// workgroups by 1/4 or 1/2 tile (so epilogues do not coincide across CUs) changed nothing.
__device__ __forceinline__ void resid_full(const GemmArgs& g, f32x4 (&acc)[8][4], int rowbase, int colw, int lr,
                                           int lg) {
  const sr_gemm_epi& ep = g.ep;
  f32x4 gm[4], bs[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int col = colw + ni * 16 + 4 * lg;
    gm[ni] = *(const f32x4*)(ep.gamma + col);
    bs[ni] = ep.bias ? *(const f32x4*)(ep.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float* xb = (float*)g.out + (int64_t)(rowbase + lr) * g.ldo + colw + 4 * lg;
  const int64_t rs = 16 * g.ldo;
  // quarters of 2 row blocks (8 float4 per lane); quarter q+1's loads are in flight while
  // quarter q is added and stored
  f32x4 xq[2][2][4];
  auto load = [&](int q) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) xq[q & 1][i][ni] = *(const f32x4*)(xb + (2 * q + i) * rs + ni * 16);
  };
  load(0);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q < 3) load(q + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        f32x4& xv = xq[q & 1][i][ni];
        xv += (acc[2 * q + i][ni] + bs[ni]) * gm[ni];
        *(f32x4*)(xb + (2 * q + i) * rs + ni * 16) = xv;
      }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---- RESID epilogue staged through LDS (GemmArgs.resid_lds), 256x256 tiles (a partial last row tile
// reads row M - 1 for the rows past M and stores only rows < M).
// The register form above keeps 8 KiB of x loads in flight per wave (64 KiB per CU) in 4 dependent
// rounds, each wave instruction touching 16 rows x 64 B; the epilogue then costs about as much as
// the K = 1024 k-loop (0.15 of proj's 0.30 ms) and is bound by that latency, not by HBM.
// Here the x tile moves as 1-KiB rows by LDS-DMA, in 64-row quarters through the two 64-KiB stage
// buffers: quarter 0 goes out under the last k-tile's MFMAs (into the stage buffer that k-tile does
// not read), quarter 1 right after it, and quarter k+2 as soon as quarter k's copy-out has read its
// buffer, so two quarters (128 KiB) are in flight while the owner waves add gamma * (acc + bias)
// in LDS and all eight waves store whole rows.  16-B chunk c of quarter row r sits at c ^ (r & 15):
// the DMA's per-lane source chunk, the owners' accumulator-layout read-modify-write (16 rows x one
// chunk column per 16 lanes) and the copy-out's row reads are all bank-conflict free.
// Per element the same fp32 operations as resid_full: x + (acc + bias) * gamma.  The tile's gamma and
// bias columns ride along with quarter 0 (1 KiB each, waves 0 / 1, past the stage buffers): the
// epilogue issues no compiler-visible load, so the compiler's wait counting never waits on the
// LDS-DMA it cannot see.
constexpr int RESID_GB = 2048;  // LDS past the two stages: gamma | bias of the tile's 256 columns
__device__ __forceinline__ void resid_dma_quarter(const GemmArgs& g, char* smem, int m0, int n0, int q, int buf,
                                                  int lane, int wave_u) {
  if (q == 0 && wave_u < 2 && (wave_u == 0 || g.ep.bias))
    sr::dma16_s(wave_u == 0 ? g.ep.gamma + n0 : g.ep.bias + n0, (uint32_t)lane * 16,
                __builtin_amdgcn_readfirstlane(sr::lds_addr(smem) + 2 * STAGE_BIG + wave_u * 1024));
  const uint32_t base = sr::lds_addr(smem) + buf * STAGE_BIG + wave_u * 8 * 1024;
  const int r0 = m0 + q * 64 + wave_u * 8;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int swz = ((wave_u & 1) << 3) | i;  // (quarter row 8 wave + i) & 15
    const int r = min(r0 + i, g.M - 1);       // rows past M (a partial last row tile): any valid row
    sr::dma16_s((const char*)g.out + ((int64_t)r * g.ldo + n0) * 4, (uint32_t)((lane ^ swz) << 4),
                __builtin_amdgcn_readfirstlane(base + i * 1024));
  }
}

__device__ __forceinline__ void resid_add_quarter(f32x4 (&acc)[8][4], char* smem, int buf, int q, int wc, int lr,
                                                  int lg, const f32x4 (&gm)[4], const f32x4 (&bs)[4]) {
  // one 16-row block at a time (16 x VGPRs live: the accumulators already fill the AGPRs and the
  // epilogue must not spill -- a scratch reload's vmcnt(0) would also wait out the LDS-DMA in flight)
  char* sb = smem + buf * STAGE_BIG + lr * 1024;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    f32x4 xv[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) xv[ni] = *(const f32x4*)(sb + m * 16 * 1024 + (((wc * 16 + ni * 4 + lg) ^ lr) << 4));
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      xv[ni] += (acc[(q & 1) * 4 + m][ni] + bs[ni]) * gm[ni];
      *(f32x4*)(sb + m * 16 * 1024 + (((wc * 16 + ni * 4 + lg) ^ lr) << 4)) = xv[ni];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

__device__ __forceinline__ void resid_store_quarter(const GemmArgs& g, const char* smem, int buf, int m0, int n0,
                                                    int q, int lane, int wave_u) {
  const char* sb = smem + buf * STAGE_BIG + wave_u * 8 * 1024;
  f32x4 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = *(const f32x4*)(sb + i * 1024 + lane * 16);
  const int r0 = m0 + q * 64 + wave_u * 8;
  float* xr = (float*)g.out + (int64_t)r0 * g.ldo + n0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int swz = ((wave_u & 1) << 3) | i;
    if (r0 + i < g.M) *(f32x4*)(xr + (int64_t)i * g.ldo + ((lane ^ swz) << 2)) = v[i];  // wave-uniform
  }
}

// After the k-loop: quarter 0 is in flight into buffer fb (issued under the last k-tile), the last
// k-tile read buffer fb ^ 1.  vmcnt counts this wave's LDS-DMA pieces (8 per quarter) and its row
// stores (8 per quarter) in issue order.
__device__ __forceinline__ void resid_lds_epilogue(const GemmArgs& g, f32x4 (&acc)[8][4], char* smem, int m0, int n0,
                                                   int fb, int wr, int wc, int lr, int lg, int lane, int wave_u) {
  const int kb = fb ^ 1;
  // a partial last row tile skips the stores of rows >= M, so the store counts below do not hold:
  // it waits for everything instead (one tile per launch at most)
  const bool partial = m0 + BIG > g.M;
  auto wait_q = [&]() {  // the quarter two DMA issues back landed: 16 younger ops (its successor's
    if (partial) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // 8 pieces, 8 row stores)
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  };
  sr::barrier_raw();                                          // every wave is done reading buffer kb
  resid_dma_quarter(g, smem, m0, n0, 1, kb, lane, wave_u);   // in flight: Q0 Q1
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");           // Q0 (+ gamma / bias) landed: this wave's
  sr::barrier_raw();                                          // ... every wave's
  f32x4 gm[4], bs[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int off = (wc * 64 + ni * 16 + 4 * lg) * 4;
    gm[ni] = *(const f32x4*)(smem + 2 * STAGE_BIG + off);
    bs[ni] = g.ep.bias ? *(const f32x4*)(smem + 2 * STAGE_BIG + 1024 + off) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (wr == 0) resid_add_quarter(acc, smem, fb, 0, wc, lr, lg, gm, bs);
  sr::wait_lgkm0();
  sr::barrier_raw();
  resid_store_quarter(g, smem, fb, m0, n0, 0, lane, wave_u);  // Q1 S0
  sr::wait_lgkm0();
  sr::barrier_raw();                                          // buffer fb read out
  resid_dma_quarter(g, smem, m0, n0, 2, fb, lane, wave_u);   // Q1 S0 Q2
  wait_q();                                                  // Q1 landed
  sr::barrier_raw();
  if (wr == 0) resid_add_quarter(acc, smem, kb, 1, wc, lr, lg, gm, bs);
  sr::wait_lgkm0();
  sr::barrier_raw();
  resid_store_quarter(g, smem, kb, m0, n0, 1, lane, wave_u);  // S0 Q2 S1
  sr::wait_lgkm0();
  sr::barrier_raw();                                          // buffer kb read out
  resid_dma_quarter(g, smem, m0, n0, 3, kb, lane, wave_u);   // S0 Q2 S1 Q3
  wait_q();                                                  // Q2 landed
  sr::barrier_raw();
  if (wr == 1) resid_add_quarter(acc, smem, fb, 2, wc, lr, lg, gm, bs);
  sr::wait_lgkm0();
  sr::barrier_raw();
  resid_store_quarter(g, smem, fb, m0, n0, 2, lane, wave_u);  // S1 Q3 S2
  if (partial) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // Q3 landed (8 younger: S2)
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  sr::barrier_raw();
  if (wr == 1) resid_add_quarter(acc, smem, kb, 3, wc, lr, lg, gm, bs);
  sr::wait_lgkm0();
  sr::barrier_raw();
  resid_store_quarter(g, smem, kb, m0, n0, 3, lane, wave_u);
}

// bias (+ erf-GELU) -> bf16 for a full 256x256 tile (every row < M; N % 256 == 0 here; no aux):
// the guarded produce/emit form compiles to an exec branch around every one of the 32 stores
// per lane; here they are plain stores with the math of the next vectors in between.
template <int EPI>
__device__ __forceinline__ void bias_full(const GemmArgs& g, f32x4 (&acc)[8][4], int rowbase, int colw, int lr,
                                          int lg) {
  const sr_gemm_epi& ep = g.ep;
  f32x4 bs[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
    bs[ni] = ep.bias ? *(const f32x4*)(ep.bias + colw + ni * 16 + 4 * lg) : f32x4{0.f, 0.f, 0.f, 0.f};
  bf16* ob = (bf16*)g.out + (int64_t)(rowbase + lr) * g.ldo + colw + 4 * lg;
  // the Q block of a plain-bias QKV projection, scaled (see produce)
  const float qs = EPI == SR_EPI_BIAS && ep.q_scale != 0.f && colw < ep.q_cols ? ep.q_scale : 1.f;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      f32x4 v = acc[mi][ni] + bs[ni];
      if (qs != 1.f) v *= qs;
      if constexpr (EPI == SR_EPI_BIAS_GELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = sr::gelu_erf_fast(v[r]);
      }
      const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      *(bf16x4*)(ob + (int64_t)mi * 16 * g.ldo + ni * 16) = o;
    }
}

// 256x256 bf16 epilogue staged through the (free) stage buffers so that global traffic is
// whole rows with 16 B per lane (the register epilogue's per-lane 8-B stores touch 16 rows
// per wave instruction).  bf16 outputs: the whole 256x256 tile (128 KiB, 512-B rows);
// RESID: two 128-row fp32 passes (1-KiB rows), each a batched coalesced read-add-write of x.
// 16-B chunk c of LDS row r sits at chunk c ^ (r & 15): the producers' 16-row column writes
// and the copy-out's row reads are both bank-conflict free.
template <int EPI>
__device__ __forceinline__ void epilogue256(const GemmArgs& g, f32x4 (&acc)[8][4], char* smem, int m0, int n0,
                                            int wr, int wc, int lr, int lg, int lane, int wave,
                                            const char* rope_lds = nullptr) {
  if constexpr (EPI == SR_EPI_PATCH) {
    epilogue<bf16, EPI, 8>(g, acc, m0 + wr * 128, n0 + wc * 64, lr, lg);
  } else if constexpr (EPI == SR_EPI_BIAS_RESID) {
    float* x = (float*)g.out;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      sr::barrier_raw();  // LDS free: k-loop reads / the previous pass's copy-out are done
      if (wr == p)
        produce<bf16, EPI, 8>(g, acc, m0 + wr * 128, n0 + wc * 64, lr, lg, [&](int row, int col, const float (&v)[4]) {
          const int rl = row - m0 - p * 128, cl = col - n0;
          *(float4*)(smem + rl * 1024 + (((cl >> 2) ^ (rl & 15)) << 4)) = make_float4(v[0], v[1], v[2], v[3]);
        });
      sr::barrier_raw();
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // 8 rows in flight per wave
        float4 xv[8];
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int row = m0 + p * 128 + wave * 16 + h * 8 + it;
          if (row < g.M) xv[it] = *(const float4*)(x + (int64_t)row * g.ldo + n0 + lane * 4);
        }
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int rl = wave * 16 + h * 8 + it, row = m0 + p * 128 + rl;
          if (row < g.M) {
            const float4 a = *(const float4*)(smem + rl * 1024 + ((lane ^ (rl & 15)) << 4));
            xv[it].x += a.x;
            xv[it].y += a.y;
            xv[it].z += a.z;
            xv[it].w += a.w;
            *(float4*)(x + (int64_t)row * g.ldo + n0 + lane * 4) = xv[it];
          }
        }
      }
    }
  } else {
    sr::barrier_raw();  // LDS free: every wave's k-loop reads are done
    produce<bf16, EPI, 8>(g, acc, m0 + wr * 128, n0 + wc * 64, lr, lg, [&](int row, int col, const float (&v)[4]) {
      const int rl = row - m0, cl = col - n0;
      const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      *(bf16x4*)(smem + rl * 512 + (((cl >> 3) ^ (rl & 15)) << 4) + ((cl & 7) << 1)) = o;
    }, rope_lds);
    sr::barrier_raw();
    bf16* out = (bf16*)g.out;
    if (m0 + 256 <= g.M) {
      // full tile: all 16 row reads in flight, then 16 unguarded stores (the guarded form waits
      // out each read's LDS latency behind an exec branch)
      uint4 v[16];
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int rl = wave * 32 + it * 2 + (lane >> 5), c = lane & 31;
        v[it] = *(const uint4*)(smem + rl * 512 + ((c ^ (rl & 15)) << 4));
      }
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int rl = wave * 32 + it * 2 + (lane >> 5), c = lane & 31;
        *(uint4*)(out + (int64_t)(m0 + rl) * g.ldo + n0 + c * 8) = v[it];
      }
      return;
    }
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int rl = wave * 32 + it * 2 + (lane >> 5), c = lane & 31, row = m0 + rl;
      if (row < g.M)
        *(uint4*)(out + (int64_t)row * g.ldo + n0 + c * 8) = *(const uint4*)(smem + rl * 512 + ((c ^ (rl & 15)) << 4));
    }
  }
}

// TBM x TBN output tile, 4 waves of 64 x 64 (128 x 128 as 2 x 2; few-row problems, M <= 64, as
// 64 x 256 = 1 x 4, so that no wave computes padding rows: the camera trunk's fp32 GEMMs at M = 2N)
template <typename T, int EPI, bool CONV = false, int TBM = BM, int TBN = BN>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_kernel(GemmArgs g) {
  static_assert(TBM % 64 == 0 && TBN % 64 == 0 && (TBM / 64) * (TBN / 64) == 4, "4 waves of 64 x 64");
  static_assert(!CONV || (TBM == 128 && TBN == 128), "the implicit conv stages A with waves 0-1");
  constexpr int STAGE = (TBM + TBN) * ROWB;
  constexpr int NPW = (TBM + TBN) / 32;  // LDS-DMA pieces (8 rows of 128 B) per wave per stage
  constexpr int WC = TBN / 64;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (g.N + TBN - 1) / TBN, ntm = (g.M + TBM - 1) / TBM;  // N % 4 == 0; last column tile ragged
  const int tile = sr::xcd_remap(blockIdx.x, ntn * ntm);
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const int m0 = tm * TBM, n0 = tn * TBN;

  // LDS-DMA sources: instruction i of wave w fills tile rows (w*NPW+i)*8 .. +8 (rows < TBM: A, else W).
  const char* src[NPW];
  // CONV: A rows come from the 3x3 window of output pixel m (waves 0-1 stage A, 2-3 stage W)
  const bool a_wave = __builtin_amdgcn_readfirstlane(wave) < 2;
  int cy[NPW], cx[NPW];  // CONV: window top-left (yo*s - 1, xo*s - 1) of this lane's pixel per piece
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    const int tr = (wave * NPW + i) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((tr >> 1) & 7);
    if (tr < TBM) {
      const int r = min(m0 + tr, g.M - 1);
      if constexpr (CONV) {
        const int hw = g.conv.Ho * g.conv.Wo;
        const int n = r / hw, rem = r - n * hw, yo = rem / g.conv.Wo, xo = rem - yo * g.conv.Wo;
        cy[i] = yo * g.conv.stride - 1;
        cx[i] = xo * g.conv.stride - 1;
        // pixel (n, cy, cx) of x, + this lane's 16-B chunk (may point before x: used only in-image)
        src[i] = g.conv.x + ((((int64_t)n * g.conv.H + cy[i]) * g.conv.W + cx[i]) * g.conv.C) * 4 + chunk * 16;
      } else {
        src[i] = g.A + (int64_t)r * g.lda_b + chunk * 16;
      }
    } else {
      const int r = min(n0 + tr - TBM, g.N - 1);  // ragged last column tile: re-read the last W row
      src[i] = g.W + (int64_t)r * g.ldw_b + chunk * 16;
    }
  }
  const uint32_t dst0 = __builtin_amdgcn_readfirstlane(sr::lds_addr(smem) + wave * NPW * 1024);
  auto stage = [&](int kt, int buf) {
    const uint32_t base = dst0 + buf * STAGE;
    if (CONV && a_wave) {
      // k-tile kt = 32 channels [ci0, ci0 + 32) of tap (ky, kx): C % 32 == 0, no tile straddles taps
      const int k0 = kt * 32, tap = k0 / g.conv.C, ci0 = k0 - tap * g.conv.C;
      const int ky = tap / 3, kx = tap - 3 * ky;
      const int64_t off = ((int64_t)ky * g.conv.W + kx) * g.conv.C * 4 + (int64_t)ci0 * 4;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int yy = cy[i] + ky, xx = cx[i] + kx;
        const bool in = (unsigned)yy < (unsigned)g.conv.H && (unsigned)xx < (unsigned)g.conv.W;
        sr::dma16(in ? src[i] + off : g.conv.zero + (lane & 7) * 16, base + i * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NPW; ++i) sr::dma16(src[i] + (int64_t)kt * ROWB, base + i * 1024);
    }
  };

  const int wr = wave / WC, wc = wave % WC;
  const int lr = lane & 15, lg = lane >> 4;
  const int swz = lr >> 1;  // (row>>1)&7 for every fragment row of this lane
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // split-K: slice blockIdx.y covers k-tiles [kt0, kt1)
  const int kt0 = g.partial ? blockIdx.y * g.kt_per_split : 0;
  const int kt1 = g.partial ? min(kt0 + g.kt_per_split, g.ktiles) : g.ktiles;
  stage(kt0, 0);
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    if (kt + 1 < kt1) {
      stage(kt + 1, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sr::barrier_raw();
    const char* sb = smem + buf * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int coff = (((ks * 4 + lg) ^ swz) * 16);
      uint4 a[4], b[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) a[mi] = *(const uint4*)(sb + (wr * 64 + mi * 16 + lr) * ROWB + coff);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) b[ni] = *(const uint4*)(sb + (TBM + wc * 64 + ni * 16 + lr) * ROWB + coff);
      if constexpr (CONV) {
        if (g.conv.relu) {  // the RCU's ReLU on the conv input (zero padding stays zero)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) {
            f32x4 v = __builtin_bit_cast(f32x4, a[mi]);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
            a[mi] = __builtin_bit_cast(uint4, v);
          }
        }
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) Mma<T>::run(b[ni], a[mi], acc[mi][ni]);  // C^T tile
    }
    sr::wait_lgkm0();
    sr::barrier_raw();
  }

  if (g.partial) {  // raw fp32 partial tile of this K slice
    float* part = g.partial + (int64_t)blockIdx.y * g.M * g.N;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int row = m0 + wr * 64 + mi * 16 + lr;
      if (row < g.M) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          if (n0 + wc * 64 + ni * 16 + 4 * lg < g.N)
            *(f32x4*)(part + (int64_t)row * g.N + n0 + wc * 64 + ni * 16 + 4 * lg) = acc[mi][ni];
      }
    }
    return;
  }
  epilogue<T, EPI, 4>(g, acc, m0 + wr * 64, n0 + wc * 64, lr, lg);
}

// Split-K reduction + epilogue: thread = 4 consecutive columns of one row; slices summed in
// order (deterministic).  out row stride ldo; RESID adds gamma*(sum+bias) to the fp32 out.
template <typename T, int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs g, int slices) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // float4 index
  const int nq = g.N >> 2;
  if (q >= (int64_t)g.M * nq) return;
  const int row = (int)(q / nq), col = (int)(q - (int64_t)row * nq) * 4;
  f32x4 v = *(const f32x4*)(g.partial + (int64_t)row * g.N + col);
  for (int z = 1; z < slices; ++z) v += *(const f32x4*)(g.partial + ((int64_t)z * g.M + row) * g.N + col);
  if (g.ep.bias) v += *(const f32x4*)(g.ep.bias + col);
  if (EPI == SR_EPI_BIAS && g.ep.q_scale != 0.f && col < g.ep.q_cols) v *= g.ep.q_scale;
  if constexpr (EPI == SR_EPI_BIAS_GELU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = sr::is_bf16<T>::value ? sr::gelu_erf_fast(v[r]) : sr::gelu_erf(v[r]);
  }
  if constexpr (EPI == SR_EPI_BIAS_RESID) {
    f32x4* xp = (f32x4*)((float*)g.out + (int64_t)row * g.ldo + col);
    *xp += v * *(const f32x4*)(g.ep.gamma + col);
  } else if constexpr (EPI == SR_EPI_F32) {  // fp32 output whatever the operand type
    *(f32x4*)((float*)g.out + (int64_t)row * g.ldo + col) = v;
  } else if constexpr (sr::is_bf16<T>::value) {
    const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    *(bf16x4*)((T*)g.out + (int64_t)row * g.ldo + col) = o;
  } else {
    *(f32x4*)((T*)g.out + (int64_t)row * g.ldo + col) = v;
  }
}

// ---------------------------------------------------------------------------------------
// 256x256 bf16 GEMM for the large-M aggregator GEMMs (M = S*P tokens).
//   * 512 threads = 8 waves as 2 (M) x 4 (N); per wave 128 x 64 outputs = 8 x 4 C^T tiles
//     (128 accumulator VGPRs); one workgroup per CU (128 KiB LDS);
//   * K-tile = 64 (128 B rows), 2 LDS stages of 64 KiB [A 256 rows | W 256 rows], XOR-swizzled;
//   * ONE barrier per K-tile: after it, the next stage is issued by LDS-DMA (8 per wave, 4 ahead
//     of each of the first two MFMA phases) and lands while the 64 MFMAs of the current tile run;
//   * the tile is computed as 4 quadrant phases (64 rows x 32 cols, 16 MFMAs each) ordered so
//     consecutive quadrants share A or B fragments (28 ds_read_b128 per 64 MFMAs);
//   * s_setprio 1 around each MFMA cluster keeps the cluster intact (cdna_hip_programming.md T5).

// Output tile -> (m0, n0): column-major inside groups of group_m row tiles, else row-major.
__device__ __forceinline__ void tile_origin(const GemmArgs& g, int tile, int& m0, int& n0) {
  const int ntn = g.N / BIG, ntm = (g.M + BIG - 1) / BIG;
  int tm, tn;
  if (g.group_m > 1) {
    const int per = g.group_m * ntn, grp = tile / per, first = grp * g.group_m;
    const int gm = min(g.group_m, ntm - first), r = tile - grp * per;
    tm = first + r % gm;
    tn = r / gm;
  } else {
    tm = tile / ntn;
    tn = tile - tm * ntn;
  }
  m0 = tm * BIG;
  n0 = tn * BIG;
}

// QKV: the RoPE cos / sin tables into LDS (ROPE_LDS bytes past the two K stages) by LDS-DMA, one
// 1-KiB piece per wave (8 waves: pieces 0-3 of cos, 0-3 of sin); lanes past a table's end re-read its
// last 16 B (no read past the allocation).  Issued before the first K stage, so the first k-tile's
// vmcnt(0) + barrier covers it.  Returns the tables' LDS base, or nullptr when they do not fit (the
// epilogue then reads them from global memory).
template <int EPI>
__device__ __forceinline__ const char* stage_rope(const GemmArgs& g, char* smem) {
  if constexpr (EPI != SR_EPI_QKV) {
    return nullptr;
  } else {
    const sr_gemm_epi& ep = g.ep;
    if (!ep.rope_cos || ep.rope_npos > ROPE_LDS_POS || !g.rope_lds) return nullptr;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bytes = ep.rope_npos * 64, piece = wave & 3;
    if (piece * 1024 < bytes) {
      const char* tab = (const char*)(wave < 4 ? ep.rope_cos : ep.rope_sin);
      const int off = min(piece * 1024 + lane * 16, bytes - 16);
      sr::dma16(tab + off, __builtin_amdgcn_readfirstlane(sr::lds_addr(smem) + 2 * STAGE_BIG +
                                                          (wave < 4 ? 0 : ROPE_LDS / 2) + piece * 1024));
    }
    return smem + 2 * STAGE_BIG;
  }
}

// One output tile over k-tiles [kb, ke) (the one-tile-per-workgroup 256x256 kernels).  RLDS: the RESID
// epilogue through LDS (resid_lds_epilogue, full and partial row tiles) -- a template parameter, not
// a run-time branch, so that no other epilogue's compiler-counted loads and stores share its control
// flow (a merged path made the compiler wait vmcnt(0) on the epilogue's LDS-DMA).
template <int EPI, bool RLDS = false>
__device__ __forceinline__ void gemm256_tile(const GemmArgs& g, char* smem, int tile, int kb, int ke,
                                             const char* rope_lds = nullptr) {
  static_assert(!RLDS || EPI == SR_EPI_BIAS_RESID, "the LDS-staged epilogue is RESID's");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int m0, n0;
  tile_origin(g, tile, m0, n0);

  // LDS-DMA sources: wave w, instruction i fills stage rows (w*8 + i)*8 .. +8 of the 512-row
  // stage: waves 0-3 stage A rows m0 + 64w + 8i + lane/8, waves 4-7 W rows n0 + 64(w-4) + 8i +
  // lane/8.  The 16-B chunk lane&7 goes to chunk ^ ((row>>1)&7) = ^ (4(i&1) + lane/16), so a
  // piece is a wave-uniform (scalar) base + one of two per-lane 32-bit offsets (no 64-bit vector
  // pointers: 14 VGPRs fewer).  Only the A waves of a ragged last row tile clamp rows per lane.
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const bool a_wave = wave_u < 4;
  const int64_t ld_b = a_wave ? g.lda_b : g.ldw_b;
  const uint32_t voA = (uint32_t)((lane >> 3) * ld_b + (((lane & 7) ^ (lane >> 4)) << 4));
  const uint32_t voB = (uint32_t)((lane >> 3) * ld_b + (((lane & 7) ^ (4 + (lane >> 4))) << 4));
  const uint32_t dst0 = __builtin_amdgcn_readfirstlane(sr::lds_addr(smem) + wave * 8 * 1024);
  // pieces [i0, i1) of stage kt (one wave-uniform branch per call): this wave's first staged row
  // (A rows clamped to M - 1 for a ragged last row tile)
  auto dma_pieces = [&](int kt, int i0, int i1) {
    const int brow0 = a_wave ? min(m0 + wave_u * 64, g.M - 1) : n0 + (wave_u - 4) * 64;
    const char* sp = (a_wave ? g.A : g.W) + (int64_t)brow0 * ld_b + (int64_t)kt * ROWB;
    const uint32_t base = dst0 + (kt & 1) * STAGE_BIG;
    if (!(a_wave && m0 + BIG > g.M)) {
#pragma unroll
      for (int i = i0; i < i1; ++i) sr::dma16_s(sp + (int64_t)i * 8 * ld_b, (i & 1) ? voB : voA, base + i * 1024);
    } else {
      const int rlim = g.M - 1 - brow0;  // last valid row relative to brow0
#pragma unroll
      for (int i = i0; i < i1; ++i) {
        const int r = min(i * 8 + (lane >> 3), rlim);
        const int chunk = (lane & 7) ^ (4 * (i & 1) + (lane >> 4));
        sr::dma16_s(sp, (uint32_t)(r * ld_b + chunk * 16), base + i * 1024);
      }
    }
  };
  auto stage = [&](int kt) { dma_pieces(kt, 0, 8); };

  const int wr = wave >> 2, wc = wave & 3;
  const int lr = lane & 15, lg = lane >> 4;
  const int swz = lr >> 1;
  // fragment row offsets (bytes) inside a stage
  const int arow = (wr * 128 + lr) * ROWB;        // + (qm*64 + mi*16) * ROWB
  const int brow = (BIG + wc * 64 + lr) * ROWB;   // + (qn*32 + ni*16) * ROWB
  const int coff0 = ((0 + lg) ^ swz) * 16, coff1 = ((4 + lg) ^ swz) * 16;  // k-substep 0 / 1

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(kb);
  for (int kt = kb; kt < ke; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of stage kt landed
    sr::barrier_raw();                                  // ... every wave's; all done with kt-1
    const bool more = kt + 1 < ke;
    // the 8 DMA pieces of stage kt+1 (overwriting the buffer of kt-1) go out 4 before each of the
    // first two MFMA phases rather than as one burst after the barrier (same-box A/B: qkv +4 %,
    // fc1 +2 %, proj / fc2 even; 2 per phase over all four phases, or waves 0-3 / 4-7 in turn,
    // measured no better)
    auto dma_phase = [&](int ph) {
      if (!more) {  // last k-tile: the RESID x tile's first quarter into the stage buffer it does not read
        if (RLDS && ph == 0) resid_dma_quarter(g, smem, m0, n0, 0, (kt + 1) & 1, lane, wave_u);
        return;
      }
      if (ph < 2) dma_pieces(kt + 1, 4 * ph, 4 * ph + 4);
    };
    const char* sb = smem + (kt & 1) * STAGE_BIG;
    // fragments double-buffered by quadrant: the next quadrant's ds_reads are issued before
    // the current quadrant's MFMA cluster so their LDS latency hides under it
    uint4 aX[4][2], aY[4][2], bX[2][2], bY[2][2];
    auto load_a = [&](uint4 (&a)[4][2], int qm) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const char* p = sb + arow + (qm * 64 + mi * 16) * ROWB;
        a[mi][0] = *(const uint4*)(p + coff0);
        a[mi][1] = *(const uint4*)(p + coff1);
      }
    };
    auto load_b = [&](uint4 (&b)[2][2], int qn) {
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const char* p = sb + brow + (qn * 32 + ni * 16) * ROWB;
        b[ni][0] = *(const uint4*)(p + coff0);
        b[ni][1] = *(const uint4*)(p + coff1);
      }
    };
    auto mma = [&](const uint4 (&a)[4][2], const uint4 (&b)[2][2], int qm, int qn) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) Mma<bf16>::run(b[ni][ks], a[mi][ks], acc[qm * 4 + mi][qn * 2 + ni]);
      __builtin_amdgcn_s_setprio(0);
    };
    load_a(aX, 0);
    load_b(bX, 0);
    load_b(bY, 1);
    dma_phase(0);
    mma(aX, bX, 0, 0);
    load_a(aY, 1);
    dma_phase(1);
    mma(aX, bY, 0, 1);
    load_b(bX, 0);
    dma_phase(2);
    mma(aY, bY, 1, 1);
    dma_phase(3);
    mma(aY, bX, 1, 0);
  }
  if constexpr (RLDS) {
    resid_lds_epilogue(g, acc, smem, m0, n0, ke & 1, wr, wc, lr, lg, lane, wave_u);
    return;
  }
  if constexpr (EPI == SR_EPI_BIAS_RESID) {
    if (m0 + BIG <= g.M && !g.lds_epi) {
      resid_full(g, acc, m0 + wr * 128, n0 + wc * 64, lr, lg);
      return;
    }
  }
  if constexpr (EPI == SR_EPI_BIAS || EPI == SR_EPI_BIAS_GELU) {
    if (m0 + BIG <= g.M && !g.lds_epi && !g.ep.aux) {
      bias_full<EPI>(g, acc, m0 + wr * 128, n0 + wc * 64, lr, lg);
      return;
    }
  }
  if (g.lds_epi) {
    epilogue256<EPI>(g, acc, smem, m0, n0, wr, wc, lr, lg, lane, wave, rope_lds);
    return;
  }
  epilogue<bf16, EPI, 8>(g, acc, m0 + wr * 128, n0 + wc * 64, lr, lg, rope_lds);
}

// LDS of the 256x256 kernels: two K stages, plus the RoPE tables for QKV / the gamma | bias columns
// for RESID (one array: a second __shared__ object can make hipcc drain the LDS-DMA ring,
// cdna_hip_programming.md §5 item 4(a))
template <int EPI> constexpr int smem256() {
  return 2 * STAGE_BIG + (EPI == SR_EPI_QKV ? ROPE_LDS : EPI == SR_EPI_BIAS_RESID ? RESID_GB : 0);
}

template <int EPI, bool RLDS>
__global__ __launch_bounds__(512, 1) void gemm256_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[smem256<EPI>()];
  const int nt = (g.N / BIG) * ((g.M + BIG - 1) / BIG);
  const char* rope = stage_rope<EPI>(g, smem);
  gemm256_tile<EPI, RLDS>(g, smem, sr::xcd_remap(blockIdx.x, nt), 0, g.ktiles, rope);
}

// Up to 4 independent 256x256 GEMMs of one epilogue kind in ONE launch (sr_gemm_group): problem
// p owns workgroups [start[p], start[p+1]), each range a multiple of 8 (padding workgroups exit) so
// that the XCD remap within a problem keeps its tiles on one XCD as a launch of its own would.
// The problems' last partial rounds merge: the layer's three QKV GEMMs after a frame block
// (queries, anchors, anchor subsample: 2,064 + 2,064 + 312 tiles at C3) run in 18 rounds, not 20.
constexpr int GROUP_MAX = 4;
struct GemmGroup {
  GemmArgs g[GROUP_MAX];
  int start[GROUP_MAX + 1];
  int n;
};

template <int EPI, bool RLDS>
__global__ __launch_bounds__(512, 1) void gemm256_group_kernel(GemmGroup gg) {
  __shared__ __attribute__((aligned(16))) char smem[smem256<EPI>()];
  int p = 0;
#pragma unroll
  for (int i = 1; i < GROUP_MAX; ++i) p += (i < gg.n && (int)blockIdx.x >= gg.start[i]) ? 1 : 0;
  const GemmArgs& g = gg.g[p];
  const int nt = (g.N / BIG) * ((g.M + BIG - 1) / BIG);
  const int lin = blockIdx.x - gg.start[p];
  if (lin >= nt) return;  // padding
  const char* rope = stage_rope<EPI>(g, smem);
  gemm256_tile<EPI, RLDS>(g, smem, sr::xcd_remap(lin, nt), 0, g.ktiles, rope);
}


// 256x256 tile order (sr_gemm and sr_gemm_group): column-major inside groups of 4 row tiles for
// the wide outputs (fc1, QKV: N >= 3072; kbench A/B fc1 -3 %, qkv -1.5 %), row-major for N = 1024
// (proj / fc2, where grouping measured neutral to +1-2 % slower).  SR_TUNE_GEMM_GROUP_M = g >= 0
// overrides (<= 1: row-major).
static int tile_group_m(int N) {
  const int g = sr::tune(SR_TUNE_GEMM_GROUP_M);
  return g >= 0 ? g : (N >= 3072 ? 4 : 0);
}

template <int EPI>
int launch256(GemmArgs a, hipStream_t s) {
  const int nwg = (a.N / BIG) * ((a.M + BIG - 1) / BIG);
  a.group_m = tile_group_m(a.N);
  if constexpr (EPI == SR_EPI_BIAS_RESID) {
    if (a.resid_lds) {
      hipLaunchKernelGGL((gemm256_kernel<EPI, true>), dim3(nwg), dim3(512), 0, s, a);
      sr::note_kernel("gemm256_kernel<%d, true>", EPI);
      return sr::check_launch("sr_gemm(256)");
    }
  }
  hipLaunchKernelGGL((gemm256_kernel<EPI, false>), dim3(nwg), dim3(512), 0, s, a);
  sr::note_kernel("gemm256_kernel<%d, false>", EPI);
  return sr::check_launch("sr_gemm(256)");
}

template <typename T, int EPI>
int launch(const GemmArgs& a, hipStream_t s) {
  const int slices = a.partial ? (a.ktiles + a.kt_per_split - 1) / a.kt_per_split : 1;
  // few rows (the camera trunk, M = 2N views): 64 x 256 tiles, no padding rows computed
  // (SR_GEMM_SMALLM=0: 128 x 128)
  const bool small_m = sr::tune(SR_TUNE_GEMM_SMALLM) != 0;
  const char* tn = sr::is_bf16<T>::value ? "__bf16" : "float";
  if (small_m && a.M <= 64 && a.N > 128) {
    const int nwg = (a.N + 255) / 256;
    hipLaunchKernelGGL((gemm_kernel<T, EPI, false, 64, 256>), dim3(nwg, slices), dim3(NTHREADS), 0, s, a);
    sr::note_kernel("gemm_kernel<%s, %d, false, 64, 256>", tn, EPI);
  } else {
    const int nwg = ((a.N + BN - 1) / BN) * ((a.M + BM - 1) / BM);
    hipLaunchKernelGGL((gemm_kernel<T, EPI>), dim3(nwg, slices), dim3(NTHREADS), 0, s, a);
    sr::note_kernel("gemm_kernel<%s, %d, false>", tn, EPI);
  }
  if (a.partial) {
    const int64_t nq = (int64_t)a.M * (a.N / 4);
    hipLaunchKernelGGL((splitk_reduce_kernel<T, EPI>), dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, a,
                       slices);
  }
  return sr::check_launch("sr_gemm");
}

// Rows [r0, r0 + rows) of a bf16 GEMM as a GEMM of its own: A / out / aux and the QKV epilogue's row
// positions advanced by r0 (every epilogue but PATCH, whose row remap is absolute).  Element sizes
// come from OutT / AuxT, the types the epilogues store (no hand-kept table).
template <int EPI>
static GemmArgs row_slice(const GemmArgs& a, int r0, int rows) {
  static_assert(EPI != SR_EPI_PATCH, "PATCH rows map to absolute output rows");
  GemmArgs b = a;
  b.A += (int64_t)r0 * a.lda_b;
  b.out = (char*)a.out + (int64_t)r0 * a.ldo * (int64_t)sizeof(OutT<bf16, EPI>);
  if (a.ep.aux) b.ep.aux = (char*)a.ep.aux + (int64_t)r0 * a.ep.ld_aux * (int64_t)sizeof(AuxT<bf16>);
  if (a.ep.colsum) b.ep.colsum = a.ep.colsum + (int64_t)(r0 / 64) * a.N;  // r0: whole 256-row tiles
  if (a.ep.pos_yx) b.ep.pos_yx += 2 * (int64_t)r0;
  else if (a.ep.pos_rowmap) b.ep.pos_rowmap += r0;
  else b.ep.pos_row_base += r0;
  b.M = rows;
  return b;
}

template <int EPI>
int launch256_tail(GemmArgs a, hipStream_t s) {
  // Last-round quantisation (SR_TUNE_GEMM_TAIL): with T tiles of 256x256 on C CUs (one workgroup
  // each) the last round runs T % C tiles while the rest of the chip idles.  When the rows past the
  // last whole round fit ONE round of the 128x128 kernel (two workgroups per CU), they go there as a
  // second launch: the frame QKV at C3 is 4,128 tiles = 16 rounds + 32 tiles, so 341 row tiles run
  // in 16 rounds and the last 640 rows in 120 small tiles.  Same MFMA and k order per output tile.
  if (sr::tune(SR_TUNE_GEMM_TAIL) && EPI != SR_EPI_PATCH) {
    const int ntn = a.N / BIG, cus = sr::cu_count();
    const long tiles = (long)ntn * ((a.M + BIG - 1) / BIG);
    const long whole = tiles / cus * cus;
    const int main_rows = (int)(whole / ntn) * BIG;
    const int rest = a.M - main_rows;
    const long small = (long)((rest + BM - 1) / BM) * (a.N / BN);
    if (tiles % cus != 0 && main_rows > 0 && rest > 0 && small <= 2L * cus) {
      GemmArgs head = a;
      head.M = main_rows;
      int rc = launch256<EPI>(head, s);
      if (rc != SR_OK) return rc;
      rc = launch<bf16, EPI>(row_slice<EPI>(a, main_rows, rest), s);
      // the launch the time goes to
      sr::note_kernel("gemm256_kernel<%d, %s>", EPI, EPI == SR_EPI_BIAS_RESID && a.resid_lds ? "true" : "false");
      return rc;
    }
  }
  return launch256<EPI>(a, s);
}

template <typename T>
int dispatch(int epi, const GemmArgs& a, hipStream_t s) {
  if constexpr (sr::is_bf16<T>::value) {
    const bool no_big = sr::tune(SR_TUNE_GEMM_NO256) != 0;
    // 256x256 tiles (one WG per CU) only when they still give >= 2 WGs per CU; smaller
    // problems (frame-sharded ranks, small scenes) keep 4x more 128x128 workgroups.
    const long tiles256 = (long)(a.N / BIG) * ((a.M + BIG - 1) / BIG);
    if (!no_big && a.N % BIG == 0 && tiles256 >= 512) {
      switch (epi) {
        case SR_EPI_BIAS: return launch256_tail<SR_EPI_BIAS>(a, s);
        case SR_EPI_BIAS_GELU: return launch256_tail<SR_EPI_BIAS_GELU>(a, s);
        case SR_EPI_BIAS_RESID: return launch256_tail<SR_EPI_BIAS_RESID>(a, s);
        case SR_EPI_QKV: return launch256_tail<SR_EPI_QKV>(a, s);
        case SR_EPI_PATCH: return launch256<SR_EPI_PATCH>(a, s);
        case SR_EPI_F32: return launch256_tail<SR_EPI_F32>(a, s);
        case SR_EPI_GELU_BWD: return launch256_tail<SR_EPI_GELU_BWD>(a, s);
      }
    }
  }
  switch (epi) {
    case SR_EPI_BIAS: return launch<T, SR_EPI_BIAS>(a, s);
    case SR_EPI_BIAS_GELU: return launch<T, SR_EPI_BIAS_GELU>(a, s);
    case SR_EPI_BIAS_RESID: return launch<T, SR_EPI_BIAS_RESID>(a, s);
    case SR_EPI_QKV: return launch<T, SR_EPI_QKV>(a, s);
    case SR_EPI_PATCH: return launch<T, SR_EPI_PATCH>(a, s);
    case SR_EPI_F32: return launch<T, SR_EPI_F32>(a, s);
    case SR_EPI_GELU_BWD: return launch<T, SR_EPI_GELU_BWD>(a, s);
  }
  sr::set_error("sr_gemm: unknown epilogue %d", epi);
  return SR_EINVAL;
}

// Narrow implicit-GEMM 3x3 conv for Cout <= 32 (DPT output_conv2[0]: 128 -> 32 at full
// resolution, dpt_head.py:105-108): a 128-wide tile would leave 3/4 of its MFMAs on padding
// columns, so this tile is 256 output pixels x 32 channels: 4 waves x 64 rows, stage = 256 A
// rows + 32 W rows (36 KiB), 9 LDS-DMA pieces per wave, same swizzle and fragments as
// gemm_kernel<float, EPI, true>.  Epilogue BIAS.
constexpr int NBM = 256, NBN = 32;
constexpr int NSTAGE = (NBM + NBN) * ROWB;  // 36 KiB

__global__ __launch_bounds__(256, 2) void conv_narrow_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[2 * NSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = sr::xcd_remap(blockIdx.x, gridDim.x) * NBM;
  constexpr int PW = (NBM + NBN) / 8 / 4;  // 9 pieces per wave
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const char* src[PW];
  int cy[PW], cx[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int gi = wave_u * PW + i;
    const int tr = gi * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((tr >> 1) & 7);
    if (gi < NBM / 8) {
      const int r = min(m0 + tr, g.M - 1);
      const int hw = g.conv.Ho * g.conv.Wo;
      const int n = r / hw, rem = r - n * hw, yo = rem / g.conv.Wo, xo = rem - yo * g.conv.Wo;
      cy[i] = yo * g.conv.stride - 1;
      cx[i] = xo * g.conv.stride - 1;
      src[i] = g.conv.x + ((((int64_t)n * g.conv.H + cy[i]) * g.conv.W + cx[i]) * g.conv.C) * 4 + chunk * 16;
    } else {
      const int r = min(tr - NBM, g.N - 1);
      cy[i] = cx[i] = 0;
      src[i] = g.W + (int64_t)r * g.ldw_b + chunk * 16;
    }
  }
  const uint32_t dst0 = __builtin_amdgcn_readfirstlane(sr::lds_addr(smem) + wave * PW * 1024);
  auto stage = [&](int kt, int buf) {
    const uint32_t base = dst0 + buf * NSTAGE;
    const int k0 = kt * 32, tap = k0 / g.conv.C, ci0 = k0 - tap * g.conv.C;
    const int ky = tap / 3, kx = tap - 3 * ky;
    const int64_t off = ((int64_t)ky * g.conv.W + kx) * g.conv.C * 4 + (int64_t)ci0 * 4;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      if (wave_u * PW + i < NBM / 8) {
        const int yy = cy[i] + ky, xx = cx[i] + kx;
        const bool in = (unsigned)yy < (unsigned)g.conv.H && (unsigned)xx < (unsigned)g.conv.W;
        sr::dma16(in ? src[i] + off : g.conv.zero + (lane & 7) * 16, base + i * 1024);
      } else {
        sr::dma16(src[i] + (int64_t)kt * ROWB, base + i * 1024);
      }
    }
  };
  const int lr = lane & 15, lg = lane >> 4;
  const int swz = lr >> 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  stage(0, 0);
  for (int kt = 0; kt < g.ktiles; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < g.ktiles) {
      stage(kt + 1, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sr::barrier_raw();
    const char* sb = smem + buf * NSTAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int coff = (((ks * 4 + lg) ^ swz) * 16);
      uint4 a[4], b[2];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) a[mi] = *(const uint4*)(sb + (wave * 64 + mi * 16 + lr) * ROWB + coff);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) b[ni] = *(const uint4*)(sb + (NBM + ni * 16 + lr) * ROWB + coff);
      if (g.conv.relu) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          f32x4 v = __builtin_bit_cast(f32x4, a[mi]);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
          a[mi] = __builtin_bit_cast(uint4, v);
        }
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) Mma<float>::run(b[ni], a[mi], acc[mi][ni]);
    }
    sr::wait_lgkm0();
    sr::barrier_raw();
  }
  // columns 32..63 (acc[.][2..3], zeros) fall outside N and are dropped by the sink
  epilogue<float, SR_EPI_BIAS, 4>(g, acc, m0 + wave * 64, 0, lr, lg);
}

template <int EPI>
int launch_conv(const GemmArgs& a, hipStream_t s) {
  const int nwg = ((a.N + BN - 1) / BN) * ((a.M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_kernel<float, EPI, true>), dim3(nwg), dim3(NTHREADS), 0, s, a);
  return sr::check_launch("sr_conv3x3_f32");
}

}  // namespace

static int gemm_args(GemmArgs& a, int dtype, int epi, const void* A, int64_t lda, const void* W, int64_t ldw,
                     void* out, int64_t ldo, int M, int N, int K, const sr_gemm_epi* ep) {
  SR_CHECK(A && W && out && ep, SR_EINVAL, "sr_gemm: null pointer");
  SR_CHECK(dtype == SR_F32 || dtype == SR_BF16, SR_EINVAL, "sr_gemm: bad dtype %d", dtype);
  SR_CHECK(M > 0 && N > 0 && K > 0, SR_EINVAL, "sr_gemm: bad shape M=%d N=%d K=%d", M, N, K);
  const int kt = dtype == SR_BF16 ? Mma<bf16>::KT : Mma<float>::KT;
  const int esz = dtype == SR_BF16 ? 2 : 4;
  SR_CHECK(N % 4 == 0, SR_EUNSUPPORTED, "sr_gemm: N=%d must be a multiple of 4", N);
  SR_CHECK(K % kt == 0, SR_EUNSUPPORTED, "sr_gemm: K=%d must be a multiple of %d", K, kt);
  SR_CHECK(lda >= K && ldw >= K && (lda * esz) % 16 == 0 && (ldw * esz) % 16 == 0, SR_EINVAL,
           "sr_gemm: bad leading dims lda=%lld ldw=%lld", (long long)lda, (long long)ldw);
  SR_CHECK(((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0, SR_EINVAL, "sr_gemm: A/W must be 16-B aligned");
  if (epi == SR_EPI_BIAS_RESID) SR_CHECK(ep->gamma, SR_EINVAL, "sr_gemm: RESID needs gamma");
  if (epi == SR_EPI_GELU_BWD) SR_CHECK(ep->aux && ep->ld_aux >= N && (ep->ld_aux * esz) % 8 == 0, SR_EINVAL,
                                       "sr_gemm: GELU_BWD needs aux (the saved pre-activation)");
  SR_CHECK(!ep->colsum || (epi == SR_EPI_GELU_BWD && ((uintptr_t)ep->colsum % 16) == 0), SR_EINVAL,
           "sr_gemm: colsum needs the GELU_BWD epilogue and a 16-B aligned buffer");
  if (ep->aux && (epi == SR_EPI_BIAS_GELU || epi == SR_EPI_QKV))
    SR_CHECK(ep->ld_aux >= N && (ep->ld_aux * esz) % 8 == 0 && ((uintptr_t)ep->aux % 8) == 0, SR_EINVAL,
             "sr_gemm: bad aux buffer");
  if (epi == SR_EPI_F32)
    SR_CHECK(ldo % 4 == 0 && ((uintptr_t)out % 16) == 0, SR_EINVAL, "sr_gemm: F32 output must be 16-B aligned");
  if (epi == SR_EPI_PATCH)
    SR_CHECK(ep->row_add && ep->seg_rows > 0 && ep->seg_stride >= ep->seg_rows, SR_EINVAL, "sr_gemm: PATCH params");
  if (ep->q_scale != 0.f)
    SR_CHECK((epi == SR_EPI_BIAS || epi == SR_EPI_QKV) && ep->q_cols >= 0 && ep->q_cols % 64 == 0 && ep->q_cols <= N &&
                 ep->q_scale == ep->q_scale,
             SR_EINVAL, "sr_gemm: q_scale needs the BIAS or QKV epilogue and q_cols a multiple of 64 within N");
  if (epi == SR_EPI_QKV) {
    SR_CHECK(ep->head_dim == 64 && ep->embed_dim % 64 == 0 && ep->embed_dim > 0, SR_EUNSUPPORTED,
             "sr_gemm: QKV epilogue needs head_dim 64 (got %d)", ep->head_dim);
    if (ep->rope_cos)
      SR_CHECK(ep->rope_sin && ep->rope_npos > 0 &&
                   (ep->pos_yx || (ep->tokens_per_frame > ep->patch_start && ep->grid_w > 0)),
               SR_EINVAL, "sr_gemm: QKV rope params");
  }
  a = GemmArgs{};
  a.A = (const char*)A;
  a.lda_b = lda * esz;
  a.W = (const char*)W;
  a.ldw_b = ldw * esz;
  a.out = out;
  a.ldo = ldo;
  a.M = M;
  a.N = N;
  a.K = K;
  a.ktiles = K / kt;
  // LDS-staged epilogue (256x256 tiles): measured +8 % on bf16 BIAS / QKV outputs, -7 % on the
  // fp32 residual update and -2 % with GELU (DESIGN.md "GEMM"), so only the former use it.
  const bool no_lds_epi = sr::tune(SR_TUNE_GEMM_REG_EPI) != 0;
  a.lds_epi = !no_lds_epi && (epi == SR_EPI_BIAS || (epi == SR_EPI_QKV && !ep->aux)) &&
              ((uintptr_t)out % 16) == 0 && (ldo * esz) % 16 == 0;
  a.ep = *ep;
  a.partial = nullptr;
  a.kt_per_split = a.ktiles;
  a.resid_lds = epi == SR_EPI_BIAS_RESID && dtype == SR_BF16 && sr::tune(SR_TUNE_GEMM_RESID_LDS) != 0 &&
                ((uintptr_t)out % 16) == 0 && ldo % 4 == 0 && ((uintptr_t)ep->gamma % 16) == 0 &&
                ((uintptr_t)ep->bias % 16) == 0;
  a.rope_lds = sr::tune(SR_TUNE_GEMM_ROPE_LDS) != 0;
  return SR_OK;
}

static int gemm_common(sr_stream_t stream, int dtype, int epi, const void* A, int64_t lda, const void* W,
                       int64_t ldw, void* out, int64_t ldo, int M, int N, int K, int splits, float* workspace,
                       const sr_gemm_epi* ep) {
  GemmArgs a;
  const int rc = gemm_args(a, dtype, epi, A, lda, W, ldw, out, ldo, M, N, K, ep);
  if (rc != SR_OK) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (splits > 1) {
    SR_CHECK(epi == SR_EPI_BIAS || epi == SR_EPI_BIAS_GELU || epi == SR_EPI_BIAS_RESID || epi == SR_EPI_F32,
             SR_EUNSUPPORTED, "sr_gemm_splitk: epilogue %d not supported", epi);
    SR_CHECK(workspace && ((uintptr_t)workspace % 16) == 0 && ((uintptr_t)out % 16) == 0 && ldo % 4 == 0 && N % 4 == 0,
             SR_EINVAL, "sr_gemm_splitk: workspace / out must be 16-B aligned");
    SR_CHECK(a.ktiles % splits == 0, SR_EUNSUPPORTED, "sr_gemm_splitk: %d k-tiles not divisible into %d slices",
             a.ktiles, splits);
    a.partial = workspace;
    a.kt_per_split = a.ktiles / splits;
    switch (epi) {  // always the 128x128 kernel (few rows)
      case SR_EPI_BIAS: return dtype == SR_BF16 ? launch<bf16, SR_EPI_BIAS>(a, s) : launch<float, SR_EPI_BIAS>(a, s);
      case SR_EPI_BIAS_GELU:
        return dtype == SR_BF16 ? launch<bf16, SR_EPI_BIAS_GELU>(a, s) : launch<float, SR_EPI_BIAS_GELU>(a, s);
      case SR_EPI_F32: return dtype == SR_BF16 ? launch<bf16, SR_EPI_F32>(a, s) : launch<float, SR_EPI_F32>(a, s);
      default:
        return dtype == SR_BF16 ? launch<bf16, SR_EPI_BIAS_RESID>(a, s) : launch<float, SR_EPI_BIAS_RESID>(a, s);
    }
  }
  return dtype == SR_BF16 ? dispatch<bf16>(epi, a, s) : dispatch<float>(epi, a, s);
}

extern "C" int sr_gemm_group(sr_stream_t stream, int dtype, int epi, int n, const sr_gemm_problem* pr) {
  SR_CHECK(pr && n >= 1 && n <= GROUP_MAX, SR_EINVAL, "sr_gemm_group: 1..%d problems (got %d)", GROUP_MAX, n);
  SR_CHECK(dtype == SR_BF16, SR_EUNSUPPORTED, "sr_gemm_group: bf16 only");
  SR_CHECK(epi == SR_EPI_BIAS || epi == SR_EPI_QKV || epi == SR_EPI_BIAS_GELU || epi == SR_EPI_BIAS_RESID ||
               epi == SR_EPI_F32 || epi == SR_EPI_GELU_BWD,
           SR_EUNSUPPORTED, "sr_gemm_group: epilogue %d not supported", epi);
  GemmGroup gg{};
  gg.n = n;
  gg.start[0] = 0;
  for (int i = 0; i < n; ++i) {
    const sr_gemm_problem& q = pr[i];
    const int rc = gemm_args(gg.g[i], dtype, epi, q.A, q.lda, q.W, q.ldw, q.out, q.ldo, q.M, q.N, q.K, &q.ep);
    if (rc != SR_OK) return rc;
    SR_CHECK(q.N % BIG == 0, SR_EUNSUPPORTED, "sr_gemm_group: N=%d must be a multiple of %d", q.N, BIG);
    GemmArgs& a = gg.g[i];
    a.group_m = tile_group_m(a.N);  // launch256's tile order
    const int nt = (a.N / BIG) * ((a.M + BIG - 1) / BIG);
    gg.start[i + 1] = gg.start[i] + (nt + 7) / 8 * 8;
  }
  for (int i = n + 1; i <= GROUP_MAX; ++i) gg.start[i] = gg.start[n];
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(gg.start[n]);
  // the LDS-staged RESID epilogue when every problem qualifies (gemm_args: alignment, the switch)
  bool rlds = epi == SR_EPI_BIAS_RESID;
  for (int i = 0; i < n; ++i) rlds = rlds && gg.g[i].resid_lds;
#define SR_GROUP_LAUNCH(E) hipLaunchKernelGGL((gemm256_group_kernel<E, false>), grid, dim3(512), 0, s, gg)
  switch (epi) {
    case SR_EPI_BIAS: SR_GROUP_LAUNCH(SR_EPI_BIAS); break;
    case SR_EPI_QKV: SR_GROUP_LAUNCH(SR_EPI_QKV); break;
    case SR_EPI_BIAS_GELU: SR_GROUP_LAUNCH(SR_EPI_BIAS_GELU); break;
    case SR_EPI_F32: SR_GROUP_LAUNCH(SR_EPI_F32); break;
    case SR_EPI_GELU_BWD: SR_GROUP_LAUNCH(SR_EPI_GELU_BWD); break;
    default:
      if (rlds) hipLaunchKernelGGL((gemm256_group_kernel<SR_EPI_BIAS_RESID, true>), grid, dim3(512), 0, s, gg);
      else SR_GROUP_LAUNCH(SR_EPI_BIAS_RESID);
  }
#undef SR_GROUP_LAUNCH
  sr::note_kernel("gemm256_group_kernel<%d, %s>", epi, rlds ? "true" : "false");  // as rocprofv3 names it
  return sr::check_launch("sr_gemm_group");
}

extern "C" int sr_gemm(sr_stream_t stream, int dtype, int epi, const void* A, int64_t lda, const void* W,
                       int64_t ldw, void* out, int64_t ldo, int M, int N, int K, const sr_gemm_epi* ep) {
  return gemm_common(stream, dtype, epi, A, lda, W, ldw, out, ldo, M, N, K, 1, nullptr, ep);
}

extern "C" int sr_gemm_splitk(sr_stream_t stream, int dtype, int epi, const void* A, int64_t lda, const void* W,
                              int64_t ldw, void* out, int64_t ldo, int M, int N, int K, int splits, float* workspace,
                              const sr_gemm_epi* ep) {
  SR_CHECK(splits >= 1, SR_EINVAL, "sr_gemm_splitk: splits=%d", splits);
  return gemm_common(stream, dtype, epi, A, lda, W, ldw, out, ldo, M, N, K, splits, workspace, ep);
}

extern "C" int sr_conv3x3_f32(sr_stream_t stream, const float* x, int n, int h, int w, int c, int stride, int relu_in,
                              const float* wgt, int cout, int epi, const sr_gemm_epi* ep, float* out, int64_t ldo,
                              const float* zero) {
  SR_CHECK(x && wgt && out && ep && zero, SR_EINVAL, "sr_conv3x3_f32: null pointer");
  SR_CHECK(n > 0 && h > 0 && w > 0 && c > 0 && c % 32 == 0 && (stride == 1 || stride == 2), SR_EUNSUPPORTED,
           "sr_conv3x3_f32: needs C %% 32 == 0 and stride 1 | 2 (n=%d h=%d w=%d c=%d stride=%d)", n, h, w, c, stride);
  SR_CHECK(cout > 0 && cout % 4 == 0 && ldo >= cout && ldo % 4 == 0, SR_EINVAL, "sr_conv3x3_f32: bad cout / ldo");
  SR_CHECK(epi == SR_EPI_BIAS || epi == SR_EPI_BIAS_RESID, SR_EUNSUPPORTED, "sr_conv3x3_f32: epilogue %d", epi);
  if (epi == SR_EPI_BIAS_RESID) SR_CHECK(ep->gamma, SR_EINVAL, "sr_conv3x3_f32: RESID needs gamma");
  SR_CHECK(((uintptr_t)x % 16) == 0 && ((uintptr_t)wgt % 16) == 0 && ((uintptr_t)out % 16) == 0 &&
               ((uintptr_t)zero % 16) == 0, SR_EINVAL, "sr_conv3x3_f32: pointers must be 16-B aligned");
  const int ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  SR_CHECK((int64_t)n * ho * wo < (1ll << 31), SR_EINVAL, "sr_conv3x3_f32: too many output pixels");
  GemmArgs a{};
  a.A = nullptr;
  a.lda_b = 0;
  a.W = (const char*)wgt;
  a.ldw_b = (int64_t)9 * c * 4;
  a.out = out;
  a.ldo = ldo;
  a.M = n * ho * wo;
  a.N = cout;
  a.K = 9 * c;
  a.ktiles = a.K / Mma<float>::KT;
  a.lds_epi = 0;
  a.kt_per_split = a.ktiles;
  a.partial = nullptr;
  a.ep = *ep;
  a.conv.x = (const char*)x;
  a.conv.zero = (const char*)zero;
  a.conv.H = h;
  a.conv.W = w;
  a.conv.C = c;
  a.conv.Ho = ho;
  a.conv.Wo = wo;
  a.conv.stride = stride;
  a.conv.relu = relu_in;
  hipStream_t s = (hipStream_t)stream;
  const bool no_narrow = sr::tune(SR_TUNE_CONV_NO_NARROW) != 0;
  if (!no_narrow && epi == SR_EPI_BIAS && cout <= NBN) {
    hipLaunchKernelGGL(conv_narrow_kernel, dim3((a.M + NBM - 1) / NBM), dim3(256), 0, s, a);
    return sr::check_launch("sr_conv3x3_f32(narrow)");
  }
  return epi == SR_EPI_BIAS ? launch_conv<SR_EPI_BIAS>(a, s) : launch_conv<SR_EPI_BIAS_RESID>(a, s);
}
