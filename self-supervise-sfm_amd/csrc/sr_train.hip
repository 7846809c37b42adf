// Training-step kernels for gfx950 (train_imc.py:320-429): the parts of
// the Block backward that are not attention (sr_attn_bwd.hip) or a dgrad GEMM (sr_gemm.hip
// with the GELU_BWD / F32 epilogues), plus the optimizer step.
//
//   sr_gemm_wgrad       dW = dY^T X  (nn.Linear weight grads), MFMA 32x32x16 bf16 with both
//                       operands read transposed from row-major LDS tiles (ds_read_b64_tr_b16)
//   sr_colsum           bias / token / positional-embedding grads (column sums)
//   sr_layernorm_bwd    LayerNorm backward with the residual accumulate and the bf16 operand copy
//   sr_qk_bwd           RoPE^T + qk-LayerNorm backward of the fused QKV epilogue
//   sr_cast_bf16, sr_nonfinite_check, sr_adam_f32
#include <algorithm>
#include <cfloat>
#include <cmath>

#include "sr_common.h"

namespace {

// ================================================================ weight gradient GEMM
// G[N,K] = sum_m A[m,n] B[m,k].  Workgroup = 128 (n) x 128 (k) output tile, 4 waves as 2 x 2,
// each 64 x 64 = 2 x 2 tiles of v_mfma_f32_32x32x16_bf16.  The reduction walks M in tiles of 64
// rows; a stage holds A[m0:m0+64, n0:n0+128] and B[m0:m0+64, k0:k0+128] as four 64-row x 64-col
// sub-tiles (128-B rows, 16-B chunk c of row r at c ^ (((r >> 1) & 1) << 2), the layout the
// transposed reads of sr_attn_bwd.hip expect), filled by LDS-DMA with the swizzle applied on the
// source address, double-buffered with one barrier per m-tile.  Operand fragments: A^T (rows = n)
// and B^T (columns = k) by ds_read_b64_tr_b16, both with the same k (= m) permutation.
constexpr int WT = 128;
constexpr int SUB = 64 * 128;    // one sub-tile, bytes
constexpr int WSTAGE = 4 * SUB;  // 32 KiB

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

struct TrOff {
  int off[2];
};
__device__ __forceinline__ TrOff tr_offsets(int lane) {
  const int hi = lane >> 5, G = lane >> 4, gi = lane & 15;
  const int vrow_in = gi >> 2;
  const int vcol_in = 16 * (G & 1) + 4 * (gi & 3);
  const int vsw = ((vrow_in >> 1) & 1) << 2;
  TrOff t;
  t.off[0] = (4 * hi + vrow_in) * 128 + (((vcol_in >> 3) ^ vsw) * 16) + (vcol_in & 7) * 2;
  t.off[1] = (4 * hi + vrow_in) * 128 + (((4 + (vcol_in >> 3)) ^ vsw) * 16) + (vcol_in & 7) * 2;
  return t;
}
// operand with rows = the tile's 32-column block db, k = tile rows row0 + {(e&3) + 8(e>>2) + 4hi}
__device__ __forceinline__ bf16x8 tr_frag(const char* tile, int row0, int off) {
  const char* pa = tile + row0 * 128 + off;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)pa);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)(pa + 8 * 128));
  const bf16x4 a4 = __builtin_bit_cast(bf16x4, a), b4 = __builtin_bit_cast(bf16x4, b);
  return bf16x8{a4[0], a4[1], a4[2], a4[3], b4[0], b4[1], b4[2], b4[3]};
}
__device__ __forceinline__ int acc_row(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

struct WgradArgs {
  const char* A;
  int64_t lda_b;
  const char* B;
  int64_t ldb_b;
  float* part;  // [splits][N][K]
  int M, N, K, mtiles, mt_per_split;
};

__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgradArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[2 * WSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int ntk = g.K / WT, ntiles = (g.N / WT) * ntk;
  const int tile = sr::xcd_remap(blockIdx.x, ntiles);
  const int tn = tile / ntk, tk = tile - tn * ntk;
  const int n0 = tn * WT, k0 = tk * WT;

  // wave w fills sub-tile w (0,1: A columns n0 + 64w; 2,3: B columns k0 + 64(w-2)), 8 DMAs of
  // 8 rows each; lane -> row 8i + (lane >> 3), LDS chunk slot lane & 7 <- source chunk slot ^ swz
  const char* base = wave < 2 ? g.A + (int64_t)(n0 + 64 * wave) * 2 : g.B + (int64_t)(k0 + 64 * (wave - 2)) * 2;
  const int64_t ld = wave < 2 ? g.lda_b : g.ldb_b;
  const int rsub = lane >> 3, slot = lane & 7;
  const uint32_t dst0 = __builtin_amdgcn_readfirstlane(sr::lds_addr(smem) + wave * SUB);
  auto stage = [&](int mt, int buf) {
    const uint32_t db = dst0 + buf * WSTAGE;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 8 * i + rsub;
      const int chunk = slot ^ (((r >> 1) & 1) << 2);
      const int row = min(mt * 64 + r, g.M - 1);
      sr::dma16(base + (int64_t)row * ld + chunk * 16, db + i * 1024);
    }
  };

  const int wr = wave >> 1, wc = wave & 1;
  const TrOff tro = tr_offsets(lane);
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int mt0 = blockIdx.y * g.mt_per_split;
  const int mt1 = min(mt0 + g.mt_per_split, g.mtiles);
  if (mt0 < mt1) stage(mt0, 0);
  for (int mt = mt0; mt < mt1; ++mt) {
    const int buf = (mt - mt0) & 1;
    sr::wait_vmcnt0();   // this wave's part of stage mt landed
    sr::barrier_raw();   // ... every wave's; every wave is done reading the other buffer
    if (mt + 1 < mt1) stage(mt + 1, buf ^ 1);
    char* sb = smem + buf * WSTAGE;
    const int valid = g.M - mt * 64;
    if (valid < 64) {  // ragged last m-tile: zero the clamped rows (uniform branch)
      for (int e = tid; e < 4 * 64 * 8; e += 256) {
        const int st = e >> 9, r = (e >> 3) & 63, c = e & 7;
        if (r >= valid) *(uint4*)(sb + st * SUB + r * 128 + c * 16) = uint4{0u, 0u, 0u, 0u};
      }
      __syncthreads();
    }
    const char* ta = sb + wr * SUB;
    const char* tb = sb + (2 + wc) * SUB;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = tr_frag(ta, 16 * s, tro.off[i]);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = tr_frag(tb, 16 * s, tro.off[j]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  // lane: column k = k0 + 64 wc + 32 j + l32, rows n = n0 + 64 wr + 32 i + acc_row(e, hi)
  float* part = g.part + (int64_t)blockIdx.y * g.N * g.K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = n0 + 64 * wr + 32 * i + acc_row(e, hi), k = k0 + 64 * wc + 32 * j + l32;
        part[(int64_t)n * g.K + k] = acc[i][j][e];
      }
}

// The same G = A^T B over 256 (n) x 256 (k) output tiles: 8 waves as 2 (n) x 4 (k), each 128 x 64 =
// 4 x 2 tiles of v_mfma_f32_32x32x16_bf16 (128 accumulator VGPRs), one workgroup per CU (128 KiB of
// LDS: two 64 KiB stages of eight 64-row x 64-col sub-tiles, A columns n0.. in sub-tiles 0-3 and B
// columns k0.. in 4-7, one per wave, same swizzle and transposed reads as wgrad_kernel).  Half the
// staged bytes per FLOP of the 128 x 128 tile; the reduction over M splits into gridDim.y slices
// whose fp32 partials wgrad_reduce_kernel sums.
constexpr int WT2 = 256;

// MT rows per m-tile, NST LDS stages (MT/8 DMA pieces per wave and stage): <64, 2> stages the next
// 64-row tile while computing the current one (a <48, 3> form with two 48-row tiles in flight measured
// no faster and was removed in round 6).
// Two problems of equal N and K in one launch (sr_gemm_wgrad_pair): slices blockIdx.y < y0 belong to
// g0, the rest to g1 (a single problem passes g1 = g0, y0 = its slice count).
template <int MT, int NST>
__global__ __launch_bounds__(512, 1) void wgrad256_kernel(WgradArgs g0, WgradArgs g1, int y0) {
  const bool second = (int)blockIdx.y >= y0;
  const WgradArgs g = second ? g1 : g0;
  const int ys = second ? (int)blockIdx.y - y0 : (int)blockIdx.y;
  constexpr int SUBT = MT * 128;  // one sub-tile: MT rows x 64 bf16 columns
  constexpr int STG = 8 * SUBT;
  constexpr int PCS = MT / 8;     // DMA wave-instructions per wave and stage
  __shared__ __attribute__((aligned(16))) char smem[NST * STG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int ntk = g.K / WT2, ntiles = (g.N / WT2) * ntk;
  const int tile = sr::xcd_remap(blockIdx.x, ntiles);
  const int tn = tile / ntk, tk = tile - tn * ntk;
  const int n0 = tn * WT2, k0 = tk * WT2;

  // wave w fills sub-tile w (0-3: A columns n0 + 64w; 4-7: B columns k0 + 64(w-4)), PCS DMAs of 8 rows
  const char* base = wave < 4 ? g.A + (int64_t)(n0 + 64 * wave) * 2 : g.B + (int64_t)(k0 + 64 * (wave - 4)) * 2;
  const int64_t ld = wave < 4 ? g.lda_b : g.ldb_b;
  const int rsub = lane >> 3, slot = lane & 7;
  const uint32_t dst0 = __builtin_amdgcn_readfirstlane(sr::lds_addr(smem) + wave * SUBT);
  auto stage = [&](int mt, int buf) {
    const uint32_t db = dst0 + buf * STG;
#pragma unroll
    for (int i = 0; i < PCS; ++i) {
      const int r = 8 * i + rsub;
      const int chunk = slot ^ (((r >> 1) & 1) << 2);
      const int row = min(mt * MT + r, g.M - 1);
      sr::dma16(base + (int64_t)row * ld + chunk * 16, db + i * 1024);
    }
  };

  const int wr = wave >> 2, wc = wave & 3;
  const TrOff tro = tr_offsets(lane);
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int mt0 = ys * g.mt_per_split;
  const int mt1 = min(mt0 + g.mt_per_split, g.mtiles);
#pragma unroll
  for (int j = 0; j < NST - 1; ++j)
    if (mt0 + j < mt1) stage(mt0 + j, j);
  int buf = 0;
  for (int mt = mt0; mt < mt1; ++mt) {
    // this wave's part of stage mt landed (the NST-2 later stages may stay in flight) ...
    if constexpr (NST == 3) {
      if (mt + 1 < mt1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PCS) : "memory");
      else sr::wait_vmcnt0();
    } else {
      sr::wait_vmcnt0();
    }
    sr::barrier_raw();   // ... every wave's; every wave is done reading the buffer restaged next
    if (mt + NST - 1 < mt1) stage(mt + NST - 1, buf == 0 ? NST - 1 : buf - 1);
    char* sb = smem + buf * STG;
    const int valid = g.M - mt * MT;
    if (valid < MT) {  // ragged last m-tile: zero the clamped rows (uniform branch)
      for (int e = tid; e < 8 * MT * 8; e += 512) {
        const int st = e / (MT * 8), r = (e >> 3) % MT, c = e & 7;
        if (r >= valid) *(uint4*)(sb + st * SUBT + r * 128 + c * 16) = uint4{0u, 0u, 0u, 0u};
      }
      __syncthreads();
    }
    const char* tb = sb + (4 + wc) * SUBT;
#pragma unroll
    for (int s = 0; s < MT / 16; ++s) {
      bf16x8 a[4], b[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = tr_frag(sb + (2 * wr + (i >> 1)) * SUBT, 16 * s, tro.off[i & 1]);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = tr_frag(tb, 16 * s, tro.off[j]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    buf = buf == NST - 1 ? 0 : buf + 1;
  }
  // lane: column k = k0 + 64 wc + 32 j + l32, rows n = n0 + 128 wr + 32 i + acc_row(e, hi)
  float* part = g.part + (int64_t)ys * g.N * g.K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = n0 + 128 * wr + 32 * i + acc_row(e, hi), k = k0 + 64 * wc + 32 * j + l32;
        part[(int64_t)n * g.K + k] = acc[i][j][e];
      }
}

// per output row n (one workgroup): slices summed in order, then scale / accumulate / rowdot
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int N, int K,
                                                           float* dW, int64_t lddw, int accumulate,
                                                           const float* __restrict__ rowscale,
                                                           const float* __restrict__ wdot, int64_t ldwd, float* rowdot) {
  __shared__ float red[4];
  const int n = blockIdx.x, tid = threadIdx.x;
  const float sc = rowscale ? rowscale[n] : 1.f;
  float dot = 0.f;
  for (int k = tid * 4; k < K; k += 1024) {
    f32x4 gsum = *(const f32x4*)(part + (int64_t)n * K + k);
    for (int z = 1; z < splits; ++z) gsum += *(const f32x4*)(part + ((int64_t)z * N + n) * K + k);
    if (wdot) {
      const f32x4 w = *(const f32x4*)(wdot + (int64_t)n * ldwd + k);
      dot += w[0] * gsum[0] + w[1] * gsum[1] + w[2] * gsum[2] + w[3] * gsum[3];
    }
    f32x4* o = (f32x4*)(dW + (int64_t)n * lddw + k);
    *o = accumulate ? *o + gsum * sc : gsum * sc;
  }
  if (wdot) {
    dot = sr::wave_sum(dot);
    if ((tid & 63) == 0) red[tid >> 6] = dot;
    __syncthreads();
    if (tid == 0) rowdot[n] += (red[0] + red[1]) + (red[2] + red[3]);
  }
}

// ================================================================ column sums
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const T* __restrict__ X, int64_t ldx, int M, int N,
                                                             int rows_per_chunk, float* __restrict__ part) {
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= N) return;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(M, r0 + rows_per_chunk);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  int r = r0;
  for (; r + 4 <= r1; r += 4) {  // 4 rows in flight
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const T* p = X + (int64_t)(r + u) * ldx + c;
      if constexpr (sr::is_bf16<T>::value) {
        const bf16x4 t = *(const bf16x4*)p;
        v[u] = f32x4{(float)t[0], (float)t[1], (float)t[2], (float)t[3]};
      } else {
        v[u] = *(const f32x4*)p;
      }
    }
    s += (v[0] + v[1]) + (v[2] + v[3]);
  }
  for (; r < r1; ++r) {
    const T* p = X + (int64_t)r * ldx + c;
    if constexpr (sr::is_bf16<T>::value) {
      const bf16x4 t = *(const bf16x4*)p;
      s += f32x4{(float)t[0], (float)t[1], (float)t[2], (float)t[3]};
    } else {
      s += *(const f32x4*)p;
    }
  }
  *(f32x4*)(part + (int64_t)blockIdx.y * N + c) = s;
}

// partial rows [chunks][N] -> out: workgroup = 16 column quads x 16 chunk groups; each thread sums
// its chunks z = g, g + 16, ... in order, then a fixed LDS tree over the 16 groups (deterministic)
// FMA form (sr_colsum_fma): out[c] += m1[c] * s[c] and o2[c] += m2[c] * s[c] for the pairs given
// (each as sr_vec_fma_f32 on the plain colsum's result: the same sum and the same fused multiply-add)
template <bool FMA = false>
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int chunks, int N,
                                                           float* out, int accumulate, float scale,
                                                           const float* __restrict__ m1 = nullptr, float* o2 = nullptr,
                                                           const float* __restrict__ m2 = nullptr) {
  __shared__ f32x4 red[16][16];
  const int qi = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t c = ((int64_t)blockIdx.x * 16 + qi) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    // four chunks in flight per step (independent sums, combined in a fixed order)
    f32x4 s1 = s, s2 = s, s3 = s;
    int z = g;
    for (; z + 48 < chunks; z += 64) {
      s += *(const f32x4*)(part + (int64_t)z * N + c);
      s1 += *(const f32x4*)(part + (int64_t)(z + 16) * N + c);
      s2 += *(const f32x4*)(part + (int64_t)(z + 32) * N + c);
      s3 += *(const f32x4*)(part + (int64_t)(z + 48) * N + c);
    }
    for (; z < chunks; z += 16) s += *(const f32x4*)(part + (int64_t)z * N + c);
    s = (s + s1) + (s2 + s3);
  }
  red[g][qi] = s;
  __syncthreads();
  for (int w = 8; w > 0; w >>= 1) {
    if (g < w) red[g][qi] += red[g + w][qi];
    __syncthreads();
  }
  if (g == 0 && c < N) {
    if constexpr (FMA) {
      const f32x4 sv = red[0][qi];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (out) out[c + e] = __builtin_fmaf(m1[c + e], sv[e], out[c + e]);
        if (o2) o2[c + e] = __builtin_fmaf(m2[c + e], sv[e], o2[c + e]);
      }
    } else {
      f32x4* o = (f32x4*)(out + c);
      *o = accumulate ? *o + red[0][qi] * scale : red[0][qi] * scale;
    }
  }
}

// row chunks of the partial pass (~1024 partial workgroups of >= 16 rows): the workspace holds
// chunks x N floats (sr_colsum_workspace_floats)
static int colsum_chunks(int M, int N, int& rpc) {
  const int64_t gx = (N / 4 + 255) / 256;
  const int chunks = (int)std::max<int64_t>(1, std::min<int64_t>((1024 + gx - 1) / gx, (M + 15) / 16));
  rpc = (M + chunks - 1) / chunks;
  return (M + rpc - 1) / rpc;
}

int colsum_launch(hipStream_t s, int dtype, const void* X, int64_t ldx, int M, int N, float* out, int accumulate,
                  float scale, float* ws, const float* m1 = nullptr, float* o2 = nullptr, const float* m2 = nullptr,
                  bool fma = false) {
  // ~1024 partial workgroups of >= 16 rows, then the parallel final reduction
  const int64_t gx = (N / 4 + 255) / 256;
  int rpc;
  const int chunks = colsum_chunks(M, N, rpc);
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(colsum_partial_kernel<bf16>, dim3((unsigned)gx, chunks), dim3(256), 0, s, (const bf16*)X, ldx,
                       M, N, rpc, ws);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<float>, dim3((unsigned)gx, chunks), dim3(256), 0, s, (const float*)X, ldx,
                       M, N, rpc, ws);
  if (fma)
    hipLaunchKernelGGL(colsum_final_kernel<true>, dim3((unsigned)((N / 4 + 15) / 16)), dim3(256), 0, s, ws, chunks, N,
                       out, 1, 1.f, m1, o2, m2);
  else
    hipLaunchKernelGGL(colsum_final_kernel<false>, dim3((unsigned)((N / 4 + 15) / 16)), dim3(256), 0, s, ws, chunks, N,
                       out, accumulate, scale, nullptr, nullptr, nullptr);
  return sr::check_launch("sr_colsum");
}

// dw | db (| dx_colsum) from layernorm_bwd_kernel's partial rows [nrows][np * cols] in ONE launch
// (was a partial + final colsum pair per output): workgroup = 4 column quads x 64 row groups, each
// thread sums rows g, g + 64, ... (four in flight), then a fixed LDS tree over the 64 groups
// (deterministic).  dw / db accumulate, dx_colsum is assigned.
__global__ __launch_bounds__(256) void lnb_final_kernel(const float* __restrict__ part, int nrows, int cols, int np,
                                                        float* dw, float* db, float* dxs) {
  __shared__ f32x4 red[64][4];
  const int qi = threadIdx.x & 3, g = threadIdx.x >> 2;
  const int N = np * cols;
  const int c = (blockIdx.x * 4 + qi) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    f32x4 s1 = s, s2 = s, s3 = s;
    int z = g;
    for (; z + 192 < nrows; z += 256) {
      s += *(const f32x4*)(part + (int64_t)z * N + c);
      s1 += *(const f32x4*)(part + (int64_t)(z + 64) * N + c);
      s2 += *(const f32x4*)(part + (int64_t)(z + 128) * N + c);
      s3 += *(const f32x4*)(part + (int64_t)(z + 192) * N + c);
    }
    for (; z < nrows; z += 64) s += *(const f32x4*)(part + (int64_t)z * N + c);
    s = (s + s1) + (s2 + s3);
  }
  red[g][qi] = s;
  __syncthreads();
  for (int w = 32; w > 0; w >>= 1) {
    if (g < w) red[g][qi] += red[g + w][qi];
    __syncthreads();
  }
  if (g == 0 && c < N) {  // cols % 4 == 0: a quad never straddles two outputs
    const int seg = c / cols, cc = c - seg * cols;
    f32x4* o = (f32x4*)((seg == 0 ? dw : seg == 1 ? db : dxs) + cc);
    *o = seg < 2 ? *o + red[0][qi] : red[0][qi];
  }
}

// ================================================================ LayerNorm backward
// One wave per row (grid-stride); lane owns columns (i*64 + lane)*VEC + j as sr_layernorm.
// dw / db: per-wave partial sums in registers, written to workspace [nwaves][2][cols] and
// reduced by colsum.
constexpr int LNB_WGS = 256;  // workgroups (x 4 waves = partial rows)

template <int NPL, int VEC, typename TD>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                            const int32_t* __restrict__ rowmap,
                                                            const TD* __restrict__ dy, int64_t lddy,
                                                            const float* __restrict__ w, float eps, float* dx,
                                                            int64_t lddx, bf16* dxb, int64_t lddxb, int want_params,
                                                            int want_sum, float* part, int rows) {
  constexpr int NV = NPL / VEC;
  constexpr int COLS = NPL * 64;
  // the column sum of the updated dx rows rides along as a third partial (cols <= 2048: the
  // register file of the 4,096-column form has no room for it)
  constexpr bool CAN_SUM = NPL <= 32;
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  float wv[NPL], dws[NPL], dbs[NPL], dss[CAN_SUM ? NPL : 1];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      wv[i * VEC + j] = w ? w[(i * 64 + lane) * VEC + j] : 1.f;
      dws[i * VEC + j] = 0.f;
      dbs[i * VEC + j] = 0.f;
      if constexpr (CAN_SUM) dss[i * VEC + j] = 0.f;
    }
  // Two rows per wave per iteration, and the dx each adds into loaded with x and dy: all loads of
  // both rows are in flight before the first reduction (one memory latency per two rows, not two
  // per row -- 1,024 waves alone do not cover HBM latency).
  auto load = [&](int64_t xr, int row, float* v, float* g, float* a) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = (i * 64 + lane) * VEC;
      const float* xp = x + xr * ldx + col;
      const TD* gp = dy + (int64_t)row * lddy + col;
      const float* ap = dx + xr * lddx + col;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        v[i * VEC + j] = xp[j];
        g[i * VEC + j] = sr::to_f32(gp[j]);
        if constexpr (NPL <= 32) a[i * VEC + j] = ap[j];
      }
    }
  };
  auto finish = [&](int64_t xr, int row, float* v, float* g, const float* a) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) s += v[i];
    const float mean = sr::wave_sum(s) * (1.f / COLS);
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      v[i] -= mean;
      s2 += v[i] * v[i];
    }
    const float rstd = rsqrtf(sr::wave_sum(s2) * (1.f / COLS) + eps);
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      v[i] *= rstd;  // xhat
      if (want_params) {
        dws[i] += g[i] * v[i];
        dbs[i] += g[i];
      }
      g[i] *= wv[i];
      sg += g[i];
      sgx += g[i] * v[i];
    }
    const float mg = sr::wave_sum(sg) * (1.f / COLS), mgx = sr::wave_sum(sgx) * (1.f / COLS);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = (i * 64 + lane) * VEC;
      float* dp = dx + xr * lddx + col;
      float o[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        o[j] = (NPL <= 32 ? a[i * VEC + j] : dp[j]) + rstd * (g[i * VEC + j] - mg - v[i * VEC + j] * mgx);
        if constexpr (CAN_SUM)
          if (want_sum) dss[i * VEC + j] += o[j];
      }
      if constexpr (VEC == 4) {
        *(float4*)dp = make_float4(o[0], o[1], o[2], o[3]);
        if (dxb) *(bf16x4*)(dxb + (int64_t)row * lddxb + col) = bf16x4{(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
      } else {
        *(float2*)dp = make_float2(o[0], o[1]);
        if (dxb) {
          bf16* q = dxb + (int64_t)row * lddxb + col;
          q[0] = (bf16)o[0];
          q[1] = (bf16)o[1];
        }
      }
    }
  };
  if constexpr (NPL > 32) {  // 4,096 columns: one row per iteration, dx read late (register file)
    for (int row = gw; row < rows; row += nw) {
      const int64_t xr = rowmap ? (int64_t)rowmap[row] : row;
      float v[NPL], g[NPL];
      load(xr, row, v, g, nullptr);
      finish(xr, row, v, g, nullptr);
    }
  } else for (int row = gw; row < rows; row += 2 * nw) {
    const int rowb = row + nw;
    const bool has_b = rowb < rows;  // wave-uniform
    const int64_t xa = rowmap ? (int64_t)rowmap[row] : row;
    const int64_t xb = has_b ? (rowmap ? (int64_t)rowmap[rowb] : rowb) : xa;
    float va[NPL], ga[NPL], aa[NPL], vb[NPL], gb[NPL], ab[NPL];
    load(xa, row, va, ga, aa);
    load(xb, has_b ? rowb : row, vb, gb, ab);
    finish(xa, row, va, ga, aa);
    if (has_b) finish(xb, rowb, vb, gb, ab);
  }
  if (want_params) {  // [nw][2 or 3][COLS]: dw, db (, dx) partials
    const int np = (CAN_SUM && want_sum) ? 3 : 2;
    float* pw = part + (int64_t)gw * np * COLS;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const int col = (i * 64 + lane) * VEC + j;
        pw[col] = dws[i * VEC + j];
        pw[COLS + col] = dbs[i * VEC + j];
        if constexpr (CAN_SUM)
          if (want_sum) pw[2 * COLS + col] = dss[i * VEC + j];
      }
  }
}

// ================================================================ qk-norm + RoPE backward
// One wave per row; 4 heads per pass (16 lanes x 4 values per head: dims 4 li .. 4 li + 3).
// RoPE pairs (d, d + 16) of each half sit in lanes li and li ^ 4.
// T = bf16 (autocast blocks) or float (fp32 blocks): the type of raw and out.
// The column blocks of 1,024 are the OUTER loop (each wave walks its rows once per block), so that
// with ep.colsum a lane sums the values it stores for its 16 columns of the block in registers
// (rows in order); at the end of a block the workgroup's 4 wave rows meet in LDS and sum into one
// partial row [blockIdx.x][ncols] of cpart; the host sums those rows into ep.colsum (a fixed order).
// (An LDS row per wave across the whole row loop cost 48 KiB of LDS per workgroup: 3 workgroups per
// CU, and 1.5x the kernel time.)
constexpr int QKB_PASSES = 3;  // ncols <= 3072 with ep.colsum
template <typename T, bool CS>
__global__ __launch_bounds__(256) void qk_bwd_kernel(const T* __restrict__ raw, int64_t ldr,
                                                     const float* __restrict__ dsrc, int64_t lds, T* out,
                                                     int64_t ldo, int rows, int ncols, sr_gemm_epi ep, float* part,
                                                     float* cpart) {
  __shared__ float csl[4][1024];  // ep.colsum: the 4 waves' sums of one column block
  constexpr bool BF = sr::is_bf16<T>::value;
  const int lane = threadIdx.x & 63, li = lane & 15;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  const int C = ep.embed_dim;
  const bool norm = ep.qn_w != nullptr;
  const bool rope = ep.rope_cos != nullptr;
  const bool first = (li & 4) == 0;  // first element of its RoPE pair
  const int fj = 4 * (li & 3);       // frequency index of element 0
  const bool xhalf = li >= 8;
  float wq[4], bq[4], wk[4], bk[4];
  float acc[4][4];  // dqn_w, dqn_b, dkn_w, dkn_b (this lane's 4 dims, summed over rows and heads)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    wq[e] = norm ? ep.qn_w[4 * li + e] : 1.f;
    bq[e] = norm ? ep.qn_b[4 * li + e] : 0.f;
    wk[e] = norm ? ep.kn_w[4 * li + e] : 1.f;
    bk[e] = norm ? ep.kn_b[4 * li + e] : 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t][e] = 0.f;
  }
  (void)bq;
  (void)bk;
  // CS (ep.colsum): the column blocks outer, one per row pass; otherwise every block of a row in turn
  for (int cbo = 0; cbo < (CS ? ncols : 1); cbo += 1024) {
  f32x4 csa[4] = {};  // CS: this lane's columns cbo + 256 p + 4 lane .. + 4, summed over its rows
  for (int row = gw; row < rows; row += nw) {
    float cs[4] = {1.f, 1.f, 1.f, 1.f}, sn[4] = {0.f, 0.f, 0.f, 0.f};
    if (rope) {
      int py, px;
      sr::rope_pos(ep, row, py, px);
      const int p = xhalf ? px : py;
      const float4 c4 = *(const float4*)(ep.rope_cos + p * 16 + fj);
      const float4 s4 = *(const float4*)(ep.rope_sin + p * 16 + fj);
      cs[0] = c4.x; cs[1] = c4.y; cs[2] = c4.z; cs[3] = c4.w;
      sn[0] = s4.x; sn[1] = s4.y; sn[2] = s4.z; sn[3] = s4.w;
    }
    // passes of 4 heads (256 columns) in groups of 4: every load of a group is issued before its
    // math (16 heads of loads in flight per wave; one pass at a time left HBM latency exposed).
    // cb re-read per row: hoisting the 4 passes' column / region / weight selections out of the
    // row loop costs more registers than it saves instructions
    for (int cb_ = CS ? cbo : 0; cb_ < (CS ? cbo + 1 : ncols); cb_ += 1024) {
      int cb = cb_;
      if constexpr (CS) asm volatile("" : "+s"(cb));
      float4 d4s[4];
      f32x4 r4s[4] = {};
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        // a short last pass computes on clamped columns and stores nothing
        const int col = min(cb + 256 * p + 4 * lane, ncols - 4);
        d4s[p] = *(const float4*)(dsrc + (int64_t)row * lds + col);
        if (norm && (col + ep.col_offset) / C < 2) {
          if constexpr (BF) {
            const bf16x4 r = *(const bf16x4*)(raw + (int64_t)row * ldr + col);
            r4s[p] = f32x4{(float)r[0], (float)r[1], (float)r[2], (float)r[3]};
          } else {
            r4s[p] = *(const f32x4*)(raw + (int64_t)row * ldr + col);
          }
        }
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
      const int c0 = cb + 256 * p;
      if (c0 < ncols) {
      const bool live = c0 + 4 * lane < ncols;
      const int col = min(c0 + 4 * lane, ncols - 4);
      const int region = (col + ep.col_offset) / C;
      const float4 d4 = d4s[p];
      float d[4] = {d4.x, d4.y, d4.z, d4.w};
      if (region < 2) {
        if (rope) {  // inverse rotation: first a: da = c dA + s dB; second b: db = c dB - s dA
          float pd[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) pd[e] = sr::dpp_xor4(d[e]);
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = first ? fmaf(cs[e], d[e], sn[e] * pd[e]) : fmaf(cs[e], d[e], -sn[e] * pd[e]);
        }
        if (norm) {
          const f32x4 r4 = r4s[p];
          float v[4] = {r4[0], r4[1], r4[2], r4[3]};
          const float mean = sr::dpp_sum16((v[0] + v[1]) + (v[2] + v[3])) * (1.f / 64.f);
          float s2 = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] -= mean;
            s2 += v[e] * v[e];
          }
          s2 = sr::dpp_sum16(s2);
          const float rstd = rsqrtf(s2 * (1.f / 64.f) + ep.qk_eps);
          float wv[4];  // selected per element: a pointer / index select here demoted the arrays to scratch
#pragma unroll
          for (int e = 0; e < 4; ++e) wv[e] = region == 0 ? wq[e] : wk[e];
          float g[4], sg = 0.f, sgx = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] *= rstd;
            if (live) {
              const float gw_ = d[e] * v[e];
              if (region == 0) {
                acc[0][e] += gw_;
                acc[1][e] += d[e];
              } else {
                acc[2][e] += gw_;
                acc[3][e] += d[e];
              }
            }
            g[e] = d[e] * wv[e];
            sg += g[e];
            sgx += g[e] * v[e];
          }
          sg = sr::dpp_sum16(sg);
          sgx = sr::dpp_sum16(sgx);
          sg *= 1.f / 64.f;
          sgx *= 1.f / 64.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = rstd * (g[e] - sg - v[e] * sgx);
        }
      }
      if (live) {
        if constexpr (BF)
          *(bf16x4*)(out + (int64_t)row * ldo + col) = bf16x4{(bf16)d[0], (bf16)d[1], (bf16)d[2], (bf16)d[3]};
        else
          *(f32x4*)(out + (int64_t)row * ldo + col) = f32x4{d[0], d[1], d[2], d[3]};
        if constexpr (CS) {
#pragma unroll
          for (int e = 0; e < 4; ++e) csa[p][e] += sr::to_f32(sr::from_f32<T>(d[e]));
        }
      }
      }
      }
    }
  }
  if constexpr (CS) {  // the workgroup's 4 wave sums of this block -> its partial row (fixed order)
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int p = 0; p < 4; ++p) *(f32x4*)(&csl[w][256 * p + 4 * lane]) = csa[p];
    __syncthreads();
    for (int c = threadIdx.x; c < 1024 && cbo + c < ncols; c += 256)
      cpart[(int64_t)blockIdx.x * ncols + cbo + c] = (csl[0][c] + csl[1][c]) + (csl[2][c] + csl[3][c]);
    __syncthreads();
  }
  }
  if (norm) {  // lanes li, li+16, li+32, li+48 hold the same dims
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[t][e] += __shfl_xor(acc[t][e], 16, 64);
        acc[t][e] += __shfl_xor(acc[t][e], 32, 64);
      }
    if (lane < 16) {
      float* pw = part + (int64_t)gw * 256;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) pw[t * 64 + 4 * li + e] = acc[t][e];
    }
  }
}

// ================================================================ elementwise / optimizer
__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ src, int64_t lds, bf16* dst,
                                                        int64_t ldd, int rows, int cols, float scale) {
  const int cq = cols / 4;
  const int64_t n = (int64_t)rows * cq;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int r = (int)(e / cq), c = (int)(e - (int64_t)r * cq) * 4;
    const float4 v = *(const float4*)(src + (int64_t)r * lds + c);
    *(bf16x4*)(dst + (int64_t)r * ldd + c) =
        bf16x4{(bf16)(v.x * scale), (bf16)(v.y * scale), (bf16)(v.z * scale), (bf16)(v.w * scale)};
  }
}

__global__ __launch_bounds__(256) void nonfinite_kernel(const float* __restrict__ g, int64_t n,
                                                        const float* __restrict__ scale, int* found) {
  const float inv = scale ? 1.f / *scale : 1.f;
  int bad = 0;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    bad |= !isfinite(g[e] * inv);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(found, 1);
}

// One element of the Adam update, in the operation order of torch.optim.Adam's single-tensor step
// (the reference's optimizer, train_imc.py:475) with its pointwise kernels' contractions:
//   grad.add(p, alpha=wd)            -> fma(wd, p, g)
//   m.lerp_(g, 1 - b1)  (weight < .5) -> fma(1 - b1, g - m, m)
//   v.mul_(b2).addcmul_(g, g, 1 - b2) -> fma((1 - b2) g, g, b2 v)
//   p.addcdiv_(m, denom, -step_size)  -> fma(-step_size, m / denom, p)
// Contraction is off and every FMA is explicit, so the float4 path and the scalar tail round
// identically (one function, one rounding sequence).
__device__ __forceinline__ void adam_elem(float g, float& p, float& m, float& v, float inv, float beta1, float beta2,
                                          float eps, float wd, float bc2_sqrt, float step_size) {
#pragma clang fp contract(off)
  float gr = g * inv;
  if (wd != 0.f) gr = fmaf(wd, p, gr);
  const float mn = fmaf(1.f - beta1, gr - m, m);
  const float vn = fmaf((1.f - beta2) * gr, gr, beta2 * v);
  const float denom = sqrtf(vn) / bc2_sqrt + eps;
  p = fmaf(-step_size, mn / denom, p);
  m = mn;
  v = vn;
}

__global__ __launch_bounds__(256) void adam_kernel(float* p, const float* __restrict__ g, float* m, float* v,
                                                   int64_t n, float lr, float beta1, float beta2, float eps, float wd,
                                                   float bc1, float bc2_sqrt, const float* __restrict__ scale,
                                                   const int* __restrict__ found) {
  if (found && *found) return;  // GradScaler.step skips the update on inf / nan
  const float inv = scale ? 1.f / *scale : 1.f;
  const float step_size = lr / bc1;
  int64_t e0 = 0;
  if ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0) {
    // 16-B aligned (the flat parameter buffers): four elements per thread and iteration; the scalar
    // loop below then takes the n % 4 tail
    const int64_t n4 = n >> 2;
    for (int64_t q = blockIdx.x * 256ll + threadIdx.x; q < n4; q += (int64_t)gridDim.x * 256) {
      const f32x4 g4 = ((const f32x4*)g)[q];
      f32x4 p4 = ((const f32x4*)p)[q], m4 = ((const f32x4*)m)[q], v4 = ((const f32x4*)v)[q];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = p4[j], mj = m4[j], vj = v4[j];
        adam_elem(g4[j], pj, mj, vj, inv, beta1, beta2, eps, wd, bc2_sqrt, step_size);
        p4[j] = pj;
        m4[j] = mj;
        v4[j] = vj;
      }
      ((f32x4*)m)[q] = m4;
      ((f32x4*)v)[q] = v4;
      ((f32x4*)p)[q] = p4;
    }
    e0 = n4 << 2;
  }
  for (int64_t e = e0 + blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    float pe = p[e], me = m[e], ve = v[e];
    adam_elem(g[e], pe, me, ve, inv, beta1, beta2, eps, wd, bc2_sqrt, step_size);
    m[e] = me;
    v[e] = ve;
    p[e] = pe;
  }
}


// ================================================================ weight packs for the dgrad GEMMs
// dst[c][r] = T(rowscale[r] * src[r][c])  (the W^T operand of dX = dY . W, with LayerScale gamma
// folded into the rows of W); 64 x 64 LDS tiles, padded against bank conflicts.
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ src, int64_t lds, int R, int C,
                                                        const float* __restrict__ rowscale, T* dst, int64_t ldd) {
  __shared__ float tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? src[(int64_t)r * lds + c] * (rowscale ? rowscale[r] : 1.f) : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) dst[(int64_t)c * ldd + r] = sr::from_f32<T>(tile[tx][i]);
  }
}

// ================================================================ small fp32 backward (camera head)
// dW[n][k] (+)= sum_m A[m][n] B[m][k] for few rows M (camera trunk / pose branch: M = 2N views);
// thread = one (n, k); db[n] (+)= sum_m A[m][n] from the k == 0 threads.
__global__ __launch_bounds__(256) void wgrad_small_kernel(const float* __restrict__ A, int64_t lda,
                                                          const float* __restrict__ B, int64_t ldb, float* dW,
                                                          int64_t lddw, int M, int N, int K, int accumulate, float* db) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)N * K) return;
  const int n = (int)(e / K), k = (int)(e - (int64_t)n * K);
  float s = 0.f, sb = 0.f;
  for (int m = 0; m < M; ++m) {
    const float a = A[(int64_t)m * lda + n];
    s = fmaf(a, B[(int64_t)m * ldb + k], s);
    sb += a;
  }
  float* o = dW + (int64_t)n * lddw + k;
  *o = accumulate ? *o + s : s;
  if (db && k == 0) db[n] = accumulate ? db[n] + sb : sb;
}

// Masked fp32 attention backward for one batch item of few rows (camera trunk: L = 2N tokens,
// head_dim 128, SR_MASK_CAMERA = ~build_lr_mask, camera_head.py:165,197-228).
// Pass 1, one workgroup per (query row i, head): scores over all allowed keys, softmax, P and
// dS = P (dP - sum_j P dP) into workspace [heads][L][L].  Pass 2: dQ = c dS K, dK = c dS^T Q,
// dV = P^T dO, one thread per output element.
__device__ __forceinline__ bool cam_allowed(int mask_mode, int n_anchor, int i, int j) {
  return mask_mode != SR_MASK_CAMERA || j < n_anchor || j == i;
}

__global__ __launch_bounds__(256) void attn_bwd_small_p_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                               const float* __restrict__ v, int64_t ld,
                                                               const float* __restrict__ dout, int64_t lddo, int L, int D,
                                                               float scale, int mask_mode, int n_anchor, float* P,
                                                               float* dS) {
  __shared__ float red[2][4];
  const int i = blockIdx.x, h = blockIdx.y, tid = threadIdx.x;
  const float* qi = q + (int64_t)i * ld + h * D;
  const float* gi = dout + (int64_t)i * lddo + h * D;
  float* Pi = P + ((int64_t)h * L + i) * L;
  float* dSi = dS + ((int64_t)h * L + i) * L;
  // scores / dP for keys j = tid, tid + 256, ...  (L <= 1024: 4 per thread)
  float sc[4], dp[4];
  float mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = tid + 256 * u;
    sc[u] = -INFINITY;
    dp[u] = 0.f;
    if (j < L && cam_allowed(mask_mode, n_anchor, i, j)) {
      const float* kj = k + (int64_t)j * ld + h * D;
      const float* vj = v + (int64_t)j * ld + h * D;
      float s = 0.f, d = 0.f;
      for (int c = 0; c < D; ++c) {
        s = fmaf(qi[c], kj[c], s);
        d = fmaf(gi[c], vj[c], d);
      }
      sc[u] = s * scale;
      dp[u] = d;
      mx = fmaxf(mx, sc[u]);
    }
  }
  mx = sr::wave_max(mx);
  if ((tid & 63) == 0) red[0][tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
  float sum = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    sc[u] = sc[u] == -INFINITY ? 0.f : expf(sc[u] - mx);
    sum += sc[u];
  }
  sum = sr::wave_sum(sum);
  __syncthreads();
  if ((tid & 63) == 0) red[0][tid >> 6] = sum;
  __syncthreads();
  const float inv = 1.f / ((red[0][0] + red[0][1]) + (red[0][2] + red[0][3]));
  float pd = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    sc[u] *= inv;
    pd += sc[u] * dp[u];
  }
  pd = sr::wave_sum(pd);
  if ((tid & 63) == 0) red[1][tid >> 6] = pd;
  __syncthreads();
  const float delta = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = tid + 256 * u;
    if (j < L) {
      Pi[j] = sc[u];
      dSi[j] = sc[u] * (dp[u] - delta);
    }
  }
}

__global__ __launch_bounds__(256) void attn_bwd_small_grad_kernel(const float* __restrict__ q,
                                                                  const float* __restrict__ k, int64_t ld,
                                                                  const float* __restrict__ dout, int64_t lddo, int L,
                                                                  int D, int H, float scale, const float* __restrict__ P,
                                                                  const float* __restrict__ dS, float* dq, float* dk,
                                                                  float* dv, int64_t ldg) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per = (int64_t)L * H * D;
  if (e >= 3 * per) return;
  const int which = (int)(e / per);
  const int64_t r = e - which * per;
  const int row = (int)(r / (H * D)), hc = (int)(r - (int64_t)row * H * D), h = hc / D;
  const float* Ph = P + (int64_t)h * L * L;
  const float* dSh = dS + (int64_t)h * L * L;
  float s = 0.f;
  if (which == 0) {  // dQ[i] = c sum_j dS[i][j] K[j]
    for (int j = 0; j < L; ++j) s = fmaf(dSh[(int64_t)row * L + j], k[(int64_t)j * ld + hc], s);
    dq[(int64_t)row * ldg + hc] = s * scale;
  } else if (which == 1) {  // dK[j] = c sum_i dS[i][j] Q[i]
    for (int i = 0; i < L; ++i) s = fmaf(dSh[(int64_t)i * L + row], q[(int64_t)i * ld + hc], s);
    dk[(int64_t)row * ldg + hc] = s * scale;
  } else {  // dV[j] = sum_i P[i][j] dO[i]
    for (int i = 0; i < L; ++i) s = fmaf(Ph[(int64_t)i * L + row], dout[(int64_t)i * lddo + hc], s);
    dv[(int64_t)row * ldg + hc] = s;
  }
}

// adaLN backward (camera_head.py:156-161): xm = gate * (xn (1 + scale) + shift) + x
//   dxn = dxm gate (1 + scale);  dmod = [dshift | dscale | dgate] = [dxm gate | dxm gate xn | dxm (xn (1 + scale) + shift)]
__global__ void adaln_bwd_kernel(const float* __restrict__ xn, const float* __restrict__ mod,
                                 const float* __restrict__ dxm, float* dxn, float* dmod, int rows, int cols) {
  const int64_t total = (int64_t)rows * cols;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % cols);
    const int64_t r = e / cols;
    const float* mr = mod + r * 3 * cols;
    const float shift = mr[c], scale = mr[cols + c], gate = mr[2 * cols + c];
    const float g = dxm[e], x = xn[e];
    dxn[e] = g * gate * (1.f + scale);
    float* dm = dmod + r * 3 * cols;
    dm[c] = g * gate;
    dm[cols + c] = g * gate * x;
    dm[2 * cols + c] = g * (x * (1.f + scale) + shift);
  }
}

// elementwise activation backward: mode 0 SiLU (poseLN_modulation[0]), 1 erf-GELU (Mlp.act)
__global__ void act_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* dx, int64_t n,
                               int mode) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[e];
    float d;
    if (mode == 0) {
      const float sg = 1.f / (1.f + expf(-v));
      d = sg * (1.f + v * (1.f - sg));
    } else {
      d = sr::gelu_erf_grad<false>(v);
    }
    dx[e] = dy[e] * d;
  }
}

// dst[rowmap[r]] (+)= src[r]  (lds 0: one broadcast row), cols % 4 == 0
__global__ __launch_bounds__(256) void scatter_rows_kernel(float* dst, int64_t ldd, const int32_t* __restrict__ rowmap,
                                                           const float* __restrict__ src, int64_t lds, int rows,
                                                           int cols, int accumulate) {
  const int cq = cols / 4;
  const int64_t n = (int64_t)rows * cq;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int r = (int)(e / cq), c = (int)(e - (int64_t)r * cq) * 4;
    const f32x4 v = *(const f32x4*)(src + (int64_t)r * lds + c);
    f32x4* d = (f32x4*)(dst + (int64_t)rowmap[r] * ldd + c);
    *d = accumulate ? *d + v : v;
  }
}

// dst[r][c] (+)= src[r][c] for any cols (strided fp32 2-D copy / accumulate)
__global__ __launch_bounds__(256) void copy2d_kernel(float* dst, int64_t ldd, const float* __restrict__ src,
                                                     int64_t lds, int rows, int cols, int accumulate) {
  const int64_t n = (int64_t)rows * cols;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int r = (int)(e / cols), c = (int)(e - (int64_t)r * cols);
    const float v = src[(int64_t)r * lds + c];
    float* d = dst + (int64_t)r * ldd + c;
    *d = accumulate ? *d + v : v;
  }
}

// activate_pose backward (head_act.py:12-60, linear T / quat, ReLU FoV) for the camera head's
// last iteration: dd[r] = 0 for anchor rows r < n_anchor, else d_act[r - n_anchor] * (c < 7 || act > 0)
__global__ void pose_act_bwd_kernel(float* dd, const float* __restrict__ d_act, const float* __restrict__ act, int rows,
                                    int n_anchor) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * 9) return;
  const int r = e / 9, c = e - r * 9;
  float v = 0.f;
  if (r >= n_anchor) {
    v = d_act[(r - n_anchor) * 9 + c];
    if (c >= 7 && !(act[e] > 0.f)) v = 0.f;
  }
  dd[e] = v;
}

// out[i] += a[i] * b[i]  (LayerScale gamma / bias grads from column sums)
__global__ void vec_fma_kernel(float* out, const float* __restrict__ a, const float* __restrict__ b, int n,
                               float* out2, const float* __restrict__ a2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    out[i] = __builtin_fmaf(a[i], b[i], out[i]);
    if (out2) out2[i] = __builtin_fmaf(a2[i], b[i], out2[i]);
  }
}

unsigned grid_for(int64_t n, int64_t cap = 4096) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, cap));
}

}  // namespace

// ---------------------------------------------------------------------------------------
namespace {
int wgrad_check(const void* A, int64_t lda, const void* B, int64_t ldb, float* dW, int64_t lddw, int M, int N, int K,
                const float* wdot, int64_t ldwd, float* rowdot, int splits, float* workspace) {
  SR_CHECK(A && B && dW && workspace, SR_EINVAL, "sr_gemm_wgrad: null pointer");
  SR_CHECK(M > 0 && N > 0 && K > 0 && N % WT == 0 && K % WT == 0, SR_EUNSUPPORTED,
           "sr_gemm_wgrad: N=%d, K=%d must be multiples of 128 (M=%d)", N, K, M);
  SR_CHECK(lda >= N && ldb >= K && lda % 8 == 0 && ldb % 8 == 0 && lddw >= K && lddw % 4 == 0 &&
               ((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0 && ((uintptr_t)dW % 16) == 0,
           SR_EINVAL, "sr_gemm_wgrad: bad leading dims / alignment");
  SR_CHECK(!wdot || (rowdot && ldwd >= K && ldwd % 4 == 0), SR_EINVAL, "sr_gemm_wgrad: wdot needs rowdot");
  SR_CHECK(splits >= 1, SR_EINVAL, "sr_gemm_wgrad: splits=%d", splits);
  return SR_OK;
}

// kernel arguments of one problem; `splits` is clamped to the slices that get m-tiles
WgradArgs wgrad_args(const void* A, int64_t lda, const void* B, int64_t ldb, int M, int N, int K, int mt, int& splits,
                     float* workspace) {
  WgradArgs g;
  g.A = (const char*)A;
  g.lda_b = lda * 2;
  g.B = (const char*)B;
  g.ldb_b = ldb * 2;
  g.part = workspace;
  g.M = M;
  g.N = N;
  g.K = K;
  g.mtiles = (M + mt - 1) / mt;
  splits = std::min(splits, g.mtiles);
  g.mt_per_split = (g.mtiles + splits - 1) / splits;
  splits = (g.mtiles + g.mt_per_split - 1) / g.mt_per_split;
  return g;
}
}  // namespace

extern "C" int sr_gemm_wgrad(sr_stream_t stream, const void* A, int64_t lda, const void* B, int64_t ldb, float* dW,
                             int64_t lddw, int M, int N, int K, int accumulate, const float* rowscale,
                             const float* wdot, int64_t ldwd, float* rowdot, int splits, float* workspace) {
  const int rc = wgrad_check(A, lda, B, ldb, dW, lddw, M, N, K, wdot, ldwd, rowdot, splits, workspace);
  if (rc != SR_OK) return rc;
  // 256 x 256 tiles (one workgroup per CU) for the aggregator shapes; SR_WGRAD256=0: 128 x 128
  const bool big = sr::tune(SR_TUNE_WGRAD256) != 0 && N % WT2 == 0 && K % WT2 == 0;
  const WgradArgs g = wgrad_args(A, lda, B, ldb, M, N, K, 64, splits, workspace);
  hipStream_t s = (hipStream_t)stream;
  if (big) {
    hipLaunchKernelGGL((wgrad256_kernel<64, 2>), dim3((N / WT2) * (K / WT2), splits), dim3(512), 0, s, g, g, splits);
    sr::note_kernel("wgrad256_kernel");
  } else {
    hipLaunchKernelGGL(wgrad_kernel, dim3((N / WT) * (K / WT), splits), dim3(256), 0, s, g);
    sr::note_kernel("wgrad_kernel");
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(N), dim3(256), 0, s, workspace, splits, N, K, dW, lddw, accumulate,
                     rowscale, wdot, ldwd, rowdot);
  return sr::check_launch("sr_gemm_wgrad");
}

extern "C" int sr_gemm_wgrad_pair(sr_stream_t stream, const sr_wgrad_problem* p) {
  SR_CHECK(p, SR_EINVAL, "sr_gemm_wgrad_pair: null problems");
  for (int i = 0; i < 2; ++i) {
    const int rc = wgrad_check(p[i].A, p[i].lda, p[i].B, p[i].ldb, p[i].dW, p[i].lddw, p[i].M, p[i].N, p[i].K,
                               p[i].wdot, p[i].ldwd, p[i].rowdot, p[i].splits, p[i].workspace);
    if (rc != SR_OK) return rc;
  }
  const int N = p[0].N, K = p[0].K;
  SR_CHECK(p[1].N == N && p[1].K == K && N % WT2 == 0 && K % WT2 == 0, SR_EUNSUPPORTED,
           "sr_gemm_wgrad_pair: both problems need the same N, K, multiples of %d (%dx%d, %dx%d)", WT2, N, K, p[1].N,
           p[1].K);
  SR_CHECK(sr::tune(SR_TUNE_WGRAD256) != 0, SR_EUNSUPPORTED, "sr_gemm_wgrad_pair: needs the 256x256 kernel");
  int sp[2] = {p[0].splits, p[1].splits};
  WgradArgs g[2];
  for (int i = 0; i < 2; ++i)
    g[i] = wgrad_args(p[i].A, p[i].lda, p[i].B, p[i].ldb, p[i].M, N, K, 64, sp[i], p[i].workspace);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((N / WT2) * (K / WT2), sp[0] + sp[1]);
  hipLaunchKernelGGL((wgrad256_kernel<64, 2>), grid, dim3(512), 0, s, g[0], g[1], sp[0]);
  sr::note_kernel("wgrad256_kernel");
  for (int i = 0; i < 2; ++i)
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(N), dim3(256), 0, s, p[i].workspace, sp[i], N, K, p[i].dW, p[i].lddw,
                       p[i].accumulate, p[i].rowscale, p[i].wdot, p[i].ldwd, p[i].rowdot);
  return sr::check_launch("sr_gemm_wgrad_pair");
}

extern "C" int64_t sr_colsum_workspace_floats(int M, int N) {
  if (M <= 0 || N <= 0 || N % 4) return 0;
  int rpc;
  return (int64_t)colsum_chunks(M, N, rpc) * N;
}

extern "C" int sr_colsum(sr_stream_t stream, int dtype, const void* X, int64_t ldx, int M, int N, float* out,
                         int accumulate, float scale, float* workspace, int64_t workspace_floats) {
  SR_CHECK(X && out && workspace, SR_EINVAL, "sr_colsum: null pointer");
  SR_CHECK(dtype == SR_F32 || dtype == SR_BF16, SR_EINVAL, "sr_colsum: bad dtype");
  SR_CHECK(M > 0 && N > 0 && N % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)out % 16) == 0, SR_EINVAL,
           "sr_colsum: bad shape M=%d N=%d ldx=%lld", M, N, (long long)ldx);
  SR_CHECK(workspace_floats >= sr_colsum_workspace_floats(M, N) && ((uintptr_t)workspace % 16) == 0, SR_EINVAL,
           "sr_colsum: workspace of %lld floats, needs %lld (sr_colsum_workspace_floats), 16-B aligned",
           (long long)workspace_floats, (long long)sr_colsum_workspace_floats(M, N));
  return colsum_launch((hipStream_t)stream, dtype, X, ldx, M, N, out, accumulate, scale, workspace);
}

extern "C" int sr_colsum_fma(sr_stream_t stream, int dtype, const void* X, int64_t ldx, int M, int N, float* out1,
                             const float* mul1, float* out2, const float* mul2, float* workspace,
                             int64_t workspace_floats) {
  SR_CHECK(X && workspace && (out1 || out2) && (!out1 || mul1) && (!out2 || mul2), SR_EINVAL,
           "sr_colsum_fma: null pointer (X, workspace, and at least one out / mul pair)");
  SR_CHECK(dtype == SR_F32 || dtype == SR_BF16, SR_EINVAL, "sr_colsum_fma: bad dtype");
  SR_CHECK(M > 0 && N > 0 && N % 4 == 0 && ldx % 4 == 0, SR_EINVAL, "sr_colsum_fma: bad shape M=%d N=%d ldx=%lld", M,
           N, (long long)ldx);
  SR_CHECK(workspace_floats >= sr_colsum_workspace_floats(M, N) && ((uintptr_t)workspace % 16) == 0, SR_EINVAL,
           "sr_colsum_fma: workspace of %lld floats, needs %lld (sr_colsum_workspace_floats), 16-B aligned",
           (long long)workspace_floats, (long long)sr_colsum_workspace_floats(M, N));
  return colsum_launch((hipStream_t)stream, dtype, X, ldx, M, N, out1, 1, 1.f, workspace, mul1, out2, mul2, true);
}

extern "C" int sr_layernorm_bwd(sr_stream_t stream, int dtype, const float* x, int64_t ldx, const int32_t* rowmap,
                                const void* dy, int64_t lddy, const float* w, float eps, float* dx, int64_t lddx,
                                void* dxb, int64_t lddxb, float* dw, float* db, int rows, int cols, float* workspace,
                                float* dx_colsum) {
  SR_CHECK(x && dy && dx && rows > 0, SR_EINVAL, "sr_layernorm_bwd: null pointer / no rows");
  SR_CHECK(dtype == SR_F32 || dtype == SR_BF16, SR_EINVAL, "sr_layernorm_bwd: bad dtype");
  SR_CHECK(!(dw || db) || (dw && db && workspace), SR_EINVAL, "sr_layernorm_bwd: dw and db need workspace");
  SR_CHECK(!dx_colsum || (dw && cols <= 2048), SR_EINVAL,
           "sr_layernorm_bwd: dx_colsum needs dw / db (their workspace) and cols <= 2048");
  hipStream_t s = (hipStream_t)stream;
  const int want = dw != nullptr;
  const int want_sum = dx_colsum != nullptr;
  const int np = want_sum ? 3 : 2;
  const int wgs = std::min(LNB_WGS, (rows + 3) / 4);
#define LNB_CASE(C, V)                                                                                          \
  case C:                                                                                                       \
    if (dtype == SR_BF16)                                                                                       \
      hipLaunchKernelGGL((layernorm_bwd_kernel<C / 64, V, bf16>), dim3(wgs), dim3(256), 0, s, x, ldx, rowmap,  \
                         (const bf16*)dy, lddy, w, eps, dx, lddx, (bf16*)dxb, lddxb, want, want_sum, workspace, \
                         rows);                                                                                \
    else                                                                                                        \
      hipLaunchKernelGGL((layernorm_bwd_kernel<C / 64, V, float>), dim3(wgs), dim3(256), 0, s, x, ldx, rowmap, \
                         (const float*)dy, lddy, w, eps, dx, lddx, (bf16*)dxb, lddxb, want, want_sum, workspace, \
                         rows);                                                                                \
    break;
  switch (cols) {
    LNB_CASE(128, 2)
    LNB_CASE(256, 4)
    LNB_CASE(384, 2)
    LNB_CASE(512, 4)
    LNB_CASE(768, 4)
    LNB_CASE(1024, 4)
    LNB_CASE(1536, 4)
    LNB_CASE(2048, 4)
    LNB_CASE(4096, 4)
    default:
      sr::set_error("sr_layernorm_bwd: unsupported cols=%d", cols);
      return SR_EUNSUPPORTED;
  }
#undef LNB_CASE
  if (want)  // partial rows [wgs*4][np*cols] -> dw | db (| dx_colsum, assigned), one launch
    hipLaunchKernelGGL(lnb_final_kernel, dim3((unsigned)((np * cols / 4 + 3) / 4)), dim3(256), 0, s, workspace,
                       wgs * 4, cols, np, dw, db, dx_colsum);
  return sr::check_launch("sr_layernorm_bwd");
}

// one resident round: the column-sum form (138 VGPRs) runs 3 waves per SIMD, the plain one (110) 4
static int qk_bwd_wgs(int rows, bool cs) { return std::min(cs ? 768 : 1024, (rows + 3) / 4); }

extern "C" int64_t sr_qk_bwd_workspace_floats(int rows, int ncols) {
  if (rows <= 0 || ncols <= 0 || ncols % 4) return 0;
  const int wgs = qk_bwd_wgs(rows, false) > qk_bwd_wgs(rows, true) ? qk_bwd_wgs(rows, false) : qk_bwd_wgs(rows, true);
  int rpc;
  const int64_t norm = (int64_t)wgs * 4 * 256 + (int64_t)colsum_chunks(wgs * 4, 256, rpc) * 256;
  return norm + (int64_t)wgs * ncols + (int64_t)colsum_chunks(wgs, ncols, rpc) * ncols;
}

template <typename T>
static int qk_bwd(const char* who, sr_stream_t stream, const void* raw, int64_t ldr, const float* dsrc, int64_t lds,
                  void* out, int64_t ldo, int rows, int ncols, const sr_gemm_epi* ep, float* grads, float* workspace) {
  SR_CHECK(dsrc && out && ep && rows > 0, SR_EINVAL, "%s: null pointer / no rows", who);
  SR_CHECK(ep->head_dim == 64 && ep->embed_dim % 64 == 0 && ncols % 64 == 0, SR_EUNSUPPORTED,
           "%s: head_dim 64 and ncols %% 64 == 0 only (ncols=%d)", who, ncols);
  const bool norm = ep->qn_w != nullptr;
  SR_CHECK(!norm || (raw && ep->qn_b && ep->kn_w && ep->kn_b && grads && workspace), SR_EINVAL,
           "%s: qk-norm needs raw, the four norm params, grads and workspace", who);
  SR_CHECK(!ep->rope_cos || (ep->rope_sin && (ep->pos_yx || (ep->tokens_per_frame > ep->patch_start && ep->grid_w > 0))),
           SR_EINVAL, "%s: rope params", who);
  SR_CHECK(!ep->colsum || (ncols <= QKB_PASSES * 1024 && workspace && ((uintptr_t)ep->colsum % 16) == 0),
           SR_EINVAL, "%s: colsum needs ncols <= %d, a workspace and a 16-B aligned output", who, QKB_PASSES * 1024);
  hipStream_t s = (hipStream_t)stream;
  const int wgs = qk_bwd_wgs(rows, ep->colsum != nullptr);
  int rpc;
  // workspace: norm partials [wgs*4][256] | their colsum scratch | colsum partials [wgs][ncols] | scratch
  float* cpart = workspace ? workspace + (int64_t)wgs * 4 * 256 + (int64_t)colsum_chunks(wgs * 4, 256, rpc) * 256
                           : nullptr;
  if (ep->colsum)
    hipLaunchKernelGGL((qk_bwd_kernel<T, true>), dim3(wgs), dim3(256), 0, s,
                       (const T*)raw, ldr, dsrc, lds, (T*)out, ldo, rows, ncols, *ep, workspace, cpart);
  else
    hipLaunchKernelGGL((qk_bwd_kernel<T, false>), dim3(wgs), dim3(256), 0, s,
                       (const T*)raw, ldr, dsrc, lds, (T*)out, ldo, rows, ncols, *ep, workspace, cpart);
  sr::note_kernel("qk_bwd_kernel<%s, %s>", sr::is_bf16<T>::value ? "__bf16" : "float", ep->colsum ? "true" : "false");
  if (norm) {  // [wgs*4][4][64] -> grads[4][64]
    const int rc = colsum_launch(s, SR_F32, workspace, 256, wgs * 4, 256, grads, 1, 1.f,
                                 workspace + (int64_t)wgs * 4 * 256);
    if (rc) return rc;
  }
  if (ep->colsum) {  // [wgs][ncols] -> colsum[ncols] (accumulated)
    const int rc = colsum_launch(s, SR_F32, cpart, ncols, wgs, ncols, ep->colsum, 1, 1.f, cpart + (int64_t)wgs * ncols);
    if (rc) return rc;
  }
  return sr::check_launch(who);
}

extern "C" int sr_qk_bwd(sr_stream_t stream, const void* raw, int64_t ldr, const float* dsrc, int64_t lds, void* out,
                         int64_t ldo, int rows, int ncols, const sr_gemm_epi* ep, float* grads, float* workspace) {
  return qk_bwd<bf16>("sr_qk_bwd", stream, raw, ldr, dsrc, lds, out, ldo, rows, ncols, ep, grads, workspace);
}

extern "C" int sr_qk_bwd_f32(sr_stream_t stream, const float* raw, int64_t ldr, const float* dsrc, int64_t lds,
                             float* out, int64_t ldo, int rows, int ncols, const sr_gemm_epi* ep, float* grads,
                             float* workspace) {
  return qk_bwd<float>("sr_qk_bwd_f32", stream, raw, ldr, dsrc, lds, out, ldo, rows, ncols, ep, grads, workspace);
}

extern "C" int sr_cast_bf16(sr_stream_t stream, const float* src, int64_t lds, void* dst, int64_t ldd, int rows,
                            int cols, float scale) {
  SR_CHECK(src && dst && rows > 0 && cols > 0 && cols % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0, SR_EINVAL,
           "sr_cast_bf16: bad arguments");
  const int64_t n = (int64_t)rows * (cols / 4);
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for(n, 8192)), dim3(256), 0, (hipStream_t)stream, src, lds,
                     (bf16*)dst, ldd, rows, cols, scale);
  return sr::check_launch("sr_cast_bf16");
}

extern "C" int sr_nonfinite_check(sr_stream_t stream, const float* g, int64_t n, const float* scale, int* found_inf) {
  SR_CHECK(g && found_inf && n >= 0, SR_EINVAL, "sr_nonfinite_check: bad arguments");
  if (n == 0) return SR_OK;
  hipLaunchKernelGGL(nonfinite_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, g, n, scale, found_inf);
  return sr::check_launch("sr_nonfinite_check");
}

extern "C" int sr_adam_f32(sr_stream_t stream, float* p, const float* g, float* m, float* v, int64_t n, float lr,
                           float beta1, float beta2, float eps, float weight_decay, int step, const float* scale,
                           const int* found_inf) {
  SR_CHECK(p && g && m && v && n >= 0 && step >= 1, SR_EINVAL, "sr_adam_f32: bad arguments");
  if (n == 0) return SR_OK;
  const float bc1 = 1.f - (float)std::pow((double)beta1, step);
  const float bc2 = 1.f - (float)std::pow((double)beta2, step);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, beta1,
                     beta2, eps, weight_decay, bc1, std::sqrt(bc2), scale, found_inf);
  return sr::check_launch("sr_adam_f32");
}

// sr_weight_refresh_bf16: up to SR_WEIGHT_REFRESH_MAX fp32 weights in one launch, each 64 x 64
// source tile read once and written as its bf16 cast (same layout) and its transposed bf16 copy
// with the row scale folded in.  Workgroup -> (item, tile) by the tile-count prefix.
struct WeightRefresh {
  sr_weight_item it[SR_WEIGHT_REFRESH_MAX];
  int start[SR_WEIGHT_REFRESH_MAX + 1];
  int n;
};

// One 64 x 64 tile t of weight w: read once, written as the bf16 cast and / or the rowscaled bf16
// transpose.
__device__ __forceinline__ void refresh_tile(const sr_weight_item& w, int t, float (*tile)[65]) {
  const int ntc = (w.cols + 63) / 64;
  const int r0 = (t / ntc) * 64, c0 = (t % ntc) * 64;
  // whole tile with 16-B source rows and 8-B bf16 destination rows (the aggregator's weights):
  // float4 loads, bf16x4 stores of the cast and of the transpose (same values as the scalar path)
  const bool vec = r0 + 64 <= w.rows && c0 + 64 <= w.cols && (w.lds & 3) == 0 && ((uintptr_t)w.src & 15) == 0 &&
                   (!w.cast || ((w.ldc & 3) == 0 && ((uintptr_t)w.cast & 7) == 0)) &&
                   (!w.trans || ((w.ldt & 3) == 0 && ((uintptr_t)w.trans & 7) == 0));
  if (vec) {
    const int q = threadIdx.x & 15, rr = threadIdx.x >> 4;  // column quad, row (+16 i)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = rr + 16 * i;
      f32x4 v = *(const f32x4*)(w.src + (int64_t)(r0 + r) * w.lds + c0 + 4 * q);
      if (w.cast)
        *(bf16x4*)((bf16*)w.cast + (int64_t)(r0 + r) * w.ldc + c0 + 4 * q) =
            bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      if (w.rowscale) v *= w.rowscale[r0 + r];
#pragma unroll
      for (int j = 0; j < 4; ++j) tile[r][4 * q + j] = v[j];
    }
    if (!w.trans) return;  // workgroup-uniform
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // transposed row c0 + c, rows r0 + 4q .. + 3
      const int c = rr + 16 * i;
      *(bf16x4*)((bf16*)w.trans + (int64_t)(c0 + c) * w.ldt + r0 + 4 * q) =
          bf16x4{(bf16)tile[4 * q][c], (bf16)tile[4 * q + 1][c], (bf16)tile[4 * q + 2][c], (bf16)tile[4 * q + 3][c]};
    }
    return;
  }
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    float v = 0.f;
    if (r < w.rows && c < w.cols) {
      v = w.src[(int64_t)r * w.lds + c];
      if (w.cast) ((bf16*)w.cast)[(int64_t)r * w.ldc + c] = (bf16)v;
      if (w.rowscale) v *= w.rowscale[r];
    }
    tile[i][tx] = v;
  }
  if (!w.trans) return;  // workgroup-uniform
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < w.cols && r < w.rows) ((bf16*)w.trans)[(int64_t)c * w.ldt + r] = (bf16)tile[tx][i];
  }
}

__global__ __launch_bounds__(256) void weight_refresh_kernel(WeightRefresh wr) {
  __shared__ float tile[64][65];
  int p = 0;
#pragma unroll
  for (int i = 1; i < SR_WEIGHT_REFRESH_MAX; ++i) p += (i < wr.n && (int)blockIdx.x >= wr.start[i]) ? 1 : 0;
  refresh_tile(wr.it[p], blockIdx.x - wr.start[p], tile);
}

// sr_weight_refresh_list_bf16: every item of a device-resident table in ONE launch (the whole model's
// per-step refresh); workgroup -> item by a binary search of the tile-count prefix start[0..n].
__global__ __launch_bounds__(256) void weight_refresh_list_kernel(const sr_weight_item* __restrict__ items,
                                                                  const int* __restrict__ start, int n) {
  __shared__ float tile[64][65];
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;  // the last item whose start <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (start[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  const sr_weight_item w = items[lo];
  refresh_tile(w, b - start[lo], tile);
}

extern "C" int sr_weight_refresh_bf16(sr_stream_t stream, int n, const sr_weight_item* items) {
  SR_CHECK(items && n > 0 && n <= SR_WEIGHT_REFRESH_MAX, SR_EINVAL, "sr_weight_refresh_bf16: 1..%d items (got %d)",
           SR_WEIGHT_REFRESH_MAX, n);
  WeightRefresh wr{};
  wr.n = n;
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    const sr_weight_item& w = items[i];
    SR_CHECK(w.src && w.rows > 0 && w.cols > 0 && w.lds >= w.cols && (w.cast || w.trans) &&
                 (!w.cast || w.ldc >= w.cols) && (!w.trans || w.ldt >= w.rows),
             SR_EINVAL, "sr_weight_refresh_bf16: item %d: bad shape / pointers", i);
    wr.it[i] = w;
    wr.start[i] = tiles;
    tiles += ((w.rows + 63) / 64) * ((w.cols + 63) / 64);
  }
  wr.start[n] = tiles;
  hipLaunchKernelGGL(weight_refresh_kernel, dim3(tiles), dim3(256), 0, (hipStream_t)stream, wr);
  sr::note_kernel("weight_refresh_kernel");
  return sr::check_launch("sr_weight_refresh_bf16");
}

extern "C" int sr_weight_refresh_plan(int n, const sr_weight_item* items, int* start) {
  SR_CHECK(items && start && n > 0, SR_EINVAL, "sr_weight_refresh_plan: null items / start or n <= 0");
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    const sr_weight_item& w = items[i];
    SR_CHECK(w.src && w.rows > 0 && w.cols > 0 && w.lds >= w.cols && (w.cast || w.trans) &&
                 (!w.cast || w.ldc >= w.cols) && (!w.trans || w.ldt >= w.rows),
             SR_EINVAL, "sr_weight_refresh_plan: item %d: bad shape / pointers", i);
    start[i] = tiles;
    const int64_t t = (int64_t)tiles + (int64_t)((w.rows + 63) / 64) * ((w.cols + 63) / 64);
    SR_CHECK(t < (1ll << 31), SR_EINVAL, "sr_weight_refresh_plan: too many tiles");
    tiles = (int)t;
  }
  start[n] = tiles;
  return SR_OK;
}

extern "C" int sr_weight_refresh_list_bf16(sr_stream_t stream, int n, const sr_weight_item* items_dev,
                                           const int* start_dev, int tiles) {
  SR_CHECK(items_dev && start_dev && n > 0 && tiles > 0, SR_EINVAL,
           "sr_weight_refresh_list_bf16: null table or empty plan");
  hipLaunchKernelGGL(weight_refresh_list_kernel, dim3(tiles), dim3(256), 0, (hipStream_t)stream, items_dev, start_dev,
                     n);
  sr::note_kernel("weight_refresh_list_kernel");
  return sr::check_launch("sr_weight_refresh_list_bf16");
}

extern "C" int sr_transpose_f32(sr_stream_t stream, int out_dtype, const float* src, int64_t lds, int rows, int cols,
                                const float* rowscale, void* dst, int64_t ldd) {
  SR_CHECK(src && dst && rows > 0 && cols > 0 && lds >= cols && ldd >= rows, SR_EINVAL, "sr_transpose_f32: bad args");
  const dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  if (out_dtype == SR_BF16)
    hipLaunchKernelGGL(transpose_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, src, lds, rows, cols, rowscale,
                       (bf16*)dst, ldd);
  else
    hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, src, lds, rows, cols, rowscale,
                       (float*)dst, ldd);
  return sr::check_launch("sr_transpose_f32");
}

extern "C" int sr_wgrad_small_f32(sr_stream_t stream, const float* A, int64_t lda, const float* B, int64_t ldb,
                                  float* dW, int64_t lddw, int M, int N, int K, int accumulate, float* db,
                                  const float* rowscale, const float* wdot, int64_t ldwd, float* rowdot,
                                  float* workspace) {
  SR_CHECK(A && B && dW && M > 0 && N > 0 && K > 0 && lda >= N && ldb >= K && lddw >= K, SR_EINVAL,
           "sr_wgrad_small_f32: bad args");
  const bool fin = rowscale || wdot;
  SR_CHECK(!fin || (workspace && K % 4 == 0 && lddw % 4 == 0 && (!wdot || (rowdot && ldwd % 4 == 0))), SR_EINVAL,
           "sr_wgrad_small_f32: rowscale / wdot need workspace, K %% 4 == 0 and rowdot");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = (int64_t)N * K;
  if (!fin) {
    hipLaunchKernelGGL(wgrad_small_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, lda, B, ldb, dW,
                       lddw, M, N, K, accumulate, db);
  } else {  // G -> workspace, then the per-row finish of sr_gemm_wgrad (scale, accumulate, rowdot)
    hipLaunchKernelGGL(wgrad_small_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, lda, B, ldb,
                       workspace, (int64_t)K, M, N, K, 0, db);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(N), dim3(256), 0, s, workspace, 1, N, K, dW, lddw, accumulate,
                       rowscale, wdot, ldwd, rowdot);
  }
  return sr::check_launch("sr_wgrad_small_f32");
}

extern "C" int sr_attention_bwd_small_f32(sr_stream_t stream, const float* q, const float* k, const float* v, int64_t ld,
                                          const float* dout, int64_t lddo, float* dq, float* dk, float* dv, int64_t ldg,
                                          int L, int heads, int head_dim, float scale, int mask_mode, int n_anchor,
                                          float* workspace) {
  SR_CHECK(q && k && v && dout && dq && dk && dv && workspace, SR_EINVAL, "sr_attention_bwd_small_f32: null pointer");
  SR_CHECK(L > 0 && L <= 1024 && heads > 0 && head_dim > 0, SR_EUNSUPPORTED,
           "sr_attention_bwd_small_f32: L=%d (<= 1024)", L);
  hipStream_t s = (hipStream_t)stream;
  float* P = workspace;
  float* dS = workspace + (int64_t)heads * L * L;
  hipLaunchKernelGGL(attn_bwd_small_p_kernel, dim3(L, heads), dim3(256), 0, s, q, k, v, ld, dout, lddo, L, head_dim,
                     scale, mask_mode, n_anchor, P, dS);
  const int64_t n = 3ll * L * heads * head_dim;
  hipLaunchKernelGGL(attn_bwd_small_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, q, k, ld, dout,
                     lddo, L, head_dim, heads, scale, P, dS, dq, dk, dv, ldg);
  return sr::check_launch("sr_attention_bwd_small_f32");
}

extern "C" int sr_adaln_bwd_f32(sr_stream_t stream, const float* xn, const float* mod, const float* dxm, float* dxn,
                                float* dmod, int rows, int cols) {
  SR_CHECK(xn && mod && dxm && dxn && dmod && rows > 0 && cols > 0, SR_EINVAL, "sr_adaln_bwd_f32: bad args");
  hipLaunchKernelGGL(adaln_bwd_kernel, dim3(grid_for((int64_t)rows * cols)), dim3(256), 0, (hipStream_t)stream, xn, mod,
                     dxm, dxn, dmod, rows, cols);
  return sr::check_launch("sr_adaln_bwd_f32");
}

extern "C" int sr_act_bwd_f32(sr_stream_t stream, int mode, const float* x, const float* dy, float* dx, int64_t n) {
  SR_CHECK(x && dy && dx && n > 0 && (mode == 0 || mode == 1), SR_EINVAL, "sr_act_bwd_f32: bad args");
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, dy, dx, n, mode);
  return sr::check_launch("sr_act_bwd_f32");
}

extern "C" int sr_vec_fma_f32(sr_stream_t stream, float* out, const float* a, const float* b, int n) {
  SR_CHECK(out && a && b && n > 0, SR_EINVAL, "sr_vec_fma_f32: bad args");
  hipLaunchKernelGGL(vec_fma_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, out, a, b, n, nullptr,
                     nullptr);
  return sr::check_launch("sr_vec_fma_f32");
}

extern "C" int sr_vec_fma2_f32(sr_stream_t stream, float* out1, const float* a1, float* out2, const float* a2,
                               const float* b, int n) {
  SR_CHECK(out1 && a1 && out2 && a2 && b && n > 0, SR_EINVAL, "sr_vec_fma2_f32: bad args");
  hipLaunchKernelGGL(vec_fma_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, out1, a1, b, n, out2, a2);
  return sr::check_launch("sr_vec_fma2_f32");
}

extern "C" int sr_scatter_rows_f32(sr_stream_t stream, float* dst, int64_t ldd, const int32_t* rowmap, const float* src,
                                   int64_t lds, int rows, int cols, int accumulate) {
  SR_CHECK(dst && rowmap && src && rows > 0 && cols > 0 && cols % 4 == 0 && ldd % 4 == 0 && lds % 4 == 0, SR_EINVAL,
           "sr_scatter_rows_f32: bad args");
  const int64_t n = (int64_t)rows * (cols / 4);
  hipLaunchKernelGGL(scatter_rows_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, dst, ldd, rowmap, src,
                     lds, rows, cols, accumulate);
  return sr::check_launch("sr_scatter_rows_f32");
}

extern "C" int sr_copy2d_f32(sr_stream_t stream, float* dst, int64_t ldd, const float* src, int64_t lds, int rows,
                             int cols, int accumulate) {
  SR_CHECK(dst && src && rows > 0 && cols > 0 && ldd >= cols && lds >= 0, SR_EINVAL, "sr_copy2d_f32: bad args");
  hipLaunchKernelGGL(copy2d_kernel, dim3(grid_for((int64_t)rows * cols)), dim3(256), 0, (hipStream_t)stream, dst, ldd,
                     src, lds, rows, cols, accumulate);
  return sr::check_launch("sr_copy2d_f32");
}

extern "C" int sr_pose_act_bwd_f32(sr_stream_t stream, float* dd, const float* d_act, const float* act, int rows,
                                   int n_anchor) {
  SR_CHECK(dd && d_act && act && rows > 0 && n_anchor >= 0, SR_EINVAL, "sr_pose_act_bwd_f32: bad args");
  hipLaunchKernelGGL(pose_act_bwd_kernel, dim3((rows * 9 + 255) / 256), dim3(256), 0, (hipStream_t)stream, dd, d_act,
                     act, rows, n_anchor);
  return sr::check_launch("sr_pose_act_bwd_f32");
}
