// Memory-bound kernels around the GEMM / attention hot ops:
// LayerNorm (+row gather), image normalise + patch im2col, special-token fill,
// row copies, and the small fp32 camera-head ops (camera_head.py, head_act.py,
// pose_enc.py, rotation.py).
#include "sr_common.h"

namespace {

// ------------------------------------------------------------------ LayerNorm
// One wave per row; each lane holds NPL = cols/64 values loaded as VEC-wide vectors
// (coalesced: vector i of lane l covers columns (i*64 + l)*VEC .. +VEC).
// rows in flight per wave (register budget): C = 1024 takes 4 (4.45 -> 5.2 TB/s over 2; 8 rows
// fell back to 4.6)
constexpr int ln_rows_per_wave(int npl) { return npl >= 32 ? 1 : (npl == 16 ? 4 : 2); }
template <int NPL, int VEC, typename TO>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int64_t ldx,
                                                        const int32_t* __restrict__ rowmap,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        float eps, TO* __restrict__ out, int64_t ldo, int rows,
                                                        float* __restrict__ xc, int64_t ldc) {
  // one wave per row pair (RPW rows in flight per wave: every load issued before the first
  // reduction); VEC-wide vector loads of x, w, b and VEC-wide stores
  constexpr int RPW = ln_rows_per_wave(NPL);
  constexpr int NV = NPL / VEC;
  constexpr int COLS = NPL * 64;
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= rows) return;
  float v[RPW][NPL];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int row = min(row0 + r, rows - 1);
    const int64_t src = rowmap ? (int64_t)rowmap[row] : row;
    const float* xr = x + src * ldx;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = (i * 64 + lane) * VEC;
      if constexpr (VEC == 4) {
        const float4 t = *(const float4*)(xr + col);
        v[r][i * 4 + 0] = t.x; v[r][i * 4 + 1] = t.y; v[r][i * 4 + 2] = t.z; v[r][i * 4 + 3] = t.w;
        if (xc) *(float4*)(xc + (int64_t)row * ldc + col) = t;  // the row's fp32 copy (training tape)
      } else {
        const float2 t = *(const float2*)(xr + col);
        v[r][i * 2 + 0] = t.x; v[r][i * 2 + 1] = t.y;
        if (xc) *(float2*)(xc + (int64_t)row * ldc + col) = t;
      }
    }
  }
  float wv[NPL], bv[NPL];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int col = (i * 64 + lane) * VEC;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      wv[i * VEC + j] = w ? w[col + j] : 1.f;
      bv[i * VEC + j] = w ? b[col + j] : 0.f;
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int row = row0 + r;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) s += v[r][i];
    const float mean = sr::wave_sum(s) * (1.f / COLS);
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      v[r][i] -= mean;
      s2 += v[r][i] * v[r][i];
    }
    const float rstd = rsqrtf(sr::wave_sum(s2) * (1.f / COLS) + eps);
    if (row >= rows) break;
    TO* orow = out + (int64_t)row * ldo;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = (i * 64 + lane) * VEC;
      float y[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) y[j] = fmaf(v[r][i * VEC + j] * rstd, wv[i * VEC + j], bv[i * VEC + j]);
      if constexpr (VEC == 4) {
        if constexpr (sr::is_bf16<TO>::value) {
          const bf16x4 o = {(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
          *(bf16x4*)(orow + col) = o;
        } else {
          *(float4*)(orow + col) = make_float4(y[0], y[1], y[2], y[3]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) orow[col + j] = sr::from_f32<TO>(y[j]);
      }
    }
  }
}

template <typename TO>
int layernorm_dispatch(hipStream_t s, const float* x, int64_t ldx, const int32_t* rowmap, const float* w,
                       const float* b, float eps, TO* out, int64_t ldo, int rows, int cols, float* xc = nullptr,
                       int64_t ldc = 0) {
  const dim3 block(256);  // 4 waves x ln_rows_per_wave rows
#define LN_CASE(C, V)                                                                                    \
  case C:                                                                                                \
    hipLaunchKernelGGL((layernorm_kernel<C / 64, V, TO>),                                                \
                       dim3((rows + 4 * ln_rows_per_wave(C / 64) - 1) / (4 * ln_rows_per_wave(C / 64))), block, \
                       0, s, x, ldx, rowmap, w, b, eps, out, ldo, rows, xc, ldc);                         \
    return sr::check_launch("sr_layernorm");
  switch (cols) {
    LN_CASE(128, 2)
    LN_CASE(256, 4)
    LN_CASE(384, 2)
    LN_CASE(512, 4)
    LN_CASE(768, 4)
    LN_CASE(1024, 4)
    LN_CASE(1536, 4)
    LN_CASE(2048, 4)
    LN_CASE(4096, 4)
  }
#undef LN_CASE
  sr::set_error("sr_layernorm: unsupported cols=%d", cols);
  return SR_EUNSUPPORTED;
}

// ------------------------------------------------------------------ residual + LayerNorm
// x += gamma * y (y = the projection GEMM's bias-epilogue output, in the compute dtype as the
// reference's autocast Linear returns it), then out = LN(x): block.py:86-89's `x + ls1(attn(..))`
// followed by norm2, in one pass over the rows (the GEMM's fp32 residual read-modify-write
// epilogue ran serialized behind each CU's MFMAs; here it streams at the HBM rate).  One wave per
// row, ln_rows_per_wave rows in flight, 4-wide vectors.
// W = columns per lane-vector: 4 (float4 x, 8-B bf16 y / out) or 8 (two float4 of x, ONE 16-B
// bf16x8 of y and of out: every load and store of the row is 16 B wide).
template <int NPL, int RPW, typename TY, typename TO, int W = 4, bool NT = false>
__global__ __launch_bounds__(256) void residual_layernorm_kernel(float* x, int64_t ldx, const TY* __restrict__ y,
                                                                 int64_t ldy, const float* __restrict__ gamma,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ b, float eps,
                                                                 TO* __restrict__ out, int64_t ldo, int rows) {
  static_assert(W == 4 || W == 8, "lane vector width");
  constexpr int NV = NPL / W;
  constexpr int COLS = NPL * 64;
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= rows) return;
  float v[RPW][NPL];
  float yv[RPW][NPL];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int row = min(row0 + r, rows - 1);
    const float* xr = x + (int64_t)row * ldx;
    const TY* yr = y + (int64_t)row * ldy;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = (i * 64 + lane) * W;
#pragma unroll
      for (int h = 0; h < W / 4; ++h) {
        const float4 t = *(const float4*)(xr + col + 4 * h);
        v[r][i * W + 4 * h + 0] = t.x; v[r][i * W + 4 * h + 1] = t.y;
        v[r][i * W + 4 * h + 2] = t.z; v[r][i * W + 4 * h + 3] = t.w;
      }
      if constexpr (sr::is_bf16<TY>::value && W == 8) {
        const bf16x8 u = *(const bf16x8*)(yr + col);
#pragma unroll
        for (int j = 0; j < 8; ++j) yv[r][i * 8 + j] = (float)u[j];
      } else if constexpr (sr::is_bf16<TY>::value) {
        const bf16x4 u = *(const bf16x4*)(yr + col);
#pragma unroll
        for (int j = 0; j < 4; ++j) yv[r][i * 4 + j] = (float)u[j];
      } else {
#pragma unroll
        for (int h = 0; h < W / 4; ++h) {
          const float4 u = *(const float4*)(yr + col + 4 * h);
          yv[r][i * W + 4 * h + 0] = u.x; yv[r][i * W + 4 * h + 1] = u.y;
          yv[r][i * W + 4 * h + 2] = u.z; yv[r][i * W + 4 * h + 3] = u.w;
        }
      }
    }
  }
  float gv[NPL], wv[NPL], bv[NPL];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int col = (i * 64 + lane) * W;
#pragma unroll
    for (int j = 0; j < W; ++j) {
      gv[i * W + j] = gamma ? gamma[col + j] : 1.f;
      wv[i * W + j] = w ? w[col + j] : 1.f;
      bv[i * W + j] = w ? b[col + j] : 0.f;
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int row = row0 + r;
    float* xr = x + (int64_t)row * ldx;
#pragma unroll
    for (int i = 0; i < NPL; ++i) v[r][i] = fmaf(gv[i], yv[r][i], v[r][i]);
    if (row < rows) {
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int h = 0; h < W / 4; ++h) {
          const int k = i * W + 4 * h;
          if constexpr (NT) {
            const f32x4 xv = {v[r][k], v[r][k + 1], v[r][k + 2], v[r][k + 3]};
            __builtin_nontemporal_store(xv, (f32x4*)(xr + (i * 64 + lane) * W + 4 * h));
          } else {
            *(float4*)(xr + (i * 64 + lane) * W + 4 * h) = make_float4(v[r][k], v[r][k + 1], v[r][k + 2], v[r][k + 3]);
          }
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) s += v[r][i];
    const float mean = sr::wave_sum(s) * (1.f / COLS);
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      v[r][i] -= mean;
      s2 += v[r][i] * v[r][i];
    }
    const float rstd = rsqrtf(sr::wave_sum(s2) * (1.f / COLS) + eps);
    if (row >= rows) break;
    TO* orow = out + (int64_t)row * ldo;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = (i * 64 + lane) * W;
      float ow[W];
#pragma unroll
      for (int j = 0; j < W; ++j) ow[j] = fmaf(v[r][i * W + j] * rstd, wv[i * W + j], bv[i * W + j]);
      if constexpr (sr::is_bf16<TO>::value && W == 8) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)ow[j];
        *(bf16x8*)(orow + col) = o;
      } else if constexpr (sr::is_bf16<TO>::value) {
        const bf16x4 o = {(bf16)ow[0], (bf16)ow[1], (bf16)ow[2], (bf16)ow[3]};
        *(bf16x4*)(orow + col) = o;
      } else {
#pragma unroll
        for (int h = 0; h < W / 4; ++h)
          *(float4*)(orow + col + 4 * h) = make_float4(ow[4 * h], ow[4 * h + 1], ow[4 * h + 2], ow[4 * h + 3]);
      }
    }
  }
}

template <typename TY, typename TO>
int residual_layernorm_dispatch(hipStream_t s, float* x, int64_t ldx, const TY* y, int64_t ldy, const float* gamma,
                                const float* w, const float* b, float eps, TO* out, int64_t ldo, int rows, int cols) {
  // rows in flight per wave as the LayerNorm (kbench M = 87,936, C = 1024: 1 row 3.5 TB/s, 2 rows
  // 4.86, 4 rows 4.96 TB/s of the 12 B per element moved)
  // Variants (SR_TUNE_RLN_WIDE, a kbench A/B switch; default 0): bit 0 = 16-B lane vectors (W = 8:
  // rows of 512-column blocks, 16-B aligned; kbench M = 87,936: 0.242 ms against round 3's
  // 0.218 ms for W = 4), bit 1 = 2 rows in flight per wave instead of 4, bit 2 = non-temporal x stores
  const int var = sr::tune(SR_TUNE_RLN_WIDE);
  const bool w8 = (var & 1) && cols % 512 == 0 && ldy % 8 == 0 && ldo % 8 == 0 && ldx % 4 == 0 &&
                  (((uintptr_t)y | (uintptr_t)out | (uintptr_t)x) & 15) == 0;
  const bool r2 = (var & 2) != 0, nt = (var & 4) != 0;
#define RLN_GO(C, R, W_, NT_)                                                                                     \
  hipLaunchKernelGGL((residual_layernorm_kernel<C / 64, R, TY, TO, W_, NT_>), dim3((rows + 4 * R - 1) / (4 * R)), \
                     dim3(256), 0, s, x, ldx, y, ldy, gamma, w, b, eps, out, ldo, rows)
#define RLN_LAUNCH(C, R)                                                                                          \
  do {                                                                                                            \
    if constexpr (C % 512 == 0 && R == 4) {                                                                       \
      if (w8 || r2 || nt) {                                                                                       \
        if (w8 && r2) { if (nt) RLN_GO(C, 2, 8, true); else RLN_GO(C, 2, 8, false); }                           \
        else if (w8) { if (nt) RLN_GO(C, 4, 8, true); else RLN_GO(C, 4, 8, false); }                           \
        else if (r2) { if (nt) RLN_GO(C, 2, 4, true); else RLN_GO(C, 2, 4, false); }                           \
        else RLN_GO(C, 4, 4, true);                                                                               \
        break;                                                                                                    \
      }                                                                                                           \
    }                                                                                                             \
    RLN_GO(C, R, 4, false);                                                                                       \
  } while (0)
#define RLN_CASE(C)                                                                                             \
  case C:                                                                                                       \
    RLN_LAUNCH(C, ln_rows_per_wave(C / 64));                                                                    \
    return sr::check_launch("sr_residual_layernorm");
  switch (cols) {
    RLN_CASE(256)
    RLN_CASE(512)
    RLN_CASE(768)
    RLN_CASE(1024)
    RLN_CASE(1536)
    RLN_CASE(2048)
  }
#undef RLN_CASE
#undef RLN_LAUNCH
#undef RLN_GO
  sr::set_error("sr_residual_layernorm: unsupported cols=%d", cols);
  return SR_EUNSUPPORTED;
}

// ------------------------------------------------------------------ im2col
template <typename T>
__global__ void im2col_kernel(const float* __restrict__ img, int frames, int H, int W, int ps, float m0, float m1,
                              float m2, float s0, float s1, float s2, T* __restrict__ out, int kpad) {
  const int gh = H / ps, gw = W / ps, kk = 3 * ps * ps;
  const int64_t total = (int64_t)frames * gh * gw * kpad;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % kpad);
    const int64_t r = e / kpad;
    float v = 0.f;
    if (k < kk) {
      const int px = (int)(r % gw), py = (int)((r / gw) % gh);
      const int64_t f = r / ((int64_t)gw * gh);
      const int c = k / (ps * ps), ky = (k / ps) % ps, kx = k % ps;
      const float raw = img[((f * 3 + c) * H + (py * ps + ky)) * (int64_t)W + px * ps + kx];
      const float mean = c == 0 ? m0 : (c == 1 ? m1 : m2);
      const float sd = c == 0 ? s0 : (c == 1 ? s1 : s2);
      v = (raw - mean) / sd;
    }
    out[e] = sr::from_f32<T>(v);
  }
}

// ------------------------------------------------------------------ token fills / copies
__global__ void special_tokens_kernel(float* __restrict__ x, int64_t ldx, int frames, int tpf, int nspec,
                                      const float* __restrict__ table, const int32_t* __restrict__ type_of_frame,
                                      int cols) {
  const int64_t total = (int64_t)frames * nspec * cols;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % cols);
    const int t = (int)((e / cols) % nspec);
    const int f = (int)(e / ((int64_t)cols * nspec));
    x[((int64_t)f * tpf + t) * ldx + c] = table[((int64_t)type_of_frame[f] * nspec + t) * cols + c];
  }
}

__global__ void copy_rows_kernel(float* __restrict__ dst, int64_t ldd, const float* __restrict__ src, int64_t lds,
                                 const int32_t* __restrict__ rowmap, int rows, int cols4) {
  const int64_t total = (int64_t)rows * cols4;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % cols4);
    const int r = (int)(e / cols4);
    const int64_t sr_ = rowmap ? (int64_t)rowmap[r] : r;
    ((float4*)(dst + r * ldd))[c] = ((const float4*)(src + sr_ * lds))[c];
  }
}

// LayerScale (layer_scale.py:22-23) as a standalone op: out[r][c] = x[r][c] * gamma[c]
template <typename T>
__global__ void mul_cols_kernel(const T* __restrict__ x, int64_t ldx, const float* __restrict__ g, T* __restrict__ out,
                                int64_t ldo, int rows, int cols) {
  const int64_t total = (int64_t)rows * cols;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % cols);
    const int64_t r = e / cols;
    out[r * ldo + c] = sr::from_f32<T>(sr::to_f32(x[r * ldx + c]) * g[c]);
  }
}

// ------------------------------------------------------------------ small fp32 ops (camera head)
__device__ __forceinline__ float silu(float v) { return v / (1.f + expf(-v)); }

// K <= 64: one thread per output
__global__ void linear_small_thread_kernel(const float* A, int64_t lda, const float* W, const float* bias, float* out,
                                           int64_t ldo, int M, int N, int K, int act) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= (int64_t)M * N) return;
  const int n = (int)(e % N), m = (int)(e / N);
  float acc = 0.f;
  for (int k = 0; k < K; ++k) {
    float a = A[m * lda + k];
    if (act) a = silu(a);
    acc = fmaf(a, W[(int64_t)n * K + k], acc);
  }
  out[m * ldo + n] = acc + (bias ? bias[n] : 0.f);
}

// K > 64: one wave per output, lanes stride K
__global__ void linear_small_wave_kernel(const float* A, int64_t lda, const float* W, const float* bias, float* out,
                                         int64_t ldo, int M, int N, int K, int act) {
  const int64_t e = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= (int64_t)M * N) return;
  const int n = (int)(e % N), m = (int)(e / N);
  float acc = 0.f;
  for (int k = lane; k < K; k += 64) {
    float a = A[m * lda + k];
    if (act) a = silu(a);
    acc = fmaf(a, W[(int64_t)n * K + k], acc);
  }
  acc = sr::wave_sum(acc);
  if (lane == 0) out[m * ldo + n] = acc + (bias ? bias[n] : 0.f);
}

__global__ void silu_kernel(const float* x, float* y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = silu(x[i]);
}

__global__ void adaln_kernel(const float* xn, const float* x, const float* mod, float* out, int rows, int cols) {
  const int64_t total = (int64_t)rows * cols;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % cols);
    const int64_t r = e / cols;
    const float* mr = mod + r * 3 * cols;
    const float shift = mr[c], scale = mr[cols + c], gate = mr[2 * cols + c];
    out[e] = gate * (xn[e] * (1.f + scale) + shift) + x[e];
  }
}

__global__ void pose_update_kernel(float* pred, const float* delta, int64_t ldd, float* act, int rows, int first) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * 9) return;
  const int r = e / 9, c = e % 9;
  const float dv = delta[r * ldd + c];
  const float p = first ? dv : pred[e] + dv;
  pred[e] = p;
  act[e] = c >= 7 ? fmaxf(p, 0.f) : p;
}

__global__ void pose_decode_kernel(const float* enc, int64_t ld, int n, float H, float W, float* ext, float* intr) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const float* e = enc + r * ld;
  const float i = e[3], j = e[4], k = e[5], q = e[6];  // xyzw, scalar last (rotation.py:14-44)
  const float two_s = 2.0f / (i * i + j * j + k * k + q * q);
  float* E = ext + r * 12;
  E[0] = 1 - two_s * (j * j + k * k);
  E[1] = two_s * (i * j - k * q);
  E[2] = two_s * (i * k + j * q);
  E[3] = e[0];
  E[4] = two_s * (i * j + k * q);
  E[5] = 1 - two_s * (i * i + k * k);
  E[6] = two_s * (j * k - i * q);
  E[7] = e[1];
  E[8] = two_s * (i * k - j * q);
  E[9] = two_s * (j * k + i * q);
  E[10] = 1 - two_s * (i * i + j * j);
  E[11] = e[2];
  float* K = intr + r * 9;
  const float fy = (H / 2.0f) / tanf(e[7] / 2.0f);
  const float fx = (W / 2.0f) / tanf(e[8] / 2.0f);
  K[0] = fx; K[1] = 0.f; K[2] = W / 2;
  K[3] = 0.f; K[4] = fy; K[5] = H / 2;
  K[6] = 0.f; K[7] = 0.f; K[8] = 1.f;
}

inline dim3 grid_for(int64_t n, int block = 256) {
  int64_t g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return dim3((unsigned)g);
}

}  // namespace

extern "C" int sr_residual_layernorm(sr_stream_t stream, int dtype, float* x, int64_t ldx, const void* y, int64_t ldy,
                                     const float* gamma, const float* w, const float* b, float eps, void* out,
                                     int64_t ldo, int rows, int cols) {
  SR_CHECK(x && y && out && rows > 0 && cols > 0, SR_EINVAL, "sr_residual_layernorm: bad args");
  SR_CHECK((w == nullptr) == (b == nullptr), SR_EINVAL, "sr_residual_layernorm: w and b must both be set or both NULL");
  SR_CHECK(ldx % 4 == 0 && ldy % 4 == 0 && ldo % 4 == 0 && ((uintptr_t)x & 15) == 0, SR_EINVAL,
           "sr_residual_layernorm: leading dims must be multiples of 4, x 16-B aligned");
  SR_CHECK((const void*)x != y && (const void*)x != out, SR_EINVAL, "sr_residual_layernorm: y / out alias x");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    return residual_layernorm_dispatch<bf16, bf16>(s, x, ldx, (const bf16*)y, ldy, gamma, w, b, eps, (bf16*)out, ldo,
                                                   rows, cols);
  SR_CHECK(dtype == SR_F32, SR_EINVAL, "sr_residual_layernorm: bad dtype");
  return residual_layernorm_dispatch<float, float>(s, x, ldx, (const float*)y, ldy, gamma, w, b, eps, (float*)out, ldo,
                                                   rows, cols);
}

extern "C" int sr_layernorm(sr_stream_t stream, int out_dtype, const float* x, int64_t ldx, const int32_t* rowmap,
                            const float* w, const float* b, float eps, void* out, int64_t ldo, int rows, int cols) {
  SR_CHECK(x && out && rows > 0 && cols > 0, SR_EINVAL, "sr_layernorm: bad args");
  SR_CHECK((w == nullptr) == (b == nullptr), SR_EINVAL, "sr_layernorm: w and b must both be set or both NULL");
  SR_CHECK(ldx % 4 == 0, SR_EINVAL, "sr_layernorm: ldx must be a multiple of 4");
  hipStream_t s = (hipStream_t)stream;
  if (out_dtype == SR_BF16)
    return layernorm_dispatch<bf16>(s, x, ldx, rowmap, w, b, eps, (bf16*)out, ldo, rows, cols);
  SR_CHECK(out_dtype == SR_F32, SR_EINVAL, "sr_layernorm: bad dtype");
  return layernorm_dispatch<float>(s, x, ldx, rowmap, w, b, eps, (float*)out, ldo, rows, cols);
}

extern "C" int sr_layernorm_copy(sr_stream_t stream, int out_dtype, const float* x, int64_t ldx, const float* w,
                                 const float* b, float eps, void* out, int64_t ldo, float* x_copy, int64_t ldc,
                                 int rows, int cols) {
  SR_CHECK(x && out && x_copy && rows > 0 && cols > 0, SR_EINVAL, "sr_layernorm_copy: bad args");
  SR_CHECK((w == nullptr) == (b == nullptr), SR_EINVAL, "sr_layernorm_copy: w and b must both be set or both NULL");
  SR_CHECK(ldx % 4 == 0 && ldc % 4 == 0 && ldc >= cols && ((uintptr_t)x_copy & 15) == 0, SR_EINVAL,
           "sr_layernorm_copy: ldx / ldc multiples of 4, ldc >= cols, 16-B aligned x_copy");
  hipStream_t s = (hipStream_t)stream;
  if (out_dtype == SR_BF16)
    return layernorm_dispatch<bf16>(s, x, ldx, nullptr, w, b, eps, (bf16*)out, ldo, rows, cols, x_copy, ldc);
  SR_CHECK(out_dtype == SR_F32, SR_EINVAL, "sr_layernorm_copy: bad dtype");
  return layernorm_dispatch<float>(s, x, ldx, nullptr, w, b, eps, (float*)out, ldo, rows, cols, x_copy, ldc);
}

extern "C" int sr_im2col_normalize(sr_stream_t stream, int dtype, const float* img, int frames, int H, int W,
                                   int patch, const float* mean3, const float* std3, void* out, int kpad) {
  SR_CHECK(img && out && mean3 && std3, SR_EINVAL, "sr_im2col_normalize: null pointer");
  SR_CHECK(frames > 0 && patch > 0 && H % patch == 0 && W % patch == 0, SR_EINVAL,
           "sr_im2col_normalize: H=%d W=%d not multiples of patch %d", H, W, patch);
  SR_CHECK(kpad >= 3 * patch * patch, SR_EINVAL, "sr_im2col_normalize: kpad too small");
  const int64_t total = (int64_t)frames * (H / patch) * (W / patch) * kpad;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(im2col_kernel<bf16>, grid_for(total), dim3(256), 0, s, img, frames, H, W, patch, mean3[0],
                       mean3[1], mean3[2], std3[0], std3[1], std3[2], (bf16*)out, kpad);
  else
    hipLaunchKernelGGL(im2col_kernel<float>, grid_for(total), dim3(256), 0, s, img, frames, H, W, patch, mean3[0],
                       mean3[1], mean3[2], std3[0], std3[1], std3[2], (float*)out, kpad);
  return sr::check_launch("sr_im2col_normalize");
}

extern "C" int sr_set_special_tokens(sr_stream_t stream, float* x, int64_t ldx, int frames, int tokens_per_frame,
                                     int n_special, const float* table, const int32_t* type_of_frame, int cols) {
  SR_CHECK(x && table && type_of_frame && frames > 0 && n_special > 0 && n_special <= tokens_per_frame, SR_EINVAL,
           "sr_set_special_tokens: bad args");
  const int64_t total = (int64_t)frames * n_special * cols;
  hipLaunchKernelGGL(special_tokens_kernel, grid_for(total), dim3(256), 0, (hipStream_t)stream, x, ldx, frames,
                     tokens_per_frame, n_special, table, type_of_frame, cols);
  return sr::check_launch("sr_set_special_tokens");
}

extern "C" int sr_copy_rows_f32(sr_stream_t stream, float* dst, int64_t ldd, const float* src, int64_t lds,
                                const int32_t* rowmap, int rows, int cols) {
  SR_CHECK(dst && src && rows > 0 && cols > 0 && cols % 4 == 0 && ldd % 4 == 0 && lds % 4 == 0, SR_EINVAL,
           "sr_copy_rows_f32: bad args (cols and lds must be multiples of 4)");
  hipLaunchKernelGGL(copy_rows_kernel, grid_for((int64_t)rows * cols / 4), dim3(256), 0, (hipStream_t)stream, dst, ldd,
                     src, lds, rowmap, rows, cols / 4);
  return sr::check_launch("sr_copy_rows_f32");
}

extern "C" int sr_mul_cols(sr_stream_t stream, int dtype, const void* x, int64_t ldx, const float* gamma, void* out,
                           int64_t ldo, int rows, int cols) {
  SR_CHECK(x && gamma && out && rows > 0 && cols > 0, SR_EINVAL, "sr_mul_cols: bad args");
  const int64_t total = (int64_t)rows * cols;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(mul_cols_kernel<bf16>, grid_for(total), dim3(256), 0, s, (const bf16*)x, ldx, gamma, (bf16*)out,
                       ldo, rows, cols);
  else {
    SR_CHECK(dtype == SR_F32, SR_EINVAL, "sr_mul_cols: bad dtype %d", dtype);
    hipLaunchKernelGGL(mul_cols_kernel<float>, grid_for(total), dim3(256), 0, s, (const float*)x, ldx, gamma,
                       (float*)out, ldo, rows, cols);
  }
  return sr::check_launch("sr_mul_cols");
}

extern "C" int sr_linear_small_f32(sr_stream_t stream, const float* A, int64_t lda, const float* W, const float* bias,
                                   float* out, int64_t ldo, int M, int N, int K, int act_in) {
  SR_CHECK(A && W && out && M > 0 && N > 0 && K > 0, SR_EINVAL, "sr_linear_small_f32: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = (int64_t)M * N;
  if (K <= 64)
    hipLaunchKernelGGL(linear_small_thread_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, lda, W, bias,
                       out, ldo, M, N, K, act_in);
  else
    hipLaunchKernelGGL(linear_small_wave_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, A, lda, W, bias, out,
                       ldo, M, N, K, act_in);
  return sr::check_launch("sr_linear_small_f32");
}

extern "C" int sr_silu_f32(sr_stream_t stream, const float* x, float* y, int64_t n) {
  SR_CHECK(x && y && n > 0, SR_EINVAL, "sr_silu_f32: bad args");
  hipLaunchKernelGGL(silu_kernel, grid_for(n), dim3(256), 0, (hipStream_t)stream, x, y, n);
  return sr::check_launch("sr_silu_f32");
}

extern "C" int sr_adaln_modulate_f32(sr_stream_t stream, const float* xn, const float* x, const float* mod,
                                     float* out, int rows, int cols) {
  SR_CHECK(xn && x && mod && out && rows > 0 && cols > 0, SR_EINVAL, "sr_adaln_modulate_f32: bad args");
  hipLaunchKernelGGL(adaln_kernel, grid_for((int64_t)rows * cols), dim3(256), 0, (hipStream_t)stream, xn, x, mod, out,
                     rows, cols);
  return sr::check_launch("sr_adaln_modulate_f32");
}

extern "C" int sr_pose_update_f32(sr_stream_t stream, float* pred, const float* delta, int64_t ld_delta, float* act,
                                  int rows, int first) {
  SR_CHECK(pred && delta && act && rows > 0, SR_EINVAL, "sr_pose_update_f32: bad args");
  hipLaunchKernelGGL(pose_update_kernel, dim3((rows * 9 + 255) / 256), dim3(256), 0, (hipStream_t)stream, pred, delta,
                     ld_delta, act, rows, first);
  return sr::check_launch("sr_pose_update_f32");
}

extern "C" int sr_pose_decode_f32(sr_stream_t stream, const float* enc, int64_t ld_enc, int n, int H, int W,
                                  float* extrinsic, float* intrinsic) {
  SR_CHECK(enc && extrinsic && intrinsic && n > 0, SR_EINVAL, "sr_pose_decode_f32: bad args");
  hipLaunchKernelGGL(pose_decode_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, enc, ld_enc, n,
                     (float)H, (float)W, extrinsic, intrinsic);
  return sr::check_launch("sr_pose_decode_f32");
}
