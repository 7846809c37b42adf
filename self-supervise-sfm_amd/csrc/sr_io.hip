// Input formation (train/utils/io.py:75-153 ImagePreprocessor.process_image_with_matrices,
// SURVEY §8(f) rank 2): zero-pad to a centred square, PIL BICUBIC resize to the target side,
// ToTensor (RGB / 255) or depth (uint16 / 1000) — bit-exact with Pillow's separable resampler.
//
// The coefficient tables (per output pixel: first input index, tap count, weights) are built on
// the host exactly as Pillow builds them (double arithmetic; 8-bit modes quantise them to 22-bit
// fixed point) and uploaded once per (input side, target) pair.  The device does the two passes:
//   h pass: canvas rows x canvas columns -> [rows][tw][c] (uint8 or uint16), the zero padding of
//           the canvas folded into the read (pixels outside the pasted image are 0);
//   v pass: [rows][tw][c] -> [c][th][tw] fp32, fused with the ToTensor scaling and written
//           straight into the caller's frame slot (strided: crops, pads and the aggregator's
//           input tensor need no extra copy).  Tables may start at any output row (crop).
// 8-bit modes accumulate in int32 with the +2^21 rounding bias and clip to 0..255 after each pass;
// 'I;16' accumulates in double in tap order (no contraction), rounds half away from zero and
// stores (v % 256 clipped) | (v >> 8 clipped) << 8, as Pillow's 16-bit path does.
#include <cmath>

#include "sr_common.h"

namespace {

constexpr int TPB = 256;
constexpr int PREC = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ int clip8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

__device__ __forceinline__ int store16(double ss) {
  const int v = (int)(ss >= 0.0 ? ss + 0.5 : ss - 0.5);
  return clip8(v % 256) + (clip8(v >> 8) << 8);
}

// ---------------------------------------------------------------- horizontal pass, 8-bit modes
__global__ void pil_h_u8_kernel(const uint8_t* __restrict__ img, int n, int h, int w, int c, int rows, int pl,
                                int pt, const int* __restrict__ bounds, const int* __restrict__ kk, int ksize,
                                int tw, uint8_t* __restrict__ tmp) {
  const int64_t total = (int64_t)n * rows * tw;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int xx = (int)(e % tw);
    const int64_t r = e / tw;
    const int y = (int)(r % rows);
    const int f = (int)(r / rows);
    const int ys = y - pt;
    int acc[4] = {1 << (PREC - 1), 1 << (PREC - 1), 1 << (PREC - 1), 1 << (PREC - 1)};
    if (ys >= 0 && ys < h) {
      const int xmin = bounds[2 * xx], cnt = bounds[2 * xx + 1];
      const int* k = kk + (int64_t)xx * ksize;
      const uint8_t* row = img + ((int64_t)f * h + ys) * w * c;
      for (int t = 0; t < cnt; ++t) {
        const int xs = xmin + t - pl;
        if (xs < 0 || xs >= w) continue;  // zero padding contributes nothing
        const int kw = k[t];
        for (int ch = 0; ch < c; ++ch) acc[ch] += (int)row[(int64_t)xs * c + ch] * kw;
      }
    }
    uint8_t* o = tmp + e * c;
    for (int ch = 0; ch < c; ++ch) o[ch] = (uint8_t)clip8(acc[ch] >> PREC);
  }
}

// ---------------------------------------------------------------- vertical pass, 8-bit modes
__global__ void pil_v_u8_kernel(const uint8_t* __restrict__ tmp, int n, int rows, int tw, int c,
                                const int* __restrict__ bounds, const int* __restrict__ kk, int ksize, int th,
                                float divisor, float* __restrict__ out, int64_t fstride, int64_t cstride,
                                int64_t ldo) {
  const int64_t total = (int64_t)n * c * th * tw;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int xx = (int)(e % tw);
    int64_t r = e / tw;
    const int yy = (int)(r % th);
    r /= th;
    const int ch = (int)(r % c);
    const int f = (int)(r / c);
    const int ymin = bounds[2 * yy], cnt = bounds[2 * yy + 1];
    const int* k = kk + (int64_t)yy * ksize;
    const uint8_t* col = tmp + ((int64_t)f * rows * tw + xx) * c + ch;
    int acc = 1 << (PREC - 1);
    for (int t = 0; t < cnt; ++t) acc += (int)col[(int64_t)(ymin + t) * tw * c] * k[t];
    out[f * fstride + ch * cstride + yy * ldo + xx] = (float)clip8(acc >> PREC) / divisor;
  }
}

// ---------------------------------------------------------------- 'I;16' passes (double)
__global__ void pil_h_u16_kernel(const uint16_t* __restrict__ img, int n, int h, int w, int rows, int pl, int pt,
                                 const int* __restrict__ bounds, const double* __restrict__ kk, int ksize, int tw,
                                 uint16_t* __restrict__ tmp) {
#pragma clang fp contract(off)
  const int64_t total = (int64_t)n * rows * tw;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int xx = (int)(e % tw);
    const int64_t r = e / tw;
    const int y = (int)(r % rows);
    const int f = (int)(r / rows);
    const int ys = y - pt;
    double ss = 0.0;
    if (ys >= 0 && ys < h) {
      const int xmin = bounds[2 * xx], cnt = bounds[2 * xx + 1];
      const double* k = kk + (int64_t)xx * ksize;
      const uint16_t* row = img + ((int64_t)f * h + ys) * w;
      for (int t = 0; t < cnt; ++t) {
        const int xs = xmin + t - pl;
        // padding pixels are 0: adding 0 * k keeps Pillow's summation order and -0/+0 behaviour
        const double v = (xs >= 0 && xs < w) ? (double)row[xs] : 0.0;
        ss += v * k[t];
      }
    }
    tmp[e] = (uint16_t)store16(ss);
  }
}

__global__ void pil_v_u16_kernel(const uint16_t* __restrict__ tmp, int n, int rows, int tw,
                                 const int* __restrict__ bounds, const double* __restrict__ kk, int ksize, int th,
                                 float divisor, float* __restrict__ out, int64_t fstride, int64_t ldo) {
#pragma clang fp contract(off)
  const int64_t total = (int64_t)n * th * tw;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int xx = (int)(e % tw);
    const int64_t r = e / tw;
    const int yy = (int)(r % th);
    const int f = (int)(r / th);
    const int ymin = bounds[2 * yy], cnt = bounds[2 * yy + 1];
    const double* k = kk + (int64_t)yy * ksize;
    const uint16_t* col = tmp + (int64_t)f * rows * tw + xx;
    double ss = 0.0;
    for (int t = 0; t < cnt; ++t) ss += (double)col[(int64_t)(ymin + t) * tw] * k[t];
    out[f * fstride + yy * ldo + xx] = (float)store16(ss) / divisor;
  }
}

unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>((n + TPB - 1) / TPB, 1 << 20); }

}  // namespace

extern "C" int sr_pil_resample_h(sr_stream_t stream, int mode, const void* img, int n, int h, int w, int c,
                                 int canvas_h, int canvas_w, int pad_left, int pad_top, const int* bounds,
                                 const void* coeffs, int ksize, int tw, void* tmp) {
  SR_CHECK(img && bounds && coeffs && tmp && n > 0 && h > 0 && w > 0 && pad_left >= 0 && pad_top >= 0 &&
               pad_left + w <= canvas_w && pad_top + h <= canvas_h && ksize > 0 && tw > 0,
           SR_EINVAL, "sr_pil_resample_h: bad args (h=%d w=%d canvas=%dx%d pad=%d,%d)", h, w, canvas_h, canvas_w,
           pad_left, pad_top);
  SR_CHECK((mode == 0 && c >= 1 && c <= 4) || (mode == 1 && c == 1), SR_EINVAL,
           "sr_pil_resample_h: mode %d with %d channels unsupported", mode, c);
  const int64_t total = (int64_t)n * canvas_h * tw;
  if (mode == 0)
    hipLaunchKernelGGL(pil_h_u8_kernel, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream,
                       (const uint8_t*)img, n, h, w, c, canvas_h, pad_left, pad_top, bounds, (const int*)coeffs, ksize,
                       tw, (uint8_t*)tmp);
  else
    hipLaunchKernelGGL(pil_h_u16_kernel, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream,
                       (const uint16_t*)img, n, h, w, canvas_h, pad_left, pad_top, bounds, (const double*)coeffs,
                       ksize, tw, (uint16_t*)tmp);
  return sr::check_launch("sr_pil_resample_h");
}

extern "C" int sr_pil_resample_v_f32(sr_stream_t stream, int mode, const void* tmp, int n, int rows, int tw, int c,
                                     const int* bounds, const void* coeffs, int ksize, int th, float divisor,
                                     float* out, int64_t frame_stride, int64_t chan_stride, int64_t ldo) {
  SR_CHECK(tmp && bounds && coeffs && out && n > 0 && rows > 0 && tw > 0 && th > 0 && ksize > 0 && divisor != 0.f &&
               ldo >= tw && (c == 1 || chan_stride >= (int64_t)th * ldo) && frame_stride >= (int64_t)c * th * tw,
           SR_EINVAL, "sr_pil_resample_v_f32: bad args");
  SR_CHECK((mode == 0 && c >= 1 && c <= 4) || (mode == 1 && c == 1), SR_EINVAL,
           "sr_pil_resample_v_f32: mode %d with %d channels unsupported", mode, c);
  if (mode == 0)
    hipLaunchKernelGGL(pil_v_u8_kernel, dim3(grid_for((int64_t)n * c * th * tw)), dim3(TPB), 0,
                       (hipStream_t)stream, (const uint8_t*)tmp, n, rows, tw, c, bounds, (const int*)coeffs, ksize,
                       th, divisor, out, frame_stride, chan_stride, ldo);
  else
    hipLaunchKernelGGL(pil_v_u16_kernel, dim3(grid_for((int64_t)n * th * tw)), dim3(TPB), 0, (hipStream_t)stream,
                       (const uint16_t*)tmp, n, rows, tw, bounds, (const double*)coeffs, ksize, th, divisor, out,
                       frame_stride, ldo);
  return sr::check_launch("sr_pil_resample_v_f32");
}
