// Input formation (train/utils/io.py:75-153 ImagePreprocessor.process_image_with_matrices,
// SURVEY §8(f) rank 2): zero-pad to a centred square, PIL BICUBIC resize to the target side,
// ToTensor (RGB / 255) or depth (uint16 / 1000) — bit-exact with Pillow's separable resampler.
//
// The coefficient tables (per output pixel: first input index, tap count, weights) are built on
// the host exactly as Pillow builds them (double arithmetic; 8-bit modes quantise them to 22-bit
// fixed point) and uploaded once per shape.  The zero padding of the square canvas is folded into
// them: taps on padding are dropped (Pillow adds 0 * weight for those, which changes nothing), so
// the kernels only ever touch image pixels.  The device runs the two passes:
//   h pass: a workgroup per band of image rows stages them in LDS with coalesced 16-byte loads,
//           then each thread produces 4 adjacent output columns of every channel (quad-major
//           table: one 16-byte load per tap, branch-free tap loop) and stores them as one dword /
//           8 bytes per channel into a planar intermediate tmp [n][c][h][ldt] (ldt = tw rounded
//           up to 4, tail zeroed);
//   v pass: each thread reads 4 adjacent intermediate columns per tap (one dword / 8 bytes) and
//           writes 4 fp32 outputs, ToTensor scaling fused, straight into the caller's frame slot
//           (strided: crops, pads and the aggregator's input tensor need no extra copy).
// 8-bit modes accumulate in int32 with the +2^21 rounding bias and clip to 0..255 after each pass;
// 'I;16' accumulates in double in tap order (no contraction), rounds half away from zero and
// stores (v % 256 clipped) | (v >> 8 clipped) << 8, as Pillow's 16-bit path does.
//
// A one-launch variant (both passes per band of output rows, intermediate in LDS) measured 2x
// slower at 32 x 768x1024 -> 518: its serialised phases ran latency-bound at LDS-limited occupancy.
#include <cmath>
#include <type_traits>

#include "sr_common.h"

namespace {

constexpr int TPB = 256;
constexpr int PREC = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2
constexpr int ROW_LDS = 32 << 10;
constexpr int KB = 8;  // taps whose loads are issued together

__device__ __forceinline__ int clip8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// NB bytes of LDS starting at any byte offset b, as NB/4 words: aligned dword reads (volatile, so
// the compiler cannot merge them into one unaligned wide read — LDS ds_read_b64/b128 at byte
// offsets returned wrong bytes here) funnel-shifted by v_alignbit.
template <int NB>
__device__ __forceinline__ void lds_span(const uint8_t* lds, int b, uint32_t (&sw)[NB / 4]) {
  typedef __attribute__((address_space(3))) const volatile uint32_t lds_word;
  lds_word* p = (lds_word*)(lds + (b & ~3));
  const uint32_t sh = (uint32_t)(b & 3) * 8u;
  uint32_t wv[NB / 4 + 1];
#pragma unroll
  for (int i = 0; i <= NB / 4; ++i) wv[i] = p[i];
#pragma unroll
  for (int i = 0; i < NB / 4; ++i) sw[i] = __builtin_amdgcn_alignbit(wv[i + 1], wv[i], sh);
}

__device__ __forceinline__ int store16(double ss) {
  const int v = (int)(ss >= 0.0 ? ss + 0.5 : ss - 0.5);
  return clip8(v % 256) + (clip8(v >> 8) << 8);
}

// ---------------------------------------------------------------- horizontal pass
// Block = band of rb image rows of one frame.  LDS holds the band (one contiguous range of the
// frame, copied from its 16-byte-aligned start, plus slack for the zero-weight tail taps).  A thread
// owns 4 adjacent output columns of one row for all C channels: the quad-major table gives their
// first indices and tap counts (one 16-byte load each) and per-tap weights (one 16-byte load per
// tap, KB taps in flight).  Every thread runs all ksize taps: weights past a column's taps are 0,
// which adds exactly nothing (integer, or +0.0 to a double sum that is never -0.0), so the tap
// loop has no branches; the padding of the canvas is folded into the table on the host.
template <int MODE, int C>
__global__ __launch_bounds__(TPB) void pil_h_kernel(const uint8_t* __restrict__ img, int h, int w,
                                                    const int4* __restrict__ hb, const void* __restrict__ hk_, int hks,
                                                    int ldt, int rb, uint8_t* __restrict__ tmp) {
#pragma clang fp contract(off)
  using T = typename std::conditional<MODE == 0, uint8_t, uint16_t>::type;
  constexpr int ESZ = sizeof(T);
  extern __shared__ __align__(16) uint32_t lds_dw[];
  const int bands = (h + rb - 1) / rb;
  const int f = blockIdx.x / bands, r0 = (blockIdx.x % bands) * rb, nr = min(rb, h - r0);
  const int rowbytes = w * C * ESZ;
  const uint8_t* src = img + ((int64_t)f * h + r0) * rowbytes;
  const uint4* a0 = (const uint4*)(src - ((uintptr_t)src & 15));
  const int shift = (int)((uintptr_t)src & 15);
  {
    // all of a thread's 16-byte loads in flight before its LDS stores
    const int nq = (shift + nr * rowbytes + 15) >> 4;
    uint4* l4 = (uint4*)lds_dw;
    for (int i0 = 0; i0 < nq; i0 += 8 * TPB) {
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i = i0 + k * TPB + threadIdx.x;
        if (i < nq) v[k] = a0[i];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i = i0 + k * TPB + threadIdx.x;
        if (i < nq) l4[i] = v[k];
      }
    }
  }
  __syncthreads();
  const int quads = ldt >> 2;
  const int plane = h * ldt;
  for (int it = threadIdx.x; it < nr * quads; it += TPB) {
    const int q = it % quads, j = it / quads;
    const uint8_t* lds = (const uint8_t*)lds_dw;
    const int rowb = shift + j * rowbytes;  // byte offset of this row in LDS
    const int4 xm = hb[2 * q];
    const int xo[4] = {rowb + xm.x * C * ESZ, rowb + xm.y * C * ESZ, rowb + xm.z * C * ESZ, rowb + xm.w * C * ESZ};
    uint32_t o[C][4];  // stored values (0..255 / 0..65535), packed below
    if constexpr (MODE == 0) {
      int acc[C][4];
#pragma unroll
      for (int ch = 0; ch < C; ++ch)
        for (int u = 0; u < 4; ++u) acc[ch][u] = 1 << (PREC - 1);
      const int4* k = (const int4*)hk_ + q * hks;
      for (int t0 = 0; t0 < hks; t0 += KB) {
        int4 kc[KB];
#pragma unroll
        for (int i = 0; i < KB; ++i) kc[i] = t0 + i < hks ? k[t0 + i] : make_int4(0, 0, 0, 0);
        const int kw[KB][4] = {
#define SR_KW(i) {kc[i].x, kc[i].y, kc[i].z, kc[i].w}
            SR_KW(0), SR_KW(1), SR_KW(2), SR_KW(3), SR_KW(4), SR_KW(5), SR_KW(6), SR_KW(7)};
#undef SR_KW
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          uint32_t sw[KB * C / 4];  // the KB taps' C bytes each, contiguous
          lds_span<KB * C>(lds, xo[u] + t0 * C, sw);
#pragma unroll
          for (int i = 0; i < KB; ++i)
#pragma unroll
            for (int ch = 0; ch < C; ++ch) {
              const int bi = i * C + ch;
              acc[ch][u] += (int)((sw[bi >> 2] >> ((bi & 3) * 8)) & 255u) * kw[i][u];
            }
        }
      }
#pragma unroll
      for (int ch = 0; ch < C; ++ch)
        for (int u = 0; u < 4; ++u) {
          o[ch][u] = (uint32_t)clip8(acc[ch][u] >> PREC);
          // opaque to the optimiser: ROCm 7.2 clang folds shift + clamp + byte pack into gfx950's
          // v_ashr_pk_u8_i32 and ORs its result as if bits 16-31 were zero, which they are not
          // (corrupted bytes 2-3 of the packed word, caught by tests/test_io_gpu.py)
          asm volatile("" : "+v"(o[ch][u]));
        }
    } else {
      double ss[4] = {0.0, 0.0, 0.0, 0.0};
      const double2* k = (const double2*)hk_ + q * hks * 2;
      constexpr int NT = KB / 2;
      for (int t0 = 0; t0 < hks; t0 += NT) {
        double2 kc[KB];
#pragma unroll
        for (int i = 0; i < KB; ++i) kc[i] = t0 + i / 2 < hks ? k[2 * t0 + i] : make_double2(0.0, 0.0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          uint32_t sw[NT / 2];  // NT uint16 pixels
          lds_span<NT * 2>(lds, xo[u] + t0 * 2, sw);
#pragma unroll
          for (int i = 0; i < NT; ++i) {
            const double kwu = (u & 1) ? ((u & 2) ? kc[2 * i + 1].y : kc[2 * i].y) : ((u & 2) ? kc[2 * i + 1].x : kc[2 * i].x);
            ss[u] += (double)((sw[i >> 1] >> ((i & 1) * 16)) & 65535u) * kwu;  // Pillow's tap order
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) o[0][u] = (uint32_t)store16(ss[u]);
    }
    T* dst = (T*)tmp + ((int64_t)f * C * h + r0 + j) * ldt + q * 4;
#pragma unroll
    for (int ch = 0; ch < C; ++ch) {
      T* d = dst + (int64_t)ch * plane;
      if constexpr (MODE == 0)
        *(uint32_t*)d = o[ch][0] | (o[ch][1] << 8) | (o[ch][2] << 16) | (o[ch][3] << 24);
      else
        *(uint2*)d = make_uint2(o[ch][0] | (o[ch][1] << 16), o[ch][2] | (o[ch][3] << 16));
    }
  }
}

// ---------------------------------------------------------------- vertical pass
template <int MODE>
__global__ __launch_bounds__(TPB) void pil_v_kernel(const uint8_t* __restrict__ tmp, int n, int rows, int ldt, int c,
                                                    const int* __restrict__ vb, const void* __restrict__ vk_, int vks,
                                                    int th, int tw, float divisor, float* __restrict__ out,
                                                    int64_t fs, int64_t cs, int64_t ldo) {
#pragma clang fp contract(off)
  using T = typename std::conditional<MODE == 0, uint8_t, uint16_t>::type;
  const int quads = ldt >> 2;
  const int64_t total = (int64_t)n * c * th * quads;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int q = (int)(e % quads);
    int64_t r = e / quads;
    const int yy = (int)(r % th);
    r /= th;
    const int ch = (int)(r % c), f = (int)(r / c);
    const int ymin = vb[2 * yy], cnt = vb[2 * yy + 1];
    const T* col = (const T*)tmp + ((int64_t)f * c + ch) * rows * ldt + q * 4;
    float v[4];
    if constexpr (MODE == 0) {
      const int* k = (const int*)vk_ + (int64_t)yy * vks;
      int a0 = 1 << (PREC - 1), a1 = a0, a2 = a0, a3 = a0;
      for (int t0 = 0; t0 < cnt; t0 += KB) {
        uint32_t p[KB];
        int kw[KB];
#pragma unroll
        for (int i = 0; i < KB; ++i) {
          const bool live = t0 + i < cnt;
          p[i] = live ? *(const uint32_t*)(col + (int64_t)(ymin + t0 + i) * ldt) : 0u;
          kw[i] = live ? k[t0 + i] : 0;
        }
#pragma unroll
        for (int i = 0; i < KB; ++i) {
          a0 += (int)(p[i] & 255) * kw[i];
          a1 += (int)((p[i] >> 8) & 255) * kw[i];
          a2 += (int)((p[i] >> 16) & 255) * kw[i];
          a3 += (int)(p[i] >> 24) * kw[i];
        }
      }
      v[0] = (float)clip8(a0 >> PREC);
      v[1] = (float)clip8(a1 >> PREC);
      v[2] = (float)clip8(a2 >> PREC);
      v[3] = (float)clip8(a3 >> PREC);
    } else {
      const double* k = (const double*)vk_ + (int64_t)yy * vks;
      double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
      for (int t0 = 0; t0 < cnt; t0 += KB) {
        uint2 p[KB];
        double kw[KB];
#pragma unroll
        for (int i = 0; i < KB; ++i) {
          const bool live = t0 + i < cnt;
          p[i] = live ? *(const uint2*)(col + (int64_t)(ymin + t0 + i) * ldt) : make_uint2(0u, 0u);
          kw[i] = live ? k[t0 + i] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < KB; ++i) {
          if (t0 + i < cnt) {  // tap order kept; no 0-weight terms beyond the taps
            s0 += (double)(p[i].x & 65535) * kw[i];
            s1 += (double)(p[i].x >> 16) * kw[i];
            s2 += (double)(p[i].y & 65535) * kw[i];
            s3 += (double)(p[i].y >> 16) * kw[i];
          }
        }
      }
      v[0] = (float)store16(s0);
      v[1] = (float)store16(s1);
      v[2] = (float)store16(s2);
      v[3] = (float)store16(s3);
    }
    float* o = out + f * fs + ch * cs + (int64_t)yy * ldo + q * 4;
    const int live = min(4, tw - q * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < live) o[u] = v[u] / divisor;
  }
}

unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>((n + TPB - 1) / TPB, 1 << 20); }

// ------------------------------------------------------------ reverse transform (io.py:197-259)
// torch's upsample index / weight rules with align_corners=False (ATen UpSample.h):
//   src = scale * (dst + 0.5) - 0.5, scale = in / out (float);  linear clamps src at 0, cubic does not;
//   cubic: i = floor(src) and t = src - i (clamped to [0, 1]), the 4 taps i-1..i+2 read clamped to
//   the image, Keys' convolution with A = -0.75 (get_cubic_upsample_coefficients).
__device__ __forceinline__ float cubic1(float x, float A) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; }
__device__ __forceinline__ float cubic2(float x, float A) { return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; }

struct Taps {
  int i[4];
  float w[4];
};

template <bool CUBIC>
__device__ __forceinline__ Taps taps(int dst, float scale, int in) {
  Taps t;
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  if constexpr (CUBIC) {
    const float fl = floorf(src);
    const int i0 = (int)fl;
    const float x = fminf(fmaxf(src - fl, 0.f), 1.f);
    constexpr float A = -0.75f;
    t.w[0] = cubic2(x + 1.f, A);
    t.w[1] = cubic1(x, A);
    t.w[2] = cubic1(1.f - x, A);
    t.w[3] = cubic2(2.f - x, A);
#pragma unroll
    for (int k = 0; k < 4; ++k) t.i[k] = min(max(i0 - 1 + k, 0), in - 1);
  } else {
    src = fmaxf(src, 0.f);
    const int i0 = (int)src;
    const float l1 = src - (float)i0;
    t.i[0] = i0;
    t.i[1] = i0 + (i0 < in - 1 ? 1 : 0);
    t.w[0] = 1.f - l1;
    t.w[1] = l1;
  }
  return t;
}

// out[ch][oy][ox] = resize(x[ch], (h, w) -> (hs, ws))[oy + y0][ox + x0]: one thread per output
// element, consecutive threads along a row (coalesced stores; the taps' reads hit L2)
template <bool CUBIC>
__global__ __launch_bounds__(TPB) void resize_crop_chw_kernel(const float* __restrict__ x, int c, int h, int w,
                                                              float sh, float sw, int y0, int x0, int ho, int wo,
                                                              float* __restrict__ out) {
  constexpr int NT = CUBIC ? 4 : 2;
  const int64_t total = (int64_t)c * ho * wo;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int ox = (int)(e % wo);
    const int64_t r = e / wo;
    const int oy = (int)(r % ho), ch = (int)(r / ho);
    const Taps ty = taps<CUBIC>(oy + y0, sh, h), tx = taps<CUBIC>(ox + x0, sw, w);
    const float* plane = x + (int64_t)ch * h * w;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float* row = plane + (int64_t)ty.i[j] * w;
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < NT; ++i) v += row[tx.i[i]] * tx.w[i];
      acc += v * ty.w[j];
    }
    out[e] = acc;
  }
}

}  // namespace

extern "C" int sr_resize_crop_chw_f32(sr_stream_t stream, const float* x, int c, int h, int w, int hs, int ws,
                                      int y0, int x0, int ho, int wo, int mode, float* out) {
  SR_CHECK(x && out && x != out && c > 0 && h > 0 && w > 0 && hs > 0 && ws > 0 && ho > 0 && wo > 0, SR_EINVAL,
           "sr_resize_crop_chw_f32: bad args");
  SR_CHECK(y0 >= 0 && x0 >= 0 && y0 + ho <= hs && x0 + wo <= ws, SR_EINVAL,
           "sr_resize_crop_chw_f32: crop [%d, %d) x [%d, %d) outside the %d x %d resized image", y0, y0 + ho, x0,
           x0 + wo, hs, ws);
  SR_CHECK(mode == 0 || mode == 1, SR_EINVAL, "sr_resize_crop_chw_f32: mode 0 (bilinear) or 1 (bicubic)");
  const int64_t total = (int64_t)c * ho * wo;
  const float sh = (float)h / (float)hs, sw = (float)w / (float)ws;  // area_pixel_compute_scale
  if (mode == 1)
    hipLaunchKernelGGL(resize_crop_chw_kernel<true>, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream, x, c,
                       h, w, sh, sw, y0, x0, ho, wo, out);
  else
    hipLaunchKernelGGL(resize_crop_chw_kernel<false>, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream, x,
                       c, h, w, sh, sw, y0, x0, ho, wo, out);
  sr::note_kernel("resize_crop_chw_kernel<%s>", mode == 1 ? "true" : "false");
  return sr::check_launch("sr_resize_crop_chw_f32");
}

extern "C" int sr_pil_resample_h(sr_stream_t stream, int mode, const void* img, int n, int h, int w, int c,
                                 const int* bounds, const void* coeffs, int ksize, int tw, void* tmp) {
  SR_CHECK(img && bounds && coeffs && tmp && n > 0 && h > 0 && w > 0 && ksize > 0 && tw > 0, SR_EINVAL,
           "sr_pil_resample_h: bad args (n=%d h=%d w=%d ksize=%d tw=%d)", n, h, w, ksize, tw);
  SR_CHECK((mode == 0 && c >= 1 && c <= 4) || (mode == 1 && c == 1), SR_EINVAL,
           "sr_pil_resample_h: mode %d with %d channels unsupported", mode, c);
  const int64_t esz = mode == 0 ? 1 : 2;
  const int64_t rowbytes = (int64_t)w * c * esz;
  // aligned-down start, the zero-weight tail taps (ksize rounded up to KB) and the last span word
  const int64_t slack = 48 + (int64_t)((ksize + KB - 1) / KB * KB) * c * esz;
  SR_CHECK(rowbytes + slack <= 2 * ROW_LDS, SR_EUNSUPPORTED, "sr_pil_resample_h: %lld-byte image rows exceed LDS",
           (long long)rowbytes);
  const int rb = (int)std::max<int64_t>(1, std::min<int64_t>(8, (ROW_LDS - slack) / rowbytes));
  const int ldt = (tw + 3) & ~3;
  const int bands = (h + rb - 1) / rb;
  const size_t lds = ((size_t)(rb * rowbytes + slack) + 15) & ~(size_t)15;
  const dim3 grid(n * bands), block(TPB);
  const hipStream_t st = (hipStream_t)stream;
  const uint8_t* im = (const uint8_t*)img;
  const int4* hb = (const int4*)bounds;
  uint8_t* t8 = (uint8_t*)tmp;
  switch (mode * 8 + c) {
    case 1: hipLaunchKernelGGL((pil_h_kernel<0, 1>), grid, block, lds, st, im, h, w, hb, coeffs, ksize, ldt, rb, t8); break;
    case 2: hipLaunchKernelGGL((pil_h_kernel<0, 2>), grid, block, lds, st, im, h, w, hb, coeffs, ksize, ldt, rb, t8); break;
    case 3: hipLaunchKernelGGL((pil_h_kernel<0, 3>), grid, block, lds, st, im, h, w, hb, coeffs, ksize, ldt, rb, t8); break;
    case 4: hipLaunchKernelGGL((pil_h_kernel<0, 4>), grid, block, lds, st, im, h, w, hb, coeffs, ksize, ldt, rb, t8); break;
    default: hipLaunchKernelGGL((pil_h_kernel<1, 1>), grid, block, lds, st, im, h, w, hb, coeffs, ksize, ldt, rb, t8); break;
  }
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
  const int ldt = (tw + 3) & ~3;
  const int64_t total = (int64_t)n * c * th * (ldt / 4);
  if (mode == 0)
    hipLaunchKernelGGL(pil_v_kernel<0>, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream,
                       (const uint8_t*)tmp, n, rows, ldt, c, bounds, coeffs, ksize, th, tw, divisor, out,
                       frame_stride, chan_stride, ldo);
  else
    hipLaunchKernelGGL(pil_v_kernel<1>, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream,
                       (const uint8_t*)tmp, n, rows, ldt, c, bounds, coeffs, ksize, th, tw, divisor, out,
                       frame_stride, chan_stride, ldo);
  return sr::check_launch("sr_pil_resample_v_f32");
}
