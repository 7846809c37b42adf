// DPT point / depth head (dpt_head.py:151-349) and depth unprojection
// (geometry.py:19-130): the data-movement and elementwise kernels around the fp32 GEMMs.
//
// Layout: every feature map is NHWC fp32 ([frames][y][x][channel], channels contiguous),
// so a 1x1 conv is a plain GEMM over pixels, a 3x3 conv is im2col + GEMM with K ordered
// (ky, kx, ci), and a k x k stride-k ConvTranspose is a GEMM to (ky, kx, co) columns followed
// by a scatter.  Threads work on float4 channel groups (channel counts are multiples of 4).
#include <cmath>

#include "sr_common.h"

namespace {

constexpr int TPB = 256;


// ---------------------------------------------------------------- im2col (3x3, pad 1)
// out[(f*ho + oy)*wo + ox][(ky*3 + kx)*c + ci] = act(x[f][oy*s + ky - 1][ox*s + kx - 1][ci]), 0 outside;
// act = ReLU when relu_in (ResidualConvUnit applies ReLU before each conv, dpt_head.py:470-476).
__global__ void im2col3x3_kernel(const float* __restrict__ x, int n, int h, int w, int c, int stride, int relu_in,
                                 float* __restrict__ out, int ho, int wo) {
  const int c4 = c >> 2;
  const int64_t total = (int64_t)n * ho * wo * 9 * c4;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int cq = (int)(e % c4);
    const int64_t t = e / c4;
    const int tap = (int)(t % 9);
    const int64_t pix = t / 9;
    const int ox = (int)(pix % wo);
    const int64_t r = pix / wo;
    const int oy = (int)(r % ho);
    const int f = (int)(r / ho);
    const int iy = oy * stride + tap / 3 - 1, ix = ox * stride + tap % 3 - 1;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (iy >= 0 && iy < h && ix >= 0 && ix < w) {
      v = *(const float4*)(x + (((int64_t)f * h + iy) * w + ix) * c + cq * 4);
      if (relu_in) {
        v.x = fmaxf(v.x, 0.f);
        v.y = fmaxf(v.y, 0.f);
        v.z = fmaxf(v.z, 0.f);
        v.w = fmaxf(v.w, 0.f);
      }
    }
    *(float4*)(out + pix * 9 * c + tap * c + cq * 4) = v;
  }
}

// ---------------------------------------------------------------- ConvTranspose scatter
// g[(f*h + y)*w + x][(ky*k + kx)*co + c] -> out[f][y*k + ky][x*k + kx][c] + bias[c]
// (ConvTranspose2d with kernel_size == stride, padding 0: dpt_head.py:89-104)
__global__ void convt_scatter_kernel(const float* __restrict__ g, int n, int h, int w, int k, int co,
                                     const float* __restrict__ bias, float* __restrict__ out) {
  const int c4 = co >> 2, W = w * k, H = h * k;
  const int64_t total = (int64_t)n * H * W * c4;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int cq = (int)(e % c4);
    const int64_t p = e / c4;
    const int X = (int)(p % W);
    const int64_t r = p / W;
    const int Y = (int)(r % H);
    const int f = (int)(r / H);
    const int y = Y / k, ky = Y - y * k, x = X / k, kx = X - x * k;
    float4 v = *(const float4*)(g + (((int64_t)f * h + y) * w + x) * (k * k * co) + (ky * k + kx) * co + cq * 4);
    if (bias) {
      const float4 b = *(const float4*)(bias + cq * 4);
      v.x += b.x;
      v.y += b.y;
      v.z += b.z;
      v.w += b.w;
    }
    *(float4*)(out + p * co + cq * 4) = v;
  }
}

// ---------------------------------------------------------------- bilinear resize
// F.interpolate(mode="bilinear", align_corners=True) (custom_interpolate, dpt_head.py:568-598):
// src = dst * (in - 1) / (out - 1); weights and blend in PyTorch's order.  Optional `add`
// (same shape as out) is summed after interpolation.
__global__ void resize_bilinear_kernel(const float* __restrict__ x, int n, int h, int w, int c, int ho, int wo,
                                       const float* __restrict__ add, float* __restrict__ out) {
  const int c4 = c >> 2;
  const float sy = ho > 1 ? (float)(h - 1) / (float)(ho - 1) : 0.f;
  const float sx = wo > 1 ? (float)(w - 1) / (float)(wo - 1) : 0.f;
  const int64_t total = (int64_t)n * ho * wo * c4;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int cq = (int)(e % c4);
    const int64_t p = e / c4;
    const int ox = (int)(p % wo);
    const int64_t r = p / wo;
    const int oy = (int)(r % ho);
    const int f = (int)(r / ho);
    const float fy = sy * oy, fx = sx * ox;
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < h - 1), x1 = x0 + (x0 < w - 1);
    const float ly1 = fy - y0, ly0 = 1.f - ly1, lx1 = fx - x0, lx0 = 1.f - lx1;
    const float* base = x + (int64_t)f * h * w * c + cq * 4;
    const float4 a = *(const float4*)(base + ((int64_t)y0 * w + x0) * c);
    const float4 b = *(const float4*)(base + ((int64_t)y0 * w + x1) * c);
    const float4 cc = *(const float4*)(base + ((int64_t)y1 * w + x0) * c);
    const float4 d = *(const float4*)(base + ((int64_t)y1 * w + x1) * c);
    float4 v;
    v.x = ly0 * (lx0 * a.x + lx1 * b.x) + ly1 * (lx0 * cc.x + lx1 * d.x);
    v.y = ly0 * (lx0 * a.y + lx1 * b.y) + ly1 * (lx0 * cc.y + lx1 * d.y);
    v.z = ly0 * (lx0 * a.z + lx1 * b.z) + ly1 * (lx0 * cc.z + lx1 * d.z);
    v.w = ly0 * (lx0 * a.w + lx1 * b.w) + ly1 * (lx0 * cc.w + lx1 * d.w);
    if (add) {  // one [ho][wo][c] table for every frame
      const float4 q = *(const float4*)(add + (p - (int64_t)f * ho * wo) * c + cq * 4);
      v.x += q.x;
      v.y += q.y;
      v.z += q.z;
      v.w += q.w;
    }
    *(float4*)(out + p * c + cq * 4) = v;
  }
}

__global__ void relu_kernel(float* __restrict__ x, int64_t n4) {
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < n4; e += (int64_t)gridDim.x * TPB) {
    float4 a = ((float4*)x)[e];
    a.x = fmaxf(a.x, 0.f);
    a.y = fmaxf(a.y, 0.f);
    a.z = fmaxf(a.z, 0.f);
    a.w = fmaxf(a.w, 0.f);
    ((float4*)x)[e] = a;
  }
}

__global__ void add_kernel(float* __restrict__ dst, const float* __restrict__ src, int64_t n4) {
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < n4; e += (int64_t)gridDim.x * TPB) {
    float4 a = ((float4*)dst)[e];
    const float4 b = ((const float4*)src)[e];
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
    ((float4*)dst)[e] = a;
  }
}

// ---------------------------------------------------------------- positional embedding
// x[f][y][x][ch] += ratio * emb (DPTHead._apply_pos_embed, dpt_head.py:300-315):
//   uv grid (utils.py create_uv_grid): u_x = linspace(-sx (w-1)/w, sx (w-1)/w, w),
//   v_y likewise with sy, (sx, sy) = (a, 1) / sqrt(a^2 + 1), a = W / H of the image;
//   channels [0, c/2): u, [c/2, c): v; each half = [sin(pos * om_i) | cos(pos * om_i)],
//   om_i = 100^(-i / (c/4)), i < c/4, evaluated in double and rounded to fp32 like
//   make_sincos_pos_embed.  linspace follows PyTorch's fp32 two-sided evaluation.
__device__ __forceinline__ float linspace_at(float start, float end, int steps, int i) {
  if (steps == 1) return start;
  const float step = (end - start) / (float)(steps - 1);
  return i < steps / 2 ? start + step * (float)i : end - step * (float)(steps - 1 - i);
}

__global__ void dpt_pos_embed_kernel(float* __restrict__ x, int n, int h, int w, int c, float aspect, float ratio) {
  const int half = c / 2, quarter = c / 4;
  const int64_t total = (int64_t)n * h * w * c;
  const float diag = sqrtf(aspect * aspect + 1.f);
  const float spx = aspect / diag, spy = 1.f / diag;
  const float lx = -spx * (float)(w - 1) / (float)w, rx = spx * (float)(w - 1) / (float)w;
  const float ty = -spy * (float)(h - 1) / (float)h, by = spy * (float)(h - 1) / (float)h;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int ch = (int)(e % c);
    const int64_t p = e / c;
    const int xx = (int)(p % w);
    const int y = (int)((p / w) % h);
    const int part = ch / half, j = ch - part * half;
    const float pos = part == 0 ? linspace_at(lx, rx, w, xx) : linspace_at(ty, by, h, y);
    const int i = j < quarter ? j : j - quarter;
    const double om = 1.0 / pow(100.0, (double)i / (double)quarter);
    const double arg = (double)pos * om;
    const float emb = (float)(j < quarter ? sin(arg) : cos(arg));
    x[e] += emb * ratio;
  }
}

// ---------------------------------------------------------------- output head
// hidden = output of output_conv2[0] (3x3 conv); out = conv1x1(relu(hidden)) + b, then
// activate_head (head_act.py:63-113): preds = act(out[:cout-1]), conf = conf_act(out[cout-1]).
// act: 0 inv_log sign(y) expm1(|y|), 1 exp, 2 linear, 3 relu.  conf_act: 0 expp1, 1 expp0, 2 sigmoid.
__global__ void dpt_head_out_kernel(const float* __restrict__ hid, int64_t ldh, int64_t npix, int cin,
                                    const float* __restrict__ wt, const float* __restrict__ b, int cout, int act,
                                    int conf_act, float* __restrict__ preds, float* __restrict__ conf) {
  for (int64_t p = blockIdx.x * (int64_t)TPB + threadIdx.x; p < npix; p += (int64_t)gridDim.x * TPB) {
    const float* hr = hid + p * ldh;
    for (int o = 0; o < cout; ++o) {
      const float* wr = wt + (int64_t)o * cin;
      float s = 0.f;
      for (int i = 0; i < cin; i += 4) {
        const float4 hv = *(const float4*)(hr + i);
        const float4 wv = *(const float4*)(wr + i);
        s = fmaf(fmaxf(hv.x, 0.f), wv.x, s);
        s = fmaf(fmaxf(hv.y, 0.f), wv.y, s);
        s = fmaf(fmaxf(hv.z, 0.f), wv.z, s);
        s = fmaf(fmaxf(hv.w, 0.f), wv.w, s);
      }
      s += b ? b[o] : 0.f;
      if (o < cout - 1) {
        float y = s;
        if (act == 0) y = copysignf(expm1f(fabsf(s)), s);
        else if (act == 1) y = expf(s);
        else if (act == 3) y = fmaxf(s, 0.f);
        preds[p * (cout - 1) + o] = y;
      } else {
        conf[p] = conf_act == 0 ? 1.f + expf(s) : (conf_act == 1 ? expf(s) : 1.f / (1.f + expf(-s)));
      }
    }
  }
}

// ---------------------------------------------------------------- depth unprojection
// world = R^T (cam - t), cam = ((u - cu) d / fu, (v - cv) d / fv, d)
// (depth_to_world_coords_points + closed_form_inverse_se3, geometry.py:53-186)
__global__ void unproject_kernel(const float* __restrict__ depth, const float* __restrict__ extr,
                                 const float* __restrict__ intr, int s, int h, int w, float* __restrict__ out) {
  const int64_t total = (int64_t)s * h * w;
  for (int64_t e = blockIdx.x * (int64_t)TPB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TPB) {
    const int u = (int)(e % w);
    const int v = (int)((e / w) % h);
    const int f = (int)(e / ((int64_t)w * h));
    const float* E = extr + f * 12;
    const float* K = intr + f * 9;
    const float d = depth[e];
    const float xc = ((float)u - K[2]) * d / K[0], yc = ((float)v - K[5]) * d / K[4], zc = d;
    // t_c2w = -R^T t;  world = R^T cam + t_c2w
    const float t0 = -(E[0] * E[3] + E[4] * E[7] + E[8] * E[11]);
    const float t1 = -(E[1] * E[3] + E[5] * E[7] + E[9] * E[11]);
    const float t2 = -(E[2] * E[3] + E[6] * E[7] + E[10] * E[11]);
    out[e * 3 + 0] = xc * E[0] + yc * E[4] + zc * E[8] + t0;
    out[e * 3 + 1] = xc * E[1] + yc * E[5] + zc * E[9] + t1;
    out[e * 3 + 2] = xc * E[2] + yc * E[6] + zc * E[10] + t2;
  }
}

unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>((n + TPB - 1) / TPB, 1 << 20); }

}  // namespace

extern "C" int sr_im2col3x3_f32(sr_stream_t stream, const float* x, int n, int h, int w, int c, int stride,
                                int relu_in, float* out) {
  SR_CHECK(x && out && n > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0 && (stride == 1 || stride == 2), SR_EINVAL,
           "sr_im2col3x3_f32: bad args (c=%d stride=%d)", c, stride);
  const int ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  const int64_t total = (int64_t)n * ho * wo * 9 * (c / 4);
  hipLaunchKernelGGL(im2col3x3_kernel, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream, x, n, h, w, c,
                     stride, relu_in, out, ho, wo);
  return sr::check_launch("sr_im2col3x3_f32");
}

extern "C" int sr_convt_scatter_f32(sr_stream_t stream, const float* g, int n, int h, int w, int k, int co,
                                    const float* bias, float* out) {
  SR_CHECK(g && out && n > 0 && h > 0 && w > 0 && k > 0 && co > 0 && co % 4 == 0, SR_EINVAL,
           "sr_convt_scatter_f32: bad args");
  const int64_t total = (int64_t)n * h * k * w * k * (co / 4);
  hipLaunchKernelGGL(convt_scatter_kernel, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream, g, n, h, w, k,
                     co, bias, out);
  return sr::check_launch("sr_convt_scatter_f32");
}

extern "C" int sr_resize_bilinear_f32(sr_stream_t stream, const float* x, int n, int h, int w, int c, int ho, int wo,
                                      const float* add, float* out) {
  SR_CHECK(x && out && n > 0 && h > 0 && w > 0 && ho > 0 && wo > 0 && c % 4 == 0 && x != out, SR_EINVAL,
           "sr_resize_bilinear_f32: bad args");
  const int64_t total = (int64_t)n * ho * wo * (c / 4);
  hipLaunchKernelGGL(resize_bilinear_kernel, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream, x, n, h, w,
                     c, ho, wo, add, out);
  return sr::check_launch("sr_resize_bilinear_f32");
}

extern "C" int sr_add_f32(sr_stream_t stream, float* dst, const float* src, int64_t n) {
  SR_CHECK(dst && src && n > 0 && n % 4 == 0, SR_EINVAL, "sr_add_f32: bad args");
  hipLaunchKernelGGL(add_kernel, dim3(grid_for(n / 4)), dim3(TPB), 0, (hipStream_t)stream, dst, src, n / 4);
  return sr::check_launch("sr_add_f32");
}

extern "C" int sr_relu_f32(sr_stream_t stream, float* x, int64_t n) {
  SR_CHECK(x && n > 0 && n % 4 == 0, SR_EINVAL, "sr_relu_f32: bad args");
  hipLaunchKernelGGL(relu_kernel, dim3(grid_for(n / 4)), dim3(TPB), 0, (hipStream_t)stream, x, n / 4);
  return sr::check_launch("sr_relu_f32");
}

extern "C" int sr_dpt_pos_embed_f32(sr_stream_t stream, float* x, int n, int h, int w, int c, float aspect,
                                    float ratio) {
  SR_CHECK(x && n > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0, SR_EINVAL, "sr_dpt_pos_embed_f32: bad args");
  const int64_t total = (int64_t)n * h * w * c;
  hipLaunchKernelGGL(dpt_pos_embed_kernel, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream, x, n, h, w, c,
                     aspect, ratio);
  return sr::check_launch("sr_dpt_pos_embed_f32");
}

extern "C" int sr_dpt_head_out_f32(sr_stream_t stream, const float* hidden, int64_t ldh, int64_t npix, int cin,
                                   const float* w, const float* b, int cout, int act, int conf_act, float* preds,
                                   float* conf) {
  SR_CHECK(hidden && w && preds && conf && npix > 0 && cin % 4 == 0 && ldh % 4 == 0 && cout >= 2 && act >= 0 &&
               act <= 3 && conf_act >= 0 && conf_act <= 2,
           SR_EINVAL, "sr_dpt_head_out_f32: bad args");
  hipLaunchKernelGGL(dpt_head_out_kernel, dim3(grid_for(npix)), dim3(TPB), 0, (hipStream_t)stream, hidden, ldh, npix,
                     cin, w, b, cout, act, conf_act, preds, conf);
  return sr::check_launch("sr_dpt_head_out_f32");
}

extern "C" int sr_unproject_depth_f32(sr_stream_t stream, const float* depth, const float* extrinsic,
                                      const float* intrinsic, int s, int h, int w, float* out) {
  SR_CHECK(depth && extrinsic && intrinsic && out && s > 0 && h > 0 && w > 0, SR_EINVAL,
           "sr_unproject_depth_f32: bad args");
  const int64_t total = (int64_t)s * h * w;
  hipLaunchKernelGGL(unproject_kernel, dim3(grid_for(total)), dim3(TPB), 0, (hipStream_t)stream, depth, extrinsic,
                     intrinsic, s, h, w, out);
  return sr::check_launch("sr_unproject_depth_f32");
}
