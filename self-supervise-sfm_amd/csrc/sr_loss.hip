// Self-supervised IMC training loss on gfx950: compute_loss
// (train/train_imc.py:141-246) = pose decode (pose_enc.py:68-135) -> K' -> K recovery (+ shared
// focal averaging) -> relative poses -> backproject / reproject (exact and fixed-depth variants,
// train/utils/geometry.py:89-303) -> log1p residuals -> CDFLossIndexPytorch (per-node weighted
// histograms, CDF, Sobel + Gaussian PDF, lookup; train/losses/cdf_loss.py:88-242), forward value
// AND its gradient with respect to the pose encodings, in one call:
//
//   imc_views_kernel   per view: K (FoV), Kr = K'K, E = [R(q) | T]             (1 workgroup)
//   imc_pairs_kernel   per pair: Ks^-1, Kd, T = Ed Es^-1 (4x4, general inverse)
//   imc_points_kernel  per point: residuals of both variants + histogram atomics (counts are
//                      sums of 1.0: exact, order-independent)
//   imc_cdf_kernel     per (variant, node): pmf, cumsum CDF, reflect-padded Sobel + Gaussian PDF
//   imc_back_kernel    per point: CDF lookup (loss terms) and the chain rule down to per-pair
//                      dKd, dT, dKs^-1, reduced per workgroup into fixed partial slots
//   imc_final_kernel   partials summed in fixed order -> per-pair -> per-view grads -> shared
//                      focal / K' / FoV / quaternion backward -> d enc; the loss value
// Points are float32 like the reference; the 3x3 / 4x4 algebra runs in double.
#include <cmath>

#include "sr_common.h"

namespace {

constexpr int PTB = 256;  // points per workgroup in the per-point kernels
constexpr int NPG = 30;   // per-pair gradient slots: dKd 9 | dT 12 | dKsinv 9
constexpr int VIEW_SLOTS = 21;  // Kr 9 | E 12
constexpr int PAIR_SLOTS = 9 + 9 + 12 + 16 + 16;  // Ksinv | Kd | T (3x4) | Es^-1 (4x4) | Ed (4x4)

struct Ws {  // workspace carve-up (floats unless noted)
  float* views;   // [n_views][21]
  float* pairs;   // [n_pairs][62]
  float* hist;    // [2][n_nodes][bins]
  float* tot;     // [2][n_nodes]
  float* cdf;     // [2][n_nodes][bins]
  float* pdf;     // [2][n_nodes][bins]
  float* part;    // [n_pairs][chunks][NPG + 1]  (+1: loss partial)
};

__host__ __device__ inline int64_t ws_floats(int nv, int np, int nn, int bins, int chunks) {
  return (int64_t)nv * VIEW_SLOTS + (int64_t)np * PAIR_SLOTS + 2ll * nn * bins + 2ll * nn + 4ll * nn * bins +
         (int64_t)np * chunks * (NPG + 1);
}

__device__ inline Ws carve(float* w, int nv, int np, int nn, int bins) {
  Ws s;
  s.views = w;
  s.pairs = s.views + (int64_t)nv * VIEW_SLOTS;
  s.hist = s.pairs + (int64_t)np * PAIR_SLOTS;
  s.tot = s.hist + 2ll * nn * bins;
  s.cdf = s.tot + 2ll * nn;
  s.pdf = s.cdf + 2ll * nn * bins;
  s.part = s.pdf + 2ll * nn * bins;
  return s;
}

// ---------------------------------------------------------------- small dense algebra (double)
__device__ inline void mat3_inv(const double* a, double* o) {
  const double c00 = a[4] * a[8] - a[5] * a[7], c01 = a[5] * a[6] - a[3] * a[8], c02 = a[3] * a[7] - a[4] * a[6];
  const double det = a[0] * c00 + a[1] * c01 + a[2] * c02;
  const double id = 1.0 / det;
  o[0] = c00 * id;
  o[1] = (a[2] * a[7] - a[1] * a[8]) * id;
  o[2] = (a[1] * a[5] - a[2] * a[4]) * id;
  o[3] = c01 * id;
  o[4] = (a[0] * a[8] - a[2] * a[6]) * id;
  o[5] = (a[2] * a[3] - a[0] * a[5]) * id;
  o[6] = c02 * id;
  o[7] = (a[1] * a[6] - a[0] * a[7]) * id;
  o[8] = (a[0] * a[4] - a[1] * a[3]) * id;
}

// general 4x4 inverse, Gauss-Jordan with partial pivoting (torch.inverse on [R|t;0 0 0 1])
__device__ inline void mat4_inv(const double* a, double* o) {
  double m[4][8];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      m[i][j] = a[i * 4 + j];
      m[i][4 + j] = i == j ? 1.0 : 0.0;
    }
  for (int c = 0; c < 4; ++c) {
    int p = c;
    for (int r = c + 1; r < 4; ++r)
      if (fabs(m[r][c]) > fabs(m[p][c])) p = r;
    if (p != c)
      for (int j = 0; j < 8; ++j) {
        const double t = m[c][j];
        m[c][j] = m[p][j];
        m[p][j] = t;
      }
    const double iv = 1.0 / m[c][c];
    for (int j = 0; j < 8; ++j) m[c][j] *= iv;
    for (int r = 0; r < 4; ++r)
      if (r != c) {
        const double f = m[r][c];
        for (int j = 0; j < 8; ++j) m[r][j] -= f * m[c][j];
      }
  }
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) o[i * 4 + j] = m[i][4 + j];
}

// ---------------------------------------------------------------- views
__global__ void imc_views_kernel(sr_imc_loss_desc d, float* wsp) {
  const Ws w = carve(wsp, d.n_views, d.n_pairs, d.n_nodes, d.num_bins);
  __shared__ double kr[64][9];
  const int n = d.n_views;
  for (int v = threadIdx.x; v < n; v += blockDim.x) {
    const float* e = d.enc + v * 9;
    // K (pose_enc.py:116-130): fy = (H/2)/tan(fov_h/2), fx = (W/2)/tan(fov_w/2), pp = (W/2, H/2)
    const float fy = (d.H / 2.0f) / tanf(e[7] / 2.0f), fx = (d.W / 2.0f) / tanf(e[8] / 2.0f);
    const double K[9] = {fx, 0, d.W / 2.0, 0, fy, d.H / 2.0, 0, 0, 1};
    const float* kp = d.kp2k + v * 9;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double s = 0;
        for (int t = 0; t < 3; ++t) s += (double)kp[i * 3 + t] * K[t * 3 + j];
        if (v < 64) kr[v][i * 3 + j] = s;
        w.views[v * VIEW_SLOTS + i * 3 + j] = (float)s;
      }
    // E = [quat_to_mat(q) | T] (rotation.py:14-44, xyzw)
    const float i_ = e[3], j_ = e[4], k_ = e[5], r_ = e[6];
    const float s2 = 2.0f / (i_ * i_ + j_ * j_ + k_ * k_ + r_ * r_);
    const float R[9] = {1 - s2 * (j_ * j_ + k_ * k_), s2 * (i_ * j_ - k_ * r_), s2 * (i_ * k_ + j_ * r_),
                        s2 * (i_ * j_ + k_ * r_), 1 - s2 * (i_ * i_ + k_ * k_), s2 * (j_ * k_ - i_ * r_),
                        s2 * (i_ * k_ - j_ * r_), s2 * (j_ * k_ + i_ * r_), 1 - s2 * (i_ * i_ + j_ * j_)};
    float* E = w.views + v * VIEW_SLOTS + 9;
    for (int i = 0; i < 3; ++i) {
      E[i * 4 + 0] = R[i * 3 + 0];
      E[i * 4 + 1] = R[i * 3 + 1];
      E[i * 4 + 2] = R[i * 3 + 2];
      E[i * 4 + 3] = e[i];
    }
  }
  __syncthreads();
  if (d.shared_focal && threadIdx.x == 0) {  // Kr_i = mean_j Kr_j (train_imc.py:169-174)
    for (int t = 0; t < 9; ++t) {
      double s = 0;
      for (int v = 0; v < n; ++v) s += (float)kr[v][t];
      const float m = (float)(s / n);
      for (int v = 0; v < n; ++v) w.views[v * VIEW_SLOTS + t] = m;
    }
  }
}

// ---------------------------------------------------------------- pairs
__global__ void imc_pairs_kernel(sr_imc_loss_desc d, float* wsp) {
  const Ws w = carve(wsp, d.n_views, d.n_pairs, d.n_nodes, d.num_bins);
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= d.n_pairs) return;
  const float* vs = w.views + d.src_idx[p] * VIEW_SLOTS;
  const float* vd = w.views + d.dst_idx[p] * VIEW_SLOTS;
  double Ks[9], Ksi[9], Es[16], Esi[16], Ed[16];
  for (int t = 0; t < 9; ++t) Ks[t] = vs[t];
  mat3_inv(Ks, Ksi);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      Es[i * 4 + j] = i < 3 ? vs[9 + i * 4 + j] : (j == 3 ? 1.0 : 0.0);
      Ed[i * 4 + j] = i < 3 ? vd[9 + i * 4 + j] : (j == 3 ? 1.0 : 0.0);
    }
  mat4_inv(Es, Esi);
  float* o = w.pairs + (int64_t)p * PAIR_SLOTS;
  for (int t = 0; t < 9; ++t) {
    o[t] = (float)Ksi[t];
    o[9 + t] = vd[t];
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = 0;
      for (int t = 0; t < 4; ++t) s += Ed[i * 4 + t] * Esi[t * 4 + j];
      o[18 + i * 4 + j] = (float)s;
    }
  for (int t = 0; t < 16; ++t) {
    o[30 + t] = (float)Esi[t];
    o[46 + t] = (float)Ed[t];
  }
}

// forward geometry of one point: returns X (3), Y (3), p (3) and both predictions
struct PointGeo {
  float X[3], Y[3], p[3], pred[2][2], r[2];
};

__device__ inline PointGeo point_geo(const sr_imc_loss_desc& d, const float* pr, int p, int k) {
  PointGeo g;
  const int64_t e = (int64_t)p * d.n_points + k;
  const float u = d.src_coords[2 * e], v = d.src_coords[2 * e + 1];
  const float ds = d.src_depth[e], dd = d.dst_depth[e];
  const float* Ksi = pr;
  const float* Kd = pr + 9;
  const float* T = pr + 18;
  for (int i = 0; i < 3; ++i) g.X[i] = (Ksi[i * 3] * u + Ksi[i * 3 + 1] * v + Ksi[i * 3 + 2]) * ds;
  for (int i = 0; i < 3; ++i) g.Y[i] = T[i * 4] * g.X[0] + T[i * 4 + 1] * g.X[1] + T[i * 4 + 2] * g.X[2] + T[i * 4 + 3];
  for (int i = 0; i < 3; ++i) g.p[i] = Kd[i * 3] * g.Y[0] + Kd[i * 3 + 1] * g.Y[1] + Kd[i * 3 + 2] * g.Y[2];
  const float ox = d.dst_coords[2 * e], oy = d.dst_coords[2 * e + 1];
  const float den[2] = {g.p[2] + 1e-6f, dd + 1e-6f};  // from_homogeneous / fixed-depth variant
  for (int vv = 0; vv < 2; ++vv) {
    g.pred[vv][0] = g.p[0] / den[vv];
    g.pred[vv][1] = g.p[1] / den[vv];
    const float a = g.pred[vv][0] - ox, b = g.pred[vv][1] - oy;
    g.r[vv] = sqrtf(a * a + b * b);
  }
  return g;
}

// ---------------------------------------------------------------- residuals + histograms
__global__ __launch_bounds__(PTB) void imc_points_kernel(sr_imc_loss_desc d, float* wsp) {
  const Ws w = carve(wsp, d.n_views, d.n_pairs, d.n_nodes, d.num_bins);
  const int p = blockIdx.y, k = blockIdx.x * PTB + threadIdx.x;
  if (k >= d.n_points) return;
  const PointGeo g = point_geo(d, w.pairs + (int64_t)p * PAIR_SLOTS, p, k);
  const float bw = (d.max_val - d.min_val) / d.num_bins;
  const int ns = d.node_src[p], nd = d.node_dst[p];
  for (int vv = 0; vv < 2; ++vv) {
    const float rl = log1pf(g.r[vv]);
    const long b = (long)((rl - d.min_val) / bw);  // .long(): truncation (cdf_loss.py:137)
    float* h = w.hist + (int64_t)vv * d.n_nodes * d.num_bins;
    if (b >= 0 && b < d.num_bins) {  // weights are the all-ones validity masks
      atomicAdd(h + (int64_t)ns * d.num_bins + b, 1.0f);
      atomicAdd(h + (int64_t)nd * d.num_bins + b, 1.0f);
    }
    atomicAdd(w.tot + vv * d.n_nodes + ns, 1.0f);
    atomicAdd(w.tot + vv * d.n_nodes + nd, 1.0f);
  }
}

// ---------------------------------------------------------------- per-node CDF / PDF
__global__ void imc_cdf_kernel(sr_imc_loss_desc d, float* wsp) {
  const Ws w = carve(wsp, d.n_views, d.n_pairs, d.n_nodes, d.num_bins);
  const int vv = blockIdx.y, node = blockIdx.x, nb = d.num_bins;
  const int64_t o = ((int64_t)vv * d.n_nodes + node) * nb;
  float* cdf = w.cdf + o;
  float* pdf = w.pdf + o;
  __shared__ float raw[1024];
  if (threadIdx.x == 0) {  // pmf = hist / (total + 1e-10); cumsum in bin order (cdf_loss.py:177-178)
    const float t = w.tot[vv * d.n_nodes + node] + 1e-10f;
    float s = 0.f;
    for (int i = 0; i < nb; ++i) {
      s += w.hist[o + i] / t;
      cdf[i] = s;
    }
  }
  __syncthreads();
  const float bw = (d.max_val - d.min_val) / nb;
  auto refl = [nb](int i) { return i < 0 ? -i : (i >= nb ? 2 * (nb - 1) - i : i); };
  for (int i = threadIdx.x; i < nb; i += blockDim.x)  // Sobel [-1, 0, 1] / (2 bw), reflect padding
    raw[i] = (-cdf[refl(i - 1)] + cdf[refl(i + 1)]) / (2.0f * bw);
  __syncthreads();
  const int R = d.smooth_radius;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    float s = 0.f;
    for (int t = -R; t <= R; ++t) s += d.smooth_w[t + R] * raw[refl(i + t)];
    pdf[i] = s;
  }
}

// ---------------------------------------------------------------- lookup + chain rule per point
__global__ __launch_bounds__(PTB) void imc_back_kernel(sr_imc_loss_desc d, float* wsp, int chunks) {
  const Ws w = carve(wsp, d.n_views, d.n_pairs, d.n_nodes, d.num_bins);
  __shared__ float red[PTB / 64][NPG + 1];
  const int p = blockIdx.y, k = blockIdx.x * PTB + threadIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc[NPG + 1];
#pragma unroll
  for (int t = 0; t <= NPG; ++t) acc[t] = 0.f;
  if (k < d.n_points) {
    const float* pr = w.pairs + (int64_t)p * PAIR_SLOTS;
    const PointGeo g = point_geo(d, pr, p, k);
    const int64_t e = (int64_t)p * d.n_points + k;
    const float ox = d.dst_coords[2 * e], oy = d.dst_coords[2 * e + 1];
    const float u = d.src_coords[2 * e], v = d.src_coords[2 * e + 1];
    const float ds = d.src_depth[e], dd = d.dst_depth[e];
    const float bw = (d.max_val - d.min_val) / d.num_bins;
    const int ns = d.node_src[p], nd = d.node_dst[p];
    const float inv4 = d.grad_scale / (4.0f * (float)d.n_pairs * (float)d.n_points);
    float gp[3] = {0.f, 0.f, 0.f};
    for (int vv = 0; vv < 2; ++vv) {
      const float rl = log1pf(g.r[vv]);
      const long b = (long)((rl - d.min_val) / bw + 0.5f);  // lookup bin (cdf_loss.py:207-210)
      const bool ok = b >= 0 && b < d.num_bins;
      const int64_t base = (int64_t)vv * d.n_nodes * d.num_bins;
      const float cs = ok ? w.cdf[base + (int64_t)ns * d.num_bins + b] : 2.0f;
      const float cd = ok ? w.cdf[base + (int64_t)nd * d.num_bins + b] : 2.0f;
      acc[NPG] += cs + cd;  // loss = sum over both variants / (4 P K)
      const float grl = ok ? (w.pdf[base + (int64_t)ns * d.num_bins + b] + w.pdf[base + (int64_t)nd * d.num_bins + b]) *
                                 inv4
                           : 0.f;
      const float gr = grl / (1.f + g.r[vv]);
      if (g.r[vv] > 0.f && gr != 0.f) {
        const float gx = gr * (g.pred[vv][0] - ox) / g.r[vv], gy = gr * (g.pred[vv][1] - oy) / g.r[vv];
        const float den = vv == 0 ? g.p[2] + 1e-6f : dd + 1e-6f;
        gp[0] += gx / den;
        gp[1] += gy / den;
        if (vv == 0) gp[2] -= (gx * g.p[0] + gy * g.p[1]) / (den * den);
      }
    }
    const float* Ksi = pr;
    const float* Kd = pr + 9;
    const float* T = pr + 18;
    float gY[3], gX[3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) acc[i * 3 + j] += gp[i] * g.Y[j];  // dKd
    for (int j = 0; j < 3; ++j) gY[j] = Kd[j] * gp[0] + Kd[3 + j] * gp[1] + Kd[6 + j] * gp[2];
    for (int i = 0; i < 3; ++i) {  // dT
      for (int j = 0; j < 3; ++j) acc[9 + i * 4 + j] += gY[i] * g.X[j];
      acc[9 + i * 4 + 3] += gY[i];
    }
    for (int j = 0; j < 3; ++j) gX[j] = T[j] * gY[0] + T[4 + j] * gY[1] + T[8 + j] * gY[2];
    const float h[3] = {u * ds, v * ds, ds};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) acc[21 + i * 3 + j] += gX[i] * h[j];  // dKs^-1
    (void)Ksi;
  }
#pragma unroll
  for (int t = 0; t <= NPG; ++t) {
    const float s = sr::wave_sum(acc[t]);
    if (lane == 0) red[wave][t] = s;
  }
  __syncthreads();
  if (threadIdx.x <= NPG) {
    float s = 0.f;
    for (int q = 0; q < PTB / 64; ++q) s += red[q][threadIdx.x];
    w.part[((int64_t)p * chunks + blockIdx.x) * (NPG + 1) + threadIdx.x] = s;
  }
}

// ---------------------------------------------------------------- per-pair -> per-view -> d enc
__global__ void imc_final_kernel(sr_imc_loss_desc d, float* wsp, int chunks) {
  const Ws w = carve(wsp, d.n_views, d.n_pairs, d.n_nodes, d.num_bins);
  if (threadIdx.x != 0) return;
  const int nv = d.n_views;
  double gKr[64][9], gE[64][12];
  for (int v = 0; v < nv; ++v) {
    for (int t = 0; t < 9; ++t) gKr[v][t] = 0;
    for (int t = 0; t < 12; ++t) gE[v][t] = 0;
  }
  double loss = 0;
  for (int p = 0; p < d.n_pairs; ++p) {
    double g[NPG + 1];
    for (int t = 0; t <= NPG; ++t) g[t] = 0;
    for (int c = 0; c < chunks; ++c)
      for (int t = 0; t <= NPG; ++t) g[t] += w.part[((int64_t)p * chunks + c) * (NPG + 1) + t];
    loss += g[NPG];
    const float* pr = w.pairs + (int64_t)p * PAIR_SLOTS;
    const int s = d.src_idx[p], dv = d.dst_idx[p];
    // dKs = -Ks^-T dKsinv Ks^-T
    double Ksi[9], tmp[9];
    for (int t = 0; t < 9; ++t) Ksi[t] = pr[t];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double a = 0;
        for (int t = 0; t < 3; ++t) a += Ksi[t * 3 + i] * g[21 + t * 3 + j];  // Ksi^T dKsinv
        tmp[i * 3 + j] = a;
      }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double a = 0;
        for (int t = 0; t < 3; ++t) a += tmp[i * 3 + t] * Ksi[j * 3 + t];  // (.) Ksi^T
        gKr[s][i * 3 + j] -= a;
      }
    for (int t = 0; t < 9; ++t) gKr[dv][t] += g[t];
    // T = Ed Es^-1:  dEd = dT Es^-T;  dEs^-1 = Ed^T dT;  dEs = -Es^-T dEs^-1 Es^-T  (4x4, dT row 3 = 0)
    double dT[16], Esi[16], Ed[16], dEsi[16], t2[16];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) dT[i * 4 + j] = i < 3 ? g[9 + i * 4 + j] : 0.0;
    for (int t = 0; t < 16; ++t) {
      Esi[t] = pr[30 + t];
      Ed[t] = pr[46 + t];
    }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 4; ++j) {
        double a = 0;
        for (int t = 0; t < 4; ++t) a += dT[i * 4 + t] * Esi[j * 4 + t];
        gE[dv][i * 4 + j] += a;
      }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        double a = 0;
        for (int t = 0; t < 4; ++t) a += Ed[t * 4 + i] * dT[t * 4 + j];
        dEsi[i * 4 + j] = a;
      }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        double a = 0;
        for (int t = 0; t < 4; ++t) a += Esi[t * 4 + i] * dEsi[t * 4 + j];
        t2[i * 4 + j] = a;
      }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 4; ++j) {
        double a = 0;
        for (int t = 0; t < 4; ++t) a += t2[i * 4 + t] * Esi[j * 4 + t];
        gE[s][i * 4 + j] -= a;
      }
  }
  if (d.loss) d.loss[0] = (float)(loss / (4.0 * (double)d.n_pairs * (double)d.n_points));
  if (d.shared_focal) {  // every Kr_i is the mean of all: dKr'_j = (1/N) sum_i dKr_i
    for (int t = 0; t < 9; ++t) {
      double s = 0;
      for (int v = 0; v < nv; ++v) s += gKr[v][t];
      for (int v = 0; v < nv; ++v) gKr[v][t] = s / nv;
    }
  }
  for (int v = 0; v < nv; ++v) {
    const float* e = d.enc + v * 9;
    const float* kp = d.kp2k + v * 9;
    double gK[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double a = 0;
        for (int t = 0; t < 3; ++t) a += (double)kp[t * 3 + i] * gKr[v][t * 3 + j];  // K'^T dKr
        gK[i * 3 + j] = a;
      }
    float* o = d.d_enc + v * 9;
    // f = (S/2) / tan(fov/2):  df/dfov = -(S/4) / sin^2(fov/2)
    const double sh = sin(e[7] / 2.0), sw = sin(e[8] / 2.0);
    o[7] = (float)(gK[4] * (-(d.H / 4.0) / (sh * sh)));
    o[8] = (float)(gK[0] * (-(d.W / 4.0) / (sw * sw)));
    for (int i = 0; i < 3; ++i) o[i] = (float)gE[v][i * 4 + 3];
    // quat_to_mat backward: R = I + s A(q), s = 2 / |q|^2
    const double qi = e[3], qj = e[4], qk = e[5], qr = e[6];
    const double nq = qi * qi + qj * qj + qk * qk + qr * qr, s2 = 2.0 / nq;
    double gR[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) gR[i * 3 + j] = gE[v][i * 4 + j];
    const double A[9] = {-(qj * qj + qk * qk), qi * qj - qk * qr, qi * qk + qj * qr, qi * qj + qk * qr,
                         -(qi * qi + qk * qk), qj * qk - qi * qr, qi * qk - qj * qr, qj * qk + qi * qr,
                         -(qi * qi + qj * qj)};
    const double dAi[9] = {0, qj, qk, qj, -2 * qi, -qr, qk, qr, -2 * qi};
    const double dAj[9] = {-2 * qj, qi, qr, qi, 0, qk, -qr, qk, -2 * qj};
    const double dAk[9] = {-2 * qk, -qr, qi, qr, -2 * qk, qj, qi, qj, 0};
    const double dAr[9] = {0, -qk, qj, qk, 0, -qi, -qj, qi, 0};
    double gA = 0, gi = 0, gj = 0, gk = 0, gr = 0;
    for (int t = 0; t < 9; ++t) {
      gA += gR[t] * A[t];
      gi += gR[t] * dAi[t];
      gj += gR[t] * dAj[t];
      gk += gR[t] * dAk[t];
      gr += gR[t] * dAr[t];
    }
    const double ds_coef = -s2 * 2.0 / nq * gA;  // d s / d q = -s * 2 q / |q|^2
    o[3] = (float)(s2 * gi + ds_coef * qi);
    o[4] = (float)(s2 * gj + ds_coef * qj);
    o[5] = (float)(s2 * gk + ds_coef * qk);
    o[6] = (float)(s2 * gr + ds_coef * qr);
  }
}

}  // namespace

extern "C" int64_t sr_imc_loss_workspace(int n_views, int n_pairs, int n_points, int n_nodes, int num_bins) {
  const int chunks = (n_points + PTB - 1) / PTB;
  return ws_floats(n_views, n_pairs, n_nodes, num_bins, chunks);
}

extern "C" int sr_imc_loss(sr_stream_t stream, const sr_imc_loss_desc* desc) {
  SR_CHECK(desc, SR_EINVAL, "sr_imc_loss: null desc");
  const sr_imc_loss_desc& d = *desc;
  SR_CHECK(d.enc && d.kp2k && d.src_idx && d.dst_idx && d.src_coords && d.dst_coords && d.src_depth && d.dst_depth &&
               d.node_src && d.node_dst && d.d_enc && d.workspace && d.smooth_w,
           SR_EINVAL, "sr_imc_loss: null pointer");
  SR_CHECK(d.n_views > 0 && d.n_views <= 64 && d.n_pairs > 0 && d.n_points > 0 && d.n_nodes > 0 &&
               d.num_bins > 2 && d.num_bins <= 1024 && d.smooth_radius >= 0 && 2 * d.smooth_radius + 1 <= d.num_bins &&
               d.max_val > d.min_val && d.H > 0 && d.W > 0,
           SR_EUNSUPPORTED, "sr_imc_loss: bad sizes (views <= 64, bins <= 1024)");
  hipStream_t s = (hipStream_t)stream;
  const int chunks = (d.n_points + PTB - 1) / PTB;
  float* w = d.workspace;
  const int64_t nn = d.n_nodes, nb = d.num_bins;
  // histograms / totals start at zero (one memset of their contiguous range)
  const int64_t hist_off = (int64_t)d.n_views * VIEW_SLOTS + (int64_t)d.n_pairs * PAIR_SLOTS;
  SR_CHECK(hipMemsetAsync(w + hist_off, 0, (2 * nn * nb + 2 * nn) * sizeof(float), s) == hipSuccess, SR_ELAUNCH,
           "sr_imc_loss: memset");
  hipLaunchKernelGGL(imc_views_kernel, dim3(1), dim3(64), 0, s, d, w);
  hipLaunchKernelGGL(imc_pairs_kernel, dim3((d.n_pairs + 63) / 64), dim3(64), 0, s, d, w);
  hipLaunchKernelGGL(imc_points_kernel, dim3(chunks, d.n_pairs), dim3(PTB), 0, s, d, w);
  hipLaunchKernelGGL(imc_cdf_kernel, dim3(d.n_nodes, 2), dim3(256), 0, s, d, w);
  hipLaunchKernelGGL(imc_back_kernel, dim3(chunks, d.n_pairs), dim3(PTB), 0, s, d, w, chunks);
  hipLaunchKernelGGL(imc_final_kernel, dim3(1), dim3(64), 0, s, d, w, chunks);
  return sr::check_launch("sr_imc_loss");
}
