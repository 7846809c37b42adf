// Attention backward for gfx950 (training step): the gradient of
// F.scaled_dot_product_attention in Attention.forward (attention.py:103-109) for the forward's
// key segments (frame / global / global_reloc), bf16 operands, fp32 accumulation, head_dim 64.
//
//   delta = rowsum(dO * O)                                  (attn_bwd_delta_kernel)
//   P = exp2(c q.k - lse)   c = scale * log2(e), lse from the forward (log2 domain)
//   dS = P * (dO.v - delta)
//   dK = scale dS^T Q,  dV = P^T dO                          (attn_bwd_dkdv_kernel: one workgroup per
//                                                            128 keys, sweeping every query that sees them)
//   dQ = scale dS K                                          (attn_bwd_dq_kernel: one workgroup per
//                                                            128 query rows, sweeping their keys)
// Both sweeps recompute P (no atomics: dQ by atomics would move ~(L/64)^2 x 16 KB per head).
//
// MFMA layout (v_mfma_f32_32x32x16_bf16; lane = l32 + 32 hi): A rows / B columns come from row
// reads of a row-major tile (16 B at d = 16 s + 8 hi), the transposed operands (dO^T, Q^T, K^T)
// from ds_read_b64_tr_b16 reads exactly as the forward reads V^T, and the P / dS operands straight
// from the accumulators: a 32x32 accumulator holds in lane (l32, hi) the column l32 and rows
// (r & 3) + 8 (r >> 2) + 4 hi, r = 0..15, which is the k order the tr-reads produce.
// Tiles are 64 rows x 128 B (swizzle: see swz below).
#include <cfloat>
#include <type_traits>

#include "sr_common.h"

namespace {

constexpr int TB = 64 * 128;  // one 64-row tile, bytes

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Tiles are read both as rows (ds_read_b128 for S / dP: 16 lanes = 16 rows, one chunk) and
// transposed (ds_read_b64_tr_b16 for dV / dK / dQ: 4 rows x 4 chunks per 32 lanes).  16-B chunk c
// of row r sits at c ^ f((r >> 1) & 7) with f(g) = b0 b1 b2 reversed: bijective on g (the 8 rows of
// one parity in a b128 lane group hit 8 distinct chunks) and rows r, r + 2 of a transposed read
// land in opposite 4-chunk halves — bank-conflict free for both (the forward's
// c ^ ((r >> 1) & 1) << 2 only serves the transposed reads: 4-way conflicts on the row reads).
__device__ __forceinline__ int swz(int r, int chunk) {
  const int g = (r >> 1) & 7;
  return chunk ^ (((g & 1) << 2) | (g & 2) | (g >> 2));
}

// 64 rows x 64 bf16 tiles staged through registers (256 threads: 2 x 16 B each per tile): the
// next tile's global loads are issued before the current tile's MFMAs and written to the other
// LDS buffer after them, so one barrier per tile separates the two (rows >= nrows clamped).
struct TileRegs {  // named members (an array member here was demoted to scratch)
  uint4 a, b;
};
__device__ __forceinline__ TileRegs fetch_tile(const bf16* base, int64_t ld, int row0, int nrows, int tid) {
  const int r = tid >> 3, c = tid & 7;  // rows r and r + 32
  TileRegs t;
  t.a = *(const uint4*)(base + (int64_t)min(row0 + r, nrows - 1) * ld + c * 8);
  t.b = *(const uint4*)(base + (int64_t)min(row0 + r + 32, nrows - 1) * ld + c * 8);
  return t;
}
__device__ __forceinline__ void store_tile(char* lds, const TileRegs& t, int tid) {
  const int r = tid >> 3, c = tid & 7;
  *(uint4*)(lds + r * 128 + swz(r, c) * 16) = t.a;
  *(uint4*)(lds + (r + 32) * 128 + swz(r + 32, c) * 16) = t.b;
}

// A/B fragment from a row read: row r, k-step s (d = 16 s + 8 hi)
__device__ __forceinline__ bf16x8 row_frag(const char* tile, int r, int s, int hi) {
  return *(const bf16x8*)(tile + r * 128 + swz(r, 2 * s + hi) * 16);
}

struct TrOff {
  int off[2][2];  // [column block db = 0 / 1][rows +0 / +8]
};
__device__ __forceinline__ TrOff tr_offsets(int lane) {
  const int hi = lane >> 5, G = lane >> 4, gi = lane & 15;
  const int vrow_in = gi >> 2;
  const int vcol_in = 16 * (G & 1) + 4 * (gi & 3);
  TrOff t;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 8 * h + 4 * hi + vrow_in;  // row0 is a multiple of 16: the swizzle repeats
      t.off[db][h] = r * 128 + swz(r, 4 * db + (vcol_in >> 3)) * 16 + (vcol_in & 7) * 2;
    }
  return t;
}
// transposed operand: m = tile column (db block), k = tile rows row0 + {(r & 3) + 8 (r >> 2) + 4 hi}
__device__ __forceinline__ bf16x8 tr_frag(const char* tile, int row0, const int (&off)[2]) {
  const char* pt = tile + row0 * 128;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)(pt + off[0]));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)(pt + off[1]));
  const bf16x4 a4 = __builtin_bit_cast(bf16x4, a), b4 = __builtin_bit_cast(bf16x4, b);
  return bf16x8{a4[0], a4[1], a4[2], a4[3], b4[0], b4[1], b4[2], b4[3]};
}

__device__ __forceinline__ int acc_row(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

// ---------------------------------------------------------------- delta = rowsum(dO * O)
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(sr_attn_bwd_desc b) {
  const sr_attn_desc& f = b.f;
  const int64_t n = (int64_t)f.batch * f.heads * f.lq;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int row = (int)(e % f.lq);
    const int64_t ih = e / f.lq;
    const int head = (int)(ih % f.heads), item = (int)(ih / f.heads);
    const int64_t r = (int64_t)item * f.q_bstride + row;
    const bf16* o = (const bf16*)f.o + r * f.ldo + head * 64;
    const bf16* g = (const bf16*)b.dout + r * b.lddo + head * 64;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const bf16x8 ov = *(const bf16x8*)(o + 8 * c), gv = *(const bf16x8*)(g + 8 * c);
#pragma unroll
      for (int j = 0; j < 8; ++j) s = fmaf((float)ov[j], (float)gv[j], s);
    }
    b.delta[e] = s;
  }
}

// ---------------------------------------------------------------- dK, dV
// grid (key tiles of 128, heads, SHARED ? 1 : batch); wave w owns keys tile*128 + 32 w + l32.
template <int SEG>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_kernel(sr_attn_bwd_desc b) {
  constexpr int STG = 2 * TB + 2 * 64 * 4;  // one stage: Q tile | dO tile | lse | delta
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];
  const sr_attn_desc& f = b.f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int head = blockIdx.y, hcol = head * 64;
  const bool shared = (SEG == 0 ? f.k0_bstride : f.k1_bstride) == 0;
  const int it0 = shared ? 0 : blockIdx.z, it1 = shared ? f.batch : blockIdx.z + 1;
  const int len = SEG == 0 ? f.l0 : f.l1;
  const int64_t kb0 = (int64_t)(shared ? 0 : blockIdx.z) * (SEG == 0 ? f.k0_bstride : f.k1_bstride);
  const bf16* kp = (const bf16*)(SEG == 0 ? f.k0 : f.k1);
  const bf16* vp = (const bf16*)(SEG == 0 ? f.v0 : f.v1);
  const int64_t ldk = SEG == 0 ? f.ldk0 : f.ldk1, ldv = SEG == 0 ? f.ldv0 : f.ldv1;
  const int key = blockIdx.x * 128 + wave * 32 + l32;
  const int keyc = min(key, len - 1);
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *(const bf16x8*)(kp + (kb0 + keyc) * ldk + hcol + 16 * s + 8 * hi);
    vf[s] = *(const bf16x8*)(vp + (kb0 + keyc) * ldv + hcol + 16 * s + 8 * hi);
  }
  const float c = f.scale * 1.4426950408889634f;
  const TrOff tro = tr_offsets(lane);
  f32x16 dk[2], dv[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) dk[0][i] = dk[1][i] = dv[0][i] = dv[1][i] = 0.f;

  // tiles t = (item - it0) * ntq + q-tile, staged through registers one tile ahead
  const int ntq = (f.lq + 63) / 64, ntiles = (it1 - it0) * ntq;
  TileRegs rq, ro;
  float rl = 0.f, rd = 0.f;
  auto fetch = [&](int t) {
    const int item = it0 + t / ntq, q0 = (t % ntq) * 64;
    rq = fetch_tile((const bf16*)f.q + (int64_t)item * f.q_bstride * f.ldq + hcol, f.ldq, q0, f.lq, tid);
    ro = fetch_tile((const bf16*)b.dout + (int64_t)item * f.q_bstride * b.lddo + hcol, b.lddo, q0, f.lq, tid);
    if (tid < 64) {
      const bool ok = q0 + tid < f.lq;
      const int64_t o = ((int64_t)item * f.heads + head) * f.lq + q0 + tid;
      rl = ok ? f.lse[o] : INFINITY;  // padded rows: P = 0
      rd = ok ? b.delta[o] : 0.f;
    }
  };
  fetch(0);
  for (int t = 0; t < ntiles; ++t) {
    {
      char* stg = smem + (t & 1) * STG;
      char* qt = stg;
      char* ot = stg + TB;
      float* lse_s = (float*)(stg + 2 * TB);
      float* dl_s = lse_s + 64;
      store_tile(qt, rq, tid);
      store_tile(ot, ro, tid);
      if (tid < 64) {
        lse_s[tid] = rl;
        dl_s[tid] = rd;
      }
      __syncthreads();  // this stage written; every wave is past the previous use of this buffer
      if (t + 1 < ntiles) fetch(t + 1);
      // S = Q K^T and dP = dO V^T for this wave's 32 keys (2 blocks of 32 query rows)
      f32x16 sc[2], dp[2];
      const f32x16 zero = {};
      sc[0] = sc[1] = dp[0] = dp[1] = zero;
#pragma unroll
      for (int s = 0; s < 4; ++s)  // four independent accumulation chains in flight
#pragma unroll
        for (int qb2 = 0; qb2 < 2; ++qb2) {
          sc[qb2] = mfma32(row_frag(qt, qb2 * 32 + l32, s, hi), kf[s], sc[qb2]);
          dp[qb2] = mfma32(row_frag(ot, qb2 * 32 + l32, s, hi), vf[s], dp[qb2]);
        }
      // P, dS (lane: key column l32, query rows qb2*32 + acc_row(r)); dV^T += dO^T P, dK^T += Q^T dS
#pragma unroll
      for (int qb2 = 0; qb2 < 2; ++qb2)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 pf, df;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int r = 8 * s2 + j;
            const int q = qb2 * 32 + acc_row(r, hi);
            const float p = __builtin_amdgcn_exp2f(sc[qb2][r] * c - lse_s[q]);
            pf[j] = (bf16)p;
            df[j] = (bf16)(p * (dp[qb2][r] - dl_s[q]));
          }
          const int row0 = qb2 * 32 + 16 * s2;
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            dv[db] = mfma32(tr_frag(ot, row0, tro.off[db]), pf, dv[db]);
            dk[db] = mfma32(tr_frag(qt, row0, tro.off[db]), df, dk[db]);
          }
        }
    }
  }
  // dK[key][d] = scale * dK^T[d][key], dV likewise (lane: key l32, d = 32 db + acc_row(r))
  if (key < len) {
    float* dkp = (SEG == 0 ? b.dk0 : b.dk1) + (kb0 + key) * (SEG == 0 ? b.lddk0 : b.lddk1) + hcol;
    float* dvp = (SEG == 0 ? b.dv0 : b.dv1) + (kb0 + key) * (SEG == 0 ? b.lddv0 : b.lddv1) + hcol;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = db * 32 + 8 * g + 4 * hi;
        *(float4*)(dkp + d0) = make_float4(dk[db][4 * g] * f.scale, dk[db][4 * g + 1] * f.scale,
                                           dk[db][4 * g + 2] * f.scale, dk[db][4 * g + 3] * f.scale);
        *(float4*)(dvp + d0) = make_float4(dv[db][4 * g], dv[db][4 * g + 1], dv[db][4 * g + 2], dv[db][4 * g + 3]);
      }
  }
}

// ---------------------------------------------------------------- dQ
// grid (query tiles of 128, heads, batch); wave w owns query rows tile*128 + 32 w + l32.
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(sr_attn_bwd_desc b) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TB];  // 2 stages of K tile | V tile
  const sr_attn_desc& f = b.f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int head = blockIdx.y, hcol = head * 64, item = blockIdx.z;
  const int qrow = blockIdx.x * 128 + wave * 32 + l32;
  const int qrc = min(qrow, f.lq - 1);
  const int64_t qr = (int64_t)item * f.q_bstride + qrc;
  const float c = f.scale * 1.4426950408889634f;
  bf16x8 qf[4], of[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = *(const bf16x8*)((const bf16*)f.q + qr * f.ldq + hcol + 16 * s + 8 * hi);
    of[s] = *(const bf16x8*)((const bf16*)b.dout + qr * b.lddo + hcol + 16 * s + 8 * hi);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[s][j] = (bf16)((float)qf[s][j] * c);
  }
  const int64_t lrow = ((int64_t)item * f.heads + head) * f.lq + qrc;
  const float lse = f.lse[lrow], dlt = b.delta[lrow];
  const TrOff tro = tr_offsets(lane);
  f32x16 dq[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) dq[0][i] = dq[1][i] = 0.f;
  // key tiles of both segments in order (segment 0 then 1), staged through registers one ahead
  const int nt0 = (f.l0 + 63) / 64, nt1 = f.l1 > 0 ? (f.l1 + 63) / 64 : 0, ntiles = nt0 + nt1;
  TileRegs rk, rv;
  auto fetch = [&](int t) {
    const int seg = t >= nt0, k0 = (seg ? t - nt0 : t) * 64, len = seg ? f.l1 : f.l0;
    const int64_t row0 = (int64_t)item * (seg ? f.k1_bstride : f.k0_bstride);
    rk = fetch_tile((const bf16*)(seg ? f.k1 : f.k0) + row0 * (seg ? f.ldk1 : f.ldk0) + hcol, seg ? f.ldk1 : f.ldk0,
                    k0, len, tid);
    rv = fetch_tile((const bf16*)(seg ? f.v1 : f.v0) + row0 * (seg ? f.ldv1 : f.ldv0) + hcol, seg ? f.ldv1 : f.ldv0,
                    k0, len, tid);
  };
  fetch(0);
  for (int t = 0; t < ntiles; ++t) {
    {
      char* kt = smem + (t & 1) * 2 * TB;
      char* vt = kt + TB;
      store_tile(kt, rk, tid);
      store_tile(vt, rv, tid);
      __syncthreads();  // this stage written; every wave is past the previous use of this buffer
      if (t + 1 < ntiles) fetch(t + 1);
      const int seg = t >= nt0;
      const int valid = (seg ? f.l1 : f.l0) - (seg ? t - nt0 : t) * 64;
      f32x16 sc[2], dp[2];
      const f32x16 zero = {};
      sc[0] = sc[1] = dp[0] = dp[1] = zero;
#pragma unroll
      for (int s = 0; s < 4; ++s)  // four independent accumulation chains in flight
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          sc[kb] = mfma32(row_frag(kt, kb * 32 + l32, s, hi), qf[s], sc[kb]);  // S^T = K (cQ)^T
          dp[kb] = mfma32(row_frag(vt, kb * 32 + l32, s, hi), of[s], dp[kb]);  // dP^T = V dO^T
        }
      auto ds_tile = [&](auto masked) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            bf16x8 df;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int r = 8 * s2 + j;
              float p = __builtin_amdgcn_exp2f(sc[kb][r] - lse);
              if constexpr (decltype(masked)::value) p = kb * 32 + acc_row(r, hi) < valid ? p : 0.f;
              df[j] = (bf16)(p * (dp[kb][r] - dlt));
            }
            const int row0 = kb * 32 + 16 * s2;
#pragma unroll
            for (int db = 0; db < 2; ++db) dq[db] = mfma32(tr_frag(kt, row0, tro.off[db]), df, dq[db]);  // dQ^T += K^T dS^T
          }
      };
      if (valid >= 64) ds_tile(std::false_type{});  // full key tile: no per-element mask (uniform branch)
      else ds_tile(std::true_type{});
    }
  }
  if (qrow < f.lq) {
    float* dqp = b.dq + ((int64_t)item * f.q_bstride + qrow) * b.lddq + hcol;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *(float4*)(dqp + db * 32 + 8 * g + 4 * hi) =
            make_float4(dq[db][4 * g] * f.scale, dq[db][4 * g + 1] * f.scale, dq[db][4 * g + 2] * f.scale,
                        dq[db][4 * g + 3] * f.scale);
  }
}

}  // namespace

extern "C" int sr_attention_bwd(sr_stream_t stream, const sr_attn_bwd_desc* desc) {
  SR_CHECK(desc, SR_EINVAL, "sr_attention_bwd: null desc");
  const sr_attn_bwd_desc& b = *desc;
  const sr_attn_desc& f = b.f;
  SR_CHECK(f.q && f.k0 && f.v0 && f.o && f.lse && b.dout && b.delta && b.dq && b.dk0 && b.dv0, SR_EINVAL,
           "sr_attention_bwd: null pointer");
  SR_CHECK(f.head_dim == 64 && f.mask_mode == SR_MASK_NONE, SR_EUNSUPPORTED,
           "sr_attention_bwd: head_dim 64 without mask only");
  SR_CHECK(f.batch > 0 && f.heads > 0 && f.lq > 0 && f.l0 > 0 && f.l1 >= 0, SR_EINVAL, "sr_attention_bwd: bad sizes");
  SR_CHECK(f.l1 == 0 || (f.k1 && f.v1 && b.dk1 && b.dv1), SR_EINVAL, "sr_attention_bwd: segment 1 needs k1/v1/dk1/dv1");
  SR_CHECK(f.ldq % 8 == 0 && f.ldk0 % 8 == 0 && f.ldv0 % 8 == 0 && f.ldo % 8 == 0 && b.lddo % 8 == 0 &&
               b.lddq % 4 == 0 && b.lddk0 % 4 == 0 && b.lddv0 % 4 == 0 &&
               (f.l1 == 0 || (f.ldk1 % 8 == 0 && f.ldv1 % 8 == 0 && b.lddk1 % 4 == 0 && b.lddv1 % 4 == 0)),
           SR_EINVAL, "sr_attention_bwd: leading dims (bf16 multiples of 8, fp32 multiples of 4)");
  hipStream_t s = (hipStream_t)stream;
  const int64_t nrows = (int64_t)f.batch * f.heads * f.lq;
  hipLaunchKernelGGL(attn_bwd_delta_kernel, dim3((unsigned)std::min<int64_t>((nrows + 255) / 256, 1 << 20)),
                     dim3(256), 0, s, b);
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3((f.lq + 127) / 128, f.heads, f.batch), dim3(256), 0, s, b);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel<0>, dim3((f.l0 + 127) / 128, f.heads, f.k0_bstride == 0 ? 1 : f.batch),
                     dim3(256), 0, s, b);
  if (f.l1 > 0)
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<1>, dim3((f.l1 + 127) / 128, f.heads, f.k1_bstride == 0 ? 1 : f.batch),
                       dim3(256), 0, s, b);
  return sr::check_launch("sr_attention_bwd");
}
