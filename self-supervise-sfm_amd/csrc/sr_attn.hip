// Fused multi-head attention for gfx950.
//
// Replaces F.scaled_dot_product_attention (attention.py:103-109) for
//   frame attention      (one item per frame, keys = the frame),
//   global attention     (one item, keys = every anchor token),
//   global_reloc         (one item per query frame; keys = [anchor subsample (shared
//                         segment 0) ; own frame (segment 1)] — exactly the rows the
//                         reference's dense bool mask allows, aggregator.py:302-311,
//                         832-851, without materialising the O((S*P)^2) mask),
//   camera trunk         (camera_head.py:165, build_lr_mask :197-228) — fp32 kernel.
//
// attn_bf16 (performance path, head_dim 64):
//   * workgroup = 4 waves = 128 query rows; each wave owns 32 rows for the whole key sweep;
//   * K/V tiles of 64 keys staged by LDS-DMA, double-buffered, XOR-swizzled rows;
//   * S^T = K.Q^T with v_mfma_f32_32x32x16_bf16 (Q fragments live in registers), so each
//     lane holds 32 scores of ONE query row: the row max / sum are in-lane plus one
//     lane^32 exchange (cdna_hip_programming.md App. B "Fused attention prefill");
//   * online softmax in fp32 with exp2; the O rescale is skipped when no row max moved;
//   * P (accumulator) feeds the PV MFMA as the B operand directly (no LDS round trip);
//     V^T fragments come from ds_read_b64_tr_b16 on the row-major V tile.
// attn_f32 (parity mode + camera trunk, head_dim 64 | 128): exact fp32 VALU kernel,
//   K/V tiles broadcast from LDS, per-key online softmax.
#include <cfloat>
#include <cstdlib>

#include "sr_common.h"

namespace {

struct AttnArgs {
  sr_attn_desc d;
  int ntile0, ntile1;  // key tiles per segment
};

// ------------------------------------------------------------------ bf16 / MFMA
constexpr int KT = 64;               // keys per tile
constexpr int TILE_B = KT * 128;     // bytes of one K (or V) tile: 64 keys x 64 bf16
constexpr int STAGE_B = 2 * TILE_B;  // K + V

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// v and its lane^32 partner combined, via v_permlane32_swap (no LDS traffic)
__device__ __forceinline__ float max_x32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_x32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// NW waves x 64 query rows per workgroup (two 32-row q-blocks per wave); KIND only names
// the call site in profiles (0 frame, 1 global_reloc, 2 global).
//
// Tile loop (K/V ring of NBUF=4 stages, up to 3 in flight, one barrier per tile):
//   S0 = K Q0^T, S1 = K Q1^T       (16 MFMA; each K fragment read once, used twice)
//   row max / rescale per q-block  (lane^32 exchange by v_permlane32_swap)
//   P = exp2(S*c - m) -> bf16; O^T += V^T P^T  (16 MFMA; each V^T fragment used twice)
// Two workgroups per CU (<= 256 VGPRs) interleave their MFMA / VALU phases freely.
template <int NW, int KIND>
__global__ __launch_bounds__(NW * 64, 2) void attn_bf16_kernel(AttnArgs args) {
  constexpr int QROWS = NW * 64;
  constexpr int NBUF = NW >= 4 ? 4 : 2;  // ring depth (power of 2); NBUF-1 stages in flight
  constexpr int DPW = 16 / NW;  // LDS-DMA wave-instructions per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[NBUF * STAGE_B];
  const sr_attn_desc& d = args.d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qt = blockIdx.x, head = blockIdx.y, item = blockIdx.z;
  const int hcol = head * 64;
  const int l32 = lane & 31, hi = lane >> 5;
  const int ntiles = args.ntile0 + args.ntile1;
  const uint32_t lds0 = sr::lds_addr(smem);

  // ---- staging: global DMA instruction gi = wave*DPW + i; gi < 8: K rows 8gi.., else V rows.
  // Segment pointers are copied to scalars once: selecting between kernel-argument fields
  // inside the loop compiles to vector loads whose vmcnt(0) wait would drain the ring.
  const bool stage_v = wave * DPW >= 8;  // wave-uniform: a wave stages only K or only V
  const bf16* const sb0 = (const bf16*)(stage_v ? d.v0 : d.k0);
  const bf16* const sb1 = (const bf16*)(stage_v ? d.v1 : d.k1);
  const int64_t sld0 = stage_v ? d.ldv0 : d.ldk0, sld1 = stage_v ? d.ldv1 : d.ldk1;
  const int64_t srb0 = (int64_t)item * d.k0_bstride, srb1 = (int64_t)item * d.k1_bstride;
  const int nt0 = args.ntile0, len0 = d.l0, len1 = d.l1;
  auto stage = [&](int t) {
    const int buf = t & (NBUF - 1);
    const bool s1 = t >= nt0;
    const int tt = s1 ? t - nt0 : t;
    const int len = s1 ? len1 : len0;
    const bf16* base = s1 ? sb1 : sb0;
    const int64_t ld = s1 ? sld1 : sld0;
    const int64_t rbase = s1 ? srb1 : srb0;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int gi = wave * DPW + i;
      const int r = (gi & 7) * 8 + (lane >> 3);  // key row inside the tile
      const int key = min(tt * KT + r, len - 1);
      // K rows: chunk ^ ((r>>1)&7) (conflict-free ds_read_b128 fragments);
      // V rows: chunk ^ (((r>>1)&1)<<2) (conflict-free ds_read_b64_tr_b16: rows r, r+2 of a
      // 4-row transposed block land in opposite 64-B halves)
      const int chunk = (lane & 7) ^ (stage_v ? (((r >> 1) & 1) << 2) : ((r >> 1) & 7));
      const uint32_t dst =
          __builtin_amdgcn_readfirstlane(lds0 + buf * STAGE_B + (stage_v ? TILE_B : 0) + (gi & 7) * 1024);
      sr::dma16(base + (rbase + key) * ld + hcol + chunk * 8, dst);
    }
  };
#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < ntiles) stage(i);

  // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[row][16s + 8hi .. +8]
  const int qrow0 = qt * QROWS + wave * 64 + l32;  // q-block b: row qrow0 + 32b
  bf16x8 qf[2][4];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int qr = min(qrow0 + 32 * b, d.lq - 1);
    const bf16* qp = (const bf16*)d.q + (item * d.q_bstride + qr) * d.ldq + hcol + 8 * hi;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[b][s] = *(const bf16x8*)(qp + 16 * s);
  }

  const float c = d.scale * 1.4426950408889634f;  // scale * log2(e)
  float m_run[2] = {-1e30f, -1e30f}, l_run[2] = {0.f, 0.f};  // l_run: this lane's partial row sums
  f32x16 o[2][2];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      o[b][0][i] = 0.f;
      o[b][1][i] = 0.f;
    }
  // K fragment: row kb*32 + l32, chunk (2s + hi) ^ kswz
  const int kswz = (l32 >> 1) & 7;
  int koff[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) koff[s] = l32 * 128 + (((2 * s + hi) ^ kswz) * 16);
  // V tr-read: group G = lane>>4, i = lane&15 supplies row r0 + (i>>2), col db*32 + 16(G&1) + 4(i&3);
  // the V swizzle term depends only on (i>>2)
  const int G = lane >> 4, gi_ = lane & 15;
  const int vrow_in = gi_ >> 2;
  const int vcol_in = 16 * (G & 1) + 4 * (gi_ & 3);
  const int vsw = ((vrow_in >> 1) & 1) << 2;
  const int voff0 = (4 * hi + vrow_in) * 128 + (((vcol_in >> 3) ^ vsw) * 16) + (vcol_in & 7) * 2;
  const int voff1 = (4 * hi + vrow_in) * 128 + (((4 + (vcol_in >> 3)) ^ vsw) * 16) + (vcol_in & 7) * 2;

  for (int t = 0; t < ntiles; ++t) {
    // tile t must have landed (up to NBUF-2 later stages stay in flight); everyone is done
    // with tile t-1, whose buffer the next stage overwrites
    if (NBUF >= 4 && t + 2 < ntiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DPW) : "memory");
    else if (NBUF >= 3 && t + 1 < ntiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sr::barrier_raw();
    if (t + NBUF - 1 < ntiles) stage(t + NBUF - 1);
    const char* kt_lds = smem + (t & (NBUF - 1)) * STAGE_B;
    const char* vt_lds = kt_lds + TILE_B;

    // ---- S^T = K Q^T for both q-blocks (2 blocks of 32 keys each)
    f32x16 sc[2][2];  // [q-block][key block]
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[b][kb][i] = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 kf = *(const bf16x8*)(kt_lds + kb * 4096 + koff[s]);
        sc[0][kb] = mfma32(kf, qf[0][s], sc[0][kb]);
        sc[1][kb] = mfma32(kf, qf[1][s], sc[1][kb]);
      }

    // ---- mask the ragged tail of a segment
    const bool s1 = t >= nt0;
    const int valid = (s1 ? len1 : len0) - (s1 ? t - nt0 : t) * KT;
    if (valid < KT) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
            if (key >= valid) sc[b][kb][r] = -INFINITY;
          }
    }

    // ---- row max per q-block; rescale O / l when it grew
    float m_new[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float t8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        t8[i] = fmaxf(fmaxf(sc[b][0][i], sc[b][0][i + 8]), fmaxf(sc[b][1][i], sc[b][1][i + 8]));
#pragma unroll
      for (int i = 0; i < 4; ++i) t8[i] = fmaxf(t8[i], t8[i + 4]);
      m_new[b] = fmaxf(m_run[b], max_x32(fmaxf(fmaxf(t8[0], t8[1]), fmaxf(t8[2], t8[3]))) * c);
    }
    if (__any((m_new[0] > m_run[0]) | (m_new[1] > m_run[1]))) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const float alpha = __builtin_amdgcn_exp2f(m_run[b] - m_new[b]);
        l_run[b] *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          o[b][0][i] *= alpha;
          o[b][1][i] *= alpha;
        }
        m_run[b] = m_new[b];
      }
    }

    // ---- P = exp2(S*c - m) (B operand), O^T += V^T P^T; each V^T fragment feeds both q-blocks
    float ps[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 pf[2];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float p = __builtin_amdgcn_exp2f(fmaf(sc[b][kb][8 * s2 + j], c, -m_run[b]));
            ps[b][j & 1] += p;
            pf[b][j] = (bf16)p;
          }
        const int rowoff = (kb * 32 + 16 * s2) * 128;
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const char* pa = vt_lds + rowoff + (db ? voff1 : voff0);
          const s16x4 va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)pa);
          const s16x4 vb =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)(pa + 8 * 128));
          const bf16x4 a4 = __builtin_bit_cast(bf16x4, va), b4 = __builtin_bit_cast(bf16x4, vb);
          const bf16x8 vf = {a4[0], a4[1], a4[2], a4[3], b4[0], b4[1], b4[2], b4[3]};
          o[0][db] = mfma32(vf, pf[0], o[0][db]);
          o[1][db] = mfma32(vf, pf[1], o[1][db]);
        }
      }
    l_run[0] += ps[0][0] + ps[0][1];
    l_run[1] += ps[1][0] + ps[1][1];
  }

  // ---- epilogue: O[q][hcol + d] = O^T[d][q] / l
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const float inv = 1.f / sum_x32(l_run[b]);
    const int qrow = qrow0 + 32 * b;
    if (qrow < d.lq) {
      bf16* op = (bf16*)d.o + (item * d.q_bstride + qrow) * d.ldo + hcol;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[b][db][4 * g + j] * inv);
          *(bf16x4*)(op + db * 32 + 8 * g + 4 * hi) = v;
        }
    }
  }
}

// ------------------------------------------------------------------ f32 / VALU
constexpr int F32_KT = 32;       // keys per LDS tile
constexpr int F32_THREADS = 128;  // query rows per workgroup

template <int D>
__global__ __launch_bounds__(F32_THREADS) void attn_f32_kernel(AttnArgs args) {
  __shared__ float ks[F32_KT][D];
  __shared__ float vs[F32_KT][D];
  const sr_attn_desc& d = args.d;
  const int tid = threadIdx.x;
  const int head = blockIdx.y, item = blockIdx.z;
  const int hcol = head * D;
  const int qrow = blockIdx.x * F32_THREADS + tid;
  const int qrow_c = min(qrow, d.lq - 1);
  const float* qp = (const float*)d.q + (item * d.q_bstride + qrow_c) * d.ldq + hcol;
  float q[D], o[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    q[i] = qp[i];
    o[i] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  const int nkeys_total = d.l0 + d.l1;
  for (int seg = 0; seg < 2; ++seg) {
    const int len = seg ? d.l1 : d.l0;
    if (len <= 0) continue;
    const float* kb = (const float*)(seg ? d.k1 : d.k0);
    const float* vb = (const float*)(seg ? d.v1 : d.v0);
    const int64_t ldk = seg ? d.ldk1 : d.ldk0, ldv = seg ? d.ldv1 : d.ldv0;
    const int64_t rb = item * (seg ? d.k1_bstride : d.k0_bstride);
    const int key_base = seg ? d.l0 : 0;  // logical key index (for the camera mask)
    for (int t0 = 0; t0 < len; t0 += F32_KT) {
      const int n = min(F32_KT, len - t0);
      __syncthreads();
      for (int e = tid; e < F32_KT * D; e += F32_THREADS) {
        const int r = e / D, cc = e - r * D;
        const int key = min(t0 + r, len - 1);
        ks[r][cc] = kb[(rb + key) * ldk + hcol + cc];
        vs[r][cc] = vb[(rb + key) * ldv + hcol + cc];
      }
      __syncthreads();
      for (int j = 0; j < n; ++j) {
        const int kidx = key_base + t0 + j;
        if (d.mask_mode == SR_MASK_CAMERA && !(kidx < d.n_anchor || kidx == qrow)) continue;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < D; ++i) s = fmaf(q[i], ks[j][i], s);
        s *= d.scale;
        if (s > m) {
          const float corr = expf(m - s);
          l = l * corr + 1.f;
#pragma unroll
          for (int i = 0; i < D; ++i) o[i] = fmaf(o[i], corr, vs[j][i]);
          m = s;
        } else {
          const float p = expf(s - m);
          l += p;
#pragma unroll
          for (int i = 0; i < D; ++i) o[i] = fmaf(p, vs[j][i], o[i]);
        }
      }
    }
  }
  (void)nkeys_total;
  if (qrow < d.lq) {
    float* op = (float*)d.o + (item * d.q_bstride + qrow) * d.ldo + hcol;
    const float inv = 1.f / l;
#pragma unroll
    for (int i = 0; i < D; ++i) op[i] = o[i] * inv;
  }
}

}  // namespace

extern "C" int sr_attention(sr_stream_t stream, int dtype, const sr_attn_desc* desc) {
  SR_CHECK(desc, SR_EINVAL, "sr_attention: null desc");
  const sr_attn_desc& d = *desc;
  SR_CHECK(d.q && d.o && d.k0 && d.v0, SR_EINVAL, "sr_attention: null q/k0/v0/o");
  SR_CHECK(d.batch > 0 && d.heads > 0 && d.lq > 0 && d.l0 > 0 && d.l1 >= 0, SR_EINVAL,
           "sr_attention: bad sizes batch=%d heads=%d lq=%d l0=%d l1=%d", d.batch, d.heads, d.lq, d.l0, d.l1);
  SR_CHECK(d.l1 == 0 || (d.k1 && d.v1), SR_EINVAL, "sr_attention: segment 1 needs k1/v1");
  SR_CHECK(d.mask_mode == SR_MASK_NONE || (d.mask_mode == SR_MASK_CAMERA && d.l1 == 0), SR_EINVAL,
           "sr_attention: bad mask_mode %d", d.mask_mode);
  AttnArgs a;
  a.d = d;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16) {
    SR_CHECK(d.head_dim == 64, SR_EUNSUPPORTED, "sr_attention(bf16): head_dim must be 64 (got %d)", d.head_dim);
    SR_CHECK(d.mask_mode == SR_MASK_NONE, SR_EUNSUPPORTED, "sr_attention(bf16): camera mask needs the f32 kernel");
    SR_CHECK(d.ldq % 8 == 0 && d.ldk0 % 8 == 0 && d.ldv0 % 8 == 0 && d.ldo % 4 == 0 &&
                 (d.l1 == 0 || (d.ldk1 % 8 == 0 && d.ldv1 % 8 == 0)),
             SR_EINVAL, "sr_attention(bf16): leading dims must be multiples of 8");
    a.ntile0 = (d.l0 + KT - 1) / KT;
    a.ntile1 = (d.l1 + KT - 1) / KT;
    const int kind = d.l1 > 0 ? 1 : (d.batch == 1 && d.lq >= 4096 ? 2 : 0);
    // 4 waves x 64 rows = 256-row query tiles (measured fastest for the frame, reloc and global
    // stacks at N=32); 2-wave 128-row tiles when 256-row tiles would leave CUs idle (fewer than
    // 2 workgroups per CU, e.g. the per-rank query slice of a frame-sharded global block).
    // SR_ATTN_WAVES=2|4 overrides (tuning experiments).
    static const int force_nw = [] {
      const char* e = getenv("SR_ATTN_WAVES");
      return e ? atoi(e) : 0;
    }();
    const long wgs256 = (long)((d.lq + 255) / 256) * d.heads * d.batch;
    const bool wide = force_nw ? force_nw == 4 : wgs256 >= 512;
    if (wide) {
      dim3 grid((d.lq + 255) / 256, d.heads, d.batch);
      if (kind == 2) hipLaunchKernelGGL((attn_bf16_kernel<4, 2>), grid, dim3(256), 0, s, a);
      else if (kind == 1) hipLaunchKernelGGL((attn_bf16_kernel<4, 1>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((attn_bf16_kernel<4, 0>), grid, dim3(256), 0, s, a);
    } else {
      dim3 grid((d.lq + 127) / 128, d.heads, d.batch);
      if (kind == 2) hipLaunchKernelGGL((attn_bf16_kernel<2, 2>), grid, dim3(128), 0, s, a);
      else if (kind == 1) hipLaunchKernelGGL((attn_bf16_kernel<2, 1>), grid, dim3(128), 0, s, a);
      else hipLaunchKernelGGL((attn_bf16_kernel<2, 0>), grid, dim3(128), 0, s, a);
    }
    return sr::check_launch("sr_attention(bf16)");
  }
  SR_CHECK(dtype == SR_F32, SR_EINVAL, "sr_attention: bad dtype %d", dtype);
  a.ntile0 = a.ntile1 = 0;
  dim3 grid((d.lq + F32_THREADS - 1) / F32_THREADS, d.heads, d.batch);
  if (d.head_dim == 64) {
    hipLaunchKernelGGL(attn_f32_kernel<64>, grid, dim3(F32_THREADS), 0, s, a);
  } else if (d.head_dim == 128) {
    hipLaunchKernelGGL(attn_f32_kernel<128>, grid, dim3(F32_THREADS), 0, s, a);
  } else {
    sr::set_error("sr_attention(f32): head_dim must be 64 or 128 (got %d)", d.head_dim);
    return SR_EUNSUPPORTED;
  }
  return sr::check_launch("sr_attention(f32)");
}
