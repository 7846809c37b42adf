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
#include "sr_attn_bwd_pipe.inc"

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

// Tiles reach LDS by LDS-DMA through a ring of NBUF stages (tiles t+1, t+2 in flight while tile
// t is consumed; t+3 is issued right after the tile's barrier).  A workgroup stages a 64-row tile
// with 8 dwordx4 wave-instructions: instruction g copies rows 8g .. 8g+7, lane l row 8g + l/8 into
// LDS chunk l & 7, so the lane fetches source chunk swz(r, l & 7) (swz is an involution per row)
// and LDS holds the swizzled image.
constexpr int NBUF = 4;
__device__ __forceinline__ void dma_rows(const bf16* base, int64_t ld, int row0, int nrows, int g, int lane,
                                         uint32_t lds_tile) {
  const int r = 8 * g + (lane >> 3);
  sr::dma16(base + (int64_t)min(row0 + r, nrows - 1) * ld + swz(r, lane & 7) * 8, lds_tile + g * 1024);
}
// Full tiles take the wave-uniform form (sr::dma16_s): a scalar row pointer + one of two per-lane
// 32-bit byte offsets (row lane/8 of the piece, its swizzled chunk; the swizzle depends only on the
// parity of the row group g, as 4g + lane/16 mod 8).  The per-lane form above (64-bit row multiply
// and clamp per piece: ~60 VALU per tile, 12 of them quarter-rate) is kept for ragged tiles.
__device__ __forceinline__ uint32_t piece_off(int64_t ld, int parity, int lane) {
  const int r = 8 * parity + (lane >> 3);
  return (uint32_t)(((lane >> 3) * ld + swz(r, lane & 7) * 8) * 2);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
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
// Eight lanes per (row, head), one 16-B chunk of the head's 64 columns each, heads fastest: a wave
// reads 8 heads x 128 B of one row contiguously.  Each lane's 8 products, then a fixed xor tree
// over the 8 lanes (deterministic).
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(sr_attn_bwd_desc b) {
  const sr_attn_desc& f = b.f;
  const int64_t n = (int64_t)f.batch * f.heads * f.lq * 8;
  const int c = threadIdx.x & 7;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int64_t gi = e >> 3;  // (item, row, head), head fastest
    const int head = (int)(gi % f.heads);
    const int64_t ir = gi / f.heads;
    const int row = (int)(ir % f.lq), item = (int)(ir / f.lq);
    const int64_t r = (int64_t)item * f.q_bstride + row;
    const bf16x8 ov = *(const bf16x8*)((const bf16*)f.o + r * f.ldo + head * 64 + 8 * c);
    const bf16x8 gv = *(const bf16x8*)((const bf16*)b.dout + r * b.lddo + head * 64 + 8 * c);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s = fmaf((float)ov[j], (float)gv[j], s);
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    if (c == 0) b.delta[((int64_t)item * f.heads + head) * f.lq + row] = -s;  // negated: seeds the dP chains
  }
}

// ---------------------------------------------------------------- dK, dV
// One 64-query tile of the dK/dV sweep for KB key blocks of 32 per wave (lane: key l32 of block
// kb): qt = the tile's LDS stage (Q tile | dO tile | 64 lse | 64 stored -delta), qv = its valid
// rows (MASKED only: clamped duplicate rows get P = 0).  S'^T = lse - c q.k (K resident negated
// and scaled), dP'^T = dO.v - delta; P = exp2(-S'), dS = P dP'; dV^T += dO^T P, dK^T += Q^T dS.
template <int KB, bool MASKED>
__device__ __forceinline__ void dkdv_tile(const char* qt, int qv, const bf16x8 (&kf)[KB][4], const bf16x8 (&vf)[KB][4],
                                          f32x16 (&dk)[KB][2], f32x16 (&dv)[KB][2], const TrOff& tro, int l32, int hi) {
  const char* ot = qt + TB;
  const float* lse_s = (const float*)(qt + 2 * TB);
  const float* dl_s = lse_s + 64;
  // seeds in accumulator order: rows qb2*32 + acc_row(r), four consecutive per float4
  f32x16 sc[KB][2], dp[KB][2];
#pragma unroll
  for (int qb2 = 0; qb2 < 2; ++qb2)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 l4 = *(const float4*)(lse_s + qb2 * 32 + 8 * g + 4 * hi);
      const float4 d4 = *(const float4*)(dl_s + qb2 * 32 + 8 * g + 4 * hi);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        sc[kb][qb2][4 * g] = l4.x; sc[kb][qb2][4 * g + 1] = l4.y;
        sc[kb][qb2][4 * g + 2] = l4.z; sc[kb][qb2][4 * g + 3] = l4.w;
        dp[kb][qb2][4 * g] = d4.x; dp[kb][qb2][4 * g + 1] = d4.y;
        dp[kb][qb2][4 * g + 2] = d4.z; dp[kb][qb2][4 * g + 3] = d4.w;
      }
    }
  bf16x8 fq[4][2], fo[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int qb2 = 0; qb2 < 2; ++qb2) {
      fq[s][qb2] = row_frag(qt, qb2 * 32 + l32, s, hi);
      fo[s][qb2] = row_frag(ot, qb2 * 32 + l32, s, hi);
    }
#pragma unroll
  for (int s = 0; s < 4; ++s)  // 4 KB independent accumulation chains in flight
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int qb2 = 0; qb2 < 2; ++qb2) {
        sc[kb][qb2] = mfma32(fq[s][qb2], kf[kb][s], sc[kb][qb2]);
        dp[kb][qb2] = mfma32(fo[s][qb2], vf[kb][s], dp[kb][qb2]);
      }
  if constexpr (MASKED) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int qb2 = 0; qb2 < 2; ++qb2)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (qb2 * 32 + acc_row(r, hi) >= qv) sc[kb][qb2][r] = INFINITY;
  }
  // P, dS (lane: key column l32, query rows qb2*32 + acc_row(r)); dV^T += dO^T P, dK^T += Q^T dS;
  // each transposed dO / Q fragment feeds every key block
#pragma unroll
  for (int qb2 = 0; qb2 < 2; ++qb2)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 pf[KB], df[KB];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        f32x8 pv, dv8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = 8 * s2 + j;
          pv[j] = __builtin_amdgcn_exp2f(-sc[kb][qb2][r]);
          dv8[j] = pv[j] * dp[kb][qb2][r];
        }
        pf[kb] = __builtin_convertvector(pv, bf16x8);
        df[kb] = __builtin_convertvector(dv8, bf16x8);
      }
      const int row0 = qb2 * 32 + 16 * s2;
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const bf16x8 to = tr_frag(ot, row0, tro.off[db]), tq = tr_frag(qt, row0, tro.off[db]);
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          dv[kb][db] = mfma32(to, pf[kb], dv[kb][db]);
          dk[kb][db] = mfma32(tq, df[kb], dk[kb][db]);
        }
      }
    }
}

// dK[key][d] = scale * dK^T[d][key], dV likewise (lane: key key_base + 32 kb, d = 32 db + acc_row(r))
template <int SEG, int KB>
__device__ __forceinline__ void store_dkdv(const sr_attn_bwd_desc& b, int64_t kb0, int key_base, int len, int hcol,
                                           int hi, const f32x16 (&dk)[KB][2], const f32x16 (&dv)[KB][2]) {
  const float scale = b.f.scale;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int key = key_base + 32 * kb;
    if (key < len) {
      float* dkp = (SEG == 0 ? b.dk0 : b.dk1) + (kb0 + key) * (SEG == 0 ? b.lddk0 : b.lddk1) + hcol;
      float* dvp = (SEG == 0 ? b.dv0 : b.dv1) + (kb0 + key) * (SEG == 0 ? b.lddv0 : b.lddv1) + hcol;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d0 = db * 32 + 8 * g + 4 * hi;
          *(float4*)(dkp + d0) = make_float4(dk[kb][db][4 * g] * scale, dk[kb][db][4 * g + 1] * scale,
                                             dk[kb][db][4 * g + 2] * scale, dk[kb][db][4 * g + 3] * scale);
          *(float4*)(dvp + d0) = make_float4(dv[kb][db][4 * g], dv[kb][db][4 * g + 1], dv[kb][db][4 * g + 2],
                                             dv[kb][db][4 * g + 3]);
        }
    }
  }
}

// grid (key tiles of 128, heads, SHARED ? 1 : batch); wave w owns keys tile*128 + 32 w + l32.
// Q / dO tiles and their lse / delta stream through the LDS-DMA ring.  The resident K fragment is
// negated and scaled by c and the S chain is seeded with +lse straight from LDS, so it returns
// -(c q.k - lse) and P = exp2(-S') (the sign is a source modifier of v_exp); the dP chain is seeded
// with the stored -delta (attn_bwd_delta_kernel) and returns dO.v - delta, so dS = P dP' with no
// sign flips (a negated V turned into 24 v_xor per tile before the packed multiplies).
// One key block of 32 per wave, two workgroups per CU (64 keys per wave with one wave per SIMD is
// the asm sweep's form; the compiled 64-key variant measured no faster and was removed in round 6).
template <int SEG>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_kernel(sr_attn_bwd_desc b) {
  constexpr int KB = 1;
  constexpr int STG = 2 * TB + 2 * 64 * 4;  // one stage: Q tile | dO tile | lse | delta
  __shared__ __attribute__((aligned(16))) char smem[NBUF * STG];
  const sr_attn_desc& f = b.f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int head = blockIdx.y, hcol = head * 64;
  const bool shared = (SEG == 0 ? f.k0_bstride : f.k1_bstride) == 0;
  const int it0 = shared ? 0 : blockIdx.z;
  const int it1 = shared ? f.batch : blockIdx.z + 1;
  const int len = SEG == 0 ? f.l0 : f.l1;
  const int64_t kb0 = (int64_t)(shared ? 0 : blockIdx.z) * (SEG == 0 ? f.k0_bstride : f.k1_bstride);
  const bf16* kp = (const bf16*)(SEG == 0 ? f.k0 : f.k1);
  const bf16* vp = (const bf16*)(SEG == 0 ? f.v0 : f.v1);
  const int64_t ldk = SEG == 0 ? f.ldk0 : f.ldk1, ldv = SEG == 0 ? f.ldv0 : f.ldv1;
  const int key_base = blockIdx.x * (128 * KB) + wave * (32 * KB) + l32;  // key of block kb: + 32 kb
  const float c = f.scale * 1.4426950408889634f;

  // staging: wave w issues row groups g = 4 (w & 1) .. + 3 of the Q (waves 0, 1) or dO (2, 3)
  // tile; waves 0 / 1 also copy the tile's 64 lse / delta values (one dword DMA each)
  const int ntq = (f.lq + 63) / 64, ntiles = (it1 - it0) * ntq;
  const uint32_t lds0 = sr::lds_addr(smem);
  const bool stage_o = wave_u >= 2;
  const bf16* const sbase = (const bf16*)(stage_o ? b.dout : f.q) + hcol;
  const int64_t sld = stage_o ? b.lddo : f.ldq;
  const float* const lsrc = wave_u == 0 ? f.lse : b.delta;
  // tile t = (item - it0) * ntq + query tile; cursors instead of divisions (the compiler
  // expands an integer division into ~15 VALU)
  const int g0 = 4 * (wave_u & 1);
  const uint32_t offA = piece_off(sld, 0, lane), offB = piece_off(sld, 1, lane);
  auto stage = [&](int t, int item, int q0) {
    const uint32_t sb = lds0 + (t & (NBUF - 1)) * STG;
    const bf16* tb = sbase + (int64_t)item * f.q_bstride * sld;
    const float* lb = lsrc + ((int64_t)item * f.heads + head) * f.lq + q0;
    if (q0 + 64 <= f.lq) {  // full tile: scalar pointers
      const char* p = (const char*)(tb + (int64_t)(q0 + 8 * g0) * sld);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        sr::dma16_s(p + (int64_t)8 * i * sld * 2, (i & 1) ? offB : offA, sb + (stage_o ? TB : 0) + (g0 + i) * 1024);
      if (wave_u < 2) sr::dma4_s(lb, (uint32_t)lane * 4, sb + 2 * TB + wave_u * 256);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) dma_rows(tb, sld, q0, f.lq, g0 + i, lane, sb + (stage_o ? TB : 0));
      if (wave_u < 2) sr::dma4(lb + min(lane, f.lq - 1 - q0), sb + 2 * TB + wave_u * 256);
    }
  };
  int s_item = it0, s_q = 0;  // next tile to stage
  for (int i = 0; i < NBUF - 1 && i < ntiles; ++i) {
    stage(i, s_item, s_q * 64);
    if (++s_q == ntq) s_q = 0, ++s_item;
  }

  bf16x8 kf[KB][4], vf[KB][4];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int keyc = min(key_base + 32 * kb, len - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[kb][s] = *(const bf16x8*)(kp + (kb0 + keyc) * ldk + hcol + 16 * s + 8 * hi);
      vf[kb][s] = *(const bf16x8*)(vp + (kb0 + keyc) * ldv + hcol + 16 * s + 8 * hi);
    }
  }
  // retire these loads (and the prologue stages) with a wait the compiler sees: its scoreboard
  // would otherwise carry them into the loop, and a vmcnt wait there drains the ring
  __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        kf[kb][s][j] = (bf16)(-(float)kf[kb][s][j] * c);
      }
      // keep the negated fragment in registers: otherwise the compiler re-derives it inside the
      // tile loop (16 v_xor + 8 v_perm per tile and fragment set)
      asm volatile("" : "+v"(kf[kb][s]));
    }
  const TrOff tro = tr_offsets(lane);
  f32x16 dk[KB][2], dv[KB][2];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[kb][0][i] = dk[kb][1][i] = dv[kb][0][i] = dv[kb][1][i] = 0.f;

  // One tile of the sweep: wait for it, restage the ring, then dkdv_tile.  MASKED (the last,
  // ragged query tile of an item) is a separate instantiation, so the full-tile body is one basic
  // block the compiler can interleave.
  auto tile_body = [&](int t, int cq, auto masked) __attribute__((always_inline)) {
    // tile t has landed (later stages stay in flight: 5 DMA wave-instructions per stage on
    // waves 0-1, 4 on waves 2-3); every wave is done with tile t-1, whose buffer stage t+3 reuses
    if (t + 2 < ntiles) {
      if (wave_u < 2) wait_vm<10>();
      else wait_vm<8>();
    } else if (t + 1 < ntiles) {
      if (wave_u < 2) wait_vm<5>();
      else wait_vm<4>();
    } else {
      wait_vm<0>();
    }
    sr::barrier_raw();
    if (t + NBUF - 1 < ntiles) {
      stage(t + NBUF - 1, s_item, s_q * 64);
      if (++s_q == ntq) s_q = 0, ++s_item;
    }
    dkdv_tile<KB, decltype(masked)::value>(smem + (t & (NBUF - 1)) * STG, f.lq - cq * 64, kf, vf, dk, dv, tro, l32, hi);
  };
  // tiles item by item; the last query tile of an item is the only one that can be ragged
  const bool ragged = f.lq % 64 != 0;
  for (int t = 0; t < ntiles;) {
    const int full = ragged ? ntq - 1 : ntq;
    for (int cq = 0; cq < full; ++cq, ++t) tile_body(t, cq, std::false_type{});
    if (ragged) {
      tile_body(t, ntq - 1, std::true_type{});
      ++t;
    }
  }
  store_dkdv<SEG, KB>(b, kb0, key_base, len, hcol, hi, dk, dv);
}

// ---------------------------------------------------------------- dK, dV: hand-scheduled sweep
// attn_bwd_dkdv_kernel's work for one item's full query tiles as ONE inline-asm statement
// (tools/gen_attn_bwd_pipe.py, sr_attn_bwd_pipe.inc): one wave per SIMD, 64 keys per wave (two key
// blocks), 256 per workgroup; the two 32-query halves of a tile are pipelined half a tile apart so
// that one half's exp2 / dS / bf16 packing runs in the MFMA gaps of the other's chains.  A ragged
// last query tile (lq % 64) is staged up front into a fifth LDS stage and run afterwards with the
// compiled dkdv_tile, so every dK / dV accumulation happens in the compiled kernel's order (the
// outputs are bit-identical to attn_bwd_dkdv_kernel's).  The host picks this kernel for one item
// per workgroup (keys not shared across the batch) and at least 4 full query tiles.
//   LDS: ring of 4 x (Q tile | dO tile) at 0 .. 64 KB, the ring's lse | -delta at 64 KB + 512 s,
//        the ragged stage (Q | dO | lse | -delta) after them.
// CAT: keys shared by a batch > 1 whose items' queries are consecutive rows (q_bstride == lq): the
// items run as ONE query sequence of batch * lq rows (64-row tiles straddle items; a row's lse /
// -delta sit at (b H + h) lq + i, formed per tile in the asm, SR_ATTN_BWD_PIPE_ASM_CAT).  The sum
// over queries is the same, grouped into other tiles than the compiled kernel's per-item sweep.
template <int SEG, bool CAT = false>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv_pipe_kernel(sr_attn_bwd_desc b) {
  constexpr int SLOT = 2 * TB, LSE0 = 4 * SLOT, RAG = LSE0 + 4 * 512;
  __shared__ __attribute__((aligned(16))) char smem[RAG + 2 * TB + 512];
  const sr_attn_desc& f = b.f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int head = blockIdx.y, hcol = head * 64, item = CAT ? 0 : blockIdx.z;
  const int len = SEG == 0 ? f.l0 : f.l1;
  const int64_t kb0 = (int64_t)item * (SEG == 0 ? f.k0_bstride : f.k1_bstride);
  const bf16* kp = (const bf16*)(SEG == 0 ? f.k0 : f.k1);
  const bf16* vp = (const bf16*)(SEG == 0 ? f.v0 : f.v1);
  const int64_t ldk = SEG == 0 ? f.ldk0 : f.ldk1, ldv = SEG == 0 ? f.ldv0 : f.ldv1;
  const int key_base = blockIdx.x * 256 + wave * 64 + l32;  // key of block kb: + 32 kb
  const float c = f.scale * 1.4426950408889634f;
  const int lqt = CAT ? f.batch * f.lq : f.lq;  // the swept query rows
  const int nfull = lqt / 64, qv = lqt % 64;  // nfull >= 4 (host)
  // CAT: row r's lse / -delta float offset from the head's item-0 base, r + (r / lq) (H-1) lq, with
  // r / lq = mulhi(r, msh_m) >> msh (exact for r < 2^24: M lq - 2^(32+s) < lq < 2^(s+1))
  int msh = 0;
  uint32_t mgc = 0;
  if constexpr (CAT) {
    msh = 31 - __builtin_clz((uint32_t)f.lq);
    if ((1 << msh) == f.lq) --msh;
    mgc = (uint32_t)(((1ull << (32 + msh)) + (uint64_t)f.lq - 1) / (uint64_t)f.lq);
    msh = __builtin_amdgcn_readfirstlane(msh);
    mgc = __builtin_amdgcn_readfirstlane(mgc);
  }
  const uint32_t istr = __builtin_amdgcn_readfirstlane((uint32_t)((f.heads - 1) * f.lq * 4));
  auto loff = [&](int r) -> uint32_t {  // CAT: bytes from the head's base to row r's lse
    const uint32_t bi = __umulhi((uint32_t)r, mgc) >> msh;
    return (uint32_t)r * 4 + bi * istr;
  };

  // staging: wave w copies row groups 4 (w & 1) .. + 3 of the Q (waves 0, 1) or dO (2, 3) tile and
  // the tile's 64 lse (waves 0, 2) or -delta (1, 3) values: five DMA wave-instructions per tile and
  // wave (waves 2, 3 duplicate 0, 1's dword copy, so the asm's vmcnt counts are uniform)
  const uint32_t lds0 = sr::lds_addr(smem);
  const bool stage_o = wave_u >= 2;
  const int64_t sld = stage_o ? b.lddo : f.ldq;
  const bf16* const tbase = (const bf16*)(stage_o ? b.dout : f.q) + (int64_t)item * f.q_bstride * sld + hcol;
  const float* const lbase = ((wave_u & 1) ? b.delta : f.lse) + ((int64_t)item * f.heads + head) * f.lq;
  const int g0 = 4 * (wave_u & 1);
  const uint32_t offA = piece_off(sld, 0, lane), offB = piece_off(sld, 1, lane);
  const uint32_t ldsv = __builtin_amdgcn_readfirstlane(lds0 + (stage_o ? TB : 0) + g0 * 1024);
  const uint32_t ldsl = __builtin_amdgcn_readfirstlane(lds0 + LSE0 + (wave_u & 1) * 256);
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const char* p = (const char*)(tbase + (int64_t)(t * 64 + 8 * g0) * sld);
#pragma unroll
    for (int i = 0; i < 4; ++i) sr::dma16_s(p + (int64_t)8 * i * sld * 2, (i & 1) ? offB : offA, ldsv + t * SLOT + i * 1024);
    if constexpr (CAT) sr::dma4((const char*)lbase + loff(t * 64 + lane), ldsl + t * 512);
    else sr::dma4_s(lbase + t * 64, (uint32_t)lane * 4, ldsl + t * 512);
  }
  if (qv) {  // the ragged last tile: rows clamped to the last row (P = 0 for them: dkdv_tile<.., true>)
#pragma unroll
    for (int i = 0; i < 4; ++i) dma_rows(tbase, sld, nfull * 64, lqt, g0 + i, lane, lds0 + RAG + (stage_o ? TB : 0));
    const int rl = min(nfull * 64 + lane, lqt - 1);
    if constexpr (CAT) sr::dma4((const char*)lbase + loff(rl), lds0 + RAG + 2 * TB + (wave_u & 1) * 256);
    else sr::dma4(lbase + rl, lds0 + RAG + 2 * TB + (wave_u & 1) * 256);
  }

  bf16x8 kf[2][4], vf[2][4];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int keyc = min(key_base + 32 * kb, len - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[kb][s] = *(const bf16x8*)(kp + (kb0 + keyc) * ldk + hcol + 16 * s + 8 * hi);
      vf[kb][s] = *(const bf16x8*)(vp + (kb0 + keyc) * ldv + hcol + 16 * s + 8 * hi);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // the fragments and the prologue stages
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[kb][s][j] = (bf16)(-(float)kf[kb][s][j] * c);
  const TrOff tro = tr_offsets(lane);
  f32x16 dk[2][2], dv[2][2];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[kb][0][i] = dk[kb][1][i] = dv[kb][0][i] = dv[kb][1][i] = 0.f;

  // the asm's operands: fragment lane addresses (slot, block and row offsets ride in the
  // instructions' offset field), the DMA walk from tile 3 on (scalar bases, per-lane offsets that
  // step one tile per stage)
  uint32_t ra[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) ra[s] = lds0 + l32 * 128 + swz(l32, 2 * s + hi) * 16;
  const uint32_t ta00 = lds0 + tro.off[0][0], ta01 = lds0 + tro.off[0][1];
  const uint32_t ta10 = lds0 + tro.off[1][0], ta11 = lds0 + tro.off[1][1];
  const uint32_t sa = lds0 + LSE0 + 16 * hi;
  const uint64_t spu = (uint64_t)(uintptr_t)(tbase + (int64_t)(3 * 64 + 8 * g0) * sld);
  const uint32_t sp_lo = __builtin_amdgcn_readfirstlane((uint32_t)spu);
  const uint32_t sp_hi = __builtin_amdgcn_readfirstlane((uint32_t)(spu >> 32));
  const char* spb = (const char*)(uintptr_t)(((uint64_t)sp_hi << 32) | sp_lo);
  const char* spb2 = spb + 16 * sld * 2;
  const uint64_t lpu = (uint64_t)(uintptr_t)(lbase + (CAT ? 0 : 3 * 64));
  const uint32_t lp_lo = __builtin_amdgcn_readfirstlane((uint32_t)lpu);
  const uint32_t lp_hi = __builtin_amdgcn_readfirstlane((uint32_t)(lpu >> 32));
  const char* lpb = (const char*)(uintptr_t)(((uint64_t)lp_hi << 32) | lp_lo);
  uint32_t dma0 = offA, dma1 = offB + (uint32_t)(8 * sld * 2), lofs = CAT ? loff(3 * 64 + lane) : (uint32_t)lane * 4;
  const uint32_t sstep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * sld * 2));
  int nn = __builtin_amdgcn_readfirstlane((nfull - 4) >> 2);
  const int rem = __builtin_amdgcn_readfirstlane((nfull - 4) & 3);
  if constexpr (CAT) {
    uint32_t rrow = 3 * 64 + lane, tmp;
    asm volatile(SR_ATTN_BWD_PIPE_ASM_CAT
                 : [dk00] "+&a"(dk[0][0]), [dk01] "+&a"(dk[0][1]), [dk10] "+&a"(dk[1][0]), [dk11] "+&a"(dk[1][1]),
                   [dv00] "+&a"(dv[0][0]), [dv01] "+&a"(dv[0][1]), [dv10] "+&a"(dv[1][0]), [dv11] "+&a"(dv[1][1]),
                   [dma0] "+&v"(dma0), [dma1] "+&v"(dma1), [lofs] "+&v"(lofs), [n] "+&s"(nn),
                     [rrow] "+&v"(rrow), [tmp] "=&v"(tmp)
                 : [k00] "v"(kf[0][0]), [k01] "v"(kf[0][1]), [k02] "v"(kf[0][2]), [k03] "v"(kf[0][3]),
                   [k10] "v"(kf[1][0]), [k11] "v"(kf[1][1]), [k12] "v"(kf[1][2]), [k13] "v"(kf[1][3]),
                   [v00] "v"(vf[0][0]), [v01] "v"(vf[0][1]), [v02] "v"(vf[0][2]), [v03] "v"(vf[0][3]),
                   [v10] "v"(vf[1][0]), [v11] "v"(vf[1][1]), [v12] "v"(vf[1][2]), [v13] "v"(vf[1][3]),
                   [ra0] "v"(ra[0]), [ra1] "v"(ra[1]), [ra2] "v"(ra[2]), [ra3] "v"(ra[3]),
                   [ta00] "v"(ta00), [ta01] "v"(ta01), [ta10] "v"(ta10), [ta11] "v"(ta11), [sa] "v"(sa),
                   [ldsv] "s"(ldsv), [ldsl] "s"(ldsl), [sp] "s"(spb), [sp2] "s"(spb2), [lp] "s"(lpb),
                   [sstep] "s"(sstep), [rem] "s"(rem), [mgc] "s"(mgc), [msh] "s"(msh), [istr] "s"(istr)
                 : SR_ATTN_BWD_PIPE_CLOBBERS, "memory", "m0", "scc");
  } else {
    asm volatile(SR_ATTN_BWD_PIPE_ASM
                 : [dk00] "+&a"(dk[0][0]), [dk01] "+&a"(dk[0][1]), [dk10] "+&a"(dk[1][0]), [dk11] "+&a"(dk[1][1]),
                   [dv00] "+&a"(dv[0][0]), [dv01] "+&a"(dv[0][1]), [dv10] "+&a"(dv[1][0]), [dv11] "+&a"(dv[1][1]),
                   [dma0] "+&v"(dma0), [dma1] "+&v"(dma1), [lofs] "+&v"(lofs), [n] "+&s"(nn)
                 : [k00] "v"(kf[0][0]), [k01] "v"(kf[0][1]), [k02] "v"(kf[0][2]), [k03] "v"(kf[0][3]),
                   [k10] "v"(kf[1][0]), [k11] "v"(kf[1][1]), [k12] "v"(kf[1][2]), [k13] "v"(kf[1][3]),
                   [v00] "v"(vf[0][0]), [v01] "v"(vf[0][1]), [v02] "v"(vf[0][2]), [v03] "v"(vf[0][3]),
                   [v10] "v"(vf[1][0]), [v11] "v"(vf[1][1]), [v12] "v"(vf[1][2]), [v13] "v"(vf[1][3]),
                   [ra0] "v"(ra[0]), [ra1] "v"(ra[1]), [ra2] "v"(ra[2]), [ra3] "v"(ra[3]),
                   [ta00] "v"(ta00), [ta01] "v"(ta01), [ta10] "v"(ta10), [ta11] "v"(ta11), [sa] "v"(sa),
                   [ldsv] "s"(ldsv), [ldsl] "s"(ldsl), [sp] "s"(spb), [sp2] "s"(spb2), [lp] "s"(lpb),
                   [sstep] "s"(sstep), [rem] "s"(rem)
                 : SR_ATTN_BWD_PIPE_CLOBBERS, "memory", "m0", "scc");
  }
  if (qv) dkdv_tile<2, true>(smem + RAG, qv, kf, vf, dk, dv, tro, l32, hi);
  store_dkdv<SEG, 2>(b, kb0, key_base, len, hcol, hi, dk, dv);
}

// ---------------------------------------------------------------- dQ
// One 64-key tile of the dQ sweep for one 32-query block (lane: query l32): kt = the tile's LDS
// stage (K tile | V tile), valid = its keys (MASKED only: keys past it get P = 0), qf = c q, nl /
// nd = -lse / the stored -delta of the lane's query broadcast.  S'^T = K (cQ)^T - lse,
// dP'^T = V dO^T - delta, dS = exp2(S') dP'; dQ^T += K^T dS^T.
template <bool MASKED>
__device__ __forceinline__ void dq_tile(const char* kt, int valid, const bf16x8 (&qf)[4], const bf16x8 (&of)[4],
                                        const f32x16& nl, const f32x16& nd, f32x16 (&dq)[2], const TrOff& tro,
                                        int l32, int hi) {
  const char* vt = kt + TB;
  f32x16 sc[2], dp[2];
  bf16x8 fk[4][2], fv[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      fk[s][kb] = row_frag(kt, kb * 32 + l32, s, hi);
      fv[s][kb] = row_frag(vt, kb * 32 + l32, s, hi);
    }
#pragma unroll
  for (int s = 0; s < 4; ++s)  // four independent accumulation chains in flight
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      sc[kb] = mfma32(fk[s][kb], qf[s], s == 0 ? nl : sc[kb]);  // S^T = K (cQ)^T - lse
      dp[kb] = mfma32(fv[s][kb], of[s], s == 0 ? nd : dp[kb]);  // dP^T = V dO^T - delta
    }
  if constexpr (MASKED) {  // partial key tile: keys >= valid get S' = -inf, P = 0
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (kb * 32 + acc_row(r, hi) >= valid) sc[kb][r] = -INFINITY;
  }
  // one code path for every tile: a masked copy of the dS / dQ block made the compiler join
  // two register assignments of dq with 64 v_mov per tile
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      f32x8 d8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = 8 * s2 + j;
        d8[j] = __builtin_amdgcn_exp2f(sc[kb][r]) * dp[kb][r];
      }
      const bf16x8 df = __builtin_convertvector(d8, bf16x8);
      const int row0 = kb * 32 + 16 * s2;
#pragma unroll
      for (int db = 0; db < 2; ++db) dq[db] = mfma32(tr_frag(kt, row0, tro.off[db]), df, dq[db]);  // dQ^T += K^T dS^T
    }
}

// grid (query tiles of 128, heads, batch); wave w owns query rows tile*128 + 32 w + l32.
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(sr_attn_bwd_desc b) {
  __shared__ __attribute__((aligned(16))) char smem[NBUF * 2 * TB];  // ring of K tile | V tile stages
  const sr_attn_desc& f = b.f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int head = blockIdx.y, hcol = head * 64, item = blockIdx.z;
  const int qrow = blockIdx.x * 128 + wave * 32 + l32;
  const int qrc = min(qrow, f.lq - 1);
  const int64_t qr = (int64_t)item * f.q_bstride + qrc;
  const float c = f.scale * 1.4426950408889634f;

  // key tiles of both segments in order (segment 0 then 1) through the LDS-DMA ring: wave w
  // issues row groups g = 4 (w & 1) .. + 3 of the K (waves 0, 1) or V (2, 3) tile.  Segment
  // bases are selected once, outside the loop.
  const int nt0 = (f.l0 + 63) / 64, nt1 = f.l1 > 0 ? (f.l1 + 63) / 64 : 0, ntiles = nt0 + nt1;
  const uint32_t lds0 = sr::lds_addr(smem);
  const bool stage_v = wave_u >= 2;
  const bf16* const sb0 = (const bf16*)(stage_v ? f.v0 : f.k0) + (int64_t)item * f.k0_bstride * (stage_v ? f.ldv0 : f.ldk0) + hcol;
  const bf16* const sb1 = f.l1 > 0 ? (const bf16*)(stage_v ? f.v1 : f.k1) + (int64_t)item * f.k1_bstride * (stage_v ? f.ldv1 : f.ldk1) + hcol
                                   : sb0;
  const int64_t sld0 = stage_v ? f.ldv0 : f.ldk0, sld1 = stage_v ? f.ldv1 : f.ldk1;
  const int g0 = 4 * (wave_u & 1);
  const uint32_t offA0 = piece_off(sld0, 0, lane), offB0 = piece_off(sld0, 1, lane);
  const uint32_t offA1 = piece_off(sld1, 0, lane), offB1 = piece_off(sld1, 1, lane);
  auto stage = [&](int t) {
    const bool s1 = t >= nt0;
    const uint32_t sb = lds0 + (t & (NBUF - 1)) * 2 * TB + (stage_v ? TB : 0);
    const bf16* base = s1 ? sb1 : sb0;
    const int64_t ld = s1 ? sld1 : sld0;
    const int r0 = (s1 ? t - nt0 : t) * 64, len = s1 ? f.l1 : f.l0;
    if (r0 + 64 <= len) {  // full tile: scalar pointers
      const char* p = (const char*)(base + (int64_t)(r0 + 8 * g0) * ld);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        sr::dma16_s(p + (int64_t)8 * i * ld * 2, (i & 1) ? (s1 ? offB1 : offB0) : (s1 ? offA1 : offA0),
                    sb + (g0 + i) * 1024);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) dma_rows(base, ld, r0, len, g0 + i, lane, sb);
    }
  };
  for (int i = 0; i < NBUF - 1 && i < ntiles; ++i) stage(i);

  bf16x8 qf[4], of[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = *(const bf16x8*)((const bf16*)f.q + qr * f.ldq + hcol + 16 * s + 8 * hi);
    of[s] = *(const bf16x8*)((const bf16*)b.dout + qr * b.lddo + hcol + 16 * s + 8 * hi);
  }
  const int64_t lrow = ((int64_t)item * f.heads + head) * f.lq + qrc;
  const float lse = f.lse[lrow], dlt = b.delta[lrow];
  __builtin_amdgcn_s_waitcnt(0);  // retire these loads with a wait the compiler sees (see dK, dV)
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[s][j] = (bf16)((float)qf[s][j] * c);
  // the S / dP chains of every tile start from -lse / -delta (this lane's query row in every
  // accumulator entry; delta is stored negated), so they return S' = c q.k - lse and dP' = dO.v - delta
  f32x16 nl, nd;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    nl[i] = -lse;
    nd[i] = dlt;  // the stored -delta
  }
  const TrOff tro = tr_offsets(lane);
  f32x16 dq[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) dq[0][i] = dq[1][i] = 0.f;
  // one key tile; MASKED (a segment's ragged last tile) is its own instantiation, so the full-tile
  // body is one basic block the compiler can interleave (see attn_bwd_dkdv_kernel)
  auto tile_body = [&](int t, auto masked) __attribute__((always_inline)) {
    if (t + 2 < ntiles) wait_vm<8>();  // tile t landed; t+1, t+2 stay in flight (4 per stage)
    else if (t + 1 < ntiles) wait_vm<4>();
    else wait_vm<0>();
    sr::barrier_raw();  // every wave is done with tile t-1, whose buffer stage t+3 reuses
    if (t + NBUF - 1 < ntiles) stage(t + NBUF - 1);
    int valid = 64;
    if constexpr (decltype(masked)::value) {
      const int seg = t >= nt0;
      valid = (seg ? f.l1 : f.l0) - (seg ? t - nt0 : t) * 64;
    }
    dq_tile<decltype(masked)::value>(smem + (t & (NBUF - 1)) * 2 * TB, valid, qf, of, nl, nd, dq, tro, l32, hi);
  };
  const int rag0 = f.l0 % 64 ? nt0 - 1 : -1, rag1 = nt1 > 0 && f.l1 % 64 ? ntiles - 1 : -1;
  for (int t = 0; t < ntiles; ++t) {
    if (t == rag0 || t == rag1) tile_body(t, std::true_type{});
    else tile_body(t, std::false_type{});
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

// ---------------------------------------------------------------- dQ: hand-scheduled sweep
// attn_bwd_dq_kernel's work as ONE inline-asm statement per key segment (tools/gen_attn_bwd_pipe.py,
// SR_ATTN_BWD_DQ_ASM): one wave per SIMD, 64 queries per wave (two query blocks sharing every K / V
// fragment read), 256 per workgroup, the two blocks pipelined half a tile apart like the dK/dV
// sweep.  Per segment: its first three tiles and its ragged last tile (l % 64 rows, into a fifth LDS
// stage) are staged, the asm sweeps the full tiles, then the compiled dq_tile runs the ragged one.
// Segment 1 follows segment 0 after a barrier.  Every dQ accumulation therefore happens in the
// compiled kernel's order (segment 0's tiles, its ragged tile, segment 1's ...): bit-identical
// outputs.  The host picks this kernel when every segment has at least 4 full key tiles.
//   LDS: ring of 4 x (K tile | V tile) at 0 .. 64 KB, the ragged stage after it.
template <int NSEG>
__global__ __launch_bounds__(256, 1) void attn_bwd_dq_pipe_kernel(sr_attn_bwd_desc b) {
  constexpr int SLOT = 2 * TB, RAG = 4 * SLOT;
  __shared__ __attribute__((aligned(16))) char smem[RAG + 2 * TB];
  const sr_attn_desc& f = b.f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int head = blockIdx.y, hcol = head * 64, item = blockIdx.z;
  const int q0 = blockIdx.x * 256 + wave * 64;  // queries of block qb: q0 + 32 qb + l32
  const float c = f.scale * 1.4426950408889634f;
  const uint32_t lds0 = sr::lds_addr(smem);
  const bool stage_v = wave_u >= 2;  // wave w copies row groups 4 (w & 1) .. + 3 of the K (waves 0, 1) or V (2, 3) tile
  const int g0 = 4 * (wave_u & 1);
  const uint32_t ldsv = __builtin_amdgcn_readfirstlane(lds0 + (stage_v ? TB : 0) + g0 * 1024);

  bf16x8 qf[2][4], of[2][4];
  float lse[2], dlt[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qrc = min(q0 + 32 * qb + l32, f.lq - 1);
    const int64_t qr = (int64_t)item * f.q_bstride + qrc;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[qb][s] = *(const bf16x8*)((const bf16*)f.q + qr * f.ldq + hcol + 16 * s + 8 * hi);
      of[qb][s] = *(const bf16x8*)((const bf16*)b.dout + qr * b.lddo + hcol + 16 * s + 8 * hi);
    }
    const int64_t lrow = ((int64_t)item * f.heads + head) * f.lq + qrc;
    lse[qb] = f.lse[lrow];
    dlt[qb] = b.delta[lrow];
  }
  __builtin_amdgcn_s_waitcnt(0);
  f32x16 nl[2], nd[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[qb][s][j] = (bf16)((float)qf[qb][s][j] * c);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      nl[qb][i] = -lse[qb];
      nd[qb][i] = dlt[qb];  // the stored -delta
    }
  }
  const TrOff tro = tr_offsets(lane);
  f32x16 dq[2][2];
#pragma unroll
  for (int i = 0; i < 16; ++i) dq[0][0][i] = dq[0][1][i] = dq[1][0][i] = dq[1][1][i] = 0.f;
  uint32_t ra[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) ra[s] = lds0 + l32 * 128 + swz(l32, 2 * s + hi) * 16;
  const uint32_t ta00 = lds0 + tro.off[0][0], ta01 = lds0 + tro.off[0][1];
  const uint32_t ta10 = lds0 + tro.off[1][0], ta11 = lds0 + tro.off[1][1];

#pragma unroll
  for (int seg = 0; seg < NSEG; ++seg) {  // NSEG = 1 + (l1 > 0), a template so that one segment compiles alone
    if (seg) __syncthreads();  // every wave is done with segment 0's ring and ragged stage
    const int len = seg ? f.l1 : f.l0;
    const int nfull = len / 64, kv = len % 64;  // nfull >= 4 (host)
    const int64_t sld = stage_v ? (seg ? f.ldv1 : f.ldv0) : (seg ? f.ldk1 : f.ldk0);
    const void* kvp = stage_v ? (seg ? f.v1 : f.v0) : (seg ? f.k1 : f.k0);
    const bf16* const sb = (const bf16*)kvp + (int64_t)item * (seg ? f.k1_bstride : f.k0_bstride) * sld + hcol;
    const uint32_t offA = piece_off(sld, 0, lane), offB = piece_off(sld, 1, lane);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const char* p = (const char*)(sb + (int64_t)(t * 64 + 8 * g0) * sld);
#pragma unroll
      for (int i = 0; i < 4; ++i) sr::dma16_s(p + (int64_t)8 * i * sld * 2, (i & 1) ? offB : offA, ldsv + t * SLOT + i * 1024);
    }
    if (kv) {  // the ragged last key tile: rows clamped to len - 1 (P = 0 for them: dq_tile<true>)
#pragma unroll
      for (int i = 0; i < 4; ++i) dma_rows(sb, sld, nfull * 64, len, g0 + i, lane, lds0 + RAG + (stage_v ? TB : 0));
    }
    __builtin_amdgcn_s_waitcnt(0);  // the prologue stages
    const uint64_t spu = (uint64_t)(uintptr_t)(sb + (int64_t)(3 * 64 + 8 * g0) * sld);
    const uint32_t sp_lo = __builtin_amdgcn_readfirstlane((uint32_t)spu);
    const uint32_t sp_hi = __builtin_amdgcn_readfirstlane((uint32_t)(spu >> 32));
    const char* spb = (const char*)(uintptr_t)(((uint64_t)sp_hi << 32) | sp_lo);
    const char* spb2 = spb + 16 * sld * 2;
    uint32_t dma0 = offA, dma1 = offB + (uint32_t)(8 * sld * 2);
    const uint32_t sstep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * sld * 2));
    int nn = __builtin_amdgcn_readfirstlane((nfull - 4) >> 2);
    const int rem = __builtin_amdgcn_readfirstlane((nfull - 4) & 3);
    asm volatile(SR_ATTN_BWD_DQ_ASM
                 : [dq00] "+&a"(dq[0][0]), [dq01] "+&a"(dq[0][1]), [dq10] "+&a"(dq[1][0]), [dq11] "+&a"(dq[1][1]),
                   [dma0] "+&v"(dma0), [dma1] "+&v"(dma1), [n] "+&s"(nn)
                 : [q00] "a"(qf[0][0]), [q01] "a"(qf[0][1]), [q02] "a"(qf[0][2]), [q03] "a"(qf[0][3]),
                   [q10] "a"(qf[1][0]), [q11] "a"(qf[1][1]), [q12] "a"(qf[1][2]), [q13] "a"(qf[1][3]),
                   [o00] "a"(of[0][0]), [o01] "a"(of[0][1]), [o02] "a"(of[0][2]), [o03] "a"(of[0][3]),
                   [o10] "a"(of[1][0]), [o11] "a"(of[1][1]), [o12] "a"(of[1][2]), [o13] "a"(of[1][3]),
                   [nl0] "v"(nl[0]), [nl1] "v"(nl[1]), [nd0] "v"(nd[0]), [nd1] "v"(nd[1]),
                   [ra0] "v"(ra[0]), [ra1] "v"(ra[1]), [ra2] "v"(ra[2]), [ra3] "v"(ra[3]),
                   [ta00] "v"(ta00), [ta01] "v"(ta01), [ta10] "v"(ta10), [ta11] "v"(ta11),
                   [ldsv] "s"(ldsv), [sp] "s"(spb), [sp2] "s"(spb2), [sstep] "s"(sstep), [rem] "s"(rem)
                 : SR_ATTN_BWD_DQ_CLOBBERS, "memory", "m0", "scc");
    if (kv) {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) dq_tile<true>(smem + RAG, kv, qf[qb], of[qb], nl[qb], nd[qb], dq[qb], tro, l32, hi);
    }
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qrow = q0 + 32 * qb + l32;
    if (qrow < f.lq) {
      float* dqp = b.dq + ((int64_t)item * f.q_bstride + qrow) * b.lddq + hcol;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *(float4*)(dqp + db * 32 + 8 * g + 4 * hi) =
              make_float4(dq[qb][db][4 * g] * f.scale, dq[qb][db][4 * g + 1] * f.scale, dq[qb][db][4 * g + 2] * f.scale,
                          dq[qb][db][4 * g + 3] * f.scale);
    }
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
  SR_CHECK(!f.q_scaled, SR_EUNSUPPORTED, "sr_attention_bwd: q_scaled (a forward-only convention) is not supported");
  SR_CHECK(f.l1 == 0 || (f.k1 && f.v1 && b.dk1 && b.dv1), SR_EINVAL, "sr_attention_bwd: segment 1 needs k1/v1/dk1/dv1");
  SR_CHECK(f.ldq % 8 == 0 && f.ldk0 % 8 == 0 && f.ldv0 % 8 == 0 && f.ldo % 8 == 0 && b.lddo % 8 == 0 &&
               b.lddq % 4 == 0 && b.lddk0 % 4 == 0 && b.lddv0 % 4 == 0 &&
               (f.l1 == 0 || (f.ldk1 % 8 == 0 && f.ldv1 % 8 == 0 && b.lddk1 % 4 == 0 && b.lddv1 % 4 == 0)),
           SR_EINVAL, "sr_attention_bwd: leading dims (bf16 multiples of 8, fp32 multiples of 4)");
  hipStream_t s = (hipStream_t)stream;
  const int64_t nrows = (int64_t)f.batch * f.heads * f.lq;
  hipLaunchKernelGGL(attn_bwd_delta_kernel, dim3((unsigned)std::min<int64_t>((nrows * 8 + 255) / 256, 1 << 20)),
                     dim3(256), 0, s, b);
  // dQ: the hand-scheduled sweep (SR_ATTN_BWD_DQ_PIPE) where every key segment has at least 4 full
  // tiles and 32-bit per-lane DMA offsets, and where its 256-query workgroups pad the query count by
  // at most 2 % more than the compiled sweep's 128 or the key sweep is long enough to carry the
  // padding (frames of 1,374 tokens: 1,536 against 1,408 rows over 1,374 keys, measured 1-3 %
  // slower, forced 16 % slower; the reloc block's 1,374-row items over 9,984 + 1,374 keys: 3 %
  // faster, profiles/r05_j22_kbwd.log); else the compiled sweep
  const int64_t qpad256 = (f.lq + 255) / 256 * 256, qpad128 = (f.lq + 127) / 128 * 128;
  const bool dq_pipe = sr::tune(SR_TUNE_ATTN_BWD_DQ_PIPE) != 0 && f.l0 >= 256 && (f.l1 == 0 || f.l1 >= 256) &&
                       (int64_t)(f.l0 + 64) * std::max<int64_t>(f.ldk0, f.ldv0) * 2 < ((int64_t)1 << 31) &&
                       (f.l1 == 0 || (int64_t)(f.l1 + 64) * std::max<int64_t>(f.ldk1, f.ldv1) * 2 < ((int64_t)1 << 31)) &&
                       (sr::tune(SR_TUNE_ATTN_BWD_DQ_PIPE) == 2 || qpad256 * 100 <= qpad128 * 102 ||
                        (int64_t)f.l0 + f.l1 >= 4096);
  if (dq_pipe && f.l1 > 0)
    hipLaunchKernelGGL(attn_bwd_dq_pipe_kernel<2>, dim3((f.lq + 255) / 256, f.heads, f.batch), dim3(256), 0, s, b);
  else if (dq_pipe)
    hipLaunchKernelGGL(attn_bwd_dq_pipe_kernel<1>, dim3((f.lq + 255) / 256, f.heads, f.batch), dim3(256), 0, s, b);
  else
    hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3((f.lq + 127) / 128, f.heads, f.batch), dim3(256), 0, s, b);
  // dK / dV: the hand-scheduled sweep (SR_ATTN_BWD_PIPE) where a workgroup sweeps one item's
  // queries, at least 4 full query tiles, with 32-bit per-lane DMA offsets; else the compiled sweep
  hipStream_t ks = s;
  const int64_t ldmax = std::max<int64_t>(f.ldq, b.lddo);
  const bool pipe_ok = sr::tune(SR_TUNE_ATTN_BWD_PIPE) != 0 && f.lq >= 256 &&
                       (int64_t)(f.lq + 64) * ldmax * 2 < ((int64_t)1 << 31);
  constexpr int kr = 128;  // keys per workgroup of the compiled sweep
  const char* name = nullptr;
  for (int seg = 0; seg < (f.l1 > 0 ? 2 : 1); ++seg) {
    const int len = seg == 0 ? f.l0 : f.l1;
    const bool shared = (seg == 0 ? f.k0_bstride : f.k1_bstride) == 0;
    const int nz = shared ? 1 : f.batch;
    if (pipe_ok && (!shared || f.batch == 1)) {
      const dim3 g((len + 255) / 256, f.heads, nz);
      if (seg == 0) hipLaunchKernelGGL((attn_bwd_dkdv_pipe_kernel<0>), g, dim3(256), 0, ks, b);
      else hipLaunchKernelGGL((attn_bwd_dkdv_pipe_kernel<1>), g, dim3(256), 0, ks, b);
      if (seg == 0) name = "attn_bwd_dkdv_pipe_kernel<0>";
      continue;
    }
    // keys shared by a batch > 1 with the items' queries in consecutive rows: one asm sweep over the
    // concatenated queries (SR_ATTN_BWD_CAT)
    const int64_t lqt = (int64_t)f.batch * f.lq;
    if (shared && f.batch > 1 && sr::tune(SR_TUNE_ATTN_BWD_PIPE) != 0 && sr::tune(SR_TUNE_ATTN_BWD_CAT) != 0 &&
        f.q_bstride == f.lq && f.lq >= 2 && lqt >= 256 && lqt < (1 << 24) &&
        (lqt + 64) * ldmax * 2 < ((int64_t)1 << 31) && (int64_t)(f.heads - 1) * f.lq * 4 < (1 << 24)) {
      const dim3 g((len + 255) / 256, f.heads, 1);
      if (seg == 0) hipLaunchKernelGGL((attn_bwd_dkdv_pipe_kernel<0, true>), g, dim3(256), 0, ks, b);
      else hipLaunchKernelGGL((attn_bwd_dkdv_pipe_kernel<1, true>), g, dim3(256), 0, ks, b);
      if (seg == 0) name = "attn_bwd_dkdv_pipe_kernel<0, cat>";
      continue;
    }
    // keys shared by a batch > 1 otherwise: one workgroup sweeps every item's queries
    const dim3 g((len + kr - 1) / kr, f.heads, nz);
    if (seg == 0) {
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<0>), g, dim3(256), 0, ks, b);
      name = "attn_bwd_dkdv_kernel<0>";
    } else {
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<1>), g, dim3(256), 0, ks, b);
    }
  }
  sr::note_kernel("%s", name);
  return sr::check_launch("sr_attention_bwd");
}

// ---------------------------------------------------------------------------------------------
// Exact fp32 attention backward (sr_attention_bwd_f32): the same gradient as above for fp32
// operands, head_dim 64 | 128, any segment / batch layout of the forward, on the VALU in fp32
// with the softmax recomputed from the forward's LSE.  It serves TrainGraph's fp32 mode, whose
// gradients are checked against the oracle's fp32 autograd at 1e-4 (the bf16 graph can only be
// held to the reference's own bf16 noise).  No MFMA, no atomics: a thread owns one query row
// (dQ) or one key row (dK, dV; a key shared by every item sums over all of them in item order).
namespace {

constexpr int F32B_T = 128;  // rows (threads) per workgroup
constexpr int F32B_KT = 16;  // rows per LDS tile

__global__ __launch_bounds__(256) void attn_bwd_delta_f32_kernel(sr_attn_bwd_desc b) {
  const sr_attn_desc& f = b.f;
  const int64_t n = (int64_t)f.batch * f.heads * f.lq;
  const int64_t ob = f.o_bstride ? f.o_bstride : f.q_bstride;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int row = (int)(e % f.lq);
    const int64_t ih = e / f.lq;
    const int head = (int)(ih % f.heads), item = (int)(ih / f.heads);
    const int64_t r = (int64_t)item * ob + row;
    const float* o = (const float*)f.o + r * f.ldo + (int64_t)head * f.head_dim;
    const float* g = (const float*)b.dout + r * b.lddo + (int64_t)head * f.head_dim;
    float s = 0.f;
    for (int d = 0; d < f.head_dim; ++d) s = fmaf(g[d], o[d], s);
    b.delta[e] = s;  // [item][head][row]
  }
}

template <int D>
__global__ __launch_bounds__(F32B_T) void attn_bwd_dq_f32_kernel(sr_attn_bwd_desc b) {
  __shared__ float ks[F32B_KT][D];
  __shared__ float vs[F32B_KT][D];
  const sr_attn_desc& f = b.f;
  const int tid = threadIdx.x, head = blockIdx.y, item = blockIdx.z;
  const int hcol = head * D;
  const int qrow = blockIdx.x * F32B_T + tid, qc = min(qrow, f.lq - 1);
  const int64_t qr = (int64_t)item * f.q_bstride + qc;
  const int64_t orow = (int64_t)item * (f.o_bstride ? f.o_bstride : f.q_bstride) + qc;
  const float c = f.scale * 1.4426950408889634f;
  float q[D], g[D], dq[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    q[i] = ((const float*)f.q)[qr * f.ldq + hcol + i];
    g[i] = ((const float*)b.dout)[orow * b.lddo + hcol + i];
    dq[i] = 0.f;
  }
  const int64_t st = ((int64_t)item * f.heads + head) * f.lq + qc;
  const float lse = f.lse[st], dl = b.delta[st];
  for (int seg = 0; seg < 2; ++seg) {
    const int len = seg ? f.l1 : f.l0;
    if (len <= 0) continue;
    const float* kb = (const float*)(seg ? f.k1 : f.k0);
    const float* vb = (const float*)(seg ? f.v1 : f.v0);
    const int64_t ldk = seg ? f.ldk1 : f.ldk0, ldv = seg ? f.ldv1 : f.ldv0;
    const int64_t rb = (int64_t)item * (seg ? f.k1_bstride : f.k0_bstride);
    for (int t0 = 0; t0 < len; t0 += F32B_KT) {
      const int n = min(F32B_KT, len - t0);
      __syncthreads();
      for (int e = tid; e < F32B_KT * D; e += F32B_T) {
        const int r = e / D, cc = e - r * D, key = min(t0 + r, len - 1);
        ks[r][cc] = kb[(rb + key) * ldk + hcol + cc];
        vs[r][cc] = vb[(rb + key) * ldv + hcol + cc];
      }
      __syncthreads();
      for (int j = 0; j < n; ++j) {
        float s = 0.f, dp = 0.f;
#pragma unroll
        for (int i = 0; i < D; ++i) {
          s = fmaf(q[i], ks[j][i], s);
          dp = fmaf(g[i], vs[j][i], dp);
        }
        const float p = exp2f(s * c - lse);
        const float ds = p * (dp - dl);
#pragma unroll
        for (int i = 0; i < D; ++i) dq[i] = fmaf(ds, ks[j][i], dq[i]);
      }
    }
  }
  if (qrow < f.lq) {
    float* out = b.dq + qr * b.lddq + hcol;
#pragma unroll
    for (int i = 0; i < D; ++i) out[i] = dq[i] * f.scale;
  }
}

// key rows of segment SEG: blockIdx.z = the item owning them (bstride > 0) or 0 (shared keys: every
// item's queries, summed in item order)
template <int D, int SEG>
__global__ __launch_bounds__(F32B_T) void attn_bwd_dkdv_f32_kernel(sr_attn_bwd_desc b) {
  __shared__ float qs[F32B_KT][D];
  __shared__ float gs[F32B_KT][D];
  __shared__ float ls[F32B_KT], dls[F32B_KT];
  const sr_attn_desc& f = b.f;
  const int tid = threadIdx.x, head = blockIdx.y;
  const int hcol = head * D;
  const int len = SEG ? f.l1 : f.l0;
  const int64_t bstride = SEG ? f.k1_bstride : f.k0_bstride;
  const bool shared = bstride == 0;
  const int key = blockIdx.x * F32B_T + tid, kc = min(key, len - 1);
  const int64_t kr = (shared ? 0 : (int64_t)blockIdx.z * bstride) + kc;
  const float* kb = (const float*)(SEG ? f.k1 : f.k0);
  const float* vb = (const float*)(SEG ? f.v1 : f.v0);
  const int64_t ldk = SEG ? f.ldk1 : f.ldk0, ldv = SEG ? f.ldv1 : f.ldv0;
  const int64_t ob = f.o_bstride ? f.o_bstride : f.q_bstride;
  const float c = f.scale * 1.4426950408889634f;
  float k[D], v[D], dk[D], dv[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    k[i] = kb[kr * ldk + hcol + i];
    v[i] = vb[kr * ldv + hcol + i];
    dk[i] = 0.f;
    dv[i] = 0.f;
  }
  const int i0 = shared ? 0 : blockIdx.z, i1 = shared ? f.batch : blockIdx.z + 1;
  for (int item = i0; item < i1; ++item) {
    for (int t0 = 0; t0 < f.lq; t0 += F32B_KT) {
      const int n = min(F32B_KT, f.lq - t0);
      __syncthreads();
      for (int e = tid; e < F32B_KT * D; e += F32B_T) {
        const int r = e / D, cc = e - r * D, row = min(t0 + r, f.lq - 1);
        qs[r][cc] = ((const float*)f.q)[((int64_t)item * f.q_bstride + row) * f.ldq + hcol + cc];
        gs[r][cc] = ((const float*)b.dout)[((int64_t)item * ob + row) * b.lddo + hcol + cc];
      }
      if (tid < F32B_KT) {
        const int64_t stt = ((int64_t)item * f.heads + head) * f.lq + min(t0 + tid, f.lq - 1);
        ls[tid] = f.lse[stt];
        dls[tid] = b.delta[stt];
      }
      __syncthreads();
      for (int j = 0; j < n; ++j) {
        float s = 0.f, dp = 0.f;
#pragma unroll
        for (int i = 0; i < D; ++i) {
          s = fmaf(qs[j][i], k[i], s);
          dp = fmaf(gs[j][i], v[i], dp);
        }
        const float p = exp2f(s * c - ls[j]);
        const float ds = p * (dp - dls[j]);
#pragma unroll
        for (int i = 0; i < D; ++i) {
          dv[i] = fmaf(p, gs[j][i], dv[i]);
          dk[i] = fmaf(ds, qs[j][i], dk[i]);
        }
      }
    }
  }
  if (key < len) {
    float* odk = (SEG ? b.dk1 : b.dk0) + kr * (SEG ? b.lddk1 : b.lddk0) + hcol;
    float* odv = (SEG ? b.dv1 : b.dv0) + kr * (SEG ? b.lddv1 : b.lddv0) + hcol;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      odk[i] = dk[i] * f.scale;
      odv[i] = dv[i];
    }
  }
}

template <int D>
void launch_bwd_f32(const sr_attn_bwd_desc& b, hipStream_t s) {
  const sr_attn_desc& f = b.f;
  hipLaunchKernelGGL(attn_bwd_dq_f32_kernel<D>, dim3((f.lq + F32B_T - 1) / F32B_T, f.heads, f.batch), dim3(F32B_T),
                     0, s, b);
  const dim3 g0((f.l0 + F32B_T - 1) / F32B_T, f.heads, f.k0_bstride == 0 ? 1 : f.batch);
  hipLaunchKernelGGL((attn_bwd_dkdv_f32_kernel<D, 0>), g0, dim3(F32B_T), 0, s, b);
  if (f.l1 > 0) {
    const dim3 g1((f.l1 + F32B_T - 1) / F32B_T, f.heads, f.k1_bstride == 0 ? 1 : f.batch);
    hipLaunchKernelGGL((attn_bwd_dkdv_f32_kernel<D, 1>), g1, dim3(F32B_T), 0, s, b);
  }
}

}  // namespace

extern "C" int sr_attention_bwd_f32(sr_stream_t stream, const sr_attn_bwd_desc* desc) {
  SR_CHECK(desc, SR_EINVAL, "sr_attention_bwd_f32: null desc");
  const sr_attn_bwd_desc& b = *desc;
  const sr_attn_desc& f = b.f;
  SR_CHECK(f.q && f.k0 && f.v0 && f.o && f.lse && b.dout && b.delta && b.dq && b.dk0 && b.dv0, SR_EINVAL,
           "sr_attention_bwd_f32: null pointer");
  SR_CHECK((f.head_dim == 64 || f.head_dim == 128) && f.mask_mode == SR_MASK_NONE, SR_EUNSUPPORTED,
           "sr_attention_bwd_f32: head_dim 64 | 128 without mask only");
  SR_CHECK(f.batch > 0 && f.heads > 0 && f.lq > 0 && f.l0 > 0 && f.l1 >= 0, SR_EINVAL,
           "sr_attention_bwd_f32: bad sizes");
  SR_CHECK(!f.q_scaled, SR_EUNSUPPORTED, "sr_attention_bwd_f32: q_scaled is a bf16 forward convention");
  SR_CHECK(f.l1 == 0 || (f.k1 && f.v1 && b.dk1 && b.dv1), SR_EINVAL,
           "sr_attention_bwd_f32: segment 1 needs k1/v1/dk1/dv1");
  hipStream_t s = (hipStream_t)stream;
  const int64_t nrows = (int64_t)f.batch * f.heads * f.lq;
  hipLaunchKernelGGL(attn_bwd_delta_f32_kernel, dim3((unsigned)std::min<int64_t>((nrows + 255) / 256, 1 << 16)),
                     dim3(256), 0, s, b);
  if (f.head_dim == 64) launch_bwd_f32<64>(b, s);
  else launch_bwd_f32<128>(b, s);
  sr::note_kernel("attn_bwd_dq_f32_kernel<%d>", f.head_dim);
  return sr::check_launch("sr_attention_bwd_f32");
}
