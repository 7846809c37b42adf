// Shared device helpers for the gfx950 (CDNA4) kernels of libsfm_amd.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sfm_amd.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

namespace sr {

// thread-local error message; set by host wrappers on failure
void set_error(const char* fmt, ...);
// after a call's launches: the runtime's launch error (and, under SR_TUNE_SYNC_CHECK, a
// device synchronisation's) -> SR_ELAUNCH with the message
int check_launch(const char* what);
// thread-local name of the kernel a call launched (sr_last_kernel), as rocprofv3 prints it
void note_kernel(const char* fmt, ...);
// current value of a tuning switch (sfm_amd.h sr_tuning_key)
int tune(int key);
// compute units of the current device (read once; 256 on MI355X)
int cu_count();

template <typename T> struct is_bf16 { static constexpr bool value = false; };
template <> struct is_bf16<bf16> { static constexpr bool value = true; };

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// Sum over the 16 lanes of a DPP row, left in every lane of the row (quad swaps, then the half-row
// and row mirrors; every lane adds the same two values at each step, so all 16 hold the same bits).
__device__ __forceinline__ float dpp_sum16(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));  // row_mirror
  return v;
}
// The value of lane l ^ 4 (within a DPP row): row_half_mirror (l -> 7 - l in each half row), then
// quad_perm 3,2,1,0 (l -> 3 - l in each quad) -- two DPP moves, no LDS permute.
__device__ __forceinline__ float dpp_xor4(float v) {
  const int m = __builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false);
  return __int_as_float(__builtin_amdgcn_mov_dpp(m, 0x1B, 0xF, 0xF, false));
}

__device__ __forceinline__ float gelu_erf(float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }

// erf-GELU for bf16 outputs: erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below
// the 2^-9 rounding of the bf16 result), 2 transcendentals + ~9 VALU instead of erff's ~35.
//   erf(|z|) = 1 - t (a1 + t (a2 + t (a3 + t (a4 + t a5)))) exp(-z^2),  t = 1 / (1 + p |z|)
//   gelu(x)  = x (1 + erf(x / sqrt2)) / 2 = max(x, 0) - |x| h,  h = poly exp(-z^2) / 2
// h(x) = (1 - erf(|x| / sqrt2)) / 2 = Phi(-|x|) by A&S 7.1.26; 1/sqrt2 is folded into p and into
// the exponent, the 1/2 into the (exactly halved) coefficients.
__device__ __forceinline__ float phi_tail_fast(float x) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, fabsf(x), 1.0f));
  float poly = fmaf(0.5f * 1.061405429f, t, 0.5f * -1.453152027f);
  poly = fmaf(poly, t, 0.5f * 1.421413741f);
  poly = fmaf(poly, t, 0.5f * -0.284496736f);
  poly = fmaf(poly, t, 0.5f * 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);
  return poly * t * e;
}
__device__ __forceinline__ float gelu_erf_fast(float x) { return fmaf(-fabsf(x), phi_tail_fast(x), fmaxf(x, 0.f)); }

// d/dx gelu_erf(x) = Phi(x) + x phi(x)  (backward of mlp.py:36's nn.GELU); `fast` uses the
// A&S erf of gelu_erf_fast (bf16 gradients), otherwise erff (exact fp32).
template <bool fast>
__device__ __forceinline__ float gelu_erf_grad(float x) {
  float cdf;
  if constexpr (fast) {
    const float h = phi_tail_fast(x);
    cdf = x >= 0.f ? 1.f - h : h;
  } else {
    cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  }
  return cdf + x * 0.3989422804014327f * __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);
}

// 2-D RoPE position (y, x) of GEMM / token row `row` (rope.py:40-66 via PositionGetter):
// explicit pos_yx, else the token row (pos_rowmap[row] or pos_row_base + row) inside a frame
// of tokens_per_frame rows, patches after patch_start, (0, 0) for the special tokens.
__device__ __forceinline__ void rope_pos(const sr_gemm_epi& ep, int row, int& py, int& px) {
  py = 0;
  px = 0;
  if (ep.pos_yx) {
    py = ep.pos_yx[2 * row];
    px = ep.pos_yx[2 * row + 1];
  } else {
    const int64_t tr = ep.pos_rowmap ? (int64_t)ep.pos_rowmap[row] : ep.pos_row_base + row;
    const int t = (int)(tr % ep.tokens_per_frame);
    if (t >= ep.patch_start) {
      const int p = t - ep.patch_start;
      py = p / ep.grid_w + 1;
      px = p - (py - 1) * ep.grid_w + 1;
    }
  }
}

// v[l] + v[l ^ 16] and v[l] + v[l ^ 32] through the gfx950 row-swap permutes (one VALU op each, no
// LDS round trip as __shfl_xor's ds_bpermute has); the even row's value is always the left operand,
// so both lanes of a pair get the same bits
__device__ __forceinline__ float sum_x16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float sum_x32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// raw workgroup barrier that does NOT drain in-flight LDS-DMA (vmcnt); memory clobbers keep
// the compiler from moving LDS accesses across it.
__device__ __forceinline__ void barrier_raw() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LDS address (32-bit) of a __shared__ pointer.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// One LDS-DMA wave-instruction: lane l copies 16 B from gptr (per lane) to
// LDS[lds_base + 16*l] (lds_base wave-uniform).  Issued from inline asm so that the
// compiler's waitcnt pass does not see an aliasing LDS write and drain it with
// vmcnt(0) before every ds_read; the caller owns the counted s_waitcnt vmcnt(N).
__device__ __forceinline__ void dma16(const void* gptr, uint32_t lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr), "s"(lds_base)
               : "memory", "m0");
}
// 4-byte variant: lane l copies one dword to LDS[lds_base + 4*l] (256 B per wave-instruction).
__device__ __forceinline__ void dma4(const void* gptr, uint32_t lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(gptr), "s"(lds_base)
               : "memory", "m0");
}
// Same with a wave-uniform 64-bit base (SGPR pair) + per-lane 32-bit byte offset: the
// address arithmetic of a tile walk stays on the scalar unit.
// The base is wave-uniform by contract; readfirstlane pins it to SGPRs where the compiler's
// divergence analysis lost track (it folds away when the value already lives in SGPRs).
__device__ __forceinline__ void dma16_s(const void* sbase, uint32_t voff, uint32_t lds_base) {
  const uint64_t a = (uint64_t)(uintptr_t)sbase;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  sbase = (const void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_base)
               : "memory", "m0");
}
// 4-byte form of dma16_s (lane l's dword at sbase + voff to LDS[lds_base + 4*l]).
__device__ __forceinline__ void dma4_s(const void* sbase, uint32_t voff, uint32_t lds_base) {
  const uint64_t a = (uint64_t)(uintptr_t)sbase;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  sbase = (const void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_base)
               : "memory", "m0");
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks that share an XCD (same b % 8) get a contiguous range of logical tiles.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, local = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + local;
}

}  // namespace sr

#define SR_CHECK(cond, code, ...)     \
  do {                                \
    if (!(cond)) {                    \
      sr::set_error(__VA_ARGS__);     \
      return (code);                  \
    }                                 \
  } while (0)
