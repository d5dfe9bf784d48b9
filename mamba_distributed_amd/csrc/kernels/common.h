// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
//
// * wave64 everywhere: lane = threadIdx.x & 63, reductions over 64 lanes.
// * bf16 stored as raw 16-bit words (`bf16_t`), converted with v_cvt_pk_bf16_f32 (RNE, NaN-safe)
//   via the HIP intrinsic; loads are 16-byte vectors wherever alignment allows (Guideline 13).
// * every launcher takes an explicit hipStream_t (the caller's torch stream) and never syncs,
//   so all launches are hipGraph-capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <algorithm>
#include "types.h"

namespace mamba_amd {

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __bfloat16_as_ushort(__float2bfloat16(f));
}

// generic scalar load/store by element type
template <typename T> __device__ __forceinline__ float ld(const T* p);
template <> __device__ __forceinline__ float ld<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T> __device__ __forceinline__ void st(T* p, float v);
template <> __device__ __forceinline__ void st<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// 4-element vector load/store (8 B for bf16, 16 B for f32) — p must be aligned accordingly
template <typename T> __device__ __forceinline__ void ld4(const T* p, float (&o)[4]);
template <> __device__ __forceinline__ void ld4<float>(const float* p, float (&o)[4]) {
  float4 v = *reinterpret_cast<const float4*>(p);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <> __device__ __forceinline__ void ld4<bf16_t>(const bf16_t* p, float (&o)[4]) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
}
template <typename T> __device__ __forceinline__ void st4(T* p, const float (&o)[4]);
template <> __device__ __forceinline__ void st4<float>(float* p, const float (&o)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
}
// two floats -> two RNE bf16 in one dword (one v_cvt_pk_bf16_f32; NaN stays NaN)
typedef __bf16 mamba_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float mamba_f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((mamba_f32x2_t){a, b}, mamba_bf16x2_t));
}
template <> __device__ __forceinline__ void st4<bf16_t>(bf16_t* p, const float (&o)[4]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
}

// 8 x bf16 = 16 B
__device__ __forceinline__ void ld8bf(const bf16_t* p, float (&o)[8]) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8bf(bf16_t* p, const float (&o)[8]) {
  *reinterpret_cast<uint4*>(p) = make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]),
                                            pack2(o[6], o[7]));
}

// Whole-wave reductions on the VALU: DPP butterflies inside each 16-lane row (quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror), then the four rows meet through v_permlane32_swap / v_permlane16_swap (gfx950).
// The __shfl_xor form is six ds_bpermute_b32 LDS round trips in a dependent chain (~100 cycles each); this one is
// eight VALU instructions.  Every lane gets the total; the summation order is fixed (deterministic).
// v_permlane{32,16}_swap x, y: x <- [x_lo, y_lo], y <- [x_hi, y_hi] (32-lane halves) and x <- [x_r0, y_r0, x_r2,
// y_r2], y <- [x_r1, y_r1, x_r3, y_r3] (16-lane rows); with x = y = v, x + y is v[l] + v[l ^ 32] (resp. ^ 16).
// Inline asm: this ROCm's builtins return the first result twice.  s_nop 1: VALU write -> swap read.
__device__ __forceinline__ float wave_rows_combine_sum(float v) {
  float x = v, y = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  v = x + y;
  x = v; y = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  return x + y;
}
__device__ __forceinline__ float wave_rows_combine_max(float v) {
  float x = v, y = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  v = fmaxf(x, y);
  x = v; y = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  return fmaxf(x, y);
}
#define MAMBA_DPPF(v, ctrl) __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, (v)), (ctrl), 0xF, 0xF, false))
__device__ __forceinline__ float wave_sum(float v) {
  v += MAMBA_DPPF(v, 0xB1);
  v += MAMBA_DPPF(v, 0x4E);
  v += MAMBA_DPPF(v, 0x141);
  v += MAMBA_DPPF(v, 0x140);
  return wave_rows_combine_sum(v);
}
// Contract for wave_sum / wave_max: the whole wave is active (EXEC all ones; every call site is).  A DPP read from
// an inactive source lane returns `old`: 0 for the sum (its identity); for the max `old` is the lane's own value, so
// an inactive source can never win (a 0 would for all-negative rows).  v_permlane{32,16}_swap: gfx950 only.
#define MAMBA_DPPF_SELF(v, ctrl)                                                                              \
  __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, (v)), __builtin_bit_cast(int, (v)), \
                                                        (ctrl), 0xF, 0xF, false))
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, MAMBA_DPPF_SELF(v, 0xB1));
  v = fmaxf(v, MAMBA_DPPF_SELF(v, 0x4E));
  v = fmaxf(v, MAMBA_DPPF_SELF(v, 0x141));
  v = fmaxf(v, MAMBA_DPPF_SELF(v, 0x140));
  return wave_rows_combine_max(v);
}

// v_rcp_f32 (~1 ulp) instead of the IEEE division sequence: 1 instruction instead of ~10 and far
// fewer live registers in the unrolled element loops
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float siluf_(float x) { return x * sigmoidf_(x); }
__device__ __forceinline__ float softplusf_(float x) { return x <= 20.f ? log1pf(__expf(x)) : x; }
// softplus with hardware exp/log: log1p(y) = log(1+y) * y / ((1+y)-1) recovers the bits of y lost in
// 1+y, so the result keeps ~fp32 relative accuracy for very negative x (used where libm log1pf's
// register footprint would cost occupancy)
// Branch-free: softplus(x) = max(x, 0) + log1p(e^{-|x|}) -- inside unrolled per-element loops a
// branchy form costs an exec-mask diamond per element.
// Hardware v_exp_f32 / v_log_f32 (base 2) directly: the arguments never reach the denormal range
// the library wrappers guard against (-|x| log2e <= 0 -> y in (0, 1]; u in [1, 2]).
__device__ __forceinline__ float softplus_fast(float x) {
  const float y = __builtin_amdgcn_exp2f(-1.4426950408889634f * fabsf(x)), u = 1.f + y;
  const float l = __builtin_amdgcn_logf(u) * 0.6931471805599453f * y * __builtin_amdgcn_rcpf(u - 1.f);
  return fmaxf(x, 0.f) + (u == 1.f ? y : l);
}
// logistic with the hardware exp2 (exp2 -> +inf for very negative x gives rcp(inf) = 0)
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}

// XCD-aware remap of a linear block id (bijective for any grid size; MI355X has 8 XCDs and
// dispatches blocks round-robin over them, so ids b and b+8 share an L2).  Consecutive logical
// tiles land on the same XCD -> neighbouring tiles share L2 lines.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int nx = 8;
  int q = nblocks / nx, r = nblocks % nx;
  int xcd = bid % nx, idx = bid / nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace mamba_amd

#define MAMBA_HIP_CHECK(expr)                                                    \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess) return _e;                                             \
  } while (0)
