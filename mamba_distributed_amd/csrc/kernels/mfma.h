// MFMA / LDS fragment helpers for gfx950 (v_mfma_f32_16x16x32_bf16 + ds_read_b64_tr_b16).
//
// 16x16x32 bf16 operand maps (cdna_hip_programming.md §3):
//   A: lane l holds A[m = l&15][k = 8*(l>>4) + j], j = 0..7
//   B: lane l holds B[k = 8*(l>>4) + j][n = l&15]
//   D: lane l holds D[m = 4*(l>>4) + r][n = l&15], r = 0..3
// The hardware pairs A and B by (lane group g = l>>4, element j), so any permutation of k that
// is applied identically to both operands gives the same product.  Two orders are used:
//   STD : element j of group g <-> k = 8g + j
//   PERM: element j of group g <-> k = 4g + j (j < 4), 16 + 4g + (j-4) (j >= 4)
// PERM is the order in which two vertically stacked 16x16 accumulator tiles already sit in a
// lane (rows 4g..4g+3 of tile 0 and of tile 1), so an accumulator can feed the next MFMA
// as its A operand (summing over the tile's ROW index) with no data movement.
//
// LDS tiles are row-major bf16 [rows][ld].  Operands whose contraction index runs along an LDS
// row ("k-contiguous") are read with one ds_read_b128 (STD) or two ds_read_b64 (PERM); operands
// whose contraction index runs DOWN the rows (token-major activations, contracted over time) are
// read with two ds_read_b64_tr_b16 (hardware transpose): lane 4q+p of a 16-lane group supplies
// the address of row q, columns 4p..4p+3, and lane i receives column i of the 4 rows.
#pragma once
#include "common.h"

namespace mamba_amd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// k-contiguous operand, STD order: row r0 + (l&15), k0 + 8g .. +7
__device__ __forceinline__ bf16x8 frag_kc(const bf16_t* T, int ld, int r0, int k0) {
  const int l = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8*>(T + (r0 + (l & 15)) * ld + k0 + 8 * (l >> 4));
}
// k-contiguous operand, PERM order
__device__ __forceinline__ bf16x8 frag_kc_perm(const bf16_t* T, int ld, int r0, int k0) {
  const int l = threadIdx.x & 63, g = l >> 4;
  const bf16_t* row = T + (r0 + (l & 15)) * ld + k0;
  bf16x4 a = *reinterpret_cast<const bf16x4*>(row + 4 * g);
  bf16x4 b = *reinterpret_cast<const bf16x4*>(row + 16 + 4 * g);
  return cat8(a, b);
}

__device__ __forceinline__ bf16x4 tr4(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}
// k runs down the rows of T ([k][c] row-major); operand index = column c0 + (l&15); STD order
__device__ __forceinline__ bf16x8 frag_tr(const bf16_t* T, int ld, int k0, int c0) {
  const int l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const bf16_t* base = T + (k0 + 8 * g + (li >> 2)) * ld + c0 + 4 * (li & 3);
  return cat8(tr4(base), tr4(base + 4 * ld));
}
// same, PERM order
__device__ __forceinline__ bf16x8 frag_tr_perm(const bf16_t* T, int ld, int k0, int c0) {
  const int l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const bf16_t* base = T + (k0 + 4 * g + (li >> 2)) * ld + c0 + 4 * (li & 3);
  return cat8(tr4(base), tr4(base + 16 * ld));
}
// two stacked accumulator tiles -> operand in PERM order (tile0 = k 0..15, tile1 = k 16..31)
__device__ __forceinline__ bf16x8 acc_frag(f32x4 t0, f32x4 t1) {
  bf16x8 r;
  r[0] = (__bf16)t0[0]; r[1] = (__bf16)t0[1]; r[2] = (__bf16)t0[2]; r[3] = (__bf16)t0[3];
  r[4] = (__bf16)t1[0]; r[5] = (__bf16)t1[1]; r[6] = (__bf16)t1[2]; r[7] = (__bf16)t1[3];
  return r;
}
__device__ __forceinline__ bf16x8 scale_frag(bf16x8 v, float s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)((float)v[j] * s);
  return r;
}

// ---- global <-> LDS tile staging (16-B chunks) ---------------------------------------------
// Register staging in two halves, so several tiles' loads can be in flight before the first LDS store: rows
// >= valid re-read the last valid row (a legal address) and are zeroed at the store -- a guarded load meets its
// zero in a phi and is waited for on the spot.
template <int R, int Cn, int NT>
struct StageRegs {
  static constexpr int CPR = Cn / 8;  // 16-B chunks per row
  static constexpr int K = (R * CPR + NT - 1) / NT;
  uint4 d[K];
  int nv;
  __device__ __forceinline__ void load(const bf16_t* g, int64_t gs, int valid) {
    nv = valid;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int v = threadIdx.x + k * NT, r = min(v / CPR, R - 1), c = (v % CPR) * 8;
      if (R * CPR % NT == 0 || v < R * CPR) d[k] = *reinterpret_cast<const uint4*>(g + (int64_t)min(r, valid - 1) * gs + c);
    }
  }
  __device__ __forceinline__ void store(bf16_t* lds, int ld) const {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int v = threadIdx.x + k * NT, r = v / CPR, c = (v % CPR) * 8;
      if (R * CPR % NT != 0 && v >= R * CPR) break;
      *reinterpret_cast<uint4*>(lds + r * ld + c) = r < nv ? d[k] : make_uint4(0, 0, 0, 0);
    }
  }
};

// copy rows [0, R) x cols [0, Cn) of a bf16 global tile (row stride gs elements) into LDS [R][ld]; rows >= valid
// are zero-filled.  Cn % 8 == 0; NT threads.
template <int R, int Cn, int NT>
__device__ __forceinline__ void stage_tile(bf16_t* lds, int ld, const bf16_t* g, int64_t gs, int valid) {
  StageRegs<R, Cn, NT> t;
  t.load(g, gs, valid);
  t.store(lds, ld);
}

// accumulator tile (16x16 at rows r0.., cols c0..) -> LDS bf16 [..][ld]
__device__ __forceinline__ void acc_to_lds(bf16_t* lds, int ld, int r0, int c0, f32x4 a) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < 4; ++r) lds[(r0 + 4 * (l >> 4) + r) * ld + c0 + (l & 15)] = f2bf(a[r]);
}

// Same tile as 4-byte column pairs: lanes li and li^1 swap two values (DPP quad_perm [1,0,3,2]) so the even lane
// writes rows 4g, 4g+1 and the odd lane rows 4g+2, 4g+3 at columns (li & ~1, li | 1): 2 ds_write_b32 per lane
// instead of 4 ds_write_b16, and no dword is shared by two lanes.  With a row pitch of 4 mod 16 dwords (e.g.
// 136 or 72 bf16) the 32 lanes of each half hit 32 distinct banks.
__device__ __forceinline__ void acc_to_lds_pk(bf16_t* lds, int ld, int r0, int c0, f32x4 a) {
  const int l = threadIdx.x & 63, li = l & 15, g = l >> 4;
  const bool odd = li & 1;
  const float s0 = odd ? a[0] : a[2], s1 = odd ? a[1] : a[3];
  const float p0 = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s0), 0xB1, 0xF, 0xF, false));
  const float p1 = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s1), 0xB1, 0xF, 0xF, false));
  const int ra = r0 + 4 * g + (odd ? 2 : 0), col = c0 + (li & ~1);
  const float e0 = odd ? p0 : a[0], e1 = odd ? a[2] : p0;  // row ra
  const float f0 = odd ? p1 : a[1], f1 = odd ? a[3] : p1;  // row ra + 1
  *reinterpret_cast<uint32_t*>(lds + ra * ld + col) = pack2(e0, e1);
  *reinterpret_cast<uint32_t*>(lds + (ra + 1) * ld + col) = pack2(f0, f1);
}

// LDS [R][ld] bf16 -> global rows (row stride gs), rows >= valid skipped
template <int R, int Cn>
__device__ __forceinline__ void store_tile(bf16_t* g, int64_t gs, const bf16_t* lds, int ld, int valid) {
  constexpr int CPR = Cn / 8;
  for (int v = threadIdx.x; v < R * CPR; v += blockDim.x) {
    const int r = v / CPR, c = (v % CPR) * 8;
    if (r < valid) *reinterpret_cast<uint4*>(g + (int64_t)r * gs + c) = *reinterpret_cast<const uint4*>(lds + r * ld + c);
  }
}

// ---- cross-lane reductions without LDS: DPP butterflies inside a 16-lane row --------------------
#define MAMBA_DPP(v, ctrl) __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, (v)), (ctrl), 0xF, 0xF, false))
// sum over the 16 lanes of each row (lanes 16r..16r+15); every lane of the row gets the sum
__device__ __forceinline__ float row_sum16(float v) {
  v += MAMBA_DPP(v, 0xB1);   // quad_perm [1,0,3,2]
  v += MAMBA_DPP(v, 0x4E);   // quad_perm [2,3,0,1]
  v += MAMBA_DPP(v, 0x141);  // row_half_mirror
  v += MAMBA_DPP(v, 0x140);  // row_mirror
  return v;
}
// sum over the 4 rows (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float rows_sum4(float v) { return wave_rows_combine_sum(v); }

// read 4 consecutive rows r0+4g..+3 of column c0 + (l&15) from a [rows][ld] bf16 LDS tile (the rows /
// column an MFMA accumulator lane owns) with one ds_read_b64_tr_b16
__device__ __forceinline__ bf16x4 acc_rows4(const bf16_t* T, int ld, int r0, int c0) {
  const int l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  return tr4(T + (r0 + 4 * g + (li >> 2)) * ld + c0 + 4 * (li & 3));
}

}  // namespace mamba_amd
