// Mamba-1 selective scan (S6), forward + backward, for gfx950.
//
//   delta = softplus(delta_raw + delta_bias)            (per channel d, step t)
//   h_t[n] = exp(delta_t A[d,n]) h_{t-1}[n] + delta_t B_t[n] u_t
//   y_t    = sum_n C_t[n] h_t[n] + D[d] u_t ;  out_t = y_t * silu(z_t)
// (upstream csrc/selective_scan)
//
// Work decomposition (MI355X-first; details above each kernel):
//  * forward: one wavefront per (b, d) row, lanes over time (16 steps each), all N states per wave;
//    the cross-lane recurrence is a DPP affine prefix scan (row_shr / row_bcast, no LDS).
//  * backward: a workgroup owns 64 channels of one batch row and walks tiles of 512 steps from the
//    end; its 4 waves split the N states, replay the forward from the saved tile-start states and
//    run the adjoint as a DPP suffix scan; dB/dC sums over channels stay in registers.
//  * deterministic everywhere: every partial has exactly one writer, reductions run in fixed order.
#include "common.h"
#include "mfma.h"
#include "selective_scan.h"
#include <cstdlib>
#include <type_traits>

namespace mamba_amd {

constexpr float kLog2e = 1.4426950408889634f;
constexpr int SF_IT = 16, SF_T = 64 * SF_IT;  // forward: one wave walks a row in 1024-step tiles
constexpr int SB_IT = 8, SB_T = 64 * SB_IT;   // backward tiles; also the saved-carry granularity
constexpr int SB_W = 4;                       // waves per backward workgroup
constexpr int SB_KC = 32;                     // channels per backward workgroup (3 rounds of 2 WGs/CU at 280M)
static_assert(SF_T % SB_T == 0, "forward tiles must hold whole backward tiles");
static_assert(SB_T == kSelScanCarryTile && SB_T % kSelScanCarrySG == 0, "carry granularities");

// saved states: (B, D, nct, N) for 512-step carries; (B, nct, D, N) for 16-step ones, so that one tile's
// states of a 64-channel workgroup are one contiguous 4 KB block (coalesced stores and loads)
__device__ __forceinline__ int64_t carry_index(const SelScanArgs& a, int b, int d, int j) {
  return a.carry_t == kSelScanCarryTile ? (((int64_t)b * a.D + d) * a.nct + j) * a.N
                                        : (((int64_t)b * a.nct + j) * a.D + d) * a.N;
}

// ---- item I/O: IT consecutive steps of one (b, d) row (16-B vectors when aligned) -------------
// VEC: every row segment is a whole number of 16-B vectors inside [0, L) or entirely outside
// (host guarantees: bf16, aligned rows, L % IT == 0) -> no per-element guards in the hot kernels.
template <bool VEC, typename T, int IT>
__device__ __forceinline__ void load_items(const T* row, int t0, int L, float (&o)[IT]) {
  if constexpr (VEC) {
    static_assert(IT % 8 == 0 || IT == 4, "vector item loads are 8 or 16 bytes");
    if (t0 < L) {
      if constexpr (IT == 4) {
        const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(row) + t0);
        o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
        o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
      } else {
#pragma unroll
        for (int q = 0; q < IT / 8; ++q) {
          float tmp[8];
          ld8bf(reinterpret_cast<const bf16_t*>(row) + t0 + 8 * q, tmp);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[8 * q + j] = tmp[j];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < IT; ++i) o[i] = 0.f;
    }
  } else {
#pragma unroll
    for (int i = 0; i < IT; ++i) o[i] = (t0 + i < L) ? ld(row + t0 + i) : 0.f;
  }
}
template <bool VEC, typename T, int IT>
__device__ __forceinline__ void store_items(T* row, int t0, int L, const float (&o)[IT]) {
  if constexpr (VEC) {
    static_assert(IT % 8 == 0, "vector item stores are 16 bytes");
    if (t0 < L) {
#pragma unroll
      for (int q = 0; q < IT / 8; ++q) {
        float tmp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) tmp[j] = o[8 * q + j];
        st8bf(reinterpret_cast<bf16_t*>(row) + t0 + 8 * q, tmp);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < IT; ++i)
      if (t0 + i < L) st(row + t0 + i, o[i]);
  }
}

// ---- wave64 affine scans on DPP (no LDS round trips) -----------------------------------------
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ float dppf(float old, float src) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, src),
                                                               CTRL, RM, 0xF, false));
}
__device__ __forceinline__ float readlanef(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// Combining the map held `off` lanes away (applied first) into (a, b): (a, b) <- (a*pa, a*pb + b).
// One combine step fused into the DPP ALU ops themselves: v_fmac_f32_dpp b += b[src] * a, then
// v_mul_f32_dpp a = a[src] * a.  Without bound_ctrl a lane whose source is out of its row (or whose
// row is masked off) is simply not written, which is exactly the identity map (1, 0) -- so no
// constant "old" registers and no separate DPP moves (2 VALU ops per step instead of 6).  The
// s_nop 1 before each op covers the VALU-write -> DPP-read hazard (2 wait states) of the asm block.
#define SS_DPP2(CTRL)                                                                    \
  "s_nop 1\n\tv_fmac_f32_dpp %1, %1, %0 " CTRL "\n\t"                              \
  "s_nop 1\n\tv_mul_f32_dpp %0, %0, %0 " CTRL "\n\t"
// inclusive prefix over lanes 0..i of the maps h -> a h + b (lane 0 applied first):
// row_shr 1/2/4/8 inside each 16-lane row, then row_bcast:15 / row_bcast:31 across rows
__device__ __forceinline__ void scan_prefix(float& a, float& b) {
  asm volatile(SS_DPP2("row_shr:1 row_mask:0xf bank_mask:0xf") SS_DPP2("row_shr:2 row_mask:0xf bank_mask:0xf")
               SS_DPP2("row_shr:4 row_mask:0xf bank_mask:0xf") SS_DPP2("row_shr:8 row_mask:0xf bank_mask:0xf")
               SS_DPP2("row_bcast:15 row_mask:0xa bank_mask:0xf") SS_DPP2("row_bcast:31 row_mask:0xc bank_mask:0xf")
               "s_nop 1"
               : "+v"(a), "+v"(b));
}
// inclusive suffix over lanes i..63 (lane 63 applied first): row_shl inside rows, then the
// four row totals (lanes 0/16/32/48) are composed through readlane
__device__ __forceinline__ void scan_suffix(float& a, float& b) {
  asm volatile(SS_DPP2("row_shl:1 row_mask:0xf bank_mask:0xf") SS_DPP2("row_shl:2 row_mask:0xf bank_mask:0xf")
               SS_DPP2("row_shl:4 row_mask:0xf bank_mask:0xf") SS_DPP2("row_shl:8 row_mask:0xf bank_mask:0xf")
               "s_nop 1"
               : "+v"(a), "+v"(b));
  const float a1 = readlanef(a, 16), b1 = readlanef(b, 16);
  const float a2 = readlanef(a, 32), b2 = readlanef(b, 32);
  const float a3 = readlanef(a, 48), b3 = readlanef(b, 48);
  const float c1a = a2 * a3, c1b = fmaf(a2, b3, b2);  // rows 2..3
  const float c0a = a1 * c1a, c0b = fmaf(a1, c1b, b1);  // rows 1..3
  const int row = (threadIdx.x & 63) >> 4;
  const float ca = row == 0 ? c0a : row == 1 ? c1a : row == 2 ? a3 : 1.f;
  const float cb = row == 0 ? c0b : row == 1 ? c1b : row == 2 ? b3 : 0.f;
  b = fmaf(a, cb, b);
  a *= ca;
}
// The forward replay's prefix scan (a, b) and the adjoint's suffix scan (c, d) are independent: one
// asm block interleaves their row steps so each DPP read is >= 3 instructions after the write it
// depends on -- no s_nop inside the 4 row steps (vs. one per op when each scan runs alone).  The
// prefix's two cross-row broadcasts follow; the suffix's cross-row part is the readlane composition.
__device__ __forceinline__ void scan_prefix_suffix(float& a, float& b, float& c, float& d) {
#define SS_PAIR(K)                                                                         \
  "v_fmac_f32_dpp %1, %1, %0 row_shr:" K " row_mask:0xf bank_mask:0xf\n\t"                  \
  "v_fmac_f32_dpp %3, %3, %2 row_shl:" K " row_mask:0xf bank_mask:0xf\n\t"                  \
  "v_mul_f32_dpp %0, %0, %0 row_shr:" K " row_mask:0xf bank_mask:0xf\n\t"                   \
  "v_mul_f32_dpp %2, %2, %2 row_shl:" K " row_mask:0xf bank_mask:0xf\n\t"
  asm volatile("s_nop 1\n\t" SS_PAIR("1") SS_PAIR("2") SS_PAIR("4") SS_PAIR("8")
               SS_DPP2("row_bcast:15 row_mask:0xa bank_mask:0xf") SS_DPP2("row_bcast:31 row_mask:0xc bank_mask:0xf")
               "s_nop 1"
               : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
#undef SS_PAIR
  // suffix: compose the four row totals (lanes 0/16/32/48) through readlane, as scan_suffix
  const float a1 = readlanef(c, 16), b1 = readlanef(d, 16);
  const float a2 = readlanef(c, 32), b2 = readlanef(d, 32);
  const float a3 = readlanef(c, 48), b3 = readlanef(d, 48);
  const float c1a = a2 * a3, c1b = fmaf(a2, b3, b2);
  const float c0a = a1 * c1a, c0b = fmaf(a1, c1b, b1);
  const int row = (threadIdx.x & 63) >> 4;
  const float ca = row == 0 ? c0a : row == 1 ? c1a : row == 2 ? a3 : 1.f;
  const float cb = row == 0 ? c0b : row == 1 ? c1b : row == 2 ? b3 : 0.f;
  d = fmaf(c, cb, d);
  c *= ca;
}
#undef SS_DPP2
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dppf<0x111>(0.f, v);
  v += dppf<0x112>(0.f, v);
  v += dppf<0x114>(0.f, v);
  v += dppf<0x118>(0.f, v);
  v += dppf<0x142, 0xA>(0.f, v);
  v += dppf<0x143, 0xC>(0.f, v);
  return readlanef(v, 63);
}

// ============================== forward ========================================================
// One wavefront per (b, d) row; lane i owns SF_IT consecutive steps of the current 1024-step tile
// and ALL N states, so the sum over n for y stays in registers.  Per state: the lane composes its
// steps into one affine map, a DPP prefix scan combines the 64 lanes, the lane replays its steps
// from its true starting state.  The state at every SB_T boundary is saved for the backward.
template <typename T, int N, bool VEC>
__global__ __launch_bounds__(256) void selscan_fwd_k(SelScanArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (row >= a.B * a.D) return;
  const int b = row / a.D, d = row % a.D;
  const int g = d / (a.D / a.G);
  const T* urow = ((const T*)a.u_) + (int64_t)b * a.sub + (int64_t)d * a.sud;
  const T* drow = ((const T*)a.delta_) + (int64_t)b * a.sdb + (int64_t)d * a.sdd;
  const T* zrow = a.z_ ? ((const T*)a.z_) + (int64_t)b * a.szb + (int64_t)d * a.szd : nullptr;
  T* orow = ((T*)a.out_) + (int64_t)b * a.sob + (int64_t)d * a.sod;
  const T* Bb = ((const T*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g * a.sBg;
  const T* Cb = ((const T*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g * a.sCg;
  const float Dd = a.D_ ? a.D_[d] : 0.f;
  const float bias = a.delta_bias ? a.delta_bias[d] : 0.f;
  const int nck = (a.L + SB_T - 1) / SB_T;
  __shared__ float hcs[4][N];  // per-wave carried state (uniform), one writer lane
  float* hc = hcs[threadIdx.x >> 6];
  if (lane < N) hc[lane] = 0.f;
  for (int t0 = 0; t0 < a.L; t0 += SF_T) {
    const int tl = t0 + lane * SF_IT;
    float u[SF_IT], dl[SF_IT], y[SF_IT];
    load_items<VEC, T, SF_IT>(urow, tl, a.L, u);
    load_items<VEC, T, SF_IT>(drow, tl, a.L, dl);
    // u is only needed as dt*u (per state) and D*u (y's skip term): fold both in up front
#pragma unroll
    for (int i = 0; i < SF_IT; ++i) {
      const float v = dl[i] + bias;
      const float sp = softplus_fast(v);
      dl[i] = (tl + i < a.L) ? (a.softplus ? sp : v) : 0.f;
      y[i] = Dd * u[i];
      u[i] *= dl[i];
    }
    // vector path: B/C rows are read at a clamped (always legal) offset without a guard; lanes past
    // L have dt = 0, i.e. the identity map, so whatever they read never reaches a stored value
    const int tc = VEC ? min(tl, a.L - SF_IT) : tl;
#pragma unroll 1
    for (int n = 0; n < N; ++n) {  // keep each state's loads in its own iteration (bounded registers)
      const float A2 = a.A[d * N + n] * kLog2e;
      float Bv[SF_IT], Cv[SF_IT], av[SF_IT], xb[SF_IT];
      if constexpr (VEC) {
        static_assert(SF_IT % 8 == 0, "16-byte B/C loads");
#pragma unroll
        for (int q = 0; q < SF_IT / 8; ++q) {
          float tb[8], tcv[8];
          ld8bf(reinterpret_cast<const bf16_t*>(Bb + (int64_t)n * a.sBn) + tc + 8 * q, tb);
          ld8bf(reinterpret_cast<const bf16_t*>(Cb + (int64_t)n * a.sCn) + tc + 8 * q, tcv);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            Bv[8 * q + j] = tb[j];
            Cv[8 * q + j] = tcv[j];
          }
        }
      } else {
        load_items<VEC, T, SF_IT>(Bb + (int64_t)n * a.sBn, tl, a.L, Bv);
        load_items<VEC, T, SF_IT>(Cb + (int64_t)n * a.sCn, tl, a.L, Cv);
      }
      float ca = 1.f, cb = 0.f;
#pragma unroll
      for (int i = 0; i < SF_IT; ++i) {
        av[i] = __builtin_amdgcn_exp2f(dl[i] * A2);
        xb[i] = u[i] * Bv[i];  // u holds dt * u
        cb = fmaf(av[i], cb, xb[i]);
        ca *= av[i];
      }
      scan_prefix(ca, cb);
      const float hend = fmaf(ca, hc[n], cb);     // state after this lane's last step
      const float hin = dppf<0x138>(hc[n], hend);  // wave_shr:1 -> state before this lane's first step
      if (a.carries && (lane & (SB_T / SF_IT - 1)) == 0 && tl < a.L)
        a.carries[((int64_t)row * nck + tl / SB_T) * N + n] = hin;
      float h = hin;
#pragma unroll
      for (int i = 0; i < SF_IT; ++i) {
        h = fmaf(av[i], h, xb[i]);
        y[i] = fmaf(Cv[i], h, y[i]);
      }
      const float hnext = readlanef(hend, 63);
      if (lane == 0) hc[n] = hnext;
    }
    float zz[SF_IT];
    if (zrow) load_items<VEC, T, SF_IT>(zrow, tl, a.L, zz);
#pragma unroll
    for (int i = 0; i < SF_IT; ++i)
      if (zrow) y[i] *= siluf_(zz[i]);
    store_items<VEC, T, SF_IT>(orow, tl, a.L, y);
  }
  if (a.last_state && lane < N) a.last_state[(int64_t)row * N + lane] = hc[lane];
}

typedef float ss_f2 __attribute__((ext_vector_type(2)));

// ---- forward, wave-per-state-group form (bf16, N = 16, D % 64 == 0) ---------------------------
// A workgroup owns 64 channels of one batch row; lane = channel, wave w owns states 4w .. 4w+3.  Time is
// walked sequentially in 16-step tiles with the 4 states of a channel in registers (two float2 pairs),
// so there is no scan at all, and B / C -- which do not depend on the channel -- are the same for every
// lane of a wave: they come from SCALAR loads (SGPR operands of the packed math), so the step loop reads
// nothing per lane but dt and dt*u (staged once per tile in LDS for the 4 waves).  Per step and lane:
// 2 v_pk_mul (dt A), 4 exp, 2 v_pk_mul (dt u B), 2 v_pk_fma (h), 2 v_pk_fma (C h).  The 4 waves' partial
// y meet in LDS at the end of the tile; (y + D u) silu(z) leaves as coalesced rows.
//
// DTF (fused dt_proj, Mamba-1): delta is not read but computed per tile, delta_raw (64 channels x 16 steps) =
// W_dt[d0 .. d0+63, :R] . x_dbl[:R, tile] as one 16x16x32 MFMA chain per wave (wave w: channels 16 w .. 16 w + 15,
// K = R padded to 32 with zero weight columns and zero x rows).  The x_dbl tile (R rows x 16 steps, bf16) is staged in
// LDS over the yS buffer (not live then) and read as the hardware-transposed B operand; each lane finishes its 4
// channels x 1 step (bias, softplus, dt u) into dlS / duS behind one extra barrier.  The (B, D, L) delta tensor --
// written by a separate GEMM and read here and in the backward -- no longer exists.
constexpr int SG_T = 16, SG_D = 3;  // tile length, tiles of u / delta / z in flight
constexpr int DTF_RMAX = 128;        // largest fused dt_rank (4 MFMA K-steps)
template <int KS>  // KS = 0: delta read from memory; KS > 0: fused dt_proj with KS = ceil(R / 32) MFMA K-steps
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void selscan_fwd_sg_k(SelScanArgs a) {
  constexpr int N = 16;
  constexpr bool DTF = KS > 0;
  // ring depth: DTF drops to 2 tiles (a tile of the walk takes microseconds) to stay within 128 VGPRs
  constexpr int SGD = DTF ? 2 : SG_D;
  __shared__ __attribute__((aligned(16))) float dlS[64][SG_T + 4], duS[64][SG_T + 4];
  __shared__ __attribute__((aligned(16))) float yS[4][64][SG_T + 4];
  __shared__ __attribute__((aligned(16))) bf16_t uS[64][SG_T];
  // this tile's B / C in fp32, per step t: wave w's 4 states of B then C at [t][8 w .. 8 w + 7]; a 36-float
  // row stride puts the 64 lanes' staging writes (steps 2j / 2j+1, state n, B or C) on 64 distinct banks
  __shared__ __attribute__((aligned(16))) float bcS[SG_T][36];
  bf16_t* const xS = reinterpret_cast<bf16_t*>(&yS[0][0][0]);  // DTF: x_dbl tile [32 ceil(R / 32)][16]
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wgs_per_b = a.D / 64;
  const int b = a.binner ? blockIdx.x % a.B : blockIdx.x / wgs_per_b;
  const int d0 = (a.binner ? blockIdx.x / a.B : blockIdx.x % wgs_per_b) * 64;
  const int g = d0 / (a.D / a.G);
  const int d = d0 + lane;  // step loop: this lane's channel
  // staging / epilogue role: channel sr = tid >> 2, 4 steps at 4 * (tid & 3)
  const int sr = threadIdx.x >> 2, sc = (threadIdx.x & 3) * 4;
  const bf16_t* urow = ((const bf16_t*)a.u_) + (int64_t)b * a.sub + (int64_t)(d0 + sr) * a.sud;
  const bf16_t* drow = DTF ? nullptr : ((const bf16_t*)a.delta_) + (int64_t)b * a.sdb + (int64_t)(d0 + sr) * a.sdd;
  const bf16_t* zrow = a.z_ ? ((const bf16_t*)a.z_) + (int64_t)b * a.szb + (int64_t)(d0 + sr) * a.szd : nullptr;
  bf16_t* orow = ((bf16_t*)a.out_) + (int64_t)b * a.sob + (int64_t)(d0 + sr) * a.sod;
  const float sbias = a.delta_bias ? a.delta_bias[d0 + sr] : 0.f;
  const float sD = a.D_ ? a.D_[d0 + sr] : 0.f;
  const bf16_t* Bw = ((const bf16_t*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g * a.sBg + (int64_t)(4 * w) * a.sBn;
  const bf16_t* Cw = ((const bf16_t*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g * a.sCg + (int64_t)(4 * w) * a.sCn;
  ss_f2 A2[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) A2[p] = ss_f2{a.A[d * N + 4 * w + 2 * p], a.A[d * N + 4 * w + 2 * p + 1]} * kLog2e;
  ss_f2 h[2] = {ss_f2{0.f, 0.f}, ss_f2{0.f, 0.f}};
  const int ntile = (a.L + SG_T - 1) / SG_T;
  // SGD-deep ring of this thread's u / delta / z pieces (8 B each): each tile's data was requested
  // SGD tiles earlier, so the short tiles never wait for HBM
  // DTF: thread tid stages 16 B of the x_dbl tile (row tid / 2, steps 8 (tid % 2) ..), the lane's A operand is
  // its channel's W_dt row (L1-resident), and the lane's accumulator rows are channels 16 w + 4 (lane / 16) + r
  // (addresses recomputed at each use: registers are the limit of this kernel)
  struct Ring { uint2 u, dl, z; };
  Ring ring[SGD];
  auto fetch = [&](Ring& r, int tile) {  // clamped to L - 4 (L % 8 == 0): always legal
    const int t = min(tile * SG_T + sc, a.L - 4);
    r.u = *reinterpret_cast<const uint2*>(urow + t);
    if (!DTF) r.dl = *reinterpret_cast<const uint2*>(drow + t);
    r.z = zrow ? *reinterpret_cast<const uint2*>(zrow + t) : make_uint2(0u, 0u);
  };
  // DTF: the x_dbl chunk one tile ahead (a tile of the walk takes microseconds; x_dbl is small and cache-resident),
  // outside the SGD-deep ring to stay within the 128 VGPRs of 4 waves per SIMD
  uint4 nx = make_uint4(0u, 0u, 0u, 0u);
  auto fetch_x = [&](int tile) {  // DTF: L % 16 == 0, tile < ntile
    const int xr = threadIdx.x >> 1;
    if (xr < a.R)
      nx = *reinterpret_cast<const uint4*>((const bf16_t*)a.dtx_ + (int64_t)xr * a.sdtx + (int64_t)b * a.L +
                                           tile * SG_T + 8 * (threadIdx.x & 1));
  };
  // B / C rows (this wave's 4 states x 16 steps = 64 dwords) of the NEXT tile in flight during the
  // current one, one dword per lane (lane = 16 n + 8 [C] + j), moved to SGPRs with v_readlane
  const int bl_n = lane >> 4, bl_m = (lane >> 3) & 1, bl_j = lane & 7;
  const bf16_t* blrow = (bl_m ? Cw + (int64_t)bl_n * a.sCn : Bw + (int64_t)bl_n * a.sBn) + 2 * bl_j;
  uint32_t bc = 0u;
  auto fetch_bc = [&](int tile) { bc = *reinterpret_cast<const uint32_t*>(blrow + min(tile * SG_T, a.L - SG_T)); };
#pragma unroll
  for (int k = 0; k < SGD; ++k) fetch(ring[k], k);
  fetch_bc(0);
  if (DTF) fetch_x(0);
  auto do_tile = [&](Ring& r, int tile) {
    const int t0 = tile * SG_T;
    __syncthreads();  // the previous tile's readers are done
    // DTF: this lane's W_dt operand (zero past R) and its 4 channels' bias -- L1/L2-resident, issued here so their
    // latency overlaps the barrier, after the wait for this tile's staged data and before the next tiles' prefetches
    // (vmcnt retires loads in order); an opaque zero offset keeps the compiler from hoisting the loop-invariant
    // loads out of the walk (they would hold registers through the step loop)
    bf16x8 wk[KS > 0 ? KS : 1];
    float bias4[4];
    if (DTF) {
      *reinterpret_cast<uint2*>(&uS[sr][sc]) = r.u;
      if (threadIdx.x < 2 * 32 * KS)
        *reinterpret_cast<uint4*>(xS + 8 * threadIdx.x) = (int)(threadIdx.x >> 1) < a.R ? nx : make_uint4(0u, 0u, 0u, 0u);
      int opq = 0;
      asm volatile("" : "+v"(opq));
      const int g16 = lane >> 4, li = lane & 15;
      const bf16_t* wrow = (const bf16_t*)a.dtw_ + (int64_t)(d0 + 16 * w + li + opq) * a.R + 8 * g16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        wk[ks] = 32 * ks + 8 * g16 < a.R ? *reinterpret_cast<const bf16x8*>(wrow + 32 * ks) : bf16x8{};
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4)
        bias4[r4] = a.delta_bias ? a.delta_bias[d0 + opq + 16 * w + 4 * g16 + r4] : 0.f;
    } else {
      const float u[4] = {__uint_as_float(r.u.x << 16), __uint_as_float(r.u.x & 0xffff0000u),
                          __uint_as_float(r.u.y << 16), __uint_as_float(r.u.y & 0xffff0000u)};
      const float raw[4] = {__uint_as_float(r.dl.x << 16), __uint_as_float(r.dl.x & 0xffff0000u),
                            __uint_as_float(r.dl.y << 16), __uint_as_float(r.dl.y & 0xffff0000u)};
      float dl[4], du[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = raw[i] + sbias;
        dl[i] = (t0 + sc + i < a.L) ? (a.softplus ? softplus_fast(v) : v) : 0.f;
        du[i] = dl[i] * u[i];
      }
      *reinterpret_cast<float4*>(&dlS[sr][sc]) = make_float4(dl[0], dl[1], dl[2], dl[3]);
      *reinterpret_cast<float4*>(&duS[sr][sc]) = make_float4(du[0], du[1], du[2], du[3]);
      *reinterpret_cast<uint2*>(&uS[sr][sc]) = r.u;
    }
    const uint2 zc = r.z;
    // B / C of the tile: this lane holds steps 2 bl_j, 2 bl_j + 1 of state 4 w + bl_n (B or C); the wave stages
    // them in its own slots (no barrier needed: same-wave LDS order) and the step loop reads them back as
    // wave-uniform float4 broadcasts -- LDS-pipe work instead of 64 v_readlane + SALU unpacking per tile
    bcS[2 * bl_j][8 * w + 4 * bl_m + bl_n] = __uint_as_float(bc << 16);
    bcS[2 * bl_j + 1][8 * w + 4 * bl_m + bl_n] = __uint_as_float(bc & 0xffff0000u);
    __syncthreads();
    if (DTF) {
      const int g16 = lane >> 4, li = lane & 15;
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc = mfma16(wk[ks], frag_tr(xS, 16, 32 * ks, 0), acc);
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int ch = 16 * w + 4 * g16 + r4;
        const float v = acc[r4] + bias4[r4];
        const float dl = a.softplus ? softplus_fast(v) : v;
        dlS[ch][li] = dl;
        duS[ch][li] = dl * bf2f(uS[ch][li]);
      }
    }
    fetch(r, min(tile + SGD, ntile - 1));
    fetch_bc(min(tile + 1, ntile - 1));
    if (DTF) {
      fetch_x(min(tile + 1, ntile - 1));
      __syncthreads();  // every wave's channels of the tile are in dlS / duS
    }
    if (a.carries && t0 % a.carry_t == 0)
      *reinterpret_cast<float4*>(a.carries + carry_index(a, b, d, t0 / a.carry_t) + 4 * w) =
          make_float4(h[0].x, h[0].y, h[1].x, h[1].y);
#pragma unroll
    for (int t4 = 0; t4 < SG_T; t4 += 4) {
      const float4 dl4 = *reinterpret_cast<const float4*>(&dlS[lane][t4]);
      const float4 du4 = *reinterpret_cast<const float4*>(&duS[lane][t4]);
      const float dlv[4] = {dl4.x, dl4.y, dl4.z, dl4.w}, duv[4] = {du4.x, du4.y, du4.z, du4.w};
      float yv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int t = t4 + k;
        const float4 Bv = *reinterpret_cast<const float4*>(&bcS[t][8 * w]);
        const float4 Cv = *reinterpret_cast<const float4*>(&bcS[t][8 * w + 4]);
        ss_f2 y2 = ss_f2{0.f, 0.f};
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const ss_f2 Bp = p ? ss_f2{Bv.z, Bv.w} : ss_f2{Bv.x, Bv.y};
          const ss_f2 Cp = p ? ss_f2{Cv.z, Cv.w} : ss_f2{Cv.x, Cv.y};
          const ss_f2 e = A2[p] * dlv[k];
          const ss_f2 av = ss_f2{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
          h[p] = __builtin_elementwise_fma(av, h[p], Bp * duv[k]);
          y2 = __builtin_elementwise_fma(Cp, h[p], y2);
        }
        yv[k] = y2.x + y2.y;
      }
      *reinterpret_cast<float4*>(&yS[w][lane][t4]) = make_float4(yv[0], yv[1], yv[2], yv[3]);
    }
    __syncthreads();  // all 4 waves' partial y of the tile are in LDS
    if (t0 + sc < a.L) {
      float y[4];
      const float4 y0 = *reinterpret_cast<const float4*>(&yS[0][sr][sc]);
      const float4 y1 = *reinterpret_cast<const float4*>(&yS[1][sr][sc]);
      const float4 y2 = *reinterpret_cast<const float4*>(&yS[2][sr][sc]);
      const float4 y3 = *reinterpret_cast<const float4*>(&yS[3][sr][sc]);
      y[0] = (y0.x + y1.x) + (y2.x + y3.x);
      y[1] = (y0.y + y1.y) + (y2.y + y3.y);
      y[2] = (y0.z + y1.z) + (y2.z + y3.z);
      y[3] = (y0.w + y1.w) + (y2.w + y3.w);
      float u[4];
      ld4<bf16_t>(&uS[sr][sc], u);
      const float z[4] = {__uint_as_float(zc.x << 16), __uint_as_float(zc.x & 0xffff0000u),
                          __uint_as_float(zc.y << 16), __uint_as_float(zc.y & 0xffff0000u)};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        y[i] = fmaf(sD, u[i], y[i]);
        if (zrow) y[i] *= siluf_(z[i]);
      }
      st4<bf16_t>(orow + t0 + sc, y);
    }
  };
  int tile = 0;
  for (; tile + SGD <= ntile; tile += SGD) {
#pragma unroll
    for (int k = 0; k < SGD; ++k) do_tile(ring[k], tile + k);
  }
#pragma unroll
  for (int k = 0; k < SGD; ++k)
    if (tile + k < ntile) do_tile(ring[k], tile + k);
  if (a.last_state)
    *reinterpret_cast<float4*>(a.last_state + ((int64_t)b * a.D + d) * N + 4 * w) =
        make_float4(h[0].x, h[0].y, h[1].x, h[1].y);
}

// ============================== backward =======================================================
// A 256-thread workgroup (SB_W = 4 waves) owns SB_KC channels of one batch row and walks the SB_T-step
// tiles from the last to the first; inside a tile it takes the channels one at a time with all 4 waves:
// wave w owns states [w NW, (w+1) NW).  For its states a wave
//   * replays the forward from the saved tile-start state (DPP prefix scan) keeping h_t,
//   * runs the adjoint x_t = exp(dt_t A)(dy_t C_t + x_{t+1}) as a DPP suffix scan, whose carry into
//     the previous tile is kept in LDS per (channel, state),
//   * accumulates dB[t,n] and dC[t,n] for ITS states over all channels of the group in REGISTERS
//     (written once per tile as the group's partial; deterministic, no atomics).
// Sums over n (du, ddelta, y for dz) go through one LDS row per wave and are finished item-parallel
// (thread = time step, fixed-order sum over the SB_W rows, coalesced I/O).
template <typename T, int N, bool VEC>
__global__ __launch_bounds__(256) void selscan_bwd_k(SelScanArgs a) {
  constexpr int NW = N >= SB_W ? N / SB_W : 1;
  constexpr int IT = SB_IT;
  __shared__ __attribute__((aligned(16))) float part[2][SB_W][3][SB_T];  // double-buffered per channel
  __shared__ __attribute__((aligned(16))) bf16_t BCs[2][N][SB_T];  // this tile's B, C (group of d0), bf16 as in HBM
  __shared__ float lamc[SB_KC][N];
  __shared__ float dAacc[SB_KC][N];
  __shared__ float dDacc[SB_KC][SB_W], dbacc[SB_KC][SB_W];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int dg = blockIdx.x, b = blockIdx.y;
  const int d0 = dg * SB_KC, nch = min(SB_KC, a.D - d0);
  const int ntl = (a.L + SB_T - 1) / SB_T;
  const int ndg = (a.D + SB_KC - 1) / SB_KC;
  const bool has_states = w * NW < N;
  for (int v = threadIdx.x; v < SB_KC * N; v += 64 * SB_W) {
    (&lamc[0][0])[v] = 0.f;
    (&dAacc[0][0])[v] = 0.f;
  }
  for (int v = threadIdx.x; v < SB_KC * SB_W; v += 64 * SB_W) {
    (&dDacc[0][0])[v] = 0.f;
    (&dbacc[0][0])[v] = 0.f;
  }
  __syncthreads();
  for (int tile = ntl - 1; tile >= 0; --tile) {
    const int tl = tile * SB_T + lane * IT;
    float accB[NW][IT], accC[NW][IT];
#pragma unroll
    for (int nn = 0; nn < NW; ++nn)
#pragma unroll
      for (int i = 0; i < IT; ++i) accB[nn][i] = accC[nn][i] = 0.f;
    const int g0 = d0 / (a.D / a.G);
    {  // B and C do not depend on the channel: stage the tile once for all SB_KC channels
      const T* Bb = ((const T*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g0 * a.sBg;
      const T* Cb = ((const T*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g0 * a.sCg;
      for (int v = threadIdx.x; v < N * SB_T; v += 64 * SB_W) {
        const int n = v / SB_T, t = tile * SB_T + v % SB_T;
        BCs[0][n][v % SB_T] = f2bf(t < a.L ? ld(Bb + (int64_t)n * a.sBn + t) : 0.f);
        BCs[1][n][v % SB_T] = f2bf(t < a.L ? ld(Cb + (int64_t)n * a.sCn + t) : 0.f);
      }
    }
    __syncthreads();
    // next channel's rows, fetched while the current one is processed (VEC path)
    uint2 nu = make_uint2(0, 0), nd = nu, ng = nu, nz = nu;
    float4 nh = make_float4(0.f, 0.f, 0.f, 0.f);  // next channel's tile-start states (NW == 4)
    auto fetch = [&](int k) {
      if constexpr (VEC) {
        if (k < nch && tl < a.L) {
          const int d = d0 + k;
          nu = *reinterpret_cast<const uint2*>(((const bf16_t*)a.u_) + (int64_t)b * a.sub + (int64_t)d * a.sud + tl);
          nd = *reinterpret_cast<const uint2*>(((const bf16_t*)a.delta_) + (int64_t)b * a.sdb + (int64_t)d * a.sdd + tl);
          ng = *reinterpret_cast<const uint2*>(((const bf16_t*)a.dout_) + (int64_t)b * a.sgb + (int64_t)d * a.sgd + tl);
          if (a.z_) nz = *reinterpret_cast<const uint2*>(((const bf16_t*)a.z_) + (int64_t)b * a.szb + (int64_t)d * a.szd + tl);
        }
        if (NW == 4 && k < nch)
          nh = *reinterpret_cast<const float4*>(a.carries + carry_index(a, b, d0 + k, tile * (SB_T / a.carry_t)) + w * NW);
      }
    };
    if (has_states) fetch(0);
    for (int k = 0; k < nch; ++k) {
      const int d = d0 + k;
      const int g = d / (a.D / a.G);
      const T* urow = ((const T*)a.u_) + (int64_t)b * a.sub + (int64_t)d * a.sud;
      const T* drow = ((const T*)a.delta_) + (int64_t)b * a.sdb + (int64_t)d * a.sdd;
      const T* grow = ((const T*)a.dout_) + (int64_t)b * a.sgb + (int64_t)d * a.sgd;
      const T* zrow = a.z_ ? ((const T*)a.z_) + (int64_t)b * a.szb + (int64_t)d * a.szd : nullptr;
      const float bias = a.delta_bias ? a.delta_bias[d] : 0.f;
      const int buf = k & 1;
      uint2 craw = make_uint2(0, 0), cg = craw, cz = craw;  // this channel's raw delta / dout / z (VEC)
      float hcv[4];
      float uf[IT], dlf[IT];
      if (has_states) {
        const T* Bb = ((const T*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g * a.sBg;
        const T* Cb = ((const T*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g * a.sCg;
        float u[IT], dl[IT], dy[IT], zz[IT];
        if constexpr (VEC) {
          auto unpack4 = [](uint2 v, float (&o)[IT]) {
            o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
            o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
          };
          unpack4(nu, u); unpack4(nd, dl); unpack4(ng, dy); unpack4(nz, zz);
          craw = nd; cg = ng; cz = nz;
          hcv[0] = nh.x; hcv[1] = nh.y; hcv[2] = nh.z; hcv[3] = nh.w;
          fetch(k + 1);
        } else {
          load_items<VEC, T, IT>(urow, tl, a.L, u);
          load_items<VEC, T, IT>(drow, tl, a.L, dl);
          load_items<VEC, T, IT>(grow, tl, a.L, dy);
          if (zrow) load_items<VEC, T, IT>(zrow, tl, a.L, zz);
        }
        if (zrow) {
#pragma unroll
          for (int i = 0; i < IT; ++i) dy[i] *= siluf_(zz[i]);
        }
#pragma unroll
        for (int i = 0; i < IT; ++i) {
          const float v = dl[i] + bias;
          dl[i] = (tl + i < a.L) ? (a.softplus ? softplus_fast(v) : v) : 0.f;
        }
        float du[IT], dd[IT], yv[IT];
#pragma unroll
        for (int i = 0; i < IT; ++i) du[i] = dd[i] = yv[i] = 0.f;
        // runtime loop over this wave's states; the accumulators rotate so the live one is always
        // slot 0 (static register indices, no overlap of the states' working sets)
#pragma unroll 1
        for (int nn = 0; nn < NW; ++nn) {
          const int n = w * NW + nn;
          const float An = a.A[d * N + n];
          const float A2 = An * kLog2e;
          float Bv[IT], Cv[IT], av[IT], hs[IT];
          if (g == g0) {
            static_assert(IT == 8, "LDS B/C reads are one 16-byte read per lane");
            ld8bf(&BCs[0][n][lane * IT], Bv);
            ld8bf(&BCs[1][n][lane * IT], Cv);
          } else {
            load_items<VEC, T, IT>(Bb + (int64_t)n * a.sBn, tl, a.L, Bv);
            load_items<VEC, T, IT>(Cb + (int64_t)n * a.sCn, tl, a.L, Cv);
          }
          // forward replay from the saved tile-start state
          float ca = 1.f, cb = 0.f;
#pragma unroll
          for (int i = 0; i < IT; ++i) {
            av[i] = __builtin_amdgcn_exp2f(dl[i] * A2);
            cb = fmaf(av[i], cb, dl[i] * u[i] * Bv[i]);
            ca *= av[i];
          }
          const float prod = ca;  // the lane's decay product also seeds the adjoint composition
          scan_prefix(ca, cb);
          const float hc0 = (VEC && NW == 4) ? hcv[0] : a.carries[carry_index(a, b, d, tile * (SB_T / a.carry_t)) + n];
          if constexpr (VEC && NW == 4) {  // rotate like the accumulators: the live one is slot 0
            const float t0_ = hcv[0];
            hcv[0] = hcv[1]; hcv[1] = hcv[2]; hcv[2] = hcv[3]; hcv[3] = t0_;
          }
          const float hend = fmaf(ca, hc0, cb);
          float h = dppf<0x138>(hc0, hend);
#pragma unroll
          for (int i = 0; i < IT; ++i) {
            h = fmaf(av[i], h, dl[i] * u[i] * Bv[i]);
            hs[i] = h;
            yv[i] = fmaf(Cv[i], h, yv[i]);
          }
          // adjoint: x_t = av_t (dy_t C_t + x_{t+1}),  lambda_t = dy_t C_t + x_{t+1}
          float ma = prod, mb = 0.f;
#pragma unroll
          for (int i = IT - 1; i >= 0; --i) {
            mb = av[i] * fmaf(dy[i], Cv[i], mb);
          }
          scan_suffix(ma, mb);
          const float xc = lamc[k][n];
          const float xfirst = fmaf(ma, xc, mb);
          float x = dppf<0x130>(xc, xfirst);  // wave_shl:1 -> x after this lane's last step
          const float xnew = readlanef(xfirst, 0);
          float dAp = 0.f;
#pragma unroll
          for (int i = IT - 1; i >= 0; --i) {
            const float lam = fmaf(dy[i], Cv[i], x);
            x = av[i] * lam;
            const float dlu = dl[i] * u[i];
            accB[0][i] = fmaf(lam, dlu, accB[0][i]);
            accC[0][i] = fmaf(dy[i], hs[i], accC[0][i]);
            du[i] = fmaf(lam, Bv[i], du[i]);
            const float t1 = lam * (hs[i] - dlu * Bv[i]);  // lam * av * h_{t-1}
            dd[i] = fmaf(lam * u[i], Bv[i], fmaf(An, t1, dd[i]));
            dAp = fmaf(dl[i], t1, dAp);
          }
          dAp = wave_sum_dpp(dAp);
          if (lane == 0) {
            lamc[k][n] = xnew;
            dAacc[k][n] += dAp;
          }
#pragma unroll
          for (int i = 0; i < IT; ++i) {
            const float tb = accB[0][i], tc = accC[0][i];
#pragma unroll
            for (int q = 0; q + 1 < NW; ++q) {
              accB[q][i] = accB[q + 1][i];
              accC[q][i] = accC[q + 1][i];
            }
            accB[NW - 1][i] = tb;
            accC[NW - 1][i] = tc;
          }
        }
#pragma unroll
        for (int i = 0; i < IT; ++i) {
          uf[i] = u[i];
          dlf[i] = dl[i];
        }
        if constexpr (VEC) {
          *reinterpret_cast<float4*>(&part[buf][w][0][lane * IT]) = make_float4(du[0], du[1], du[2], du[3]);
          *reinterpret_cast<float4*>(&part[buf][w][1][lane * IT]) = make_float4(dd[0], dd[1], dd[2], dd[3]);
          *reinterpret_cast<float4*>(&part[buf][w][2][lane * IT]) = make_float4(yv[0], yv[1], yv[2], yv[3]);
        } else {
#pragma unroll
          for (int i = 0; i < IT; ++i) {
            part[buf][w][0][lane * IT + i] = du[i] * dl[i];
            part[buf][w][1][lane * IT + i] = dd[i];
            part[buf][w][2][lane * IT + i] = yv[i];
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < IT; ++i)
          part[buf][w][0][lane * IT + i] = part[buf][w][1][lane * IT + i] = part[buf][w][2][lane * IT + i] = 0.f;
      }
      __syncthreads();
      if constexpr (VEC) {
        // one wave (rotating with the channel) finishes the channel from its registers: the other waves
        // go straight on to the next channel (part[] is double-buffered, so the next channel's barrier
        // orders this wave's reads before the buffer is rewritten two channels later)
        if (w == (k & (SB_W - 1)) && has_states) {
          float s1[IT], sdd[IT], sy[IT];
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            float4 acc4 = *reinterpret_cast<const float4*>(&part[buf][0][q][lane * IT]);
#pragma unroll
            for (int v = 1; v < SB_W; ++v) {
              const float4 o = *reinterpret_cast<const float4*>(&part[buf][v][q][lane * IT]);
              acc4.x += o.x; acc4.y += o.y; acc4.z += o.z; acc4.w += o.w;
            }
            float* dst = q == 0 ? s1 : (q == 1 ? sdd : sy);
            dst[0] = acc4.x; dst[1] = acc4.y; dst[2] = acc4.z; dst[3] = acc4.w;
          }
          const float Dd = a.D_ ? a.D_[d] : 0.f;
          float gv[IT], zv[IT], rv[IT], o_du[IT], o_dd[IT], o_dz[IT];
          auto unp = [](uint2 v, float (&o)[IT]) {
            o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
            o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
          };
          unp(cg, gv); unp(cz, zv); unp(craw, rv);
          const bool inr = tl < a.L;
          float dDp = 0.f, dbp = 0.f;
#pragma unroll
          for (int i = 0; i < IT; ++i) {
            float dyv = gv[i];
            o_dz[i] = 0.f;
            if (zrow) {
              const float sg = sigmoidf_(zv[i]);
              dyv = gv[i] * zv[i] * sg;
              o_dz[i] = gv[i] * fmaf(Dd, uf[i], sy[i]) * sg * (1.f + zv[i] * (1.f - sg));
            }
            o_du[i] = fmaf(dlf[i], s1[i], Dd * dyv);
            o_dd[i] = inr ? sdd[i] * (a.softplus ? sigmoidf_(rv[i] + bias) : 1.f) : 0.f;
            dDp = fmaf(dyv, uf[i], dDp);
            dbp += o_dd[i];
          }
          if (inr) {
            auto pk = [](const float (&o)[IT]) { return make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3])); };
            *reinterpret_cast<uint2*>(((bf16_t*)a.du_) + (int64_t)b * a.sdub + (int64_t)d * a.sdud + tl) = pk(o_du);
            *reinterpret_cast<uint2*>(((bf16_t*)a.ddelta_) + (int64_t)b * a.sddb + (int64_t)d * a.sddd + tl) = pk(o_dd);
            if (zrow && a.dz_)
              *reinterpret_cast<uint2*>(((bf16_t*)a.dz_) + (int64_t)b * a.sdzb + (int64_t)d * a.sdzd + tl) = pk(o_dz);
          }
          dDp = wave_sum_dpp(dDp);
          dbp = wave_sum_dpp(dbp);
          if (lane == 0) {
            dDacc[k][0] += dDp;
            dbacc[k][0] += dbp;
          }
        }
      } else {
        // finish item-parallel: thread j <-> step tile*SB_T + j
        float dDp = 0.f, dbp = 0.f;
        for (int j = threadIdx.x; j < SB_T; j += 64 * SB_W) {  // SB_T = 2 x the workgroup size
          const int t = tile * SB_T + j;
          if (t < a.L) {
            float sdu = 0.f, sdd = 0.f, sy = 0.f;
#pragma unroll
            for (int v = 0; v < SB_W; ++v) {
              sdu += part[buf][v][0][j];
              sdd += part[buf][v][1][j];
              sy += part[buf][v][2][j];
            }
            const float Dd = a.D_ ? a.D_[d] : 0.f;
            const float uu = ld(urow + t), raw = ld(drow + t) + bias, go = ld(grow + t);
            float dyv = go, dz = 0.f;
            if (zrow) {
              const float zv = ld(zrow + t), sg = sigmoidf_(zv);
              dyv = go * zv * sg;
              dz = go * fmaf(Dd, uu, sy) * sg * (1.f + zv * (1.f - sg));
            }
            const float ddl = sdd * (a.softplus ? sigmoidf_(raw) : 1.f);
            st(((T*)a.du_) + (int64_t)b * a.sdub + (int64_t)d * a.sdud + t, fmaf(Dd, dyv, sdu));
            st(((T*)a.ddelta_) + (int64_t)b * a.sddb + (int64_t)d * a.sddd + t, ddl);
            if (zrow && a.dz_) st(((T*)a.dz_) + (int64_t)b * a.sdzb + (int64_t)d * a.sdzd + t, dz);
            dDp = fmaf(dyv, uu, dDp);
            dbp += ddl;
          }
        }
        dDp = wave_sum_dpp(dDp);
        dbp = wave_sum_dpp(dbp);
        if (lane == 0) {
          dDacc[k][w] += dDp;
          dbacc[k][w] += dbp;
        }
        __syncthreads();  // part[] consumed before the next channel overwrites it
      }
    }
    // this tile's dB / dC partial for the group's channels (this wave's states)
    if (has_states) {
#pragma unroll
      for (int nn = 0; nn < NW; ++nn) {
        const int n = w * NW + nn;
        float* pb = a.part_dB + (((int64_t)b * ndg + dg) * N + n) * a.L;
        float* pc = a.part_dC + (((int64_t)b * ndg + dg) * N + n) * a.L;
        if (tl + IT <= a.L && (a.L % 4) == 0) {
#pragma unroll
          for (int q = 0; q < IT / 4; ++q) {
            *reinterpret_cast<float4*>(pb + tl + 4 * q) =
                make_float4(accB[nn][4 * q], accB[nn][4 * q + 1], accB[nn][4 * q + 2], accB[nn][4 * q + 3]);
            *reinterpret_cast<float4*>(pc + tl + 4 * q) =
                make_float4(accC[nn][4 * q], accC[nn][4 * q + 1], accC[nn][4 * q + 2], accC[nn][4 * q + 3]);
          }
        } else {
#pragma unroll
          for (int i = 0; i < IT; ++i)
            if (tl + i < a.L) {
              pb[tl + i] = accB[nn][i];
              pc[tl + i] = accC[nn][i];
            }
        }
      }
    }
  }
  __syncthreads();
  for (int v = threadIdx.x; v < nch * N; v += 64 * SB_W)
    a.part_dA[((int64_t)b * a.D + d0 + v / N) * N + v % N] = dAacc[v / N][v % N];
  for (int v = threadIdx.x; v < nch; v += 64 * SB_W) {
    float sD = 0.f, sb = 0.f;
#pragma unroll
    for (int q = 0; q < SB_W; ++q) {
      sD += dDacc[v][q];
      sb += dbacc[v][q];
    }
    a.part_dD[(int64_t)b * a.D + d0 + v] = sD;
    a.part_dbias[(int64_t)b * a.D + d0 + v] = sb;
  }
}

// ---- backward, bf16 fast path ------------------------------------------------------------------
// Same decomposition as selscan_bwd_k (a 4-wave workgroup owns SB_KC channels of one batch row and
// walks the 512-step tiles backwards; wave w owns states [w NW, (w+1) NW)), reorganised so the VALU
// work per state-step is close to the arithmetic of the recurrence itself:
//  * 8 steps per lane (the two DPP scans per state and channel are amortised over 512 steps);
//  * the NW states of a wave are fully unrolled, so the register-resident dB/dC accumulators are
//    indexed statically (the runtime state loop of the generic kernel had to rotate them);
//  * xb_t = dt_t u_t B_t is computed once and reused by the replay and by the adjoint, whose terms
//    share S1_t = sum_n lam B:  du = dt S1 + D dy,  ddelta = (u S1 + sum_n A_n lam (h_t - xb_t)) sp',
//    dA_n = sum_t dt lam (h_t - xb_t)   (lam (h_t - xb_t) = lam a_t h_{t-1});
//  * the sums over states (S1, S2, y) meet in ONE single-buffered LDS block, and all four waves
//    finish the channel together, wave w taking steps 2w, 2w+1 of every lane's segment;
//  * B, C of the tile sit in LDS as bf16 [n][t]: one 16-B read per lane per state.
// LDS ~66 KB and <= 256 VGPRs: two workgroups per CU.  Deterministic: every partial has one writer.
template <int N>
__global__ __launch_bounds__(256) void selscan_bwd_fast_k(SelScanArgs a) {
  constexpr int NW = N / SB_W;
  constexpr int IT = SB_IT;
  static_assert(NW >= 1 && IT == 8, "bf16 fast path: 8 steps per lane, >= 1 state per wave");
  __shared__ __attribute__((aligned(16))) float part[SB_W][3][SB_T];
  __shared__ __attribute__((aligned(16))) bf16_t BCs[2][N][SB_T];
  __shared__ float lamc[SB_KC][N];
  __shared__ float dAacc[SB_KC][N];
  __shared__ float dDacc[SB_KC][SB_W], dbacc[SB_KC][SB_W];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int dg = blockIdx.x, b = blockIdx.y;
  const int d0 = dg * SB_KC, nch = min(SB_KC, a.D - d0);
  const int ntl = (a.L + SB_T - 1) / SB_T;
  const int ndg = (a.D + SB_KC - 1) / SB_KC;
  const int dpg = a.D / a.G;
  for (int v = threadIdx.x; v < SB_KC * N; v += 64 * SB_W) {
    (&lamc[0][0])[v] = 0.f;
    (&dAacc[0][0])[v] = 0.f;
  }
  for (int v = threadIdx.x; v < SB_KC * SB_W; v += 64 * SB_W) {
    (&dDacc[0][0])[v] = 0.f;
    (&dbacc[0][0])[v] = 0.f;
  }
  const bf16_t* ub = ((const bf16_t*)a.u_) + (int64_t)b * a.sub;
  const bf16_t* db_ = ((const bf16_t*)a.delta_) + (int64_t)b * a.sdb;
  const bf16_t* gb = ((const bf16_t*)a.dout_) + (int64_t)b * a.sgb;
  const bf16_t* zb = a.z_ ? ((const bf16_t*)a.z_) + (int64_t)b * a.szb : nullptr;
  for (int tile = ntl - 1; tile >= 0; --tile) {
    const int tl = tile * SB_T + lane * IT;
    const bool inr = tl < a.L;  // L % 8 == 0: a lane's 8 steps are all inside or all outside
    float accB[NW][IT], accC[NW][IT];
#pragma unroll
    for (int nn = 0; nn < NW; ++nn)
#pragma unroll
      for (int i = 0; i < IT; ++i) accB[nn][i] = accC[nn][i] = 0.f;
    const int g0 = d0 / dpg;
    __syncthreads();  // previous tile's readers of BCs are done
    {
      const bf16_t* Bb = ((const bf16_t*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g0 * a.sBg;
      const bf16_t* Cb = ((const bf16_t*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g0 * a.sCg;
      for (int v = threadIdx.x; v < N * (SB_T / 8); v += 64 * SB_W) {
        const int n = v / (SB_T / 8), c8 = (v % (SB_T / 8)) * 8, t = tile * SB_T + c8;
        uint4 bq = make_uint4(0, 0, 0, 0), cq = bq;
        if (t < a.L) {
          bq = *reinterpret_cast<const uint4*>(Bb + (int64_t)n * a.sBn + t);
          cq = *reinterpret_cast<const uint4*>(Cb + (int64_t)n * a.sCn + t);
        }
        *reinterpret_cast<uint4*>(&BCs[0][n][c8]) = bq;
        *reinterpret_cast<uint4*>(&BCs[1][n][c8]) = cq;
      }
    }
    __syncthreads();
    uint4 nu = make_uint4(0, 0, 0, 0), nd = nu, ng = nu, nz = nu;
    float nh[NW], nA[NW];
    auto fetch = [&](int k) {
      if (k < nch) {
        const int d = d0 + k;
        if (inr) {
          nu = *reinterpret_cast<const uint4*>(ub + (int64_t)d * a.sud + tl);
          nd = *reinterpret_cast<const uint4*>(db_ + (int64_t)d * a.sdd + tl);
          ng = *reinterpret_cast<const uint4*>(gb + (int64_t)d * a.sgd + tl);
          if (zb) nz = *reinterpret_cast<const uint4*>(zb + (int64_t)d * a.szd + tl);
        }
        const float* cp = a.carries + carry_index(a, b, d, tile * (SB_T / a.carry_t)) + w * NW;
#pragma unroll
        for (int nn = 0; nn < NW; ++nn) {
          nh[nn] = cp[nn];
          nA[nn] = a.A[d * N + w * NW + nn];
        }
      }
    };
    fetch(0);
    for (int k = 0; k < nch; ++k) {
      const int d = d0 + k;
      const int g = d / dpg;
      // everything this channel reads from memory is in flight before the next channel's prefetch is
      // issued, so the waits below never cover the prefetch (vmcnt counts in issue order)
      const float bias = a.delta_bias ? a.delta_bias[d] : 0.f;
      const float Dd = a.D_ ? a.D_[d] : 0.f;
      // the bf16 pairs of steps 2w, 2w+1 this wave finishes stay live packed (4 registers); the fp32
      // working set is dl, dy, dlu
      const uint4 cu = nu, craw = nd, cg = ng, cz = nz;
      unsigned wu = cu.x, wr = craw.x, wg = cg.x, wz = cz.x;
#pragma unroll
      for (int ww = 1; ww < SB_W; ++ww)
        if (w == ww) {
          wu = (&cu.x)[ww]; wr = (&craw.x)[ww]; wg = (&cg.x)[ww]; wz = (&cz.x)[ww];
        }
      float hc[NW], Ac[NW];
#pragma unroll
      for (int nn = 0; nn < NW; ++nn) {
        hc[nn] = nh[nn];
        Ac[nn] = nA[nn];
      }
      fetch(k + 1);
      float dl[IT], dy[IT], dlu[IT];
      {
        float u[IT], raw[IT], go[IT], zz[IT];
        ld8bf(reinterpret_cast<const bf16_t*>(&cu), u);
        ld8bf(reinterpret_cast<const bf16_t*>(&craw), raw);
        ld8bf(reinterpret_cast<const bf16_t*>(&cg), go);
        ld8bf(reinterpret_cast<const bf16_t*>(&cz), zz);
#pragma unroll
        for (int i = 0; i < IT; ++i) {  // branch-free: both forms computed, then selected
          const float v = raw[i] + bias;
          const float sp = softplus_fast(v);
          dl[i] = inr ? (a.softplus ? sp : v) : 0.f;
          const float gate = zz[i] * sigmoid_fast(zz[i]);
          dy[i] = go[i] * (zb ? gate : 1.f);
          dlu[i] = dl[i] * u[i];
        }
      }
      float S1[IT], S2[IT], yv[IT];
#pragma unroll
      for (int i = 0; i < IT; ++i) S1[i] = S2[i] = yv[i] = 0.f;
      // runtime loop over the wave's states (one state's working set live at a time); its dB / dC
      // contributions are added to the statically indexed accumulators through a uniform switch
#pragma unroll 1
      for (int nn = 0; nn < NW; ++nn) {
        const int n = w * NW + nn;
        float hcn = hc[0], An = Ac[0];
#pragma unroll
        for (int q = 1; q < NW; ++q)
          if (nn == q) {
            hcn = hc[q];
            An = Ac[q];
          }
        const float A2 = An * kLog2e;
        float Bv[IT], Cv[IT], av[IT], xb[IT], hs[IT], cB[IT], cC[IT];
        if (g == g0) {
          ld8bf(&BCs[0][n][lane * IT], Bv);
          ld8bf(&BCs[1][n][lane * IT], Cv);
        } else {
          load_items<true, bf16_t, IT>(((const bf16_t*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g * a.sBg +
                                       (int64_t)n * a.sBn, tl, a.L, Bv);
          load_items<true, bf16_t, IT>(((const bf16_t*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g * a.sCg +
                                       (int64_t)n * a.sCn, tl, a.L, Cv);
        }
        // forward replay from the saved tile-start state
        float ca = 1.f, cb = 0.f;
#pragma unroll
        for (int i = 0; i < IT; ++i) {
          av[i] = __builtin_amdgcn_exp2f(dl[i] * A2);
          xb[i] = dlu[i] * Bv[i];
          cb = fmaf(av[i], cb, xb[i]);
          ca *= av[i];
        }
        // adjoint x_t = a_t (dy_t C_t + x_{t+1}): this lane's map, composed before the scans so the
        // prefix (forward replay) and suffix (adjoint) scans run interleaved
        float ma = ca, mb = 0.f;
#pragma unroll
        for (int i = IT - 1; i >= 0; --i) mb = av[i] * fmaf(dy[i], Cv[i], mb);
        scan_prefix_suffix(ca, cb, ma, mb);
        const float hend = fmaf(ca, hcn, cb);
        float h = dppf<0x138>(hcn, hend);  // wave_shr:1 -> state before this lane's first step
#pragma unroll
        for (int i = 0; i < IT; ++i) {
          h = fmaf(av[i], h, xb[i]);
          hs[i] = h;
          yv[i] = fmaf(Cv[i], h, yv[i]);
        }
        const float xc = lamc[k][n];
        const float xfirst = fmaf(ma, xc, mb);
        float x = dppf<0x130>(xc, xfirst);  // wave_shl:1 -> adjoint after this lane's last step
        const float xnew = readlanef(xfirst, 0);
        float dAp = 0.f;
#pragma unroll
        for (int i = IT - 1; i >= 0; --i) {
          const float lam = fmaf(dy[i], Cv[i], x);
          x = av[i] * lam;
          cB[i] = lam * dlu[i];
          cC[i] = dy[i] * hs[i];
          S1[i] = fmaf(lam, Bv[i], S1[i]);
          const float t1 = lam * (hs[i] - xb[i]);  // lam a_t h_{t-1}
          S2[i] = fmaf(An, t1, S2[i]);
          dAp = fmaf(dl[i], t1, dAp);
        }
#pragma unroll
        for (int q = 0; q < NW; ++q)
          if (nn == q) {
#pragma unroll
            for (int i = 0; i < IT; ++i) {
              accB[q][i] += cB[i];
              accC[q][i] += cC[i];
            }
          }
        dAp = wave_sum_dpp(dAp);
        if (lane == 0) {
          lamc[k][n] = xnew;
          dAacc[k][n] += dAp;
        }
      }
      float* pw = &part[w][0][lane * IT];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        *reinterpret_cast<float4*>(pw + 4 * q) = make_float4(S1[4 * q], S1[4 * q + 1], S1[4 * q + 2], S1[4 * q + 3]);
        *reinterpret_cast<float4*>(pw + SB_T + 4 * q) =
            make_float4(S2[4 * q], S2[4 * q + 1], S2[4 * q + 2], S2[4 * q + 3]);
        *reinterpret_cast<float4*>(pw + 2 * SB_T + 4 * q) =
            make_float4(yv[4 * q], yv[4 * q + 1], yv[4 * q + 2], yv[4 * q + 3]);
      }
      __syncthreads();
      // finish the channel: wave w takes steps 2w, 2w+1 of every lane (uniform select of the pair)
      float2 su = make_float2(0.f, 0.f), s2 = su, sy = su;
#pragma unroll
      for (int v = 0; v < SB_W; ++v) {
        const float2 p0 = *reinterpret_cast<const float2*>(&part[v][0][lane * IT + 2 * w]);
        const float2 p1 = *reinterpret_cast<const float2*>(&part[v][1][lane * IT + 2 * w]);
        const float2 p2 = *reinterpret_cast<const float2*>(&part[v][2][lane * IT + 2 * w]);
        su.x += p0.x; su.y += p0.y;
        s2.x += p1.x; s2.y += p1.y;
        sy.x += p2.x; sy.y += p2.y;
      }
      float pu[2], pdl[2], pdy[2], pr[2], pg[2], pz[2];
      {
        pu[0] = __uint_as_float(wu << 16); pu[1] = __uint_as_float(wu & 0xffff0000u);
        pr[0] = __uint_as_float(wr << 16); pr[1] = __uint_as_float(wr & 0xffff0000u);
        pg[0] = __uint_as_float(wg << 16); pg[1] = __uint_as_float(wg & 0xffff0000u);
        pz[0] = __uint_as_float(wz << 16); pz[1] = __uint_as_float(wz & 0xffff0000u);
        pdl[0] = dl[0]; pdl[1] = dl[1]; pdy[0] = dy[0]; pdy[1] = dy[1];
#pragma unroll
        for (int ww = 1; ww < SB_W; ++ww)
          if (w == ww) {
            pdl[0] = dl[2 * ww]; pdl[1] = dl[2 * ww + 1]; pdy[0] = dy[2 * ww]; pdy[1] = dy[2 * ww + 1];
          }
      }
      const float s1v[2] = {su.x, su.y}, s2v[2] = {s2.x, s2.y}, syv[2] = {sy.x, sy.y};
      float o_du[2], o_dd[2], o_dz[2];
      float dDp = 0.f, dbp = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        o_du[j] = fmaf(pdl[j], s1v[j], Dd * pdy[j]);
        const float dds = fmaf(pu[j], s1v[j], s2v[j]);
        const float sd = sigmoid_fast(pr[j] + bias), sg = sigmoid_fast(pz[j]);
        o_dd[j] = inr ? dds * (a.softplus ? sd : 1.f) : 0.f;
        o_dz[j] = pg[j] * fmaf(Dd, pu[j], syv[j]) * sg * (1.f + pz[j] * (1.f - sg));
        dDp = fmaf(pdy[j], pu[j], dDp);
        dbp += o_dd[j];
      }
      if (inr) {
        const int64_t t = tl + 2 * w;
        *reinterpret_cast<unsigned*>(((bf16_t*)a.du_) + (int64_t)b * a.sdub + (int64_t)d * a.sdud + t) =
            pack2(o_du[0], o_du[1]);
        *reinterpret_cast<unsigned*>(((bf16_t*)a.ddelta_) + (int64_t)b * a.sddb + (int64_t)d * a.sddd + t) =
            pack2(o_dd[0], o_dd[1]);
        if (zb && a.dz_)
          *reinterpret_cast<unsigned*>(((bf16_t*)a.dz_) + (int64_t)b * a.sdzb + (int64_t)d * a.sdzd + t) =
              pack2(o_dz[0], o_dz[1]);
      }
      dDp = wave_sum_dpp(dDp);
      dbp = wave_sum_dpp(dbp);
      if (lane == 0) {
        dDacc[k][w] += dDp;
        dbacc[k][w] += dbp;
      }
      __syncthreads();  // part[] consumed before the next channel rewrites it
    }
    // this tile's dB / dC partial for the group's channels (this wave's states)
    if (inr) {
#pragma unroll
      for (int nn = 0; nn < NW; ++nn) {
        const int n = w * NW + nn;
        float* pb = a.part_dB + (((int64_t)b * ndg + dg) * N + n) * a.L + tl;
        float* pc = a.part_dC + (((int64_t)b * ndg + dg) * N + n) * a.L + tl;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          *reinterpret_cast<float4*>(pb + 4 * q) =
              make_float4(accB[nn][4 * q], accB[nn][4 * q + 1], accB[nn][4 * q + 2], accB[nn][4 * q + 3]);
          *reinterpret_cast<float4*>(pc + 4 * q) =
              make_float4(accC[nn][4 * q], accC[nn][4 * q + 1], accC[nn][4 * q + 2], accC[nn][4 * q + 3]);
        }
      }
    }
  }
  __syncthreads();
  for (int v = threadIdx.x; v < nch * N; v += 64 * SB_W)
    a.part_dA[((int64_t)b * a.D + d0 + v / N) * N + v % N] = dAacc[v / N][v % N];
  for (int v = threadIdx.x; v < nch; v += 64 * SB_W) {
    float sD = 0.f, sb = 0.f;
#pragma unroll
    for (int q = 0; q < SB_W; ++q) {
      sD += dDacc[v][q];
      sb += dbacc[v][q];
    }
    a.part_dD[(int64_t)b * a.D + d0 + v] = sD;
    a.part_dbias[(int64_t)b * a.D + d0 + v] = sb;
  }
}

// ---- backward, wave-per-state-group form (bf16, N = 16, D % 64 == 0, L % 16 == 0) -------------
// The mirror of selscan_fwd_sg_k: a workgroup owns 64 channels of one batch row, lane = channel, wave w
// owns states 4w .. 4w+3 (two float2 pairs), and time is walked BACKWARDS in 16-step tiles, one step after
// the other -- no scans.  The forward saved the state at every tile start (carry_t = 16), so per tile a
// wave
//   * replays the tile forward from its saved state, keeping h_t (4 states x 16 steps = 64 VGPRs);
//   * runs the adjoint lam_t = dy_t C_t + x_t, x_{t-1} = a_t lam_t backwards with packed f32 math; B / C do
//     not depend on the channel, so they are SGPR operands (one dword per lane + v_readlane, as forward);
//   * keeps dA[d, n] = sum_t dt lam a h_{t-1} in the lane (one (d, n) per lane and register);
//   * reduces dB[t, n] = sum_d lam dt u and dC[t, n] = sum_d dy h over the 64 lanes with a register
//     butterfly every 4 steps (v_permlane32_swap / v_permlane16_swap halves, then DPP row rotations):
//     one partial per 64-channel group, summed in fixed order by selscan_reduce_bc_k;
//   * meets the other 3 waves in LDS for the sums over states (lam B, A lam a h, C h), and the tile is
//     finished (du, ddelta, dz, dD, ddelta_bias) by all 256 threads: channel tid / 4, steps 2 (tid % 4)
//     and 2 (tid % 4) + 1 of each half -- the same threads that staged those steps.
// Per lane and step: 2 x (pk_mul, 2 exp, pk_mul, pk_fma) replay + 2 x (pk_mul, 2 exp, 11 pk ops) adjoint.
// Deterministic: every partial has one writer and every sum a fixed order.
constexpr int SGB_T = kSelScanCarrySG;  // backward tile = forward carry granularity
#ifndef SGB_NAV
#define SGB_NAV 16  // steps per tile whose exp(dt A) the replay keeps for the adjoint (all: 256 VGPRs, no spill; 8: -1.6%, 12: -2.8%, 16: -4..6% kernel time)
#endif
static_assert(SGB_T == SG_T, "the forward writes a carry at every one of its tiles");

// v_permlane32_swap / v_permlane16_swap (inline asm: the clang builtins of this ROCm return the first
// result twice, `v_add x, x` after the swap): x <- [x_lo, y_lo], y <- [x_hi, y_hi] (32-lane halves) and
// x <- [x_r0, y_r0, x_r2, y_r2], y <- [x_r1, y_r1, x_r3, y_r3] (16-lane rows).  The s_nop covers a VALU
// write -> swap read (2 wait states, as the compiler places between swaps).
// sums over the 64 lanes of two sets of 8 values per lane (dB and dC of two steps); lane l returns the
// totals of value (l >> 3) & 7 of each set.  The independent swaps of a stage share one asm block, so only
// its first instruction needs the wait states after the VALU writes of its inputs.
__device__ __forceinline__ void lane_sum8x2(const float (&u)[8], const float (&v)[8], float& ru, float& rv) {
  const int lane = threadIdx.x & 63;
  float a0 = u[0], a1 = u[1], a2 = u[2], a3 = u[3], b0 = u[4], b1 = u[5], b2 = u[6], b3 = u[7];
  float c0 = v[0], c1 = v[1], c2 = v[2], c3 = v[3], d0 = v[4], d1 = v[5], d2 = v[6], d3 = v[7];
  // xor 32: lanes 0-31 keep value i, lanes 32-63 value i + 4
  asm volatile("s_nop 1\n\t"
               "v_permlane32_swap_b32 %0, %4\n\tv_permlane32_swap_b32 %1, %5\n\t"
               "v_permlane32_swap_b32 %2, %6\n\tv_permlane32_swap_b32 %3, %7\n\t"
               "v_permlane32_swap_b32 %8, %12\n\tv_permlane32_swap_b32 %9, %13\n\t"
               "v_permlane32_swap_b32 %10, %14\n\tv_permlane32_swap_b32 %11, %15"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3),
                 "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));
  float e0 = a0 + b0, e1 = a1 + b1, e2 = a2 + b2, e3 = a3 + b3;
  float f0 = c0 + d0, f1 = c1 + d1, f2 = c2 + d2, f3 = c3 + d3;
  // xor 16: even rows keep i, odd rows i + 2
  asm volatile("s_nop 1\n\t"
               "v_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3\n\t"
               "v_permlane16_swap_b32 %4, %6\n\tv_permlane16_swap_b32 %5, %7"
               : "+v"(e0), "+v"(e1), "+v"(e2), "+v"(e3), "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
  const float g0 = e0 + e2, g1 = e1 + e3, h0 = f0 + f2, h1 = f1 + f3;
  // xor 8 (row_ror:8): bit 3 clear keeps value 0, set keeps value 1; then the remaining 8 lanes of each
  // half row hold the same value: half-row mirror, then the quad
  const bool hi = lane & 8;
  const float pu0 = g0 + dppf<0x128>(0.f, g0), pu1 = g1 + dppf<0x128>(0.f, g1);  // DPP on every lane,
  const float pv0 = h0 + dppf<0x128>(0.f, h0), pv1 = h1 + dppf<0x128>(0.f, h1);  // then the select
  float zu = hi ? pu1 : pu0;
  float zv = hi ? pv1 : pv0;
  zu += dppf<0x141>(0.f, zu);
  zv += dppf<0x141>(0.f, zv);
  zu += dppf<0xB1>(0.f, zu);  // quad_perm [1,0,3,2]
  zv += dppf<0xB1>(0.f, zv);
  zu += dppf<0x4E>(0.f, zu);  // quad_perm [2,3,0,1]
  zv += dppf<0x4E>(0.f, zv);
  ru = zu;
  rv = zv;
}

//
// DTF (fused dt_proj): as the forward, delta_raw of the tile is recomputed by one MFMA chain per wave from W_dt and
// the staged x_dbl tile (over sS, which is not live between the finish of one tile and the adjoint of the next), and
// each lane writes dt, dt u and softplus' of its 4 channels x 1 step behind one extra barrier.  Bitwise the same
// delta as the forward (same operands, same instruction sequence).
template <int KS>  // KS = 0: delta read from memory; KS > 0: fused dt_proj, KS = ceil(R / 32) MFMA K-steps
__global__ __launch_bounds__(256) void selscan_bwd_sg_k(SelScanArgs a) {
  constexpr int N = 16, T = SGB_T, TH = SGB_T / 2;
  constexpr bool DTF = KS > 0;
  // per step and channel: dt, dt u, dout silu(z) (adjoint) and u, softplus', dout silu'(z) (finish)
  // Rows of 64 channels, column c of step row t stored at c ^ sw(t): the step loops read / write a whole row (a
  // permutation: conflict-free), the staging and finish passes touch (t = 8 hf + 2 sp + e, c = tid / 4), whose 32-lane
  // groups then hit 32 distinct banks (a 65-float pitch put 2-3 lanes on a bank there, and a conflict-free pitch of 68
  // would not fit two workgroups per CU)
  __shared__ float dlS[T][64], duS[T][64], dyS[T][64], uS[T][64], sdS[T][64], gzS[T][64];
  __shared__ __attribute__((aligned(16))) float sS[4][3][T][64];  // per wave: sum_n lam B, A lam a h, C h
  auto sw = [](int t, int c) { return c ^ (8 * ((t >> 1) & 3)); };
  bf16_t* const xS = reinterpret_cast<bf16_t*>(&sS[0][0][0][0]);  // DTF: x_dbl tile [32 ceil(R / 32)][16]
  __shared__ __attribute__((aligned(16))) float BCs[4][T][8];  // per wave and step: B of its 4 states, C
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wgs_per_b = a.D / 64;
  const int b = a.binner ? blockIdx.x % a.B : blockIdx.x / wgs_per_b;
  const int dg = a.binner ? blockIdx.x / a.B : blockIdx.x % wgs_per_b, d0 = dg * 64;
  const int g = d0 / (a.D / a.G);
  const int d = d0 + lane;
  // staging / finishing role: channel sr, steps 2 sp, 2 sp + 1 of each half tile.  Rows are addressed
  // as a uniform base (SGPRs) plus a 32-bit per-thread offset (host: every row offset < 2^31).
  const int sr = threadIdx.x >> 2, sp = threadIdx.x & 3;
  const bf16_t* ub = (const bf16_t*)a.u_ + (int64_t)b * a.sub + (int64_t)d0 * a.sud;
  const bf16_t* db = DTF ? nullptr : (const bf16_t*)a.delta_ + (int64_t)b * a.sdb + (int64_t)d0 * a.sdd;
  const bf16_t* gb = (const bf16_t*)a.dout_ + (int64_t)b * a.sgb + (int64_t)d0 * a.sgd;
  const bf16_t* zb = a.z_ ? (const bf16_t*)a.z_ + (int64_t)b * a.szb + (int64_t)d0 * a.szd : nullptr;
  bf16_t* dub = (bf16_t*)a.du_ + (int64_t)b * a.sdub + (int64_t)d0 * a.sdud;
  bf16_t* ddb = (bf16_t*)a.ddelta_ + (int64_t)b * a.sddb + (int64_t)d0 * a.sddd;
  bf16_t* dzb = (a.z_ && a.dz_) ? (bf16_t*)a.dz_ + (int64_t)b * a.sdzb + (int64_t)d0 * a.sdzd : nullptr;
  const int ou = sr * (int)a.sud + 2 * sp, od = sr * (int)a.sdd + 2 * sp, og = sr * (int)a.sgd + 2 * sp,
            oz = sr * (int)a.szd + 2 * sp;
  const float sbias = a.delta_bias ? a.delta_bias[d0 + sr] : 0.f;
  const float sD = a.D_ ? a.D_[d0 + sr] : 0.f;
  ss_f2 A2[2], An[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    An[p] = ss_f2{a.A[d * N + 4 * w + 2 * p], a.A[d * N + 4 * w + 2 * p + 1]};
    A2[p] = An[p] * kLog2e;
  }
  const int ntile = a.L / T;
  const int ndg = a.D / 64;
  // next tile's inputs, in flight during the current one: this thread's u / delta / dout / z dwords
  // (2 steps of each half), the wave's B / C dword (lane = 16 n + 8 [C] + j) and the lane's saved state
  uint32_t nu[2], nr[2], ng[2], nz[2];
  uint32_t nbc = 0u;
  float4 nh;
  // DTF: x_dbl tile staging (thread tid: row tid / 2, steps 8 (tid % 2) ..), W_dt operand rows, accumulator channels
  const int xr = threadIdx.x >> 1, xh = threadIdx.x & 1, g16 = lane >> 4, li = lane & 15;
  const bool xld = DTF && threadIdx.x < 2 * a.R;
  const bf16_t* xrow = DTF ? (const bf16_t*)a.dtx_ + (int64_t)min(xr, a.R - 1) * a.sdtx + (int64_t)b * a.L + 8 * xh
                           : nullptr;
  // the lane's W_dt operand for every K-step and its 4 channels' bias stay in registers for the whole walk (the
  // backward has the VGPRs; reloading them per tile put an L2 round trip on every tile's critical path)
  bf16x8 wf[KS > 0 ? KS : 1];
  float bias4[4] = {0.f, 0.f, 0.f, 0.f};
  if (DTF) {
    const bf16_t* wrow = (const bf16_t*)a.dtw_ + (int64_t)(d0 + 16 * w + li) * a.R + 8 * g16;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[ks] = 32 * ks + 8 * g16 < a.R ? *reinterpret_cast<const bf16x8*>(wrow + 32 * ks) : bf16x8{};
    if (a.delta_bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bias4[r] = a.delta_bias[d0 + 16 * w + 4 * g16 + r];
    }
  }
  uint4 nx = make_uint4(0u, 0u, 0u, 0u);
  const bf16_t* Bw = ((const bf16_t*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g * a.sBg + (int64_t)(4 * w) * a.sBn;
  const bf16_t* Cw = ((const bf16_t*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g * a.sCg + (int64_t)(4 * w) * a.sCn;
  const int bl_n = lane >> 4, bl_m = (lane >> 3) & 1, bl_j = lane & 7;
  const int obc = bl_n * (int)(bl_m ? a.sCn : a.sBn) + 2 * bl_j;
  const float* cb = a.carries + carry_index(a, b, d0, 0) + 4 * w;  // (B, nct, D, N)
  const int oc = lane * N, ocj = a.D * N;
  auto fetch = [&](int tile) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int t = tile * T + TH * hf;
      nu[hf] = *reinterpret_cast<const uint32_t*>(ub + t + ou);
      if (!DTF) nr[hf] = *reinterpret_cast<const uint32_t*>(db + t + od);
      ng[hf] = *reinterpret_cast<const uint32_t*>(gb + t + og);
      nz[hf] = zb ? *reinterpret_cast<const uint32_t*>(zb + t + oz) : 0u;
    }
    if (bl_m) nbc = *reinterpret_cast<const uint32_t*>(Cw + tile * T + obc);
    else nbc = *reinterpret_cast<const uint32_t*>(Bw + tile * T + obc);
    nh = *reinterpret_cast<const float4*>(cb + tile * ocj + oc);
    if (xld) nx = *reinterpret_cast<const uint4*>(xrow + tile * T);
  };
  ss_f2 x[2] = {ss_f2{0.f, 0.f}, ss_f2{0.f, 0.f}};  // adjoint carried into the step after the tile
  ss_f2 dA[2] = {ss_f2{0.f, 0.f}, ss_f2{0.f, 0.f}};
  float dDp = 0.f, dbp = 0.f;
  // this lane's dB / dC totals (lane_sum8x2): state 4 w + ((lane >> 3) & 3), step t2 + (lane >> 5)
  // stored through buffer descriptors over the wave's 4 state rows: the lane part of the offset is one VGPR for the
  // whole walk, the tile's step in an SGPR and the step pair's in the immediate (64-bit lane addresses were
  // recomputed at every step pair)
  float* pdB = a.part_dB + (((int64_t)b * ndg + dg) * N + 4 * w) * a.L;
  float* pdC = a.part_dC + (((int64_t)b * ndg + dg) * N + 4 * w) * a.L;
  const __amdgpu_buffer_rsrc_t rdB = __builtin_amdgcn_make_buffer_rsrc(pdB, (short)0, 16 * a.L, 0x00020000);
  const __amdgpu_buffer_rsrc_t rdC = __builtin_amdgcn_make_buffer_rsrc(pdC, (short)0, 16 * a.L, 0x00020000);
  const int opd = 4 * (((lane >> 3) & 3) * a.L + (lane >> 5));
  fetch(ntile - 1);
  for (int tile = ntile - 1; tile >= 0; --tile) {
    const int t0 = tile * T;
    __syncthreads();  // the previous tile's readers of the staged rows are done
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        auto upk = [&](uint32_t q) { return __uint_as_float(e ? (q & 0xffff0000u) : (q << 16)); };
        const float u = upk(nu[hf]), go = upk(ng[hf]), zz = upk(nz[hf]);
        const float sg = sigmoid_fast(zz);
        const int tl = TH * hf + 2 * sp + e;
        if (!DTF) {
          const float v = upk(nr[hf]) + sbias;
          const float dl = a.softplus ? softplus_fast(v) : v;
          dlS[tl][sw(tl, sr)] = dl;
          duS[tl][sw(tl, sr)] = dl * u;
          sdS[tl][sw(tl, sr)] = a.softplus ? sigmoid_fast(v) : 1.f;
        }
        dyS[tl][sw(tl, sr)] = zb ? go * (zz * sg) : go;
        uS[tl][sw(tl, sr)] = u;
        gzS[tl][sw(tl, sr)] = zb ? go * sg * (1.f + zz * (1.f - sg)) : 0.f;
      }
    }
    if (DTF && threadIdx.x < 2 * 32 * KS)
      *reinterpret_cast<uint4*>(xS + 16 * xr + 8 * xh) = xld ? nx : make_uint4(0u, 0u, 0u, 0u);
    // B / C are the same for every lane: broadcast LDS reads in the step loops
    BCs[w][2 * bl_j][4 * bl_m + bl_n] = __uint_as_float(nbc << 16);
    BCs[w][2 * bl_j + 1][4 * bl_m + bl_n] = __uint_as_float(nbc & 0xffff0000u);
    const ss_f2 hst[2] = {ss_f2{nh.x, nh.y}, ss_f2{nh.z, nh.w}};
    __syncthreads();
    if (tile > 0) fetch(tile - 1);
    if (DTF) {
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc = mfma16(wf[ks], frag_tr(xS, 16, 32 * ks, 0), acc);
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int ch = 16 * w + 4 * g16 + r4;
        const float v = acc[r4] + bias4[r4];
        const float dl = a.softplus ? softplus_fast(v) : v;
        dlS[li][sw(li, ch)] = dl;
        duS[li][sw(li, ch)] = dl * uS[li][sw(li, ch)];
        sdS[li][sw(li, ch)] = a.softplus ? sigmoid_fast(v) : 1.f;
      }
      __syncthreads();  // every wave's channels of the tile are in dlS / duS / sdS
    }
    auto ldB = [&](int t, ss_f2 (&o)[2]) {
      const float4 q = *reinterpret_cast<const float4*>(&BCs[w][t][0]);
      o[0] = ss_f2{q.x, q.y};
      o[1] = ss_f2{q.z, q.w};
    };
    auto ldC = [&](int t, ss_f2 (&o)[2]) {
      const float4 q = *reinterpret_cast<const float4*>(&BCs[w][t][4]);
      o[0] = ss_f2{q.x, q.y};
      o[1] = ss_f2{q.z, q.w};
    };
    // replay the tile from its saved state, keeping h_t of every step
    // exp(dt A) of the last NAV steps is kept for the adjoint, which starts there (short-lived registers around the
    // replay -> adjoint turn); the earlier steps' are recomputed
    constexpr int NAV = SGB_NAV, TAV = T - NAV;
    ss_f2 hs[T][2];
    ss_f2 avs[NAV > 0 ? NAV : 1][2];
    {
      ss_f2 h[2] = {hst[0], hst[1]};
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const float dl = dlS[t][sw(t, lane)], du = duS[t][sw(t, lane)];
        ss_f2 Bv[2];
        ldB(t, Bv);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const ss_f2 e = A2[p] * dl;
          const ss_f2 av = ss_f2{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
          h[p] = __builtin_elementwise_fma(av, h[p], Bv[p] * du);
          hs[t][p] = h[p];
          if (t >= TAV) avs[t >= TAV ? t - TAV : 0][p] = av;
        }
      }
    }
    // re-read dt / B / C from LDS and recompute exp(dt A) below rather than keep the replay's values
    // live across the tile (register pressure)
    asm volatile("" ::: "memory");
    // the adjoint, backwards, two steps at a time (one lane butterfly per two steps for dB and dC)
#pragma unroll
    for (int t2 = T - 2; t2 >= 0; t2 -= 2) {
      float cB[8], cC[8];  // value 4 k + n_local for step t2 + k
#pragma unroll
      for (int k = 1; k >= 0; --k) {
        const int t = t2 + k;
        const float dl = dlS[t][sw(t, lane)], du = duS[t][sw(t, lane)], dy = dyS[t][sw(t, lane)];
        ss_f2 s1 = ss_f2{0.f, 0.f}, s2 = s1, yy = s1;
        ss_f2 Bv[2], Cv[2];
        ldB(t, Bv);
        ldC(t, Cv);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          ss_f2 av;
          if (t >= TAV) {
            av = avs[t >= TAV ? t - TAV : 0][p];
          } else {
            const ss_f2 e = A2[p] * dl;
            av = ss_f2{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
          }
          const ss_f2 Bp = Bv[p], Cp = Cv[p];
          const ss_f2 lam = __builtin_elementwise_fma(Cp, ss_f2{dy, dy}, x[p]);
          const ss_f2 hp = t > 0 ? hs[t > 0 ? t - 1 : 0][p] : hst[p];
          const ss_f2 t1 = lam * (av * hp);  // lam a_t h_{t-1}
          const ss_f2 cb = lam * du, cc = hs[t][p] * dy;
          cB[4 * k + 2 * p] = cb.x; cB[4 * k + 2 * p + 1] = cb.y;
          cC[4 * k + 2 * p] = cc.x; cC[4 * k + 2 * p + 1] = cc.y;
          s1 = __builtin_elementwise_fma(lam, Bp, s1);
          s2 = __builtin_elementwise_fma(An[p], t1, s2);
          yy = __builtin_elementwise_fma(Cp, hs[t][p], yy);
          dA[p] = __builtin_elementwise_fma(t1, ss_f2{dl, dl}, dA[p]);
          x[p] = av * lam;
        }
        sS[w][0][t][sw(t, lane)] = s1.x + s1.y;
        sS[w][1][t][sw(t, lane)] = s2.x + s2.y;
        sS[w][2][t][sw(t, lane)] = yy.x + yy.y;
      }
      float rb, rc;
      lane_sum8x2(cB, cC, rb, rc);
      asm volatile("" : "+v"(rb), "+v"(rc));  // finish the sums here: sunk into the branch, their last DPP add
                                             // no longer folds (v_mov 0 + v_mov_dpp + v_add instead of v_add_dpp)
      if ((lane & 7) == 0) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, rb), rdB, opd + 4 * t2, 4 * t0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, rc), rdC, opd + 4 * t2, 4 * t0, 0);
      }
    }
    __syncthreads();  // the 4 waves' sums over states of the tile are in LDS
    // finish: this thread's 2 steps of each half (the ones it staged)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      float o_du[2], o_dd[2], o_dz[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int tl = TH * hf + 2 * sp + e;
        const int cs = sw(tl, sr);
        const float S1 = (sS[0][0][tl][cs] + sS[1][0][tl][cs]) + (sS[2][0][tl][cs] + sS[3][0][tl][cs]);
        const float S2 = (sS[0][1][tl][cs] + sS[1][1][tl][cs]) + (sS[2][1][tl][cs] + sS[3][1][tl][cs]);
        const float Y = (sS[0][2][tl][cs] + sS[1][2][tl][cs]) + (sS[2][2][tl][cs] + sS[3][2][tl][cs]);
        const float dl = dlS[tl][cs], dy = dyS[tl][cs], u = uS[tl][cs];
        o_du[e] = fmaf(dl, S1, sD * dy);
        o_dd[e] = fmaf(u, S1, S2) * sdS[tl][cs];
        o_dz[e] = gzS[tl][cs] * fmaf(sD, u, Y);
        dDp = fmaf(dy, u, dDp);
        dbp += o_dd[e];
      }
      const int t = t0 + TH * hf;
      *reinterpret_cast<unsigned*>(dub + t + sr * (int)a.sdud + 2 * sp) = pack2(o_du[0], o_du[1]);
      *reinterpret_cast<unsigned*>(ddb + t + sr * (int)a.sddd + 2 * sp) = pack2(o_dd[0], o_dd[1]);
      if (dzb) *reinterpret_cast<unsigned*>(dzb + t + sr * (int)a.sdzd + 2 * sp) = pack2(o_dz[0], o_dz[1]);
    }
  }
  {
    float4* pa = reinterpret_cast<float4*>(a.part_dA + ((int64_t)b * a.D + d) * N + 4 * w);
    float4 v = make_float4(dA[0].x, dA[0].y, dA[1].x, dA[1].y);
    if (a.pacc) {
      const float4 o = *pa;
      v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
    }
    *pa = v;
  }
  // dD / ddelta_bias: the 4 threads of a channel are one quad
  dDp += dppf<0xB1>(0.f, dDp);
  dDp += dppf<0x4E>(0.f, dDp);
  dbp += dppf<0xB1>(0.f, dbp);
  dbp += dppf<0x4E>(0.f, dbp);
  if (sp == 0) {
    const int64_t o = (int64_t)b * a.D + d0 + sr;
    a.part_dD[o] = a.pacc ? a.part_dD[o] + dDp : dDp;
    a.part_dbias[o] = a.pacc ? a.part_dbias[o] + dbp : dbp;
  }
}

// dB[b,g,n,t] = sum over the channel groups that belong to group g
template <typename T>
__global__ void selscan_reduce_bc_k(SelScanArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over B*G*N*L
  const int N = a.N;
  const int64_t total = (int64_t)a.B * a.G * N * a.L;
  if (i >= total) return;
  const int t = i % a.L;
  const int n = (i / a.L) % N;
  const int g = (i / ((int64_t)a.L * N)) % a.G;
  const int b = i / ((int64_t)a.L * N * a.G);
  const int ndg = (a.D + a.Kc - 1) / a.Kc;
  const int dpg = a.D / a.G;
  const int dg0 = (g * dpg) / a.Kc, dg1 = ((g + 1) * dpg + a.Kc - 1) / a.Kc;
  float sb = 0.f, sc = 0.f;
  for (int dg = dg0; dg < dg1; ++dg) {
    const int64_t o = (((int64_t)b * ndg + dg) * N + n) * a.L + t;
    sb += a.part_dB[o];
    sc += a.part_dC[o];
  }
  st(((T*)a.dB_) + (int64_t)b * a.sdBb + (int64_t)g * a.sdBg + (int64_t)n * a.sdBn + t, sb);
  st(((T*)a.dC_) + (int64_t)b * a.sdCb + (int64_t)g * a.sdCg + (int64_t)n * a.sdCn + t, sc);
}

// the same sum, 4 consecutive steps per thread (16-B partial loads, 8-B bf16 stores) with the channel groups' loads
// unrolled 4 deep: the scalar form above kept one 4-B load pair per group in flight (48 -> see
// profiles/r6/reduce_bc_vec.txt).  Needs L % 4 == 0 and 8-B aligned dB / dC rows (host-checked).
__global__ void selscan_reduce_bc4_k(SelScanArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over B*G*N*L/4
  const int N = a.N, L4 = a.L >> 2;
  const int64_t total = (int64_t)a.B * a.G * N * L4;
  if (i >= total) return;
  const int t = (int)(i % L4) * 4;
  const int n = (int)((i / L4) % N);
  const int g = (int)((i / ((int64_t)L4 * N)) % a.G);
  const int b = (int)(i / ((int64_t)L4 * N * a.G));
  const int ndg = (a.D + a.Kc - 1) / a.Kc;
  const int dpg = a.D / a.G;
  const int dg0 = (g * dpg) / a.Kc, dg1 = ((g + 1) * dpg + a.Kc - 1) / a.Kc;
  float4 sb = make_float4(0.f, 0.f, 0.f, 0.f), sc = sb;
#pragma unroll 4
  for (int dg = dg0; dg < dg1; ++dg) {
    const int64_t o = (((int64_t)b * ndg + dg) * N + n) * a.L + t;
    const float4 pb = *reinterpret_cast<const float4*>(a.part_dB + o);
    const float4 pc = *reinterpret_cast<const float4*>(a.part_dC + o);
    sb.x += pb.x; sb.y += pb.y; sb.z += pb.z; sb.w += pb.w;
    sc.x += pc.x; sc.y += pc.y; sc.z += pc.z; sc.w += pc.w;
  }
  bf16_t* db = ((bf16_t*)a.dB_) + (int64_t)b * a.sdBb + (int64_t)g * a.sdBg + (int64_t)n * a.sdBn + t;
  bf16_t* dc = ((bf16_t*)a.dC_) + (int64_t)b * a.sdCb + (int64_t)g * a.sdCg + (int64_t)n * a.sdCn + t;
  *reinterpret_cast<uint2*>(db) = make_uint2(pack2(sb.x, sb.y), pack2(sb.z, sb.w));
  *reinterpret_cast<uint2*>(dc) = make_uint2(pack2(sc.x, sc.y), pack2(sc.z, sc.w));
}

#define SS_DISPATCH(...)                                                            \
  do {                                                                              \
    if (a.dtype == kBF16 && a.N == 16) { using TT = bf16_t; constexpr int NN = 16; __VA_ARGS__; } \
    else if (a.dtype == kF32 && a.N == 16) { using TT = float; constexpr int NN = 16; __VA_ARGS__; } \
    else if (a.dtype == kBF16 && a.N == 8) { using TT = bf16_t; constexpr int NN = 8; __VA_ARGS__; } \
    else if (a.dtype == kF32 && a.N == 8) { using TT = float; constexpr int NN = 8; __VA_ARGS__; } \
    else if (a.dtype == kBF16 && a.N == 4) { using TT = bf16_t; constexpr int NN = 4; __VA_ARGS__; } \
    else if (a.dtype == kF32 && a.N == 4) { using TT = float; constexpr int NN = 4; __VA_ARGS__; } \
    else return hipErrorInvalidValue;                                               \
  } while (0)

// the wave-per-state-group kernels: bf16 rows, 64-channel workgroups inside one B/C group
static bool sg_shape_ok(const SelScanArgs& a) {
  return a.dtype == kBF16 && a.vec && a.vecbc && (!a.z_ || a.vecz) && a.N == 16 && a.D % 64 == 0 &&
         (a.D / a.G) % 64 == 0;
}
// sequential-time forward walk when the batch has the channels to fill the GPU (>= 2048 wavefronts);
// otherwise (small batches, L not a multiple of the walk's step tile) the time-parallel DPP-scan kernel.
// Measured at B=32, D=1536, L=1024, N=16 on MI355X: 290 us vs 345 us.
static bool use_fwd_sg(const SelScanArgs& a) {
  // L >= SG_T: the per-tile B / C row reads start at min(t0, L - SG_T)
  return sg_shape_ok(a) && a.L % SF_IT == 0 && a.L >= SG_T &&
         (int64_t)a.B * a.D / 16 >= 2048;
}
// sequential-time backward: needs the forward's 16-step carries; the time-parallel backward (and 512-step
// carries) otherwise
int selscan_carry_t(const SelScanArgs& a) {
  return (use_fwd_sg(a) && a.L % SGB_T == 0) ? SGB_T : SB_T;
}
static bool use_bwd_sg(const SelScanArgs& a) {
  // 32-bit in-kernel offsets: 64 rows of every (b, d, l) tensor, 64 carry rows
  const int64_t lim = (int64_t)1 << 24;
  const bool off32 = a.sud < lim && a.sdd < lim && a.sgd < lim && (!a.z_ || a.szd < lim) && a.sdud < lim &&
                     a.sddd < lim && (!a.dz_ || a.sdzd < lim) && a.sBn < lim && a.sCn < lim && a.L < lim;
  return a.carry_t == SGB_T && sg_shape_ok(a) && a.vecg && a.L % SGB_T == 0 && a.nct == a.L / SGB_T && off32;
}
int selscan_bwd_kc(const SelScanArgs& a) { return use_bwd_sg(a) ? 64 : SB_KC; }
// fused dt_proj (DTF): the forward walk with 16-step carries (so the backward is the sequential kernel too), a dt_rank
// the 4-step MFMA chain covers, 16-B x_dbl / W_dt rows
bool selscan_dt_fusable(const SelScanArgs& a) {
  return use_fwd_sg(a) && a.L % SGB_T == 0 && a.R > 0 && a.R % 8 == 0 && a.R <= DTF_RMAX && a.sdtx % 8 == 0 &&
         (uintptr_t)a.dtx_ % 16 == 0 && (uintptr_t)a.dtw_ % 16 == 0;
}
bool selscan_bwd_sequential(const SelScanArgs& a) { return use_bwd_sg(a); }

// workgroup order of the wave-per-state-group walks: 0 = b-major (default), 1 = b fastest when the channels' rows are
// (d, b, l) memory (the Mamba-1 layout), so concurrently running workgroups read neighbouring rows.  Unlike the
// bandwidth-bound channel-first conv (15-20% faster in memory order) the VALU-bound walks lose 0.5% of the Mamba-1
// 280M step with it (profiles/r6/row_order.txt).  MAMBA_AMD_SELSCAN_ORDER sets the process default,
// set_selscan_order overrides it.
static int g_ss_order = -1;
int selscan_order() {
  if (g_ss_order < 0) {
    const char* e = getenv("MAMBA_AMD_SELSCAN_ORDER");
    g_ss_order = (e && atoi(e) == 1) ? 1 : 0;
  }
  return g_ss_order;
}
void set_selscan_order(int v) { g_ss_order = v == 1 ? 1 : 0; }
static SelScanArgs with_order(const SelScanArgs& a) {
  SelScanArgs c = a;
  c.binner = selscan_order() != 0 && a.sub < a.sud;
  return c;
}

hipError_t launch_selscan_fwd(const SelScanArgs& a_in, hipStream_t st) {
  const SelScanArgs a = with_order(a_in);
  const int64_t rows = (int64_t)a.B * a.D;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  if (a.carries && a.nct != (a.L + a.carry_t - 1) / a.carry_t) return hipErrorInvalidValue;
  if (a.dtw_) {  // fused dt_proj: the wave-per-state-group walk only
    if (!selscan_dt_fusable(a)) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(a.B * (a.D / 64)));
    switch ((a.R + 31) / 32) {
      case 1: hipLaunchKernelGGL(selscan_fwd_sg_k<1>, grid, dim3(256), 0, st, a); break;
      case 2: hipLaunchKernelGGL(selscan_fwd_sg_k<2>, grid, dim3(256), 0, st, a); break;
      case 3: hipLaunchKernelGGL(selscan_fwd_sg_k<3>, grid, dim3(256), 0, st, a); break;
      default: hipLaunchKernelGGL(selscan_fwd_sg_k<4>, grid, dim3(256), 0, st, a); break;
    }
    return hipGetLastError();
  }
  if (use_fwd_sg(a)) {
    hipLaunchKernelGGL(selscan_fwd_sg_k<0>, dim3((unsigned)(a.B * (a.D / 64))), dim3(256), 0, st, a);
    return hipGetLastError();
  }
  if (a.carry_t != SB_T) return hipErrorInvalidValue;  // the time-parallel forward saves per 512-step tile
  const bool v = a.dtype == kBF16 && a.vec && a.vecbc && (!a.z_ || a.vecz) && a.L % SF_IT == 0;
  if (v) SS_DISPATCH(hipLaunchKernelGGL((selscan_fwd_k<TT, NN, true>), grid, block, 0, st, a));
  else SS_DISPATCH(hipLaunchKernelGGL((selscan_fwd_k<TT, NN, false>), grid, block, 0, st, a));
  return hipGetLastError();
}

hipError_t launch_selscan_bwd(const SelScanArgs& a_in, hipStream_t st) {
  const SelScanArgs a = with_order(a_in);
  if (a.Kc != selscan_bwd_kc(a) || (a.carry_t != SGB_T && a.carry_t != SB_T) ||
      a.nct != (a.L + a.carry_t - 1) / a.carry_t)
    return hipErrorInvalidValue;
  if (a.pacc && !use_bwd_sg(a)) return hipErrorInvalidValue;  // only the sequential kernel adds into partials
  if (a.dtw_) {
    if (!use_bwd_sg(a) || !selscan_dt_fusable(a)) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(a.B * (a.D / 64)));
    switch ((a.R + 31) / 32) {
      case 1: hipLaunchKernelGGL(selscan_bwd_sg_k<1>, grid, dim3(256), 0, st, a); break;
      case 2: hipLaunchKernelGGL(selscan_bwd_sg_k<2>, grid, dim3(256), 0, st, a); break;
      case 3: hipLaunchKernelGGL(selscan_bwd_sg_k<3>, grid, dim3(256), 0, st, a); break;
      default: hipLaunchKernelGGL(selscan_bwd_sg_k<4>, grid, dim3(256), 0, st, a); break;
    }
  } else if (use_bwd_sg(a)) {
    hipLaunchKernelGGL(selscan_bwd_sg_k<0>, dim3((unsigned)(a.B * (a.D / 64))), dim3(256), 0, st, a);
  } else {
    dim3 grid((a.D + SB_KC - 1) / SB_KC, a.B), block(64 * SB_W);
    const bool v = a.dtype == kBF16 && a.vec && a.vecbc && a.vecg && (!a.z_ || a.vecz) && a.L % 8 == 0;
    if (v) {
      if (a.N == 16) hipLaunchKernelGGL(selscan_bwd_fast_k<16>, grid, block, 0, st, a);
      else if (a.N == 8) hipLaunchKernelGGL(selscan_bwd_fast_k<8>, grid, block, 0, st, a);
      else if (a.N == 4) hipLaunchKernelGGL(selscan_bwd_fast_k<4>, grid, block, 0, st, a);
      else return hipErrorInvalidValue;
    } else {
      SS_DISPATCH(hipLaunchKernelGGL((selscan_bwd_k<TT, NN, false>), grid, block, 0, st, a));
    }
  }
  MAMBA_HIP_CHECK(hipGetLastError());
  const int64_t total = (int64_t)a.B * a.G * a.N * a.L;
  const bool v4 = a.dtype == kBF16 && a.L % 4 == 0 && a.sdBb % 4 == 0 && a.sdBg % 4 == 0 && a.sdBn % 4 == 0 &&
                  a.sdCb % 4 == 0 && a.sdCg % 4 == 0 && a.sdCn % 4 == 0 && (uintptr_t)a.dB_ % 8 == 0 &&
                  (uintptr_t)a.dC_ % 8 == 0;
  if (v4)
    hipLaunchKernelGGL(selscan_reduce_bc4_k, dim3((unsigned)((total / 4 + 255) / 256)), dim3(256), 0, st, a);
  else if (a.dtype == kBF16)
    hipLaunchKernelGGL(selscan_reduce_bc_k<bf16_t>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(selscan_reduce_bc_k<float>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ---- single-token state update (decode), Mamba-1 and Mamba-2 forms -------------------------
// state (b, H, P, N) fp32 [Mamba-1: H = d, P = 1]; x, z (b, H, P); dt (b, H) [Mamba-1: dt per d].
// One row (b, h, p) = N contiguous states is owned by a group of LPR = min(N, 64) lanes (NPL states
// per lane, lane-strided so each load is one coalesced line); y = sum_n C_n h_n is a butterfly over
// the group.  A decode step is ~B*H*P*N*8 bytes of state traffic, so the layout is chosen for
// full-width coalesced state reads/writes and enough waves to cover the chip even at batch 1.
template <typename T, int LPR, int NPL>
__global__ __launch_bounds__(256) void ssm_update_k(SSMUpdateArgs a) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane % LPR;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const int64_t rows = (int64_t)a.B * a.H * a.P;
  float y = 0.f, xv = 0.f;
  int p = 0, h = 0, b = 0;
  if (row < rows) {
    p = row % a.P;
    h = (row / a.P) % a.H;
    b = row / ((int64_t)a.P * a.H);
    const int g = h / (a.H / a.G);
    float dt = ld((const T*)a.dt_ + (int64_t)b * a.sdtb + (int64_t)h * a.sdth + (int64_t)p * a.sdtp);
    if (a.dt_bias) dt += a.dt_bias[a.dt_bias_per_p ? h * a.P + p : h];
    if (a.softplus) dt = softplusf_(dt);
    xv = ld((const T*)a.x_ + (int64_t)b * a.sxb + (int64_t)h * a.sxh + p);
    float* st_ = a.state + row * a.N;
    const T* Bp = ((const T*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g * a.sBg;
    const T* Cp = ((const T*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g * a.sCg;
    const float dtx = dt * xv;
#pragma unroll
    for (int q = 0; q < NPL; ++q) {
      const int n = sub + q * LPR;
      const float An = a.A_per_n ? a.A[(h * a.P + p) * a.N + n] : a.A[h];
      const float nv = fmaf(st_[n], __expf(dt * An), dtx * ld(Bp + n));
      st_[n] = nv;
      y = fmaf(nv, ld(Cp + n), y);
    }
  }
#pragma unroll
  for (int off = LPR / 2; off >= 1; off >>= 1) y += __shfl_xor(y, off, 64);
  if (row < rows && sub == 0) {
    if (a.D) y += xv * a.D[a.D_per_p ? h * a.P + p : h];
    if (a.z_) y *= siluf_(ld(((const T*)a.z_) + (int64_t)b * a.szb + (int64_t)h * a.szh + p));
    st(((T*)a.out_) + (int64_t)b * a.H * a.P + (int64_t)h * a.P + p, y);
  }
}

template <typename T>
static hipError_t ssm_update_launch(const SSMUpdateArgs& a, hipStream_t st) {
  const int64_t rows = (int64_t)a.B * a.H * a.P;
#define SSM_UP(LPR, NPL)                                                                            \
  {                                                                                                 \
    const int64_t waves = (rows + (64 / LPR) - 1) / (64 / LPR);                                     \
    hipLaunchKernelGGL((ssm_update_k<T, LPR, NPL>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, a); \
    return hipGetLastError();                                                                       \
  }
  switch (a.N) {
    case 4: SSM_UP(4, 1)
    case 8: SSM_UP(8, 1)
    case 16: SSM_UP(16, 1)
    case 32: SSM_UP(32, 1)
    case 64: SSM_UP(64, 1)
    case 128: SSM_UP(64, 2)
    case 256: SSM_UP(64, 4)
    default: return hipErrorInvalidValue;
  }
#undef SSM_UP
}

hipError_t launch_ssm_update(const SSMUpdateArgs& a, hipStream_t st) {
  if (a.dtype == kBF16) return ssm_update_launch<bf16_t>(a, st);
  if (a.dtype == kF32) return ssm_update_launch<float>(a, st);
  return hipErrorInvalidValue;
}

}  // namespace mamba_amd
