// Pipelined bf16 MFMA GEMM engine for the Mamba projections (in_proj / out_proj forward,
// input gradient and weight gradient; reached from model.py:35-41 through the mixers' in_proj/out_proj).
//
//   C[M, N] (op)= A[M, K] . B[N, K]^T      fp32 accumulate, bf16 or fp32 output
//
// Each operand comes in one of two layouts, so every product of a projection runs without a transpose:
//   KC : the operand's rows hold K contiguously        (activations x[tokens, K], nn.Linear W[out, in])
//   XC : the operand is stored [K][rows], rows contiguous (dY^T / X^T for the weight gradient, W for dgrad)
// forward  y  = x W^T      A = x  (KC), B = W  (KC)
// dgrad    dx = dy W       A = dy (KC), B = W  (XC: B[n=i][k=o] = W[o][i])
// wgrad    dW = dy^T x     A = dy (XC), B = x  (XC), K = tokens, split over K into fp32 slabs
//
// MI355X design (cdna_hip_programming.md §5 "Pipelining across barriers", "glds vs register staging"):
//  * 256 x 256 (or 128 x 256) output tile per 512-thread workgroup, 8 waves as 2 (M) x 4 (N); every wave
//    owns a (BM/2) x 64 sub-tile = MI x 4 accumulators of v_mfma_f32_16x16x32_bf16 (128 acc VGPRs at 256^2).
//  * K advances in 32-deep stages through a 4-slot LDS ring filled by global_load_lds_dwordx4 (LDS-DMA:
//    no VGPR staging, no ds_write).  Stage s+4 is issued right after the barrier that retires stage s, so
//    three stages (~3k MFMA cycles) are in flight; each stage boundary waits with a COUNTED vmcnt (never 0
//    in steady state) and a raw s_barrier (no __syncthreads: its fence would drain the in-flight DMA).
//  * inside a stage the MFMAs of the first M-half run while the second half's fragments are read, and the
//    next stage's fragments are read (into a second B register set) behind the second half's MFMAs, so the
//    matrix pipe never waits on an LDS round trip.
//  * LDS images are lane-linear (what the DMA writes) with the bank-conflict swizzle applied to the
//    per-lane SOURCE address and undone on the read (rule 21):
//      KC [rows][32 k] (64-B rows): 16-B chunk c of row r at slot c ^ kc_swz(r) — the four 16-lane groups of
//         ds_read_b128 then hit 16 distinct slots (checked by hand, see kc_swz).
//      XC [32 k][128] halves (256-B rows): chunk s of k-row r at s ^ 2 xc_swz(r), read with
//         ds_read_b64_tr_b16 (hardware transpose), conflict-free for the rows one 32-lane half reads.
//  * MFMA operands are swapped (D = B_tile . A_tile^T) so each lane's 4 accumulator registers are 4
//    CONSECUTIVE output columns of one row: the epilogue stores 8 B (bf16) / 16 B (fp32) per lane and
//    needs no LDS round trip; fp32 output may accumulate in place (+=).
//  * XCD-aware bijective block remap; tiles of one M panel (and one K split) are consecutive, so they
//    share the A panel / the K slab in one XCD's L2.
//  * K tails: chunks with k >= K are DMA'd from a 16-B zero page (per-lane source), rows / columns past
//    M / N are clamped on load and never stored.
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "mfma.h"
#include "launchers.h"

namespace mamba_amd {
namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int GP_NT = 512;   // threads per workgroup
constexpr int GP_BK = 64;    // k per K-tile (one LDS buffer)

__device__ __attribute__((aligned(64))) unsigned int g_gp_zero[16];  // zero page for k >= K chunks

// KC image [rows][64 k] (128-B rows): 16-B chunk c of row r at slot c ^ (r & 7).  A ds_read_b128 lane group
// (rows 0-3 and 12-15 at chunk 4ks+g, rows 4-11 at chunk 4ks+g+1) then covers all 16 slots of a bank row.
// XC image: [64 k][128] halves (256-B rows); chunk s of k-row r at s ^ 2 xc_swz(r)
__device__ __forceinline__ int xc_swz(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

// ---- fragment reads (16 operand rows x 32 k of k-step ks, STD k order) --------------------------------------
// Lane-dependent byte offsets are computed once (lane_kc / lane_xc); the row / column block and the buffer
// are compile-time or wave-uniform, so every read is `lane VGPR + immediate` (hipcc cannot prove on its own
// that the swizzle term depends on the lane only, and otherwise keeps one address VGPR per read).
// KC: row r = r0 + (l & 15) with r0 % 16 == 0  ->  r & 7 == l & 7
__device__ __forceinline__ int lane_kc(int ks) {
  const int l = threadIdx.x & 63;
  return (l & 15) * 128 + (((4 * ks + (l >> 4)) ^ (l & 7)) << 4);
}
__device__ __forceinline__ bf16x8 ld_kc(const char* img, int lane_off, int r0) {
  return *reinterpret_cast<const bf16x8*>(img + lane_off + r0 * 128);
}
// XC: column block c0 (multiple of 16) of a [64 k][128]-halved image; k-rows 32 ks + 8 g + (li >> 2) (+4).
// The XOR mask depends on the lane only (xc_swz of those rows), the 8-B unit on c0: one offset per c0 % 128.
__device__ __forceinline__ int lane_xc(int c0) {
  const int l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int r = 8 * g + (li >> 2);
  const int u = ((c0 & 127) >> 2) + (li & 3);
  return r * 256 + ((u ^ (xc_swz(r) << 2)) << 3);
}
__device__ __forceinline__ bf16x8 ld_xc(const char* img, int lane_off, int c0, int ks) {
  const char* p = img + (c0 >> 7) * (64 * 256) + ks * (32 * 256) + lane_off;
  return cat8(tr4(reinterpret_cast<const bf16_t*>(p)), tr4(reinterpret_cast<const bf16_t*>(p + 4 * 256)));
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// pin the preceding block as [NMFMA MFMAs] with NREADS DS reads issued first, two per MFMA, then a
// scheduling fence (hipcc otherwise hoists MFMAs across the barrier and merges neighbouring K-tiles)
template <int NREADS, int NMFMA, int NVMEM = 0>
__device__ __forceinline__ void pin() {
#pragma unroll
  for (int k = 0; k < NREADS / 2; ++k) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
  }
  if constexpr (NREADS % 2) {  // odd read count (3-column-tile waves): the last read gets its own MFMA
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
  }
#pragma unroll
  for (int k = 0; k < NVMEM; ++k) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (LDS-DMA)
  }
  static_assert(NMFMA >= (NREADS + 1) / 2 + NVMEM, "pin: more reads / DMAs than MFMA slots");
  __builtin_amdgcn_sched_group_barrier(0x008, NMFMA - (NREADS + 1) / 2 - NVMEM, 0);
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace

struct GemmPipeArgs {
  const bf16_t* A; int64_t lda;
  const bf16_t* B; int64_t ldb;
  void* C; int64_t ldc; int64_t split_stride;  // elements between the fp32 slabs of consecutive K splits
  int M, N, K, kslice, splits;
  unsigned nbA, nbB;  // operand bytes covered by the buffer descriptors (gemm_wg_k)
};

// LA / LB: operand layouts (0 = KC, 1 = XC); MI: 16-row tiles per wave along M (BM = 32 MI); EPI: 0 = bf16
// store, 1 = fp32 store, 2 = fp32 +=
//
// Schedule (2 LDS buffers of one 64-deep K-tile each, t = K-tile, X = buffer t % 2, Y = the other):
//   k-step 0: read ahi | [B-half DMA of t+1 -> Y] MFMA alo x b0 | read alo, b1 (k-step 1) | MFMA ahi x b0
//   k-step 1: read ahi | MFMA alo x b1 | lgkmcnt(0), vmcnt(0) [t+1 landed in Y], s_barrier [X read by every
//             wave] | A-half DMA of t+2 -> X, read alo, b0 of t+1 from Y | MFMA ahi x b1
// so every DMA has ~one K-tile of MFMAs to land, fetches whole 128-B lines, and no block carries more than
// four LDS-DMAs or an MFMA waiting on a fragment read issued fewer than 16 MFMAs earlier.
// (A persistent variant that streams the next output tile's K-tiles behind this one's was measured slower:
// the dynamic buffer parity and tile bookkeeping cost more in the K-loop than the hidden epilogue gained.)
// WN = 4: 8 waves as 2 x 4, each 128 x 64 of the 256 x 256 tile (two per SIMD); WN = 2: 4 waves of 128 x 128
// (one per SIMD, 256 accumulator registers): half the LDS fragment reads per MFMA
// MI: 16-row tiles per wave along M (8: 256-row output tiles; 4: 128-row tiles for narrow outputs, e.g. the
// Mamba-1 x_proj's 80 rows)
template <int LA, int LB, int EPI, int WN = 4, int MI = 8>
__global__ __launch_bounds__(128 * WN) void gemm_pipe_k(GemmPipeArgs a) {
  constexpr int NT = 128 * WN;
  constexpr int NJ = 16 / WN;  // 16-col tiles per wave
  constexpr int BM = 32 * MI, BN = 16 * NJ * WN;
  constexpr int SA = BM * 128, SB = BN * 128;  // bytes per K-tile image
  constexpr int SS = SA + SB;
  constexpr int GA = BM * 8 / NT, GB = BN * 8 / NT;  // DMA instructions per thread per K-tile and operand
  constexpr int IPH = 1024 / NT;                      // XC: DMA instructions per [64][128] half
  constexpr int G = GA + GB;
  constexpr int MH = MI / 2;
  __shared__ __attribute__((aligned(1024))) char smem[2 * SS];

  const int tn = (a.N + BN - 1) / BN, tm = (a.M + BM - 1) / BM;
  const int nwg = tm * tn * a.splits;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int split = t / (tm * tn), tile = t % (tm * tn);
  const int m0 = (tile / tn) * BM, n0 = (tile % tn) * BN;
  const int kbeg = split * a.kslice, kend = min(a.K, kbeg + a.kslice);
  const int KT = (kend - kbeg + GP_BK - 1) / GP_BK;
  const int KTF = (kend - kbeg) / GP_BK;  // full K-tiles (the rest, if any, takes the zero-page check)
  const int mvalid = min(BM, a.M - m0), nvalid = min(BN, a.N - n0);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wr = w / WN, wc = w % WN;
  const int am0 = wr * (BM / 2), bn0 = wc * (BN / WN);

  // per-thread DMA sources as 32-bit BYTE offsets from the operand base at k = kbeg (host-checked to fit):
  // global_load_lds then takes the saddr + voffset form with no per-DMA 64-bit pointer registers
  unsigned off[G];
  {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const bool isA = i < GA;
      const int ii = isA ? i : i - GA;
      const int L = isA ? LA : LB;
      const int base = isA ? m0 : n0, valid = isA ? mvalid : nvalid;
      const int64_t ld = isA ? a.lda : a.ldb;
      int64_t e;
      if (L == 0) {
        const int q = ii * NT + tid, r = q >> 3, c = (q & 7) ^ (r & 7);
        e = (int64_t)(base + min(r, valid - 1)) * ld + 8 * c;
      } else {
        const int h = ii / IPH, q = (ii % IPH) * NT + tid, r = q >> 4, sx = q & 15;
        const int c = min(h * 128 + 8 * (sx ^ (2 * xc_swz(r))), valid - 8);
        e = (int64_t)r * ld + base + c;
      }
      off[i] = (unsigned)(e * 2);
    }
  }
  const int64_t stepA = LA == 0 ? GP_BK : GP_BK * a.lda;  // elements per K-tile
  const int64_t stepB = LB == 0 ? GP_BK : GP_BK * a.ldb;
  const char* baseA = reinterpret_cast<const char*>(a.A + (LA == 0 ? kbeg : (int64_t)kbeg * a.lda));
  const char* baseB = reinterpret_cast<const char*>(a.B + (LB == 0 ? kbeg : (int64_t)kbeg * a.ldb));
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // DMA of K-tile kt into buf; part 0: A's DMAs, 1: B's, 2: both
  auto dma = [&](int kt_, char* buf, bool checked, int part) {
    const int kt = __builtin_amdgcn_readfirstlane(kt_);  // opaque to LLVM's strength reduction
    const int k0 = kbeg + kt * GP_BK;
    const char* bA = baseA + kt * stepA * 2;
    const char* bB = baseB + kt * stepB * 2;
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const bool isA = i < GA;
      if ((part == 0 && !isA) || (part == 1 && isA)) continue;
      const int ii = isA ? i : i - GA;
      const void* p = (isA ? bA : bB) + off[i];
      if (checked) {  // k of this lane's chunk
        const int L = isA ? LA : LB;
        const int tid = threadIdx.x;
        int kk;
        if (L == 0) {
          const int q = ii * NT + tid, r = q >> 3;
          kk = k0 + 8 * ((q & 7) ^ (r & 7));
        } else {
          kk = k0 + (((ii % IPH) * NT + tid) >> 4);
        }
        if (kk >= kend) p = (const void*)g_gp_zero;
      }
      __builtin_amdgcn_global_load_lds(p, (lds_void*)(buf + (isA ? 0 : SA) + (ii * NT + wu * 64) * 16), 16, 0, 0);
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = zero4();

  bf16x8 alo[MH], ahi[MH], b0[NJ], b1[NJ];
  // lane offsets: KC -> one per k-step; XC -> one per 16-column block (k-step and half are immediates)
  constexpr int NOA = LA == 0 ? 2 : MI, NOB = LB == 0 ? 2 : NJ;
  int oa[NOA], ob[NOB];
#pragma unroll
  for (int i = 0; i < NOA; ++i) oa[i] = LA == 0 ? lane_kc(i) : lane_xc(am0 + 16 * i);
#pragma unroll
  for (int j = 0; j < NOB; ++j) ob[j] = LB == 0 ? lane_kc(j) : lane_xc(bn0 + 16 * j);
  auto fa = [&](const char* img, int i, int ks) -> bf16x8 {
    const int r0 = am0 + 16 * i;
    if constexpr (LA == 0) return ld_kc(img, oa[ks], r0);
    else return ld_xc(img, oa[i], r0, ks);
  };
  auto fb = [&](const char* img, int j, int ks) -> bf16x8 {
    const int c0 = bn0 + 16 * j;
    if constexpr (LB == 0) return ld_kc(img + SA, ob[ks], c0);
    else return ld_xc(img + SA, ob[j], c0, ks);
  };
  auto rd_lo = [&](const char* img, int ks, bf16x8 (&bf)[NJ]) {
#pragma unroll
    for (int i = 0; i < MH; ++i) alo[i] = fa(img, i, ks);
#pragma unroll
    for (int j = 0; j < NJ; ++j) bf[j] = fb(img, j, ks);
  };
  auto rd_hi = [&](const char* img, int ks) {
#pragma unroll
    for (int i = 0; i < MH; ++i) ahi[i] = fa(img, MH + i, ks);
  };
  auto mm_lo = [&](bf16x8 (&bf)[NJ]) {
#pragma unroll
    for (int i = 0; i < MH; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(bf[j], alo[i], acc[i][j]);
  };
  auto mm_hi = [&](bf16x8 (&bf)[NJ]) {
#pragma unroll
    for (int i = 0; i < MH; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[MH + i][j] = mfma16(bf[j], ahi[i], acc[MH + i][j]);
  };

  // one K-tile from buffer `cur` (tile kt); `nxt` holds tile kt+1 and receives tile kt+2.  `bpend`: the B
  // half of tile kt+1 is still to be issued (its A half went out at the previous K-tile's barrier)
  auto ktile = [&](int kt, char* cur, char* nxt, bool steady, bool bpend) {
    // k-step 0
    rd_hi(cur, 0);
    if (bpend) dma(kt + 1, nxt, !steady && kt + 1 >= KTF, 1);
    mm_lo(b0);
    pin<MH, MH * NJ, GB>();
    rd_lo(cur, 1, b1);
    mm_hi(b0);
    pin<MH + NJ, MH * NJ>();
    // k-step 1
    rd_hi(cur, 1);
    mm_lo(b1);
    pin<MH, MH * NJ>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave is done reading `cur`
    if (steady || kt + 1 < KT) {
      vm_wait<0>();                    // tile kt+1 has landed in `nxt`
      __builtin_amdgcn_s_barrier();    // ... for every wave; every wave is done reading `cur`
      __builtin_amdgcn_sched_barrier(0);
      if (steady) dma(kt + 2, cur, false, 0);
      else if (kt + 2 < KT) dma(kt + 2, cur, kt + 2 >= KTF, 0);
      rd_lo(nxt, 0, b0);
    }
    mm_hi(b1);
    pin<MH + NJ, MH * NJ, GA>();
  };

  if (KT > 0) {
    dma(0, smem, KTF < 1, 2);
    if (KT > 1) dma(1, smem + SS, KTF < 2, 2);
    if (KT > 1) vm_wait<G>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    rd_lo(smem, 0, b0);
  }
  int kt = 0;
  for (; kt + 4 <= KTF; kt += 2) {  // kt+2 and kt+3 exist and are full
    ktile(kt, smem, smem + SS, true, kt > 0);
    ktile(kt + 1, smem + SS, smem, true, true);
  }
  for (; kt < KT; kt += 2) {
    ktile(kt, smem, smem + SS, false, kt > 0 && kt + 1 < KT);
    if (kt + 1 < KT) ktile(kt + 1, smem + SS, smem, false, kt + 2 < KT);
  }

  // epilogue: lane holds C[m][n .. n+3], m = m0 + am0 + 16 i + (l & 15), n = n0 + bn0 + 16 j + 4 (l >> 4)
  const int mr = l & 15, nc = 4 * (l >> 4);
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int mm = am0 + 16 * i + mr;
    if (mm >= mvalid) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nn = bn0 + 16 * j + nc;
      if (nn >= nvalid) continue;
      const int64_t off = (int64_t)(m0 + mm) * a.ldc + n0 + nn;
      if constexpr (EPI == 0) {
        bf16_t* c = reinterpret_cast<bf16_t*>(a.C) + off;
        *reinterpret_cast<uint2*>(c) = make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
      } else {
        float* c = reinterpret_cast<float*>(a.C) + (int64_t)split * a.split_stride + off;
        float4 v = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        if constexpr (EPI == 2) {
          const float4 o = *reinterpret_cast<const float4*>(c);
          v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        *reinterpret_cast<float4*>(c) = v;
      }
    }
  }
}

// ---- staged-ring engine (gemm_wg_k): the split-K weight gradients and every other gp_mm product ----------------
// dW = dY^T X reduces over tokens into a small output, so each workgroup runs ONE long K-loop (171 K-tiles of 64 at
// the 280M in_proj shape) and the loop alone sets the speed.  gemm_pipe_k's 2-buffer ring gives every LDS-DMA one
// 64-deep K-tile to land and drains it with vmcnt(0) at the barrier; worse, hipcc cannot tell its
// global_load_lds writes from the LDS reads that follow (ds_read_b64_tr_b16 builtins) and waits vmcnt(0) right
// after each DMA issue.  Here:
//  * the K-loop advances in 32-deep STAGES through an NB-slot ring (NB x 32 KB at 256 x 256):
//      stage s: read ahi(s) | MFMA alo(s) x b(s) | lgkmcnt(0); vmcnt(G (NB-2)) [stage s+1 landed]; s_barrier
//               [slot s read by every wave] | DMA stage s+NB -> slot s, read alo(s+1), b(s+1) | MFMA ahi(s) x b(s)
//    so a stage's DMA has NB-1 stages to land and no wait drains the ring (b alternates between two register sets
//    by stage parity; the steady loop is unrolled to lcm(NB, 2) stages so every slot address is a constant);
//  * operands are DMA'd with buffer_load ... lds through descriptors that cover exactly the operands' bytes (rows
//    past M / N and k-rows past K read as zeros; KC k-chunks past K get an out-of-range offset), and every LDS
//    fragment read is inline asm with explicit lgkmcnt waits, so hipcc inserts no DMA drain;
//  * images: XC [32 k][128] halves (256-B rows, gemm_pipe_k's xc_swz swizzle, ds_read_b64_tr_b16 x 2 per
//    fragment); KC [rows][32 k] (64-B rows, 16-B chunk c of row r at c ^ kc32_swz(r): every 16-lane group of a
//    ds_read_b128 hits 16 distinct slots of a bank row).
// Split-K slices sit on gemm_pipe_k's 64-token grid, and the k order (one MFMA per 32 tokens, in sequence) is the
// same, so both engines write the same slabs bit for bit (MAMBA_AMD_WG_NB=0 routes gp_mm back to gemm_pipe_k).
// 4 slots measured faster than 5 at every weight-gradient shape (profiles/r5/wg_engine_ab.txt).
__device__ __forceinline__ int kc32_swz(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }  // [0, 2, 3, 1]

template <int LA, int LB, int EPI, int NB, int MI>
__global__ __launch_bounds__(512) void gemm_wg_k(GemmPipeArgs a) {
  constexpr int NT = 512, WN = 4, NJ = 4, MH = MI / 2;
  constexpr int BM = 32 * MI, BN = 256, BK = 32;
  constexpr int SA = BM * BK * 2, SB = BN * BK * 2, SS = SA + SB;  // bytes per operand image / slot
  constexpr int GA = BM / 128, GB = BN / 128, G = GA + GB;          // DMA instructions per thread per stage
  constexpr int RA = LA ? 2 : 1, RB = LB ? 2 : 1;                   // LDS read instructions per fragment
  static_assert(NB >= 3 && NB * SS <= 163840, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[NB * SS];

  const int tn = (a.N + BN - 1) / BN, tm = (a.M + BM - 1) / BM;
  const int nwg = tm * tn * a.splits;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int split = t / (tm * tn), tile = t % (tm * tn);
  const int m0 = (tile / tn) * BM, n0 = (tile % tn) * BN;
  const int kbeg = split * a.kslice, kend = min(a.K, kbeg + a.kslice);
  const int KT = (kend - kbeg + BK - 1) / BK;  // stages
  const int KTF = (kend - kbeg) / BK;          // full stages
  const int mvalid = min(BM, a.M - m0), nvalid = min(BN, a.N - n0);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, tid = threadIdx.x;
  const int wr = w / WN, wc = w % WN;
  const int am0 = wr * (BM / 2), bn0 = wc * (BN / WN);

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, (int)a.nbA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, (int)a.nbB, 0x00020000);
  // per-thread DMA byte offsets of stage 0 (32-bit, host-checked) and the per-stage step
  // XC: instruction ii = half ii of [32 k][R]: k-row tid >> 4, chunk (tid & 15) swizzled on the source (rule 21)
  // KC: instruction ii = rows 128 ii .. +127 of [R][32 k]: row (ii 512 + tid) >> 2, 16-B chunk (tid & 3) ^ kc32_swz
  auto off0 = [&](int L, int ii, int base, int valid, int64_t ld) -> unsigned {
    if (L == 1) {
      const int kr = tid >> 4, sx = tid & 15;
      return (unsigned)((((int64_t)kbeg + kr) * ld + base + min(ii * 128 + 8 * (sx ^ (2 * xc_swz(kr))), valid - 8)) * 2);
    }
    const int r = (ii * NT + tid) >> 2, c = (tid & 3) ^ kc32_swz(r);
    return (unsigned)((((int64_t)base + r) * ld + kbeg + 8 * c) * 2);
  };
  unsigned offA[GA], offB[GB];
#pragma unroll
  for (int ii = 0; ii < GA; ++ii) offA[ii] = off0(LA, ii, m0, mvalid, a.lda);
#pragma unroll
  for (int ii = 0; ii < GB; ++ii) offB[ii] = off0(LB, ii, n0, nvalid, a.ldb);
  const unsigned stepA = LA ? (unsigned)(BK * a.lda * 2) : BK * 2u, stepB = LB ? (unsigned)(BK * a.ldb * 2) : BK * 2u;
  const int kchunk = 8 * ((tid & 3) ^ kc32_swz(tid >> 2));  // KC: this thread's k offset in a stage (all ii)
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // DMA of stage s into slot buf; `chk`: KC k-chunks past kend get an out-of-range offset (zeros)
  auto dma = [&](int s_, char* buf, bool chk) {
    const unsigned s = (unsigned)__builtin_amdgcn_readfirstlane(s_);
    const unsigned ua = __builtin_amdgcn_readfirstlane(s * stepA), ub = __builtin_amdgcn_readfirstlane(s * stepB);
    const bool dead = chk && kbeg + (int)s * BK + kchunk >= kend;
#pragma unroll
    for (int ii = 0; ii < GA; ++ii) {
      const unsigned v = (LA == 0 && dead) ? 0xFFFFFFF0u : offA[ii] + ua;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(buf + ii * 8192 + wu * 1024), 16, v, 0, 0, 0);
    }
#pragma unroll
    for (int ii = 0; ii < GB; ++ii) {
      const unsigned v = (LB == 0 && dead) ? 0xFFFFFFF0u : offB[ii] + ub;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(buf + SA + ii * 8192 + wu * 1024), 16, v, 0, 0, 0);
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = zero4();
  bf16x8 alo[MH], ahi[MH], b0[NJ], b1[NJ];
  // Fragment reads as INLINE ASM with explicit lgkmcnt waits (see above).  LDS byte addresses: XC one per
  // 16-column block (its XOR swizzle is lane- and block-dependent), KC one per operand (row blocks are immediates);
  // the slot base is added per stage.
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int lkc = (l & 15) * 64 + (((l >> 4) ^ kc32_swz(l & 15)) << 4);
  constexpr int NOA = LA ? MI : 1, NOB = LB ? NJ : 1;
  unsigned oa[NOA], ob[NOB];
#pragma unroll
  for (int i = 0; i < NOA; ++i)
    oa[i] = LA ? lds0 + ((am0 + 16 * i) >> 7) * (32 * 256) + lane_xc(am0 + 16 * i) : lds0 + am0 * 64 + lkc;
#pragma unroll
  for (int j = 0; j < NOB; ++j)
    ob[j] = LB ? lds0 + SA + ((bn0 + 16 * j) >> 7) * (32 * 256) + lane_xc(bn0 + 16 * j) : lds0 + SA + bn0 * 64 + lkc;
  auto rd_xc = [&](bf16x8& d, unsigned addr) {
    u32x2 x, y;
    asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:1024" : "=&v"(x), "=&v"(y) : "v"(addr));
    d = __builtin_bit_cast(bf16x8, __builtin_shufflevector(x, y, 0, 1, 2, 3));
  };
  auto rd_kc = [&](bf16x8& d, unsigned addr, auto off) {
    u32x4 x;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x) : "v"(addr), "n"(decltype(off)::value));
    d = __builtin_bit_cast(bf16x8, x);
  };
  // fragment i of A (16 rows) / j of B (16 columns) from the slot at byte offset `so`
  auto fa = [&](bf16x8& d, auto I, unsigned so) {
    constexpr int i = decltype(I)::value;
    if constexpr (LA) rd_xc(d, oa[i] + so);
    else rd_kc(d, oa[0] + so, std::integral_constant<int, 1024 * i>{});
  };
  auto fb = [&](bf16x8& d, auto J, unsigned so) {
    constexpr int j = decltype(J)::value;
    if constexpr (LB) rd_xc(d, ob[j] + so);
    else rd_kc(d, ob[0] + so, std::integral_constant<int, 1024 * j>{});
  };
  auto lgkm = [](auto n) {  // fenced on both sides: no MFMA may cross it either way
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(decltype(n)::value) : "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mm_lo = [&](bf16x8 (&bf)[NJ]) {
#pragma unroll
    for (int i = 0; i < MH; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(bf[j], alo[i], acc[i][j]);
  };
  // compile-time loops over fragment indices (the asm immediates and register arrays need constants)
  auto rd_ahi = [&](unsigned so) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (fa(ahi[I], std::integral_constant<int, MH + I>{}, so), ...);
    }(std::make_integer_sequence<int, MH>{});
  };
  auto rd_lo = [&](unsigned so, bf16x8 (&bn)[NJ]) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (fa(alo[I], std::integral_constant<int, I>{}, so), ...);
    }(std::make_integer_sequence<int, MH>{});
    [&]<int... J>(std::integer_sequence<int, J...>) {
      (fb(bn[J], std::integral_constant<int, J>{}, so), ...);
    }(std::make_integer_sequence<int, NJ>{});
  };
  // mm_hi (ahi x bc) with the next stage's alo / bn reads spread between its MFMAs: one fragment per MFMA
  auto mm_hi_rd = [&](bf16x8 (&bc)[NJ], bf16x8 (&bn)[NJ], unsigned so, bool rd) {
    [&]<int... Q>(std::integer_sequence<int, Q...>) {
      ([&] {
        constexpr int q = Q, i = q / NJ, j = q % NJ;
        if (rd) {
          if constexpr (q < MH) fa(alo[q], std::integral_constant<int, q>{}, so);
          else if constexpr (q < MH + NJ) fb(bn[q - MH], std::integral_constant<int, q - MH>{}, so);
        }
        acc[MH + i][j] = mfma16(bc[j], ahi[i], acc[MH + i][j]);
        __builtin_amdgcn_sched_barrier(0);
      }(), ...);
    }(std::make_integer_sequence<int, MH * NJ>{});
  };
  // stage s from slot offset `cur` (which then receives stage s+NB); slot `nxt` holds stage s+1.  `steady`:
  // stages s+1 .. s+NB exist and are full (counted vmcnt wait, unchecked DMA).  Reads in flight on entry: alo / bc
  // of stage s.
  auto stage = [&](int s, unsigned cur, unsigned nxt, bf16x8 (&bc)[NJ], bf16x8 (&bn)[NJ], bool steady) {
    rd_ahi(cur);
    lgkm(std::integral_constant<int, MH * RA>{});  // alo / bc have landed (LDS returns in order)
    mm_lo(bc);
    lgkm(std::integral_constant<int, 0>{});  // ahi has landed: this wave is done reading slot s
    const bool more = steady || s + 1 < KT;
    if (more) {
      if (steady) vm_wait<G * (NB - 2)>();  // stage s+1 has landed (NB-2 younger stages stay in flight)
      else vm_wait<0>();
      __builtin_amdgcn_s_barrier();  // ... for every wave; every wave is done reading slot s
      __builtin_amdgcn_sched_barrier(0);
      if (steady) dma(s + NB, smem + cur, false);
      else if (s + NB < KT) dma(s + NB, smem + cur, s + NB >= KTF);
    }
    mm_hi_rd(bc, bn, nxt, more);
  };

  if (KT > 0) {
#pragma unroll
    for (int s = 0; s < NB; ++s)
      if (s < KT) dma(s, smem + s * SS, s >= KTF);
    if (KT >= NB) vm_wait<G * (NB - 1)>();  // stage 0 landed
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    rd_lo(0u, b0);
  }
  // steady loop: U = lcm(NB, 2) stages per iteration
  constexpr int U = NB % 2 ? 2 * NB : NB;
  int s = 0;
#pragma unroll 1
  for (; s + U + NB <= KTF; s += U) {  // stages s+1 .. s+U-1+NB exist and are full
#pragma unroll
    for (int u = 0; u < U; u += 2) {
      stage(s + u, (u % NB) * SS, ((u + 1) % NB) * SS, b0, b1, true);
      stage(s + u + 1, ((u + 1) % NB) * SS, ((u + 2) % NB) * SS, b1, b0, true);
    }
  }
  // tail (a multiple of U stages done: stage s is in slot 0): every wait vmcnt(0)
  unsigned o0 = 0, o1 = SS, o2 = 2 * SS;
  auto adv = [](unsigned o) { return o + SS == NB * SS ? 0u : o + SS; };
#pragma unroll 1
  for (; s < KT; s += 2) {
    stage(s, o0, o1, b0, b1, false);
    if (s + 1 < KT) stage(s + 1, o1, o2, b1, b0, false);
    o0 = o2; o1 = adv(o2); o2 = adv(o1);
  }
  vm_wait<0>();
  lgkm(std::integral_constant<int, 0>{});

  // epilogue: lane holds C[m][n .. n+3], m = m0 + am0 + 16 i + (l & 15), n = n0 + bn0 + 16 j + 4 (l >> 4)
  const int mr = l & 15, nc = 4 * (l >> 4);
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int mm = am0 + 16 * i + mr;
    if (mm >= mvalid) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nn = bn0 + 16 * j + nc;
      if (nn >= nvalid) continue;
      const int64_t off = (int64_t)(m0 + mm) * a.ldc + n0 + nn;
      if constexpr (EPI == 0) {
        bf16_t* c = reinterpret_cast<bf16_t*>(a.C) + off;
        *reinterpret_cast<uint2*>(c) = make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
      } else {
        float* c = reinterpret_cast<float*>(a.C) + (int64_t)split * a.split_stride + off;
        float4 v = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        if constexpr (EPI == 2) {
          const float4 o = *reinterpret_cast<const float4*>(c);
          v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        *reinterpret_cast<float4*>(c) = v;
      }
    }
  }
}

// ---- staged-ring engine with PAIRED KC images (gemm_wg_kp_k) ----------------------------------------------------
// gemm_wg_k for products with a KC operand: such an operand's 32-deep stage is a [rows][32 k] image of 64-B rows,
// DMA'd as half cache lines (4 lanes per row), and the same product runs 1.2-1.5x slower than its XC form
// (profiles/r6/wg_kc_pairs.txt).  Here a KC operand's stages 2j and 2j+1 share one [rows][64 k] image of 128-B
// rows (gemm_pipe_k's KC layout: chunk c of row r at c ^ (r & 7)), filled by ONE DMA of whole row segments at the
// odd stage that frees it; XC operands keep their per-stage images.  Everything else is gemm_wg_k.
template <int LA, int LB, int EPI, int MI>
__global__ __launch_bounds__(512) void gemm_wg_kp_k(GemmPipeArgs a) {
  constexpr int NB = 4;
  constexpr int NT = 512, WN = 4, NJ = 4, MH = MI / 2;
  constexpr int BM = 32 * MI, BN = 256, BK = 32;
  constexpr int SA = BM * BK * 2, SB = BN * BK * 2, SS = SA + SB;  // bytes per operand image / slot
  constexpr int GA = BM / 128, GB = BN / 128, G = GA + GB;          // DMA instructions per thread per stage
  constexpr int RA = LA ? 2 : 1, RB = LB ? 2 : 1;                   // LDS read instructions per fragment
  constexpr bool PA = LA == 0, PB = LB == 0;  // paired (KC) operands
  constexpr int GX = (PA ? 0 : GA) + (PB ? 0 : GB);  // per-stage DMA instructions
  constexpr int GP = (PA ? GA : 0) + (PB ? GB : 0);  // per-stage share of the pair DMAs (2 GP at odd stages)
  static_assert(GP > 0, "a KC operand");
  static_assert(NB >= 3 && NB * SS <= 163840, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[NB * SS];
  // LDS map: [A images: NB x SA][B images: NB x SB]; a paired operand's stage positions 2q, 2q+1 share the
  // 2 S-byte image q
  auto offA = [](int p) -> unsigned { return PA ? (p >> 1) * 2 * SA : p * SA; };
  auto offB = [](int p) -> unsigned { return NB * SA + (PB ? (p >> 1) * 2 * SB : p * SB); };

  const int tn = (a.N + BN - 1) / BN, tm = (a.M + BM - 1) / BM;
  const int nwg = tm * tn * a.splits;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int split = t / (tm * tn), tile = t % (tm * tn);
  const int m0 = (tile / tn) * BM, n0 = (tile % tn) * BN;
  const int kbeg = split * a.kslice, kend = min(a.K, kbeg + a.kslice);
  const int KT = (kend - kbeg + BK - 1) / BK;  // stages
  const int KTF = (kend - kbeg) / BK;          // full stages
  const int mvalid = min(BM, a.M - m0), nvalid = min(BN, a.N - n0);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, tid = threadIdx.x;
  const int wr = w / WN, wc = w % WN;
  const int am0 = wr * (BM / 2), bn0 = wc * (BN / WN);

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, (int)a.nbA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, (int)a.nbB, 0x00020000);
  // per-thread DMA byte offsets of stage 0 (32-bit, host-checked) and the per-stage step
  // XC: instruction ii = half ii of [32 k][R]: k-row tid >> 4, chunk (tid & 15) swizzled on the source (rule 21)
  // KC: instruction ii = rows 128 ii .. +127 of [R][32 k]: row (ii 512 + tid) >> 2, 16-B chunk (tid & 3) ^ kc32_swz
  // KC pair: instruction ii = rows 64 ii .. +63 of [R][64 k]: row (ii 512 + tid) >> 3, chunk (tid & 7) ^ (row & 7)
  auto off0 = [&](int L, bool pr, int ii, int base, int valid, int64_t ld) -> unsigned {
    if (L == 1) {
      const int kr = tid >> 4, sx = tid & 15;
      return (unsigned)((((int64_t)kbeg + kr) * ld + base + min(ii * 128 + 8 * (sx ^ (2 * xc_swz(kr))), valid - 8)) * 2);
    }
    if (pr) {
      const int r = (ii * NT + tid) >> 3, c = (tid & 7) ^ (r & 7);
      return (unsigned)((((int64_t)base + r) * ld + kbeg + 8 * c) * 2);
    }
    const int r = (ii * NT + tid) >> 2, c = (tid & 3) ^ kc32_swz(r);
    return (unsigned)((((int64_t)base + r) * ld + kbeg + 8 * c) * 2);
  };
  constexpr int NDA = PA ? 2 * GA : GA, NDB = PB ? 2 * GB : GB;
  unsigned offAd[NDA], offBd[NDB];
#pragma unroll
  for (int ii = 0; ii < NDA; ++ii) offAd[ii] = off0(LA, PA, ii, m0, mvalid, a.lda);
#pragma unroll
  for (int ii = 0; ii < NDB; ++ii) offBd[ii] = off0(LB, PB, ii, n0, nvalid, a.ldb);
  const unsigned stepA = LA ? (unsigned)(BK * a.lda * 2) : BK * 2u, stepB = LB ? (unsigned)(BK * a.ldb * 2) : BK * 2u;
  // this thread's k offset inside a KC stage (all ii) / inside a KC stage pair
  const int kchunk = 8 * ((tid & 7) ^ ((tid >> 3) & 7));
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // per-stage DMA of the unpaired (XC) operands of stage s into position p
  auto dma = [&](int s_, int p) {
    const unsigned s = (unsigned)__builtin_amdgcn_readfirstlane(s_);
    const unsigned ua = __builtin_amdgcn_readfirstlane(s * stepA), ub = __builtin_amdgcn_readfirstlane(s * stepB);
    char* const bufA = smem + offA(p);
    char* const bufB = smem + offB(p);
    if constexpr (!PA) {
#pragma unroll
      for (int ii = 0; ii < GA; ++ii) {
        const unsigned v = offAd[ii] + ua;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(bufA + ii * 8192 + wu * 1024), 16, v, 0, 0, 0);
      }
    }
    if constexpr (!PB) {
#pragma unroll
      for (int ii = 0; ii < GB; ++ii) {
        const unsigned v = offBd[ii] + ub;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(bufB + ii * 8192 + wu * 1024), 16, v, 0, 0, 0);
      }
    }
  };
  // the paired operands' stages s0 (even), s0 + 1 into the pair image at position p (p even); `chk`: k-chunks past
  // kend get an out-of-range offset (zeros)
  auto dma_pair = [&](int s0_, int p, bool chk) {
    {
      const unsigned s0 = (unsigned)__builtin_amdgcn_readfirstlane(s0_);
      const unsigned ua = __builtin_amdgcn_readfirstlane(s0 * stepA), ub = __builtin_amdgcn_readfirstlane(s0 * stepB);
      const bool dead = chk && kbeg + (int)s0 * BK + kchunk >= kend;
      if constexpr (PA) {
        char* const buf = smem + offA(p);
#pragma unroll
        for (int ii = 0; ii < 2 * GA; ++ii) {
          const unsigned v = dead ? 0xFFFFFFF0u : offAd[ii] + ua;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(buf + ii * 8192 + wu * 1024), 16, v, 0, 0, 0);
        }
      }
      if constexpr (PB) {
        char* const buf = smem + offB(p);
#pragma unroll
        for (int ii = 0; ii < 2 * GB; ++ii) {
          const unsigned v = dead ? 0xFFFFFFF0u : offBd[ii] + ub;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(buf + ii * 8192 + wu * 1024), 16, v, 0, 0, 0);
        }
      }
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = zero4();
  bf16x8 alo[MH], ahi[MH], b0[NJ], b1[NJ];
  // Fragment reads as in gemm_wg_k; a paired operand has one LDS address per k half (row blocks are immediates).
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  constexpr int NOA = LA ? MI : (PA ? 2 : 1), NOB = LB ? NJ : (PB ? 2 : 1);
  unsigned oa[NOA], ob[NOB];
#pragma unroll
  for (int i = 0; i < NOA; ++i)
    oa[i] = LA ? lds0 + ((am0 + 16 * i) >> 7) * (32 * 256) + lane_xc(am0 + 16 * i) : lds0 + am0 * 128 + lane_kc(i);
#pragma unroll
  for (int j = 0; j < NOB; ++j)
    ob[j] = LB ? lds0 + ((bn0 + 16 * j) >> 7) * (32 * 256) + lane_xc(bn0 + 16 * j) : lds0 + bn0 * 128 + lane_kc(j);
  auto rd_xc = [&](bf16x8& d, unsigned addr) {
    u32x2 x, y;
    asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:1024" : "=&v"(x), "=&v"(y) : "v"(addr));
    d = __builtin_bit_cast(bf16x8, __builtin_shufflevector(x, y, 0, 1, 2, 3));
  };
  auto rd_kc = [&](bf16x8& d, unsigned addr, auto off) {
    u32x4 x;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x) : "v"(addr), "n"(decltype(off)::value));
    d = __builtin_bit_cast(bf16x8, x);
  };
  // a stage position's image offsets (A / B) and k half (paired images)
  struct Pos { unsigned sa, sb; int ks; };
  auto pos = [&](int p) -> Pos { return Pos{offA(p), offB(p) - NB * SA, p & 1}; };
  // fragment i of A (16 rows) / j of B (16 columns) of the stage at position q
  auto fa = [&](bf16x8& d, auto I, const Pos& q) {
    constexpr int i = decltype(I)::value;
    if constexpr (LA) rd_xc(d, oa[i] + q.sa);
    else rd_kc(d, (q.ks ? oa[1] : oa[0]) + q.sa, std::integral_constant<int, 2048 * i>{});
  };
  constexpr unsigned bbase = NB * SA;  // the B images' region
  auto fb = [&](bf16x8& d, auto J, const Pos& q) {
    constexpr int j = decltype(J)::value;
    if constexpr (LB) rd_xc(d, ob[j] + bbase + q.sb);
    else rd_kc(d, (q.ks ? ob[1] : ob[0]) + bbase + q.sb, std::integral_constant<int, 2048 * j>{});
  };
  auto lgkm = [](auto n) {  // fenced on both sides: no MFMA may cross it either way
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(decltype(n)::value) : "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mm_lo = [&](bf16x8 (&bf)[NJ]) {
#pragma unroll
    for (int i = 0; i < MH; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(bf[j], alo[i], acc[i][j]);
  };
  // compile-time loops over fragment indices (the asm immediates and register arrays need constants)
  auto rd_ahi = [&](const Pos& q) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (fa(ahi[I], std::integral_constant<int, MH + I>{}, q), ...);
    }(std::make_integer_sequence<int, MH>{});
  };
  auto rd_lo = [&](const Pos& q, bf16x8 (&bn)[NJ]) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (fa(alo[I], std::integral_constant<int, I>{}, q), ...);
    }(std::make_integer_sequence<int, MH>{});
    [&]<int... J>(std::integer_sequence<int, J...>) {
      (fb(bn[J], std::integral_constant<int, J>{}, q), ...);
    }(std::make_integer_sequence<int, NJ>{});
  };
  // mm_hi (ahi x bc) with the next stage's alo / bn reads spread between its MFMAs: one fragment per MFMA
  auto mm_hi_rd = [&](bf16x8 (&bc)[NJ], bf16x8 (&bn)[NJ], const Pos& q, bool rd) {
    [&]<int... Q>(std::integer_sequence<int, Q...>) {
      ([&] {
        constexpr int qq = Q, i = qq / NJ, j = qq % NJ;
        if (rd) {
          if constexpr (qq < MH) fa(alo[qq], std::integral_constant<int, qq>{}, q);
          else if constexpr (qq < MH + NJ) fb(bn[qq - MH], std::integral_constant<int, qq - MH>{}, q);
        }
        acc[MH + i][j] = mfma16(bc[j], ahi[i], acc[MH + i][j]);
        __builtin_amdgcn_sched_barrier(0);
      }(), ...);
    }(std::make_integer_sequence<int, MH * NJ>{});
  };
  // stage s from position pc (which then receives the XC operands of stage s+NB; at odd s the pair image of
  // positions pc-1, pc receives the paired operands of stages s+3, s+4); position pn holds stage s+1.  `steady`: stages s+1 .. s+NB exist and are full
  // (counted vmcnt wait, unchecked DMA).  Reads in flight on entry: alo / bc of stage s.
  auto stage = [&](int s, int pc, int pn, bf16x8 (&bc)[NJ], bf16x8 (&bn)[NJ], bool steady) {
    const Pos qc = pos(pc), qn = pos(pn);
    rd_ahi(qc);
    lgkm(std::integral_constant<int, MH * RA>{});  // alo / bc have landed (LDS returns in order)
    mm_lo(bc);
    lgkm(std::integral_constant<int, 0>{});  // ahi has landed: this wave is done reading stage s
    const bool more = steady || s + 1 < KT;
    if (more) {
      // stage s+1 has landed; younger DMAs stay in flight (issue order per stage: the unpaired stage s+4, then at
      // odd stages the pair s+3, s+4): even s waits for the pair issued at s-3 (2 GX + 2 GP younger), odd s for
      // the pair issued at s-2 (GX younger); s and pc have the same parity
      if (steady) {
        if (pc & 1) vm_wait<GX>();
        else vm_wait<2 * GX + 2 * GP>();
      } else {
        vm_wait<0>();
      }
      __builtin_amdgcn_s_barrier();  // ... for every wave; every wave is done reading stage s
      __builtin_amdgcn_sched_barrier(0);
      if (steady) {
        dma(s + NB, pc);
        if (pc & 1) dma_pair(s + 3, pc - 1, false);
      } else {
        if (s + NB < KT) dma(s + NB, pc);
        if ((pc & 1) && s + 3 < KT) dma_pair(s + 3, pc - 1, true);
      }
    }
    mm_hi_rd(bc, bn, qn, more);
  };

  if (KT > 0) {
    // the steady issue order from stage -4 on: unpaired 0, 1, pair (0, 1), unpaired 2, 3, pair (2, 3)
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      if (s < KT) dma(s, s);
      if ((s & 1) && s - 1 < KT) dma_pair(s - 1, s - 1, true);
    }
    if (KT >= NB) vm_wait<2 * GX + 2 * GP>();  // stage 0 landed
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    rd_lo(pos(0), b0);
  }
  // steady loop: U = lcm(NB, 2) stages per iteration
  constexpr int U = NB % 2 ? 2 * NB : NB;
  int s = 0;
#pragma unroll 1
  for (; s + U + NB <= KTF; s += U) {  // stages s+1 .. s+U-1+NB exist and are full
#pragma unroll
    for (int u = 0; u < U; u += 2) {
      stage(s + u, u % NB, (u + 1) % NB, b0, b1, true);
      stage(s + u + 1, (u + 1) % NB, (u + 2) % NB, b1, b0, true);
    }
  }
  // tail (a multiple of U stages done: stage s is at position 0): every wait vmcnt(0)
  int p0 = 0;
  auto adv = [](int p) { return p + 1 == NB ? 0 : p + 1; };
#pragma unroll 1
  for (; s < KT; s += 2) {
    const int p1 = adv(p0), p2 = adv(p1);
    stage(s, p0, p1, b0, b1, false);
    if (s + 1 < KT) stage(s + 1, p1, p2, b1, b0, false);
    p0 = p2;
  }
  vm_wait<0>();
  lgkm(std::integral_constant<int, 0>{});

  // epilogue: lane holds C[m][n .. n+3], m = m0 + am0 + 16 i + (l & 15), n = n0 + bn0 + 16 j + 4 (l >> 4)
  const int mr = l & 15, nc = 4 * (l >> 4);
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int mm = am0 + 16 * i + mr;
    if (mm >= mvalid) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nn = bn0 + 16 * j + nc;
      if (nn >= nvalid) continue;
      const int64_t off = (int64_t)(m0 + mm) * a.ldc + n0 + nn;
      if constexpr (EPI == 0) {
        bf16_t* c = reinterpret_cast<bf16_t*>(a.C) + off;
        *reinterpret_cast<uint2*>(c) = make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
      } else {
        float* c = reinterpret_cast<float*>(a.C) + (int64_t)split * a.split_stride + off;
        float4 v = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        if constexpr (EPI == 2) {
          const float4 o = *reinterpret_cast<const float4*>(c);
          v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        *reinterpret_cast<float4*>(c) = v;
      }
    }
  }
}

// ---- persistent engine --------------------------------------------------------------------------------------
// The same K-loop as gemm_pipe_k (256 x 256 or 128 x 256 tiles, 8 waves, 64-deep K-tiles in two LDS buffers),
// but ONE workgroup per CU walks output tiles, and the K-tile stream runs across tile boundaries: the last two
// K-tiles of tile i DMA tile i+1's first two K-tiles into the LDS buffers they free, so the next tile's
// operands land while tile i's epilogue drains.  The epilogue's stores are issued AFTER those DMAs and the
// first wait of the next tile counts past them (vmcnt(NST)): the stores stay in flight under the next tile's
// first K-tile (vmcnt counts stores too, in order).  gemm_pipe_k's ablation put ~60 % of its time at the
// in_proj forward shape in that store tail (profiles/r2_v2_gemm_pipe_ablations.log).
//
// Tiles are CLAIMED, not assigned: a workgroup's first tile is its (XCD-remapped) block index, every later
// one comes from a per-launch atomic counter (one lane, issued a K-tile ahead, published through LDS).  With
// a static walk a workgroup that starts late -- its CU still busy with the other micro-batch stream's kernels
// -- holds back its whole share of tiles; a claimed walk gives late starters fewer tiles
// (profiles/r3/pk2_whole_step_engine_ab.txt: static persistent tiles lost 4 % of the overlapped step while
// winning in isolation).  Tiles are numbered in groups of 8 M-panels, column-major inside a group, so tiles
// claimed together share A and B panels.
//
// The loop body is branch-free (hipcc stops accumulating MFMAs in place across scalar branches and spills):
// every wave issues exactly NST epilogue stores (lanes outside C write a sink), and after the last tile the
// "next tile" DMAs re-read the current tile into the free buffers, drained before exit.
//
// Operands are DMA'd with buffer_load ... lds through a descriptor that covers exactly the operand's bytes,
// so rows past M / N and k-rows past K read as zeros (no clamping, no zero page); KC k-chunks past K (the
// next row's bytes, in range) get an out-of-range offset.
//
// bf16 epilogue: each wave stages its 16 x 64 accumulator rows through a private 2 KB LDS slot (XOR-swizzled,
// conflict-free both ways) so that every global store writes 8 WHOLE 128-B row segments (16 B per lane),
// instead of 16 rows x 32 B from the accumulator layout.  RS: rows scaled by an fp32 `rowscale` vector before
// rounding (a norm's rstd folded out of the A operand).
struct GemmPkArgs {
  const bf16_t* A; int64_t lda;
  const bf16_t* B; int64_t ldb;
  bf16_t* C; int64_t ldc;
  const float* rowscale;        // RS: C[m, :] *= rowscale[m]
  int* ctr;                     // this launch's counter pair {next claim, finished workgroups}, zero on entry
  unsigned nbA, nbB;            // operand bytes covered by the buffer descriptors
  int M, N, K, tm, tn, ntiles, kte; // kte: K-tiles per output tile, rounded up to even (>= 4)
};

__device__ __attribute__((aligned(64))) uint4 g_pk_sink[64];  // epilogue stores of lanes outside C

// WN: waves along N (2 x WN waves).  WN = 4: 8 waves of (16 MI) x (16 NJ), two per SIMD (the shipped form);
// WN = 2: 4 waves, one per SIMD -- half the LDS fragment reads per MFMA, but ~20% slower at every tile shape
// (192/256 x 192/224/256; profiles/r4/pk4_four_wave_tiles_rejected.txt), so not instantiated.
template <int MI, int NJ, bool RS, bool TAIL, int WN = 4>
__global__ __launch_bounds__(128 * WN) void gemm_pk_k(GemmPkArgs a) {
  constexpr int NT = 128 * WN, MH = MI / 2, NW = 2 * WN;
  constexpr int BM = 32 * MI, BN = 16 * WN * NJ;  // WN 4: NJ = 4: 256-wide tiles; NJ = 3: 192-wide (d_model = 768 outputs)
  constexpr int SA = BM * 128, SB = BN * 128, SS = SA + SB;
  constexpr int RPI = NT / 8;  // tile rows per DMA instruction (8 lanes per 128-B row)
  constexpr int GA = BM / RPI, GB = BN / RPI, G = GA + GB;
  constexpr int CH = 2 * NJ;              // 16-B chunks per staged accumulator row (16 NJ columns)
  constexpr int PCH = (CH + 7) / 8 * 8;    // staged row pitch in chunks (the XOR swizzle permutes groups of 8)
  constexpr int STW = 16 * PCH * 16;      // staging bytes per wave (16 rows)
  constexpr int STG = NW * STW;
  constexpr int SPI = (16 * CH + 63) / 64;  // epilogue store instructions per 16-row block
  constexpr int NST = SPI * MI;             // epilogue store instructions per wave
  static_assert(NST <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(1024))) char smem[2 * SS + STG + 64];
  int* const claim = reinterpret_cast<int*>(smem + 2 * SS + STG);  // the claimed next tile, LDS-broadcast

  const int nwg = gridDim.x;
  int tile = xcd_remap(blockIdx.x, nwg);
  if (tile >= a.ntiles) return;
  const int w = threadIdx.x >> 6, tid = threadIdx.x;
  const int wr = w / WN, wc = w % WN;
  const int am0 = wr * (BM / 2), bn0 = wc * (BN / WN);
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, (int)a.nbA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, (int)a.nbB, 0x00020000);
  // KC operands: DMA instruction ii moves rows RPI ii + (tid >> 3) at 16-B chunk (tid & 7) ^ (row & 7)
  // (RPI ii, a multiple of 32, does not change row & 7), so the lane part of every offset is one VGPR per operand
  const int lrow = tid >> 3, lch = (tid & 7) ^ (lrow & 7);
  const unsigned loA = (unsigned)(((int64_t)lrow * a.lda + 8 * lch) * 2);
  const unsigned loB = (unsigned)(((int64_t)lrow * a.ldb + 8 * lch) * 2);
  const int kchunk = 8 * lch;
  auto tile_mn = [&](int t, int& m0, int& n0) {  // groups of 8 M-panels, column-major inside a group
    const int gsz = 8 * a.tn, g = t / gsz, r = t - g * gsz;
    const int gm = min(8, a.tm - 8 * g);
    m0 = (8 * g + r % gm) * BM;
    n0 = (r / gm) * BN;
  };
  // DMA K-tile kt of tile t into buf; part 0: A, 1: B, 2: both
  auto dma = [&](int t, int kt_, char* buf, int part) {
    const int kt = __builtin_amdgcn_readfirstlane(kt_);
    int m0, n0;
    tile_mn(t, m0, n0);
    const unsigned ba = __builtin_amdgcn_readfirstlane((unsigned)((int64_t)m0 * a.lda * 2) + (unsigned)kt * 128u);
    const unsigned bb = __builtin_amdgcn_readfirstlane((unsigned)((int64_t)n0 * a.ldb * 2) + (unsigned)kt * 128u);
    const bool dead = TAIL && kt * 64 + kchunk >= a.K;  // KC k-chunk past K (in range: the next row's bytes)
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const bool isA = i < GA;
      if ((part == 0 && !isA) || (part == 1 && isA)) continue;
      const int ii = isA ? i : i - GA;
      unsigned v = isA ? loA + ba + (unsigned)(RPI * ii * a.lda * 2) : loB + bb + (unsigned)(RPI * ii * a.ldb * 2);
      if (dead) v = 0xFFFFFFF0u;
      lds_void* dst = (lds_void*)(buf + (isA ? 0 : SA) + (ii * NT + wu * 64) * 16);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rA : rB, dst, 16, v, 0, 0, 0);
    }
  };

  f32x4 acc[MI][NJ];
  bf16x8 alo[MH], ahi[MH], b0[NJ], b1[NJ];
  const int ok0 = lane_kc(0), ok1 = lane_kc(1);
  auto fa = [&](const char* img, int i, int ks) -> bf16x8 { return ld_kc(img, ks ? ok1 : ok0, am0 + 16 * i); };
  auto fb = [&](const char* img, int j, int ks) -> bf16x8 { return ld_kc(img + SA, ks ? ok1 : ok0, bn0 + 16 * j); };
  auto rd_lo = [&](const char* img, int ks, bf16x8 (&bf)[NJ]) {
#pragma unroll
    for (int i = 0; i < MH; ++i) alo[i] = fa(img, i, ks);
#pragma unroll
    for (int j = 0; j < NJ; ++j) bf[j] = fb(img, j, ks);
  };
  auto rd_hi = [&](const char* img, int ks) {
#pragma unroll
    for (int i = 0; i < MH; ++i) ahi[i] = fa(img, MH + i, ks);
  };
  // zc: first MFMA of every accumulator in this K-tile (k-step 0) starts from zero
  auto mm_lo = [&](bf16x8 (&bf)[NJ], bool zc) {
#pragma unroll
    for (int i = 0; i < MH; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(bf[j], alo[i], zc ? zero4() : acc[i][j]);
  };
  auto mm_hi = [&](bf16x8 (&bf)[NJ], bool zc) {
#pragma unroll
    for (int i = 0; i < MH; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[MH + i][j] = mfma16(bf[j], ahi[i], zc ? zero4() : acc[MH + i][j]);
  };

  char* const buf0 = smem;
  char* const buf1 = smem + SS;
  const int KTE = a.kte;
  int nt = a.ntiles;  // the claimed next tile (>= ntiles: none)
  // One K-tile from `cur` (`nx` holds the next K-tile, landing or landed).  bdma: the B-half DMA (bt, bk) at
  // k-step 0; the barrier's wait leaves `wst` younger VMEM ops (the previous tile's epilogue stores) in flight;
  // rdc: read the claimed next tile (published by the barrier) before the DMA (at, ak) into `cur`, both halves
  // when `aboth`, at < 0 meaning "the claimed tile, or this one again if none".  Every call site passes
  // constant selectors.
  // clm: one lane claims the tile after this one (issued at k-step 0, landed by the barrier's vmcnt(0)) and
  // stores it in LDS after the barrier; a later barrier publishes it to every wave (rdc)
  auto ktile = [&](char* cur, char* nx, bool bdma, int bt, int bk, bool wst, int at, int ak, bool aboth, bool zc,
                   bool rdc, bool clm) {
    rd_hi(cur, 0);
    if (bdma) dma(bt, bk, nx, 1);
    int old = 0;
    if (clm && tid == 0) old = __hip_atomic_fetch_add(a.ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    mm_lo(b0, zc);
    pin<MH, MH * NJ, GB>();
    rd_lo(cur, 1, b1);
    mm_hi(b0, zc);
    pin<MH + NJ, MH * NJ>();
    rd_hi(cur, 1);
    mm_lo(b1, false);
    pin<MH, MH * NJ>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (wst) vm_wait<NST>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (clm && tid == 0) *claim = nwg + old;
    if (rdc) nt = __builtin_amdgcn_readfirstlane(*claim);
    const int t = at >= 0 ? at : (nt < a.ntiles ? nt : tile);
    dma(t, ak, cur, aboth ? 2 : 0);
    rd_lo(nx, 0, b0);
    mm_hi(b1, false);
    pin<MH + NJ, MH * NJ, GA>();
  };

  // prologue: the first tile's K-tiles 0 and 1, then its K-tile 0
  dma(tile, 0, buf0, 2);
  dma(tile, 1, buf1, 2);
  vm_wait<G>();
  __builtin_amdgcn_s_barrier();
  rd_lo(buf0, 0, b0);
  ktile(buf0, buf1, false, 0, 0, false, tile, 2, false, true, false, false);

  for (;;) {
    // K-tile 1 and the steady K-tiles (KTE >= 4)
    ktile(buf1, buf0, true, tile, 2, false, tile, 3, false, false, false, true);
#pragma unroll 1
    for (int kt = 2; kt < KTE - 2; kt += 2) {
      ktile(buf0, buf1, true, tile, kt + 1, false, tile, kt + 2, false, false, false, false);
      ktile(buf1, buf0, true, tile, kt + 2, false, tile, kt + 3, false, false, false, false);
    }
    // the last two K-tiles stream the claimed tile's K-tiles 0 and 1 (both halves) into the buffers they free
    ktile(buf0, buf1, true, tile, KTE - 1, false, -1, 0, false, false, true, false);
    const int ntc = nt < a.ntiles ? nt : tile;  // past the last tile: harmless re-reads of this one
    ktile(buf1, buf0, true, ntc, 0, false, ntc, 1, true, false, false, false);

    // ---- epilogue: lane holds C[m][n .. n+3], m = m0 + am0 + 16 i + (l & 15), n = n0 + bn0 + 16 j + 4 (l >> 4)
    // Lane-derived addressing is recomputed here (lane id from mbcnt, wave id from an SGPR): hoisted out of the
    // tile loop it would stay live across the K-loop, whose accumulator and fragment registers leave no room.
    {
      int el;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(el));
      const int ew = wu;
      const int eam0 = (ew / WN) * (BM / 2), ebn0 = (ew % WN) * (BN / WN);
      int m0, n0;
      tile_mn(tile, m0, n0);
      char* stg = smem + 2 * SS + ew * STW;
      const int r = el & 15, q = el >> 4;
      // staged row = CH 16-B chunks; store h covers chunk slots el + 64 h (slots past 16 rows go to the sink)
      float rs[MI];
      if constexpr (RS) {
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int mm = m0 + eam0 + 16 * i + r;
          rs[i] = a.rowscale[mm < a.M ? mm : a.M - 1];
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int off = r * (PCH * 16) + (((2 * j + (q >> 1)) ^ (r & 7)) << 4) + ((q & 1) << 3);
          f32x4 v = acc[i][j];
          if constexpr (RS) v = v * rs[i];
          *reinterpret_cast<uint2*>(stg + off) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
#pragma unroll
        for (int h = 0; h < SPI; ++h) {
          const int sl = el + 64 * h;
          const int row = sl / CH, cc = sl % CH;
          const int rowc = row < 16 ? row : 15;
          const uint4 v = *reinterpret_cast<const uint4*>(stg + rowc * (PCH * 16) + ((cc ^ (rowc & 7)) << 4));
          const int m = m0 + eam0 + 16 * i + row, n = n0 + ebn0 + 8 * cc;
          uint4* dst = (row < 16 && m < a.M && n < a.N) ? reinterpret_cast<uint4*>(a.C + (int64_t)m * a.ldc + n)
                                                       : &g_pk_sink[el];
          *dst = v;
        }
      }
    }
    if (nt >= a.ntiles) break;
    tile = nt;
    // the next tile's K-tile 0 (its K-tile 1 landed before the stores above were issued)
    ktile(buf0, buf1, false, 0, 0, true, tile, 2, false, true, false, false);
  }
  vm_wait<0>();  // no LDS-DMA may outlive the workgroup
  // the last workgroup to finish re-arms this launch's counter pair for its next use
  if (tid == 0) {
    const int done = __hip_atomic_fetch_add(a.ctr + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == nwg - 1) {
      __hip_atomic_store(a.ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.ctr + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// out[i] (+)= sum_s part[s][i] in fixed order (the K-split slabs of a weight gradient), a float4 per thread
__global__ void gp_reduce_k(const float* __restrict__ part, int S, int64_t stride, int64_t n, float* __restrict__ out,
                            bool accumulate) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  float4 s = accumulate ? *reinterpret_cast<const float4*>(out + i) : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k = 0; k < S; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)k * stride + i);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  *reinterpret_cast<float4*>(out + i) = s;
}

// Many slabs over a small output (the 42 / 16-slab narrow weight gradients): wave w of the workgroup sums the slab
// quarter [w S / 4, (w + 1) S / 4) for 256 consecutive outputs (a float4 per lane), and the four quarter sums are
// added in quarter order through LDS (fixed order: deterministic).  The one-element-per-thread form it replaced
// issued S 4-B loads per lane; this one S / 4 16-B loads (profiles/r6/gp_reduce_quarters.txt).
__global__ __launch_bounds__(256) void gp_reduce_q_k(const float* __restrict__ part, int S, int64_t stride, int64_t n,
                                                     float* __restrict__ out, bool accumulate) {
  __shared__ float4 q[3][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = ((int64_t)blockIdx.x * 64 + lane) * 4;
  const bool ok = i < n;
  const int k0 = w * S / 4, k1 = (w + 1) * S / 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    for (int k = k0; k < k1; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)k * stride + i);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  if (w > 0) q[w - 1][lane] = s;
  __syncthreads();
  if (w == 0 && ok) {
    float4 o = accumulate ? *reinterpret_cast<const float4*>(out + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    o.x += s.x; o.y += s.y; o.z += s.z; o.w += s.w;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const float4 v = q[u][lane];
      o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
    }
    *reinterpret_cast<float4*>(out + i) = o;
  }
}

// waves per workgroup of the split-K engine (gemm_pipe_k, weight gradients): 8 (two per SIMD, 128 x 64 wave
// tiles) or 4 (one per SIMD, 128 x 128); MAMBA_AMD_PIPE_WAVES sets the process default, set_gemm_pipe_waves
// overrides it.  (The persistent engine's 4-wave form measured ~20% slower at every tile shape:
// profiles/r4/pk4_four_wave_tiles_rejected.txt.)
static int g_pipe_waves = 0;
int gemm_pipe_waves() {
  if (g_pipe_waves == 0) {
    const char* e = getenv("MAMBA_AMD_PIPE_WAVES");
    g_pipe_waves = (e && atoi(e) == 4) ? 4 : 8;
  }
  return g_pipe_waves;
}
void set_gemm_pipe_waves(int w) { g_pipe_waves = (w == 4) ? 4 : 8; }

// LDS slots of the split-K XC . XC weight-gradient engine (gemm_wg_k): 0 = route those products to gemm_pipe_k
// instead; MAMBA_AMD_WG_NB sets the process default, set_gemm_wg_nb overrides it
static int g_wg_nb = -1;
int gemm_wg_nb() {
  if (g_wg_nb < 0) {
    const char* e = getenv("MAMBA_AMD_WG_NB");
    const int v = e ? atoi(e) : 4;  // 4 slots measured fastest (profiles/r5/wg_engine_ab.txt)
    g_wg_nb = (v == 4 || v == 5) ? v : 0;
  }
  return g_wg_nb;
}
void set_gemm_wg_nb(int nb) { g_wg_nb = (nb == 4 || nb == 5) ? nb : 0; }

// paired 64-deep KC images (gemm_wg_kp_k): 0 never, 1 for wide long-K KC operands (default), 2 for every KC operand;
// MAMBA_AMD_WG_KCPAIR sets the process default, set_gemm_wg_kcpair overrides it
static int g_wg_kcpair = -1;
int gemm_wg_kcpair() {
  if (g_wg_kcpair < 0) {
    const char* e = getenv("MAMBA_AMD_WG_KCPAIR");
    const int v = e ? atoi(e) : 1;
    g_wg_kcpair = (v >= 0 && v <= 2) ? v : 1;
  }
  return g_wg_kcpair;
}
void set_gemm_wg_kcpair(int v) { g_wg_kcpair = (v >= 0 && v <= 2) ? v : 1; }

bool gemm_pipe_supported(int la, int lb, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  if (M <= 0 || N <= 0 || K <= 0) return false;
  if (lda % 8 || ldb % 8 || ldc % 4 || N % 4) return false;
  if ((la == 0 || lb == 0) && K % 8) return false;  // KC operands are DMA'd in 8-element k chunks
  if (la == 1 && M % 8) return false;  // XC operand columns are DMA'd in 8-element chunks
  if (lb == 1 && N % 8) return false;
  if (la == 0 && lda < K) return false;
  if (lb == 0 && ldb < K) return false;
  // per-thread DMA offsets are 32-bit byte offsets from the K-tile base (KC operands span all rows)
  if (la == 0 && ((int64_t)(M - 1) * lda + K) * 2 >= (int64_t)1 << 32) return false;
  if (lb == 0 && ((int64_t)(N - 1) * ldb + K) * 2 >= (int64_t)1 << 32) return false;
  return true;
}

int gemm_pipe_splits(int M, int N, int K) {
  // one workgroup per CU (128 KB of LDS), >= 8 K-tiles per split (launchers.h)
  return split_k_count(((int64_t)(M + 255) / 256) * ((N + 255) / 256), M, N, K, 8 * GP_BK);
}

// gemm_wg_k's 32-bit DMA byte offsets: XC up to one stage past K, KC up to one 256-row tile past the rows, and
// below the out-of-range sentinel
static bool gemm_wg_offsets_ok(int la, int lb, int M, int N, int K, int64_t lda, int64_t ldb) {
  const int64_t lim = ((int64_t)1 << 32) - 64;
  auto ok = [&](int L, int rows, int64_t ld) {
    return (L ? ((int64_t)K + 64) * ld : ((int64_t)rows + 256) * ld + K + 64) * 2 < lim;
  };
  return ok(la, M, lda) && ok(lb, N, ldb);
}

hipError_t launch_gemm_pipe(int la, int lb, const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                            int64_t ldc, int M, int N, int K, int splits, int64_t split_stride, int epi, int bm,
                            hipStream_t st) {
  if (!gemm_pipe_supported(la, lb, M, N, K, lda, ldb, ldc)) return hipErrorInvalidValue;
  if (splits < 1 || (splits > 1 && epi == 0) || (bm != 256 && bm != 128)) return hipErrorInvalidValue;
  GemmPipeArgs a;
  a.A = (const bf16_t*)A; a.lda = lda; a.B = (const bf16_t*)B; a.ldb = ldb;
  a.C = C; a.ldc = ldc; a.split_stride = split_stride;
  a.M = M; a.N = N; a.K = K; a.splits = splits;
  a.kslice = ((K + splits - 1) / splits + GP_BK - 1) / GP_BK * GP_BK;
  const int nwg = ((M + bm - 1) / bm) * ((N + 255) / 256) * splits;
  // every layout with an XC operand or an fp32 output: the ring measured faster on each of them
  // (wg_engine_ab.txt, wg_engine_m1.txt); KC . KC bf16 stays here (pk_ring_rejected.txt)
  if (gemm_wg_nb() != 0 && !(la == 0 && lb == 0 && epi == 0) && gemm_wg_offsets_ok(la, lb, M, N, K, lda, ldb)) {
    // the staged-ring engine (32-deep stages, 4-slot ring); split slices on the 64-token grid
    a.kslice = ((K + splits - 1) / splits + GP_BK - 1) / GP_BK * GP_BK;
    a.nbA = (unsigned)((la ? (int64_t)(K - 1) * lda + M : (int64_t)(M - 1) * lda + K) * 2);
    a.nbB = (unsigned)((lb ? (int64_t)(K - 1) * ldb + N : (int64_t)(N - 1) * ldb + K) * 2);
    const int mi = bm == 128 ? 4 : 8;
    // KC operands in paired 64-deep images (whole 128-B rows per DMA) when the KC operand is a wide one streamed
    // over a long reduction (a weight gradient): measured (profiles/r6/wg_kc_pairs.txt) 1.27x on the Mamba-1
    // in_proj weight gradient (3072 KC rows) and +0.2-0.8% whole-step with the out_proj one (1536 rows) added;
    // slower for short-K products with a small L2-resident KC operand (the out_proj forward's 768-row weight
    // +14-22%) and the 48 / 80-row x_proj / dt_proj products (+25-60%): the pair halves the prefetch distance of
    // every even stage.  256-row tiles only: the x_proj / dt_proj weight gradients on 128-row tiles pair their wide
    // (1536-row) KC operand under the size test but ran 60.8 vs 56.4 us paired (profiles/r6/prof_mamba1-280m_serial_*).
    // MAMBA_AMD_WG_KCPAIR: 0 off, 1 this rule, 2 every KC operand.
    const int kpm = gemm_wg_kcpair();
    const bool kp = kpm == 2 ? (la == 0 || lb == 0)
                             : kpm == 1 && mi == 8 && K >= 16384 && ((la == 0 && M >= 1536) || (lb == 0 && N >= 1536));
#define WG_L(LA_, LB_, E_, MI_)                                                                          \
  if constexpr (LA_ == 0 || LB_ == 0) {                                                                  \
    if (kp) hipLaunchKernelGGL((gemm_wg_kp_k<LA_, LB_, E_, MI_>), dim3(nwg), dim3(512), 0, st, a);       \
    else hipLaunchKernelGGL((gemm_wg_k<LA_, LB_, E_, 4, MI_>), dim3(nwg), dim3(512), 0, st, a);          \
  } else {                                                                                                \
    hipLaunchKernelGGL((gemm_wg_k<LA_, LB_, E_, 4, MI_>), dim3(nwg), dim3(512), 0, st, a);               \
  }
#define WG_M(LA_, LB_, MI_)                                     \
  if (epi == 0) { WG_L(LA_, LB_, 0, MI_) }                      \
  else if (epi == 1) { WG_L(LA_, LB_, 1, MI_) }                 \
  else { WG_L(LA_, LB_, 2, MI_) }
#define WG_E(LA_, LB_)                                          \
  if (mi == 4) { WG_M(LA_, LB_, 4) }                            \
  else { WG_M(LA_, LB_, 8) }
    if (la == 0 && lb == 0) { WG_E(0, 0) }
    else if (la == 0 && lb == 1) { WG_E(0, 1) }
    else if (la == 1 && lb == 1) { WG_E(1, 1) }
    else { WG_E(1, 0) }
#undef WG_E
#undef WG_M
#undef WG_L
    return hipGetLastError();
  }
  if (bm == 128 && (epi != 0 || lb != 1)) return hipErrorInvalidValue;  // gemm_pipe_k: narrow A . XC B, bf16 out
  if (bm == 128) {
    if (la == 0) hipLaunchKernelGGL((gemm_pipe_k<0, 1, 0, 4, 4>), dim3(nwg), dim3(GP_NT), 0, st, a);
    else hipLaunchKernelGGL((gemm_pipe_k<1, 1, 0, 4, 4>), dim3(nwg), dim3(GP_NT), 0, st, a);
    return hipGetLastError();
  }
#define GP_EPI(LA_, LB_)                                                                       \
  if (gemm_pipe_waves() == 4) {                                                                \
    switch (epi) {                                                                             \
      case 0: hipLaunchKernelGGL((gemm_pipe_k<LA_, LB_, 0, 2>), dim3(nwg), dim3(256), 0, st, a); break; \
      case 1: hipLaunchKernelGGL((gemm_pipe_k<LA_, LB_, 1, 2>), dim3(nwg), dim3(256), 0, st, a); break; \
      default: hipLaunchKernelGGL((gemm_pipe_k<LA_, LB_, 2, 2>), dim3(nwg), dim3(256), 0, st, a); break; \
    }                                                                                          \
  } else {                                                                                     \
    switch (epi) {                                                                             \
      case 0: hipLaunchKernelGGL((gemm_pipe_k<LA_, LB_, 0>), dim3(nwg), dim3(GP_NT), 0, st, a); break; \
      case 1: hipLaunchKernelGGL((gemm_pipe_k<LA_, LB_, 1>), dim3(nwg), dim3(GP_NT), 0, st, a); break; \
      default: hipLaunchKernelGGL((gemm_pipe_k<LA_, LB_, 2>), dim3(nwg), dim3(GP_NT), 0, st, a); break; \
    }                                                                                          \
  }
  if (la == 0 && lb == 0) { GP_EPI(0, 0) }
  else if (la == 0 && lb == 1) { GP_EPI(0, 1) }
  else if (la == 1 && lb == 1) { GP_EPI(1, 1) }
  else if (la == 1 && lb == 0) { GP_EPI(1, 0) }  // the Mamba-1 out_proj: forward (bf16) and weight gradient
  else return hipErrorInvalidValue;
#undef GP_EPI
  return hipGetLastError();
}

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}



bool gemm_pk_supported(int la, int lb, int epi, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  if (M <= 0 || N <= 0 || K <= 192) return false;  // >= 4 K-tiles
  if (la != 0 || lb != 0 || epi != 0) return false;  // instantiated: KC . KC, bf16 output
  if (lda % 8 || ldb % 8 || ldc % 8 || N % 8 || K % 8 || lda < K || ldb < K) return false;
  // every DMA byte offset, including the overhang of partial tiles, must stay below the out-of-range sentinel
  const int64_t kt = ((K + 63) / 64 + 1) / 2 * 2;
  const int64_t lim = ((int64_t)1 << 32) - 64;
  const int64_t Mp = (M + 255) / 256 * 256 + 256, Np = (N + 255) / 256 * 256 + 256;  // any tile shape's overhang
  return (Mp * lda + kt * 64) * 2 < lim && (Np * ldb + kt * 64) * 2 < lim;
}

// per-launch tile-claim counters: a ring of zeroed {next, done} pairs, each re-armed by its launch's last
// workgroup; launches in flight at once (two micro-batch streams) never share a pair.  Launches recorded into a
// HIP graph take pairs from a separate, never-recycled range (a replayed graph keeps its baked pair, which an
// eager launch must never reuse).  The buffer is allocated on the device's first eager launch; a first launch
// inside stream capture fails loudly (run one eager launch, e.g. the warm-up step, before capturing).
constexpr int PK_RING = 16384, PK_CAPTURED = 8192;  // eager ring, graph-captured range (pairs)
int gemm_pk_graph_counter_capacity() { return PK_CAPTURED; }
static int* pk_counters(int dev, hipStream_t st) {
  constexpr int R = PK_RING, RC = PK_CAPTURED;
  static int* bufs[16] = {};
  static unsigned seq[16] = {};
  static unsigned cap[16] = {};
  if (dev < 0 || dev >= 16) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return nullptr;
  const bool capturing = cs != hipStreamCaptureStatusNone;
  if (!bufs[dev]) {
    if (capturing) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, (R + RC) * 2 * sizeof(int)) != hipSuccess || hipMemset(p, 0, (R + RC) * 2 * sizeof(int)) != hipSuccess)
      return nullptr;
    bufs[dev] = (int*)p;
  }
  if (capturing) {
    if (cap[dev] >= (unsigned)RC) return nullptr;
    return bufs[dev] + 2 * (R + (int)cap[dev]++);
  }
  const int slot = (int)(seq[dev]++ % R);
  return bufs[dev] + 2 * slot;
}

hipError_t launch_gemm_pk(int la, int lb, const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                          int64_t ldc, int M, int N, int K, int epi, const float* rowscale, hipStream_t st) {
  if (!gemm_pk_supported(la, lb, epi, M, N, K, lda, ldb, ldc)) return hipErrorInvalidValue;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidValue;
  GemmPkArgs a;
  a.A = (const bf16_t*)A; a.lda = lda; a.B = (const bf16_t*)B; a.ldb = ldb;
  a.C = (bf16_t*)C; a.ldc = ldc; a.rowscale = rowscale;
  a.ctr = pk_counters(dev, st);
  if (!a.ctr) return hipErrorNotReady;  // no counter pair: first launch under capture, or the captured range is spent
  a.nbA = (unsigned)(((int64_t)(M - 1) * lda + K) * 2);
  a.nbB = (unsigned)(((int64_t)(N - 1) * ldb + K) * 2);
  a.M = M; a.N = N; a.K = K;
  a.kte = ((K + 63) / 64 + 1) / 2 * 2;
  const int ncu = cu_count();
  // tile shape: 256 x 256 unless a smaller tile fills the rounds of ncu workgroups better.  Relative tile costs:
  // 128 x 256 ~0.55, 256 x 192 ~0.78 of a 256 x 256 tile.  E.g. N = 768 outputs (out_proj fwd, in_proj / lm_head
  // dgrad at d_model 768): 384 tiles of 256 x 256 are 1.5 rounds of 256 CUs, 768 of 128 x 256 are 3 rounds
  // (1.65), 512 of 256 x 192 are exactly 2 rounds (1.56) at full-height operand reuse.
  auto rounds = [&](int bm_, int bn_) {
    const int t = ((M + bm_ - 1) / bm_) * ((N + bn_ - 1) / bn_);
    return (double)((t + ncu - 1) / ncu);
  };
  const double c256 = rounds(256, 256), c128 = 0.55 * rounds(128, 256), c192 = 0.78 * rounds(256, 192);
  int bm = 256, bn = 256;
  if (c192 < c256 && c192 <= c128) bn = 192;
  else if (c128 < c256) bm = 128;
  a.tm = (M + bm - 1) / bm; a.tn = (N + bn - 1) / bn;
  a.ntiles = a.tm * a.tn;
  const bool tail = K % 64 != 0 || a.kte * 64 != K;
  const int nwg = std::min(a.ntiles, ncu);
#define PK_L(MI_, NJ_, RS_)                                                                              \
  if (tail) hipLaunchKernelGGL((gemm_pk_k<MI_, NJ_, RS_, true>), dim3(nwg), dim3(512), 0, st, a);     \
  else hipLaunchKernelGGL((gemm_pk_k<MI_, NJ_, RS_, false>), dim3(nwg), dim3(512), 0, st, a)
  if (bn == 192) {
    if (rowscale) { PK_L(8, 3, true); } else { PK_L(8, 3, false); }
  } else if (bm == 256) {
    if (rowscale) { PK_L(8, 4, true); } else { PK_L(8, 4, false); }
  } else {
    if (rowscale) { PK_L(4, 4, true); } else { PK_L(4, 4, false); }
  }
#undef PK_L
  return hipGetLastError();
}

hipError_t launch_gp_reduce(const float* part, int S, int64_t stride, int64_t n, float* out, bool accumulate,
                            hipStream_t st) {
  if (n % 4 || stride % 4) return hipErrorInvalidValue;
  if (n / 4 < 512 * 256 && S >= 16)  // fewer than 2 float4 workgroups per CU: the slab quarters per wave
    hipLaunchKernelGGL(gp_reduce_q_k, dim3((unsigned)((n / 4 + 63) / 64)), dim3(256), 0, st, part, S, stride, n, out,
                       accumulate);
  else
    hipLaunchKernelGGL(gp_reduce_k, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, st, part, S, stride, n,
                       out, accumulate);
  return hipGetLastError();
}

}  // namespace mamba_amd
