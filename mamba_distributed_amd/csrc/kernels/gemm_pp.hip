// Ping-pong persistent bf16 GEMM for the projection forward / input-gradient products and the lm_head
// (model.py:35-46 through the mixers' in_proj / out_proj and the LM head):
//
//   C[M, N] = A[M, K] . B[N, K]^T        both operands K-contiguous (KC), fp32 accumulate, bf16 output
//
// Why a second engine next to gemm_pk_k (gemm_pipe.hip): there, the two waves sharing a SIMD run the same
// program in lockstep -- both read LDS, both wait at the same barrier, both issue MFMAs -- so every LDS round
// trip and barrier wait is a hole in the matrix pipe.  Here the 8 waves form two groups (wave rows wr = 0, 1;
// each SIMD holds one wave of each) that run the same 8-phase-per-2-K-tiles program ONE BARRIER APART: while
// group 0 issues its 16-MFMA cluster, group 1 reads its next fragments and issues its share of the LDS-DMA,
// then they swap.  The matrix pipe sees a continuous stream of clusters (cdna_hip_programming.md: the 256^2
// 8-phase template, T3+T4+T5).
//
// Geometry: 256 x 256 output tile, K-tiles of 64, 8 waves as 2 (M) x 4 (N), wave tile 128 x 64 = 8 x 4
// accumulators of v_mfma_f32_16x16x32_bf16 (operands swapped, so a lane holds 4 consecutive output columns of
// one row).  One phase = one quadrant (64 rows x 32 columns) of the wave tile over the whole K-tile: 16 MFMAs.
// Quadrant order q0 (m0, n0), q1 (m0, n1), q2 (m1, n1), q3 (m1, n0): every phase reads only the fragments that
// changed (8 A + 4 B, 4 B, 8 A, none: B(n0) stays in registers from q0).
//
// LDS: two K-tile buffers of four 16 KB half-tiles each, [128 rows][64 k] bf16 with the 16-B chunk of row r at
// slot c ^ (r & 7) (conflict-free ds_read_b128; the swizzle is applied to the DMA's per-lane SOURCE address):
//   HA0 = A rows {0-63, 128-191} (the m0 halves of both wave rows), HA1 = A rows {64-127, 192-255},
//   HB0 = B rows {64c .. 64c+31}, HB1 = B rows {64c+32 .. 64c+63}, c = 0..3 (the n0 / n1 halves of each wave).
// Each half-tile is refilled 2-3 phases after its last read:
//   phase j of K-tile g issues  j0: HB1(g+1)  j1: HA1(g+1)  j2: HA0(g+2)  j3: HB0(g+2)
// so every half-tile is DMA'd 5-6 phases before its first read (one `buffer_load ... lds` pair per thread per
// phase, counted vmcnt waits before the j0, j1, j2 reads, raw s_barrier, never vmcnt(0) in the loop).
//
// Persistent walk: one workgroup per CU takes output tiles id, id + G, ... (groups of 8 M-panels, column-major
// inside a group, XCD-remapped ids); the K-tile stream runs across tile boundaries (the DMA of the next tile's
// first K-tiles overlaps this tile's last ones), and the previous tile's accumulators are stored quadrant by
// quadrant in the read interval of the phase that restarts them (K-tile 0 of the next tile), so no phase waits
// on an epilogue.  Out-of-range rows / columns / k read as zeros through the buffer descriptor; stores outside
// C go to a sink so every wave issues the same number of VMEM operations (the vmcnt counts are exact).
#include <cstdlib>

#include "mfma.h"
#include "launchers.h"

namespace mamba_amd {
namespace {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __attribute__((aligned(64))) uint2 g_pp_sink[128];

template <int N>
__device__ __forceinline__ void pp_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void pp_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// lane byte offset of a ds_read_b128 fragment (rows r0 + (l & 15), k-step ks) in a [rows][64 k] swizzled image;
// r0 % 16 == 0, so the row's low 3 bits are the lane's
__device__ __forceinline__ int pp_lane_kc(int ks) {
  const int l = threadIdx.x & 63;
  return (l & 15) * 128 + (((4 * ks + (l >> 4)) ^ (l & 7)) << 4);
}

}  // namespace

struct GemmPPArgs {
  const bf16_t* A; int64_t lda;
  const bf16_t* B; int64_t ldb;
  bf16_t* C; int64_t ldc;
  unsigned nbA, nbB;         // operand bytes covered by the buffer descriptors
  int M, N, K, tm, tn, ntiles, KT;
};

template <bool TAIL>
__global__ __launch_bounds__(512) void gemm_pp_k(GemmPPArgs a) {
  constexpr int HT = 16384;   // half-tile bytes
  constexpr int BUF = 4 * HT; // K-tile buffer: HA0 HA1 HB0 HB1
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];

  const int G = gridDim.x;
  const int id = xcd_remap(blockIdx.x, G);
  const int nmine = (a.ntiles - id + G - 1) / G;  // >= 1: G <= ntiles
  const int tid = threadIdx.x, l = tid & 63;
  const int wu = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wu >> 2, wc = wu & 3;

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, (int)a.nbA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, (int)a.nbB, 0x00020000);
  // DMA lanes: image row 64 ii + (tid >> 3), 16-B chunk (tid & 7) ^ (row & 7) of the row's 128 B
  const int lrow = tid >> 3, lch = (tid & 7) ^ (lrow & 7);
  const unsigned loA = (unsigned)(((int64_t)lrow * a.lda + 8 * lch) * 2);
  const unsigned loB = (unsigned)(((int64_t)(64 * (lrow >> 5) + (lrow & 31)) * a.ldb + 8 * lch) * 2);
  const int kchunk = 8 * lch;

  auto tile_mn = [&](int t, int& m0, int& n0) {  // groups of 8 M-panels, column-major inside a group
    const int gsz = 8 * a.tn, g = t / gsz, r = t - g * gsz;
    const int gm = min(8, a.tm - 8 * g);
    m0 = __builtin_amdgcn_readfirstlane((8 * g + r % gm) * 256);
    n0 = __builtin_amdgcn_readfirstlane((r / gm) * 256);
  };
  // half-tile h (0 HA0, 1 HA1, 2 HB0, 3 HB1) of K-tile kt of the tile at (m0, n0) into buffer buf
  auto dma = [&](int m0, int n0, int kt_, char* buf, int h) {
    const int kt = __builtin_amdgcn_readfirstlane(kt_);
    const bool isA = h < 2;
    const int hh = h & 1;
    const bool dead = TAIL && kt * 64 + kchunk >= a.K;  // k-chunk past K (in range: the next row's bytes)
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      unsigned v;
      if (isA) {
        v = loA + __builtin_amdgcn_readfirstlane((unsigned)((int64_t)(m0 + 128 * ii + 64 * hh) * a.lda * 2) + (unsigned)kt * 128u);
      } else {
        v = loB + __builtin_amdgcn_readfirstlane((unsigned)((int64_t)(n0 + 128 * ii + 32 * hh) * a.ldb * 2) + (unsigned)kt * 128u);
      }
      if (dead) v = 0xFFFFFFF0u;
      lds_void* dst = (lds_void*)(buf + h * HT + ii * 8192 + wu * 1024);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rA : rB, dst, 16, v, 0, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero4();
  bf16x8 af[4][2], bf0[2][2], bf1[2][2];  // A of the current m-half; B of n-half 0 (q0, q3) and 1 (q1, q2)
  const int ok0 = pp_lane_kc(0), ok1 = pp_lane_kc(1);

  // reads of quadrant q from buffer buf: q0 A(m0) + B(n0), q1 B(n1), q2 A(m1), q3 none (B(n0) kept since q0)
  auto rd_a = [&](const char* buf, int mh) {
    const char* img = buf + mh * HT + (64 * wr) * 128;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i][0] = *reinterpret_cast<const bf16x8*>(img + ok0 + 16 * i * 128);
      af[i][1] = *reinterpret_cast<const bf16x8*>(img + ok1 + 16 * i * 128);
    }
  };
  auto rd_b = [&](const char* buf, int nh, bf16x8 (&bf)[2][2]) {
    const char* img = buf + (2 + nh) * HT + (32 * wc) * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf[j][0] = *reinterpret_cast<const bf16x8*>(img + ok0 + 16 * j * 128);
      bf[j][1] = *reinterpret_cast<const bf16x8*>(img + ok1 + 16 * j * 128);
    }
  };
  // the MFMA cluster, with this phase's two LDS-DMA pieces issued between its first MFMAs (their issue cost then
  // overlaps this wave's own matrix work instead of lengthening the read interval the other group waits on)
  auto mfma_q = [&](int mh, int nh, bool zc, int dm, int dn, int dk, char* dbuf, int dh) {
    bf16x8 (&bf)[2][2] = nh ? bf1 : bf0;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4& c = acc[4 * mh + i][2 * nh + j];
          c = mfma16(bf[j][s], af[i][s], (zc && s == 0) ? zero4() : c);
        }
    dma(dm, dn, dk, dbuf, dh);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (the DMA)
    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // store quadrant (mh, nh) of the tile at (m0, n0) as 16-B row pieces: a lane holds 4 consecutive columns of one
  // row in each of the quadrant's two 16-column tiles; v_permlane16_swap trades the second tile's values of lane
  // rows 0 / 2 for the first tile's of rows 1 / 3, so lane group g stores columns 16 (g & 1) + 8 (g >> 1) .. + 7 of
  // row 16 i + (l & 15): per instruction 16 rows x 64 contiguous bytes (8-B pieces issue at half the rate)
  auto store_q = [&](int mh, int nh, int m0, int n0) {
    const int lg = l >> 4;
    const int n = n0 + 64 * wc + 32 * nh + 16 * (lg & 1) + 8 * (lg >> 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + 128 * wr + 64 * mh + 16 * i + (l & 15);
      const f32x4 v0 = acc[4 * mh + i][2 * nh], v1 = acc[4 * mh + i][2 * nh + 1];
      unsigned x0 = pack2(v0[0], v0[1]), x1 = pack2(v0[2], v0[3]);
      unsigned y0 = pack2(v1[0], v1[1]), y1 = pack2(v1[2], v1[3]);
      asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3"
                   : "+v"(x0), "+v"(x1), "+v"(y0), "+v"(y1));
      uint4* dst = (m < a.M && n < a.N) ? reinterpret_cast<uint4*>(a.C + (int64_t)m * a.ldc + n)
                                        : reinterpret_cast<uint4*>(&g_pp_sink[2 * l]);
      *dst = make_uint4(x0, x1, y0, y1);
    }
  };

  // The two groups run one barrier apart: group 1 passes one extra barrier first, group 0 one at the end.
  // A wait that retires a half-tile before its first read sits at the end of the interval before the barrier
  // that precedes group 0's reads: after the MFMA cluster for group 0, after the reads + DMA for group 1.
  const bool g0 = wr == 0;
  char* const buf0 = smem;
  char* const buf1 = smem + BUF;

  // one phase: reads of quadrant q, the DMA (half-tile DH of K-tile DK at (DM, DN) into DBUF), the stores of the
  // previous tile's quadrant q (STORE), the barrier pair around the MFMA cluster, and the vmcnt wait W (< 0:
  // none) that retires the next phase's first-read half-tile, placed per group
#define PP_PHASE(q, buf, DM, DN, DK, DBUF, DH, ZC, STORE, W)                                 \
  {                                                                                          \
    constexpr int mh_ = ((q) == 2 || (q) == 3) ? 1 : 0;                                      \
    constexpr int nh_ = ((q) == 1 || (q) == 2) ? 1 : 0;                                      \
    if constexpr ((q) == 0) rd_b(buf, 0, bf0);                                               \
    if constexpr ((q) == 1) rd_b(buf, 1, bf1);                                               \
    if constexpr ((q) == 0 || (q) == 2) rd_a(buf, mh_);                                      \
    if constexpr (STORE) store_q(mh_, nh_, pm0, pn0);                                        \
    if constexpr ((W) >= 0) { if (!g0) pp_vm_wait<((W) < 2 ? 0 : (W) - 2)>(); }             \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    __builtin_amdgcn_s_barrier();                                                            \
    pp_lgkm0();                                                                              \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    mfma_q(mh_, nh_, ZC, DM, DN, DK, DBUF, DH);                                              \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    if constexpr ((W) >= 0) { if (g0) pp_vm_wait<((W) < 0 ? 0 : (W))>(); }                  \
    __builtin_amdgcn_s_barrier();                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                       \
  }
  // One K-tile (global index g: buffer g & 1).  The DMA is issued inside the MFMA cluster, so at group 1's wait (end
// of its read interval) this phase's DMA is not yet issued: group 1 waits for W - 2.  DMA schedule (j: phase): j0 HB1(g+1), j1 HA1(g+1), j2 HA0(g+2),
  // j3 HB0(g+2) -- each half-tile 2-3 phases after its last read (HA0, HB0: j0; HB1: j1; HA1: j2) and 5-6 phases
  // before its first read.  (M1, N1, K1) / (M2, N2, K2): the tile and K-tile one / two K-tiles ahead.
  // Waits (in phases 3, 0, 1 for the reads of j0, j1, j2 of the next phase): retire the half-tile issued four
  // phases back: vmcnt(8 + 8 per store phase since then).  KIND 0: K-tile 0 of a tile (stores the previous tile's
  // quadrants), 1: K-tile 1, 2: the rest.
#define PP_KTILE(KIND, cur, nx, M1, N1, K1, M2, N2, K2)                                                        \
  {                                                                                                              \
    PP_PHASE(0, cur, M1, N1, K1, nx, 3, (KIND) == 0, (KIND) == 0, ((KIND) == 0 ? 16 : (KIND) == 1 ? 40 : 8))    \
    PP_PHASE(1, cur, M1, N1, K1, nx, 1, (KIND) == 0, (KIND) == 0, ((KIND) == 0 ? 24 : (KIND) == 1 ? 32 : 8))    \
    PP_PHASE(2, cur, M2, N2, K2, cur, 0, (KIND) == 0, (KIND) == 0, -1)                                           \
    PP_PHASE(3, cur, M2, N2, K2, cur, 2, (KIND) == 0, (KIND) == 0, ((KIND) == 0 ? 40 : (KIND) == 1 ? 16 : 8))    \
  }

  int tcur = id, i = 0;
  int cm0, cn0, nm0, nn0;  // this tile and the next one (the last tile again past the end)
  tile_mn(tcur, cm0, cn0);
  if (nmine > 1) tile_mn(id + G, nm0, nn0);
  else { nm0 = cm0; nn0 = cn0; }
  int pm0 = a.M, pn0 = a.N;  // the previous tile: none yet (K-tile 0 of the first tile stores to the sink)

  // prologue: HA0(0), HB0(0), HB1(0), HA1(0), HA0(1), HB0(1) -- the steady state's half-tiles at K-tile 0; K-tile 0
  // landed, K-tile 1's first two in flight
  dma(cm0, cn0, 0, buf0, 0);
  dma(cm0, cn0, 0, buf0, 2);
  dma(cm0, cn0, 0, buf0, 3);
  dma(cm0, cn0, 0, buf0, 1);
  dma(cm0, cn0, 1, buf1, 0);
  dma(cm0, cn0, 1, buf1, 2);
  pp_vm_wait<4>();
  __builtin_amdgcn_s_barrier();
  if (!g0) __builtin_amdgcn_s_barrier();  // the stagger

  const int KT = a.KT;  // >= 4
  int g = 0;            // global K-tile index (buffer parity)
  for (;;) {
    {
      char* cur = (g & 1) ? buf1 : buf0;
      char* nx = (g & 1) ? buf0 : buf1;
      PP_KTILE(0, cur, nx, cm0, cn0, 1, cm0, cn0, 2)
      ++g;
    }
    {
      char* cur = (g & 1) ? buf1 : buf0;
      char* nx = (g & 1) ? buf0 : buf1;
      PP_KTILE(1, cur, nx, cm0, cn0, 2, cm0, cn0, 3)
      ++g;
    }
#pragma unroll 1
    for (int kt = 2; kt < KT; ++kt) {
      char* cur = (g & 1) ? buf1 : buf0;
      char* nx = (g & 1) ? buf0 : buf1;
      const bool n1 = kt + 1 >= KT, n2 = kt + 2 >= KT;  // the DMA targets cross into the next tile
      const int M1 = n1 ? nm0 : cm0, N1 = n1 ? nn0 : cn0, K1 = n1 ? kt + 1 - KT : kt + 1;
      const int M2 = n2 ? nm0 : cm0, N2 = n2 ? nn0 : cn0, K2 = n2 ? kt + 2 - KT : kt + 2;
      PP_KTILE(2, cur, nx, M1, N1, K1, M2, N2, K2)
      ++g;
    }
    pm0 = cm0; pn0 = cn0;
    if (++i >= nmine) break;
    tcur = id + i * G;
    cm0 = nm0; cn0 = nn0;
    if (i + 1 < nmine) tile_mn(id + (i + 1) * G, nm0, nn0);
  }
#undef PP_KTILE
#undef PP_PHASE
  if (g0) __builtin_amdgcn_s_barrier();  // the stagger, undone
  store_q(0, 0, pm0, pn0);
  store_q(0, 1, pm0, pn0);
  store_q(1, 1, pm0, pn0);
  store_q(1, 0, pm0, pn0);
  pp_vm_wait<0>();  // no LDS-DMA may outlive the workgroup
}

bool gemm_pp_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  if (M <= 0 || N <= 0 || K < 256) return false;  // >= 4 K-tiles
  if (lda % 8 || ldb % 8 || ldc % 8 || N % 8 || K % 8 || lda < K || ldb < K) return false;
  const int64_t kt = (K + 63) / 64;
  const int64_t lim = ((int64_t)1 << 32) - 64;
  const int64_t Mp = (M + 255) / 256 * 256 + 256, Np = (N + 255) / 256 * 256 + 256;  // tile overhang
  return (Mp * lda + kt * 64) * 2 < lim && (Np * ldb + kt * 64) * 2 < lim;
}

static int pp_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

hipError_t launch_gemm_pp(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N,
                          int K, hipStream_t st) {
  if (!gemm_pp_supported(M, N, K, lda, ldb, ldc)) return hipErrorInvalidValue;
  GemmPPArgs a;
  a.A = (const bf16_t*)A; a.lda = lda; a.B = (const bf16_t*)B; a.ldb = ldb;
  a.C = (bf16_t*)C; a.ldc = ldc;
  a.nbA = (unsigned)(((int64_t)(M - 1) * lda + K) * 2);
  a.nbB = (unsigned)(((int64_t)(N - 1) * ldb + K) * 2);
  a.M = M; a.N = N; a.K = K;
  a.tm = (M + 255) / 256; a.tn = (N + 255) / 256;
  a.ntiles = a.tm * a.tn;
  a.KT = (K + 63) / 64;
  const int nwg = std::min(a.ntiles, pp_cu_count());
  if (K % 64) hipLaunchKernelGGL((gemm_pp_k<true>), dim3(nwg), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((gemm_pp_k<false>), dim3(nwg), dim3(512), 0, st, a);
  return hipGetLastError();
}

}  // namespace mamba_amd
