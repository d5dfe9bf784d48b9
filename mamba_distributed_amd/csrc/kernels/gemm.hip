// bf16 GEMM for the forward projections: C[M, N] = A[M, K] . B[N, K]^T  (fp32 accumulate, bf16 out).
//
// Both operands are K-contiguous row-major (activations x[M, K], weights W[N, K] as nn.Linear stores
// them), which is the in_proj / out_proj forward of every Mamba block.  On the
// 280M shapes (M = 32768, K = 768 / 1536, N = 3352 / 768) the library picks 256-wide tiles that
// leave a 1.5-wave tail (N = 768) or a mostly empty last column tile (N = 3352).
//
// Structure (cdna_hip_programming.md §5 "step-3" GEMM, MI355X_MICROARCH.md LDS rules):
//  * 128 x 128 output tile per 256-thread workgroup, 4 waves as 2 x 2, each wave 64 x 64 =
//    4 x 4 v_mfma_f32_16x16x32_bf16 accumulators; BK = 64.
//  * global -> LDS with global_load_lds_dwordx4 (no VGPR staging), double-buffered: tile k+1 is
//    in flight while tile k is consumed; one vmcnt(0) + barrier per K-step.
//  * the LDS image is lane-linear (the DMA writes base + lane*16), so the bank-conflict XOR swizzle
//    (16-B chunk c of row r stored at chunk c ^ (r & 7)) is applied to the per-lane SOURCE address
//    and undone on the ds_read_b128 fragment read (both sides of the same involution).
//  * XCD-aware bijective workgroup remap: consecutive output tiles (same A row-panel) share an L2.
//  * epilogue staged through LDS so every global store is a full 16-B vector; columns >= N masked
//    (N % 8 == 0), B rows >= N are clamped on load (their results are never stored).
#include "mfma.h"
#include "launchers.h"
#include <algorithm>

namespace mamba_amd {

namespace {
constexpr int GBM = 128, GBN = 128, GBK = 64;
constexpr int GTILE_BYTES = GBM * GBK * 2;  // one operand tile: 16 KB
constexpr int GLDC = GBN + 8;               // padded epilogue row (elements)

typedef __attribute__((address_space(3))) void lds_void;

// 16-B chunk (row r, chunk c) of a [128][64] bf16 tile lives at byte r*128 + ((c ^ (r & 7)) << 4)
__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

// issue the DMA of one [128 x 64] tile: 1024 chunks, 4 per thread; LDS slot q holds the source
// chunk that the swizzle maps there
__device__ __forceinline__ void load_tile(const bf16_t* g, int64_t ld, int row0, int rows_valid, int k0,
                                          char* lds) {
  const int tid = threadIdx.x, w = tid >> 6;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = i * 256 + tid;           // LDS chunk slot written by this lane
    const int r = q >> 3, cs = q & 7;      // slot row / chunk
    const int c = cs ^ (r & 7);            // logical k-chunk stored in that slot
    const int rr = min(r, rows_valid - 1);  // clamp (tail rows are never stored)
    const bf16_t* src = g + (int64_t)(row0 + rr) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + (i * 256 + w * 64) * 16), 16, 0, 0);
  }
}

// k-contiguous MFMA operand (STD order) from a swizzled tile: rows r0 + (l & 15), k = 32 ks + 8 (l >> 4)
__device__ __forceinline__ bf16x8 frag(const char* lds, int r0, int ks) {
  const int l = threadIdx.x & 63, r = r0 + (l & 15), c = 4 * ks + (l >> 4);
  return *reinterpret_cast<const bf16x8*>(lds + swz(r, c));
}
}  // namespace

__global__ __launch_bounds__(256) void gemm_tn_bf16_k(const bf16_t* __restrict__ A, int64_t lda,
                                                      const bf16_t* __restrict__ B, int64_t ldb,
                                                      bf16_t* __restrict__ C, int64_t ldc, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[4 * GTILE_BYTES];  // [buf][A|B]; epilogue reuses it
  const int tiles_n = (N + GBN - 1) / GBN;
  const int nwg = ((M + GBM - 1) / GBM) * tiles_n;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int m0 = (t / tiles_n) * GBM, n0 = (t % tiles_n) * GBN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = w >> 1, wn = w & 1;
  const int mvalid = min(GBM, M - m0), nvalid = min(GBN, N - n0);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero4();
  const int KT = K / GBK;
  load_tile(A, lda, m0, mvalid, 0, smem);
  load_tile(B, ldb, n0, nvalid, 0, smem + GTILE_BYTES);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    char* cur = smem + (kt & 1) * 2 * GTILE_BYTES;
    if (kt + 1 < KT) {  // the other buffer was released by the previous iteration's barrier
      char* nxt = smem + ((kt + 1) & 1) * 2 * GTILE_BYTES;
      load_tile(A, lda, m0, mvalid, (kt + 1) * GBK, nxt);
      load_tile(B, ldb, n0, nvalid, (kt + 1) * GBK, nxt + GTILE_BYTES);
    }
#pragma unroll
    for (int ks = 0; ks < GBK / 32; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag(cur, wm * 64 + 16 * i, ks);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag(cur + GTILE_BYTES, wn * 64 + 16 * j, ks);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // epilogue: acc -> bf16 LDS tile [128][GLDC] -> 16-B row stores
  bf16_t* Cs = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * 64 + 16 * i + 4 * (l >> 4) + r) * GLDC + wn * 64 + 16 * j + (l & 15)] = f2bf(acc[i][j][r]);
  __syncthreads();
  for (int v = threadIdx.x; v < GBM * (GBN / 8); v += 256) {
    const int r = v / (GBN / 8), c = (v % (GBN / 8)) * 8;
    if (r < mvalid && c < nvalid)
      *reinterpret_cast<uint4*>(C + (int64_t)(m0 + r) * ldc + n0 + c) = *reinterpret_cast<const uint4*>(Cs + r * GLDC + c);
  }
}

// ================================ weight gradient ==============================================
// C[P, Q] (fp32) = dY[M, P]^T . X[M, Q]: the nn.Linear weight gradient (dW = dY^T X), reduced over the
// M = batch*seqlen tokens.  The output is small (768 x 1536 = 72 tiles of 128^2), so M is split into
// S slices (S * tiles ~ 2-3 workgroups per CU); each workgroup writes an fp32 partial and a
// second kernel sums the S partials in a fixed order (deterministic), writing fp32 directly (the
// parameter's gradient dtype: no bf16 round trip, no cast kernel).
// Both operands are token-major, i.e. the contraction index runs down the rows of the staged tiles,
// so the MFMA operands come through ds_read_b64_tr_b16 (frag_tr): A[p][k=m] from the dY tile and
// B[k=m][q] from the X tile.  Tiles are register-staged (global -> VGPR -> padded LDS) and double
// buffered: tile k+1 is loaded while tile k is multiplied, one barrier per k-step.
namespace {
constexpr int WB = 128;       // output tile (P x Q)
constexpr int WK = 64;        // token rows per k-step
constexpr int WLD = WB + 8;   // padded LDS row (elements)

struct WStage {  // one 64 x 128 bf16 tile = 1024 16-B chunks, 4 per thread
  uint4 v[4];
  __device__ __forceinline__ void load(const bf16_t* g, int64_t ld, int m0, int mlim, int c0, int clim) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = i * 256 + threadIdx.x, r = q >> 4, c = (q & 15) * 8;
      v[i] = (m0 + r < mlim && c0 + c < clim) ? *reinterpret_cast<const uint4*>(g + (int64_t)(m0 + r) * ld + c0 + c)
                                              : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(bf16_t* lds) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = i * 256 + threadIdx.x, r = q >> 4, c = (q & 15) * 8;
      *reinterpret_cast<uint4*>(lds + r * WLD + c) = v[i];
    }
  }
};
}  // namespace

__global__ __launch_bounds__(256) void gemm_wgrad_k(const bf16_t* __restrict__ dY, int64_t ldy,
                                                    const bf16_t* __restrict__ X, int64_t ldx,
                                                    float* __restrict__ part, int M, int P, int Q, int mslice,
                                                    bool pacc = false) {
  __shared__ __attribute__((aligned(16))) bf16_t As[2][WK * WLD];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][WK * WLD];
  const int tq = (Q + WB - 1) / WB, tp = (P + WB - 1) / WB;
  const int nwg = gridDim.x;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int tile = t % (tp * tq), sl = t / (tp * tq);
  const int p0 = (tile / tq) * WB, q0 = (tile % tq) * WB;
  const int mb = sl * mslice, me = min(M, mb + mslice);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wp = w >> 1, wq = w & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero4();
  WStage sa, sb;
  sa.load(dY, ldy, mb, me, p0, P);
  sb.load(X, ldx, mb, me, q0, Q);
  const int KT = (me - mb + WK - 1) / WK;
  sa.store(As[0]);
  sb.store(Bs[0]);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) {
      sa.load(dY, ldy, mb + (kt + 1) * WK, me, p0, P);
      sb.load(X, ldx, mb + (kt + 1) * WK, me, q0, Q);
    }
#pragma unroll
    for (int ks = 0; ks < WK / 32; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag_tr(As[cur], WLD, 32 * ks, wp * 64 + 16 * i);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag_tr(Bs[cur], WLD, 32 * ks, wq * 64 + 16 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < KT) {  // buffer cur^1 was last read in iteration kt-1, before its closing barrier
      sa.store(As[cur ^ 1]);
      sb.store(Bs[cur ^ 1]);
    }
    __syncthreads();
  }
  float* pc = part + (int64_t)sl * P * Q;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = p0 + wp * 64 + 16 * i + 4 * (l >> 4) + r, q = q0 + wq * 64 + 16 * j + (l & 15);
        if (p < P && q < Q) {
          float* d = pc + (int64_t)p * Q + q;
          *d = pacc ? *d + acc[i][j][r] : acc[i][j][r];  // pacc: add into persistent slabs (deferred reduce)
        }
      }
}

// Large-tile path (M % 64 == 0): tiles filled by global_load_lds_dwordx4 straight into LDS (no VGPR
// staging, double-buffered, one vmcnt(0) + barrier per k-step).  The DMA image must be lane-linear
// (unpadded 256-B rows), which puts all rows of a transposed read on the same banks (8-way); the
// 16-B chunk s of row r is therefore stored at s ^ 2 f(r), f(r) = (r & 3) | ((r >> 3) & 1) << 2,
// applied on the SOURCE address and undone on the ds_read_b64_tr_b16 address (f separates the
// rows r and r + 8 that one 32-lane half reads together: conflict-free, checked in a bank model).
namespace {
__device__ __forceinline__ int wswz(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

__device__ __forceinline__ bf16x8 wfrag(const char* lds, int k0, int c0) {
  const int l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int u = (c0 >> 2) + (li & 3);
  const int r0 = k0 + 8 * g + (li >> 2), r1 = r0 + 4;
  const char* a0 = lds + r0 * (WB * 2) + ((u ^ (wswz(r0) << 2)) << 3);
  const char* a1 = lds + r1 * (WB * 2) + ((u ^ (wswz(r1) << 2)) << 3);
  return cat8(tr4(reinterpret_cast<const bf16_t*>(a0)), tr4(reinterpret_cast<const bf16_t*>(a1)));
}
}  // namespace

// 256 x 256 output tile, 512 threads (8 waves as 2 (P) x 4 (Q), each 128 x 64 = 8 x 4 MFMA tiles).
// A 128^2 tile moves 64 FLOP per staged byte, which at the MFMA rate needs ~64 B/clk/CU of L2 read
// bandwidth (the per-CU L2 share); 256^2 halves that.  Operand tiles are [64 tokens][256 cols] stored
// as two swizzled [64][128] halves; LDS 2 buffers x (32 + 32) KB = 128 KB -> one workgroup per CU,
// so the split count targets one full round of workgroups.
// CM = true: dY is CHANNEL-major (P rows of M contiguous tokens, the Mamba-1 in_proj gradient d(xz)).
// Its [TP][64-token] tile is then k-contiguous: two [128][64] halves DMA'd with the gemm_tn XOR
// swizzle and read with the plain k-contiguous fragment (no transpose needed on that side).
// CMB = true: X is channel-major as well (Q rows of M contiguous tokens, e.g. the Mamba-1 scan output
// y for the out_proj gradient): staged and read exactly like a CM dY tile.
template <int TP, int TQ, bool CM, bool CMB = false>
__global__ __launch_bounds__(512) void gemm_wgrad_big_k(const bf16_t* __restrict__ dY, int64_t ldy,
                                                        const bf16_t* __restrict__ X, int64_t ldx,
                                                        float* __restrict__ part, int M, int P, int Q, int mslice,
                                                        bool pacc = false) {
  constexpr int HB = WK * WB * 2;            // one [64][128] half-tile: 16 KB
  constexpr int AB = (TP / WB) * HB, BB = (TQ / WB) * HB;
  constexpr int WQN = 4, WPN = 2;            // wave grid
  constexpr int MI = TP / WPN / 16, NJ = TQ / WQN / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * (AB + BB)];
  const int tq = (Q + TQ - 1) / TQ, tp = (P + TP - 1) / TP;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = t % (tp * tq), sl = t / (tp * tq);
  const int p0 = (tile / tq) * TP, q0 = (tile % tq) * TQ;
  const int mb = sl * mslice, me = min(M, mb + mslice);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wp = w / WQN, wq = w % WQN;
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = zero4();
  auto stage = [&](int m0, char* buf) {
    // each [64][128] half-tile is one 256-thread DMA pass (4 chunks per thread): waves 0-3 take the
    // even halves, waves 4-7 the odd ones; slot (r, s) receives source chunk s ^ 2 f(r)
    const int half = threadIdx.x >> 8;  // 0 or 1
#pragma unroll
    for (int hh = 0; hh < TP / WB; hh += 2) {
      const int h = hh + half;
      if (h < TP / WB) {
        const int tid = threadIdx.x & 255, w4 = tid >> 6;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if constexpr (CM) {  // [128 channels][64 tokens] half: slot (r, cs) <- source chunk cs ^ (r & 7)
            const int q = i * 256 + tid, r = q >> 3, cs = q & 7;
            const int row = min(p0 + h * WB + r, P - 1);  // rows past P are never stored
            __builtin_amdgcn_global_load_lds((const void*)(dY + (int64_t)row * ldy + m0 + 8 * (cs ^ (r & 7))),
                                             (lds_void*)(buf + h * HB + (i * 256 + w4 * 64) * 16), 16, 0, 0);
          } else {
            const int q = i * 256 + tid, r = q >> 4, s2 = q & 15;
            const int col = min(p0 + h * WB + 8 * (s2 ^ (2 * wswz(r))), P - 8);
            __builtin_amdgcn_global_load_lds((const void*)(dY + (int64_t)(m0 + r) * ldy + col),
                                             (lds_void*)(buf + h * HB + (i * 256 + w4 * 64) * 16), 16, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int hh = 0; hh < TQ / WB; hh += 2) {
      const int h = hh + half;
      if (h < TQ / WB) {
        const int tid = threadIdx.x & 255, w4 = tid >> 6;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if constexpr (CMB) {
            const int q = i * 256 + tid, r = q >> 3, cs = q & 7;
            const int row = min(q0 + h * WB + r, Q - 1);  // rows past Q are never stored
            __builtin_amdgcn_global_load_lds((const void*)(X + (int64_t)row * ldx + m0 + 8 * (cs ^ (r & 7))),
                                             (lds_void*)(buf + AB + h * HB + (i * 256 + w4 * 64) * 16), 16, 0, 0);
          } else {
            const int q = i * 256 + tid, r = q >> 4, s2 = q & 15;
            const int col = min(q0 + h * WB + 8 * (s2 ^ (2 * wswz(r))), Q - 8);
            __builtin_amdgcn_global_load_lds((const void*)(X + (int64_t)(m0 + r) * ldx + col),
                                             (lds_void*)(buf + AB + h * HB + (i * 256 + w4 * 64) * 16), 16, 0, 0);
          }
        }
      }
    }
  };
  const int KT = (me - mb) / WK;
  if (KT > 0) stage(mb, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const char* cur = smem + (kt & 1) * (AB + BB);
    if (kt + 1 < KT) stage(mb + (kt + 1) * WK, smem + ((kt + 1) & 1) * (AB + BB));
#pragma unroll
    for (int ks = 0; ks < WK / 32; ++ks) {
      bf16x8 bfr[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = wq * (TQ / WQN) + 16 * j;
        bfr[j] = CMB ? frag(cur + AB + (c / WB) * HB, c % WB, ks) : wfrag(cur + AB + (c / WB) * HB, 32 * ks, c % WB);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int c = wp * (TP / WPN) + 16 * i;
        const bf16x8 af = CM ? frag(cur + (c / WB) * HB, c % WB, ks) : wfrag(cur + (c / WB) * HB, 32 * ks, c % WB);
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(af, bfr[j], acc[i][j]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  float* pc = part + (int64_t)sl * P * Q;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = p0 + wp * (TP / WPN) + 16 * i + 4 * (l >> 4) + r;
        const int q = q0 + wq * (TQ / WQN) + 16 * j + (l & 15);
        if (p < P && q < Q) {
          float* d = pc + (int64_t)p * Q + q;
          *d = pacc ? *d + acc[i][j][r] : acc[i][j][r];  // pacc: add into persistent slabs (deferred reduce)
        }
      }
}

// out[i] = sum_s part[s][i] (fixed order), optionally += into out (gradient accumulation)
__global__ void wgrad_reduce_k(const float* __restrict__ part, int S, int64_t n, float* __restrict__ out,
                               bool accumulate) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  float4 s = *reinterpret_cast<const float4*>(part + i);
  for (int k = 1; k < S; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)k * n + i);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  if (accumulate) {
    const float4 o = *reinterpret_cast<const float4*>(out + i);
    s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
  }
  *reinterpret_cast<float4*>(out + i) = s;
}

namespace {
constexpr int BT = 256;  // big-tile size
bool wgrad_big(int M, const void* dY, const void* X) {
  return M % WK == 0 && ((uintptr_t)dY % 16) == 0 && ((uintptr_t)X % 16) == 0;
}
// split count: big tiles run one workgroup per CU -> aim at one full round (~256 workgroups) with
// >= 8 k-steps per slice; small tiles run 2 per CU -> aim at >= 512
int wgrad_splits(int M, int P, int Q, bool big) {
  if (big) {
    // one round (not launchers.h split_k_count): this kernel is the side-stream in-place wgrad of the wide
    // models, where the main stream fills a short last round and extra slabs only add traffic (Mamba-2 1.4B
    // with the rounds-aware rule: 93.8k vs 95.0k tok/s, profiles/r4/wgrad_splits.txt)
    const int tiles = ((P + BT - 1) / BT) * ((Q + BT - 1) / BT);
    int S = std::max(1, 256 / tiles);
    while (S > 1 && M / S < 8 * WK) --S;
    return S;
  }
  const int tiles = ((P + WB - 1) / WB) * ((Q + WB - 1) / WB);
  int S = 1;
  while (tiles * S < 512 && M / (S * 2) >= 4 * WK) S *= 2;
  return S;
}
}  // namespace

int gemm_wgrad_splits(int M, int P, int Q) { return wgrad_splits(M, P, Q, M % WK == 0); }

hipError_t launch_gemm_wgrad(const void* dY, int64_t ldy, const void* X, int64_t ldx, float* part, float* out,
                             int M, int P, int Q, bool accumulate, hipStream_t st) {
  if (ldy % 8 || ldx % 8 || P % 8 || Q % 8 || ((int64_t)P * Q) % 4) return hipErrorInvalidValue;
  const bool big = wgrad_big(M, dY, X);
  const int S = wgrad_splits(M, P, Q, M % WK == 0);  // same rule as gemm_wgrad_splits (part size)
  const int mslice = ((M + S - 1) / S + WK - 1) / WK * WK;
  if (big) {
    const int tiles = ((P + BT - 1) / BT) * ((Q + BT - 1) / BT);
    hipLaunchKernelGGL((gemm_wgrad_big_k<BT, BT, false>), dim3(tiles * S), dim3(512), 0, st, (const bf16_t*)dY, ldy,
                       (const bf16_t*)X, ldx, part, M, P, Q, mslice);
  } else {
    const int tiles = ((P + WB - 1) / WB) * ((Q + WB - 1) / WB);
    hipLaunchKernelGGL(gemm_wgrad_k, dim3(tiles * S), dim3(256), 0, st, (const bf16_t*)dY, ldy, (const bf16_t*)X, ldx,
                       part, M, P, Q, mslice);
  }
  MAMBA_HIP_CHECK(hipGetLastError());
  const int64_t n = (int64_t)P * Q;
  hipLaunchKernelGGL(wgrad_reduce_k, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, st, part, S, n, out,
                     accumulate);
  return hipGetLastError();
}

// ================================ small-K / small-N "skinny" GEMM ===================================
// C[N, M] (+)= A[N, K] . B[K, M] with a small weight A (K-contiguous) and activation / output rows
// that run along the token dimension M (the channel-major Mamba-1 layout, models/mamba1.py):
//   x_dbl = W_x (80 x 1536) . conv_out      delta = W_dt (1536 x 48) . x_dbl[:48]
//   dx_dbl[:48] = W_dt^T . ddelta           dconv_out += W_x^T (1536 x 80) . dx_dbl
// One side of every product is tiny (K = 48 / 80 or N = 48 / 80), so the work is a streaming pass over
// the M-long rows; hipBLASLt runs these 2-4x slower than the bytes allow.  Workgroup = TN rows of C x
// TM tokens; 4 waves split TM; K in steps of 32 through LDS (A tile [TN][32], B tile [32][TM], zero
// padded past K / N); B fragments via ds_read_b64_tr_b16 (K runs down the rows); the epilogue is staged
// through LDS so every global load / store is a 16-B vector along M (ACC adds into C in fp32).
namespace {
constexpr int SK_TN = 64;
}

// BK = K-depth per LDS stage: 32 for the small-K products (one MFMA step), 128 for the long-K ones
// (x_dbl, dx_dbl: 12 stages instead of 48, 4x the bytes in flight per barrier)
template <int TM, int BK, bool ACC>
__global__ __launch_bounds__(256) void gemm_skinny_k(const bf16_t* __restrict__ A, int64_t lda,
                                                     const bf16_t* __restrict__ B, int64_t ldb,
                                                     bf16_t* __restrict__ C, int64_t ldc, int N, int K, int M) {
  constexpr int LDA_ = BK + 8, LDB_ = TM + 8, LDC_ = TM + 8;
  constexpr int WM = TM / 4, NJ = WM / 16, MI = SK_TN / 16;
  constexpr int AB = SK_TN * LDA_ * 2, BB = BK * LDB_ * 2, CB = SK_TN * LDC_ * 2;
  constexpr int SMEM = (AB + BB) > CB ? (AB + BB) : CB;
  constexpr int QA = (SK_TN * BK / 8 + 255) / 256, QB = BK * TM / 8 / 256, QC = SK_TN * TM / 8 / 256;
  static_assert(BK * TM / 8 % 256 == 0 && SK_TN * TM / 8 % 256 == 0, "whole 16-B pieces per thread");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Bs = reinterpret_cast<bf16_t*>(smem + AB);
  const int m0 = blockIdx.x * TM, n0 = blockIdx.y * SK_TN;
  const int w = threadIdx.x >> 6;
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = zero4();
  // Every global load is unconditional, from a clamped (legal) address, and zeroed by a select where it is
  // consumed: a guarded load meets its zero in a phi and is waited for on the spot.  The stage after the
  // current one is requested before the current one's MFMAs, and (ACC) every piece of the C tile the epilogue
  // adds into is requested at once -- in the guarded form the epilogue's 8 read-add-write rounds ran one HBM
  // latency each.
  uint4 ra[QA], rb[QB], rc[QC];
  auto ld_stage = [&](int k0) {
#pragma unroll
    for (int u = 0; u < QA; ++u) {
      const int q = threadIdx.x + 256 * u, r = q / (BK / 8), c = (q % (BK / 8)) * 8;
      ra[u] = *reinterpret_cast<const uint4*>(A + (int64_t)min(n0 + r, N - 1) * lda + min(k0 + c, K - 8));
    }
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      const int q = threadIdx.x + 256 * u, kk = q / (TM / 8), c = (q % (TM / 8)) * 8;
      rb[u] = *reinterpret_cast<const uint4*>(B + (int64_t)min(k0 + kk, K - 1) * ldb + min(m0 + c, M - 8));
    }
  };
  ld_stage(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
#pragma unroll
    for (int u = 0; u < QA; ++u) {  // A tile: 64 rows x BK
      const int q = threadIdx.x + 256 * u, r = q / (BK / 8), c = (q % (BK / 8)) * 8;
      if (q < SK_TN * BK / 8)
        *reinterpret_cast<uint4*>(As + r * LDA_ + c) = (n0 + r < N && k0 + c < K) ? ra[u] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < QB; ++u) {  // B tile: BK k-rows x TM tokens
      const int q = threadIdx.x + 256 * u, kk = q / (TM / 8), c = (q % (TM / 8)) * 8;
      *reinterpret_cast<uint4*>(Bs + kk * LDB_ + c) = (k0 + kk < K && m0 + c < M) ? rb[u] : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    ld_stage(min(k0 + BK, (K - 1) / BK * BK));  // the next stage (the last one again at the end)
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 bfr[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[j] = frag_tr(Bs, LDB_, 32 * ks, w * WM + 16 * j);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const bf16x8 af = frag_kc(As, LDA_, 16 * i, 32 * ks);
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(af, bfr[j], acc[i][j]);
      }
    }
    __syncthreads();
  }
  // epilogue through LDS: lane holds rows n = 16i + 4g + r of column m = w WM + 16 j + (l & 15)
  bf16_t* Cs = reinterpret_cast<bf16_t*>(smem);
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(16 * i + 4 * (l >> 4) + r) * LDC_ + w * WM + 16 * j + (l & 15)] = f2bf(acc[i][j][r]);
  if (ACC) {  // all of the tile's C pieces in flight at once (the accumulators are dead: no register cost)
#pragma unroll
    for (int u = 0; u < QC; ++u) {
      const int q = threadIdx.x + 256 * u, r = q / (TM / 8), c = (q % (TM / 8)) * 8;
      rc[u] = *reinterpret_cast<const uint4*>(C + (int64_t)min(n0 + r, N - 1) * ldc + min(m0 + c, M - 8));
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < QC; ++u) {
    const int q = threadIdx.x + 256 * u, r = q / (TM / 8), c = (q % (TM / 8)) * 8;
    uint4 v = *reinterpret_cast<const uint4*>(Cs + r * LDC_ + c);
    if (ACC) {
      float f[8], o[8];
      ld8bf(reinterpret_cast<const bf16_t*>(&v), f);
      ld8bf(reinterpret_cast<const bf16_t*>(&rc[u]), o);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] += o[e];
      st8bf(reinterpret_cast<bf16_t*>(&v), f);
    }
    if (n0 + r < N && m0 + c < M) *reinterpret_cast<uint4*>(C + (int64_t)(n0 + r) * ldc + m0 + c) = v;
  }
}

bool gemm_skinny_supported(int N, int K, int M, int64_t lda, int64_t ldb, int64_t ldc) {
  // K, M >= 8: the clamped 16-B loads (min(k, K - 8), min(m, M - 8)) stay inside the operands
  return N > 0 && K >= 8 && M >= 8 && K % 8 == 0 && M % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0;
}

hipError_t launch_gemm_skinny(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int N,
                              int K, int M, bool accumulate, hipStream_t st) {
  if (!gemm_skinny_supported(N, K, M, lda, ldb, ldc)) return hipErrorInvalidValue;
  const int ntiles = (N + SK_TN - 1) / SK_TN;
  // wide outputs (N >= 256, small K) take 256-token tiles and one-MFMA-deep stages; narrow ones
  // (N < 256, long K) 128-token tiles (the grid still covers the CUs) and 128-deep stages
  const bool wide = ntiles >= 4;
  const dim3 block(256);
#define SK_LAUNCH(TMV, BKV)                                                                                   \
  {                                                                                                           \
    const dim3 grid((unsigned)((M + (TMV) - 1) / (TMV)), (unsigned)ntiles);                                   \
    if (accumulate)                                                                                           \
      hipLaunchKernelGGL((gemm_skinny_k<TMV, BKV, true>), grid, block, 0, st, (const bf16_t*)A, lda,             \
                         (const bf16_t*)B, ldb, (bf16_t*)C, ldc, N, K, M);                                    \
    else                                                                                                      \
      hipLaunchKernelGGL((gemm_skinny_k<TMV, BKV, false>), grid, block, 0, st, (const bf16_t*)A, lda,            \
                         (const bf16_t*)B, ldb, (bf16_t*)C, ldc, N, K, M);                                    \
  }
  // write-only wide products (delta = W_dt x_dbl[:R]) take 128-token tiles: half the LDS per workgroup, twice the
  // workgroups (and stores) in flight, 45.4 -> 40.4 us at the 280M shape; the read-add-write ones (dconv += W_x^T
  // dx_dbl) stay at 256 (81.8 vs 89.3 us at 128; scripts/skinny_bench.py, profiles/r6/skinny_tiles.txt)
  if (wide && !accumulate) SK_LAUNCH(128, 32) else if (wide) SK_LAUNCH(256, 32) else SK_LAUNCH(128, 128)
#undef SK_LAUNCH
  return hipGetLastError();
}

// dW (P, Q) (+)= dY X with a channel-major dY (P, M) (Mamba-1 d(xz)) and token-major X (M, Q).
// pacc: the split-K slabs in `part` are added into (they persist across the micro-steps of an optimizer
// step); reduce: sum the slabs into `out` (else the slabs are left for a later micro-step).
bool gemm_wgrad_cm_supported(int M, int P, int Q, int64_t ldy, int64_t ldx) {
  return M % WK == 0 && P % 8 == 0 && Q % 8 == 0 && ldy % 8 == 0 && ldx % 8 == 0 && P >= 8 && Q >= 8;
}

hipError_t launch_gemm_wgrad_cm(const void* dY, int64_t ldy, const void* X, int64_t ldx, float* part, float* out,
                                int M, int P, int Q, bool accumulate, bool dy_cm, bool x_cm, hipStream_t st,
                                bool pacc, bool reduce) {
  if (!gemm_wgrad_cm_supported(M, P, Q, ldy, ldx) || (!dy_cm && !x_cm)) return hipErrorInvalidValue;
  const int S = wgrad_splits(M, P, Q, true);
  const int mslice = ((M + S - 1) / S + WK - 1) / WK * WK;
  const int tiles = ((P + BT - 1) / BT) * ((Q + BT - 1) / BT);
  if (dy_cm && x_cm)
    hipLaunchKernelGGL((gemm_wgrad_big_k<BT, BT, true, true>), dim3(tiles * S), dim3(512), 0, st, (const bf16_t*)dY,
                       ldy, (const bf16_t*)X, ldx, part, M, P, Q, mslice, pacc);
  else if (dy_cm)
    hipLaunchKernelGGL((gemm_wgrad_big_k<BT, BT, true, false>), dim3(tiles * S), dim3(512), 0, st, (const bf16_t*)dY,
                       ldy, (const bf16_t*)X, ldx, part, M, P, Q, mslice, pacc);
  else
    hipLaunchKernelGGL((gemm_wgrad_big_k<BT, BT, false, true>), dim3(tiles * S), dim3(512), 0, st, (const bf16_t*)dY,
                       ldy, (const bf16_t*)X, ldx, part, M, P, Q, mslice, pacc);
  MAMBA_HIP_CHECK(hipGetLastError());
  if (!reduce) return hipSuccess;
  const int64_t n = (int64_t)P * Q;
  hipLaunchKernelGGL(wgrad_reduce_k, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, st, part, S, n, out,
                     accumulate);
  return hipGetLastError();
}

bool gemm_tn_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  return M > 0 && N > 0 && K > 0 && K % GBK == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0;
}

hipError_t launch_gemm_tn_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                               int N, int K, hipStream_t st) {
  if (!gemm_tn_supported(M, N, K, lda, ldb, ldc)) return hipErrorInvalidValue;
  const int nwg = ((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
  hipLaunchKernelGGL(gemm_tn_bf16_k, dim3(nwg), dim3(256), 0, st, (const bf16_t*)A, lda, (const bf16_t*)B, ldb,
                     (bf16_t*)C, ldc, M, N, K);
  return hipGetLastError();
}

// ================================ bf16 transpose (the input-gradient GEMMs' W^T operand) ===========================
// Y (C, R) = X (R, C)^T, once per optimizer step per projection weight.  64 x 64 tiles through LDS: 16-B row loads
// and 16-B row stores (R % 8 == 0, C % 8 == 0); torch's copy of a transposed view runs element-wise (strided
// reads, ~16 us for a 3392 x 768 weight).
__global__ __launch_bounds__(256) void transpose_bf16_k(const bf16_t* __restrict__ x, int64_t ldx,
                                                        bf16_t* __restrict__ y, int64_t ldy, int R, int C) {
  __shared__ __attribute__((aligned(16))) unsigned short t[64][72];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = threadIdx.x + k * 256, r = idx >> 3, c = (idx & 7) * 8;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r0 + r < R && c0 + c < C) v = *reinterpret_cast<const uint4*>(x + (int64_t)(r0 + r) * ldx + c0 + c);
    *reinterpret_cast<uint4*>(&t[r][c]) = v;
  }
  __syncthreads();
  const int i = threadIdx.x >> 2, j0 = (threadIdx.x & 3) * 16;
  if (c0 + i >= C) return;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int j = j0 + 8 * h;
    if (r0 + j >= R) break;
    unsigned q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) q[e] = (unsigned)t[j + 2 * e][i] | ((unsigned)t[j + 2 * e + 1][i] << 16);
    *reinterpret_cast<uint4*>(y + (int64_t)(c0 + i) * ldy + r0 + j) = make_uint4(q[0], q[1], q[2], q[3]);
  }
}

hipError_t launch_transpose_bf16(const void* x, int64_t ldx, void* y, int64_t ldy, int R, int C, hipStream_t st) {
  if (R <= 0 || C <= 0 || R % 8 || C % 8 || ldx % 8 || ldy % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose_bf16_k, dim3((C + 63) / 64, (R + 63) / 64), dim3(256), 0, st, (const bf16_t*)x, ldx,
                     (bf16_t*)y, ldy, R, C);
  return hipGetLastError();
}

}  // namespace mamba_amd
