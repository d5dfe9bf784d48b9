// Fused residual-add + RMSNorm and gated RMSNorm, forward and backward, for gfx950.
//
// Design (memory-bound; the roofline is HBM bytes):
//  * one wavefront per row, 4 rows per 256-thread block; each lane owns NCH chunks of 4
//    consecutive columns (col = 4*(lane + 64*c)), loaded as one 8-B (bf16) / 16-B (f32) vector,
//    so a wave instruction covers 512 B / 1 KiB of contiguous row -> fully coalesced.
//  * statistics in fp32, one wave_sum per row (no LDS, no barriers on the row path).
//  * the row stays in registers between the statistics pass and the output pass: HBM sees
//    each input byte once and each output byte once.
//  * weight gradients: each wave accumulates its rows' dy*xhat in registers over a
//    grid-stride loop, the 4 waves of a block are summed through LDS, and one row of partials
//    per block is written; a second kernel sums the partials column-wise in a fixed order
//    (bitwise deterministic, no float atomics).
// Reference semantics: upstream ops/triton/layer_norm.py and layernorm_gated.py.
#include <cstdlib>

#include "common.h"
#include "launchers.h"

namespace mamba_amd {

__device__ __forceinline__ void ld4_dyn(const void* p, int dt, int64_t i, float (&o)[4]) {
  if (dt == kF32) ld4<float>(reinterpret_cast<const float*>(p) + i, o);
  else ld4<bf16_t>(reinterpret_cast<const bf16_t*>(p) + i, o);
}
__device__ __forceinline__ void st4_dyn(void* p, int dt, int64_t i, const float (&o)[4]) {
  if (dt == kF32) st4<float>(reinterpret_cast<float*>(p) + i, o);
  else st4<bf16_t>(reinterpret_cast<bf16_t*>(p) + i, o);
}

// ------------------------------------------------------------------------------------------
template <int NCH>
__global__ __launch_bounds__(256) void add_rmsnorm_fwd_k(
    const void* __restrict__ x, int xdt, int64_t sx, const void* __restrict__ res, int rdt, int64_t sr,
    const float* __restrict__ w, void* __restrict__ y, int ydt, void* __restrict__ ro, int rodt,
    float* __restrict__ rstd, int64_t M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[NCH][4];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4;
    if (col < D) {
      ld4_dyn(x, xdt, row * sx + col, v[c]);
      if (res) {
        float r[4];
        ld4_dyn(res, rdt, row * sr + col, r);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[c][k] += r[k];
      }
      st4_dyn(ro, rodt, row * D + col, v[c]);
#pragma unroll
      for (int k = 0; k < 4; ++k) ss += v[c][k] * v[c][k];
    }
  }
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4;
    if (col < D) {
      float wv[4], o[4];
      ld4<float>(w + col, wv);
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = v[c][k] * rs * wv[k];
      st4_dyn(y, ydt, row * D + col, o);
    }
  }
  if (lane == 0) rstd[row] = rs;
}

// block-level partial reduction of per-wave dw accumulators -> part[blockIdx.x][D]
template <int NCH>
__device__ __forceinline__ void block_dw_partial(float (&acc)[NCH][4], float* part, int D, float* lds, bool pacc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4;
    if (col < D) {
#pragma unroll
      for (int k = 0; k < 4; ++k) lds[wave * D + col + k] = acc[c][k];
    }
  }
  __syncthreads();
  for (int col = threadIdx.x; col < D; col += blockDim.x) {
    const int64_t i = (int64_t)blockIdx.x * D + col;
    const float v = lds[col] + lds[D + col] + lds[2 * D + col] + lds[3 * D + col];
    part[i] = pacc ? part[i] + v : v;  // pacc: accumulate across micro-steps (reduced once per optimizer step)
  }
}

template <int NCH>
__global__ __launch_bounds__(256) void add_rmsnorm_bwd_k(
    const void* __restrict__ dy, int ydt, const void* __restrict__ dro, int drodt,
    const void* __restrict__ ro, int rodt, const float* __restrict__ w, const float* __restrict__ rstd,
    void* __restrict__ dx, int xdt, void* __restrict__ dres, int rdt, float* __restrict__ part, bool pacc,
    int64_t M, int D) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  float acc[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[c][k] = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += (int64_t)gridDim.x * 4) {
    const float rs = rstd[row];
    float xh[NCH][4], dyw[NCH][4];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      if (col < D) {
        float r[4], g[4], wv[4];
        ld4_dyn(ro, rodt, row * D + col, r);
        ld4_dyn(dy, ydt, row * D + col, g);
        ld4<float>(w + col, wv);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          xh[c][k] = r[k] * rs;
          dyw[c][k] = g[k] * wv[k];
          dot += dyw[c][k] * xh[c][k];
          acc[c][k] += g[k] * xh[c][k];
        }
      }
    }
    dot = wave_sum(dot) / (float)D;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      if (col < D) {
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = (dyw[c][k] - xh[c][k] * dot) * rs;
        if (dro) {
          float d2[4];
          ld4_dyn(dro, drodt, row * D + col, d2);
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] += d2[k];
        }
        st4_dyn(dx, xdt, row * D + col, o);
        if (dres) st4_dyn(dres, rdt, row * D + col, o);
      }
    }
  }
  block_dw_partial<NCH>(acc, part, D, lds, pacc);
}

// ------------------------------------------------------------------------------------------
// Typed fast paths for the training dtypes (x / y / dy / dx in TX, the residual stream res / ro / dro /
// dres in TR -- bf16 + fp32 with residual_in_fp32).  The dynamic-dtype kernels above branch per load,
// and the two load flavours meeting in a phi force a vmcnt(0) after EVERY load, so a row's 9-12 loads
// run one latency at a time; here a row's loads are all issued before the first wait.  Columns past D
// load a clamped (valid) address and contribute zero, so the row path has no per-lane branch either,
// and w stays in registers across the grid-stride rows.
template <int NCH, typename TX, typename TR, bool RES>
__global__ __launch_bounds__(256) void add_rmsnorm_fwd_t_k(
    const TX* __restrict__ x, int64_t sx, const TR* __restrict__ res, int64_t sr, const float* __restrict__ w,
    TX* __restrict__ y, TR* __restrict__ ro, float* __restrict__ rstd, int64_t M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[NCH][4], r[NCH][4], wv[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4, cc = col < D ? col : 0;
    ld4<TX>(x + row * sx + cc, v[c]);
    if (RES) ld4<TR>(res + row * sr + cc, r[c]);
    ld4<float>(w + cc, wv[c]);
  }
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (RES) v[c][k] += r[c][k];
      s = fmaf(v[c][k], v[c][k], s);
    }
    if (col < D) {
      ss += s;
      st4<TR>(ro + row * D + col, v[c]);
    }
  }
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4;
    if (col < D) {
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = v[c][k] * rs * wv[c][k];
      st4<TX>(y + row * D + col, o);
    }
  }
  if (lane == 0) rstd[row] = rs;
}

template <int NCH, typename TX, typename TR, bool DRO>
__global__ __launch_bounds__(256) void add_rmsnorm_bwd_t_k(
    const TX* __restrict__ dy, const TR* __restrict__ dro, const TR* __restrict__ ro, const float* __restrict__ w,
    const float* __restrict__ rstd, TX* __restrict__ dx, TR* __restrict__ dres, float* __restrict__ part, bool pacc,
    int64_t M, int D) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  float acc[NCH][4], wv[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4;
    ld4<float>(w + (col < D ? col : 0), wv[c]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[c][k] = 0.f;
      if (col >= D) wv[c][k] = 0.f;  // out-of-row lanes: dyw = 0 -> no dot / acc contribution
    }
  }
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += (int64_t)gridDim.x * 4) {
    float xh[NCH][4], g[NCH][4], d2[NCH][4];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4, cc = col < D ? col : 0;
      ld4<TR>(ro + row * D + cc, xh[c]);
      ld4<TX>(dy + row * D + cc, g[c]);
      if (DRO) ld4<TR>(dro + row * D + cc, d2[c]);
    }
    const float rs = rstd[row];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xh[c][k] *= rs;
        dot = fmaf(g[c][k] * wv[c][k], xh[c][k], dot);
        if ((lane + 64 * c) * 4 < D) acc[c][k] = fmaf(g[c][k], xh[c][k], acc[c][k]);
      }
    dot = wave_sum(dot) / (float)D;
    // d2 is only read under the (col < D) store guard: pin it here, or the compiler sinks its load into
    // that branch, behind the reduction, with a vmcnt(0) of its own
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      if (DRO) asm volatile("" : "+v"(d2[c][0]), "+v"(d2[c][1]), "+v"(d2[c][2]), "+v"(d2[c][3]));
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      if (col < D) {
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o[k] = (g[c][k] * wv[c][k] - xh[c][k] * dot) * rs;
          if (DRO) o[k] += d2[c][k];
        }
        st4<TX>(dx + row * D + col, o);
        if (dres) st4<TR>(dres + row * D + col, o);
      }
    }
  }
  block_dw_partial<NCH>(acc, part, D, lds, pacc);
}

// out[c] = sum_r part[r * rstride + c] in a fixed order.  Block = 64 columns x 16 row-groups (1024
// threads); each thread sums a strided row subset (independent loads -> deep memory-level
// parallelism), the 16 group sums are combined through LDS in index order -> bitwise deterministic.
__global__ __launch_bounds__(1024) void colsum_k(const float* __restrict__ part, int nrows, int ncols,
                                                 int64_t rstride, float* __restrict__ out) {
  __shared__ float red[16][65];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < ncols) {
    int r = rg;
    for (; r + 48 < nrows; r += 64) {
      const float a0 = part[(int64_t)r * rstride + c], a1 = part[(int64_t)(r + 16) * rstride + c];
      const float a2 = part[(int64_t)(r + 32) * rstride + c], a3 = part[(int64_t)(r + 48) * rstride + c];
      s += (a0 + a1) + (a2 + a3);
    }
    for (; r < nrows; r += 16) s += part[(int64_t)r * rstride + c];
  }
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < ncols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][cl];
    out[c] = t;
  }
}

// Stage 1 of a tall reduction: block (column tile, split s) sums rows [s*R, min((s+1)*R, nrows)) and
// writes the result over the first row of its own range (every read of that range precedes the
// write: the block barrier), so no scratch buffer is needed and blocks never touch each other's rows.
__global__ __launch_bounds__(256) void colsum_split_k(float* __restrict__ part, int nrows, int ncols, int R) {
  __shared__ float red[4][65];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * R, r1 = min(r0 + R, nrows);
  float s0 = 0.f, s1 = 0.f;
  if (c < ncols) {
    int r = r0 + rg;
    for (; r + 4 < r1; r += 8) {
      s0 += part[(int64_t)r * ncols + c];
      s1 += part[(int64_t)(r + 4) * ncols + c];
    }
    if (r < r1) s0 += part[(int64_t)r * ncols + c];
  }
  red[rg][cl] = s0 + s1;
  __syncthreads();
  if (rg == 0 && c < ncols) part[(int64_t)r0 * ncols + c] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

// Column sums of a (nrows, ncols) fp32 partial block (clobbers `part`).  Tall blocks with few column
// tiles (norm weight grads: 2048 x 768 -> 12 tiles) are split over >= ~512 workgroups first, so the
// sum is bandwidth- rather than latency-bound; the second stage reduces the RS split sums.
// (A single-launch form -- each tile's last block summing the splits behind an agent-scope release/acquire
// handoff -- measured 39-43 us against 6.5-10.6 us for the two launches at the backward's shapes: the device-scope
// release writes back the XCD's L2 (profiles/r5/colsum_single_launch_rejected.txt).)
hipError_t launch_colsum(float* part, int nrows, int ncols, float* out, hipStream_t st) {
  const int tiles = (ncols + 63) / 64;
  int RS = std::min((nrows + 15) / 16, std::max(1, 512 / tiles));
  if (RS <= 1 || nrows <= 64) {
    hipLaunchKernelGGL(colsum_k, dim3(tiles), dim3(1024), 0, st, part, nrows, ncols, (int64_t)ncols, out);
    return hipGetLastError();
  }
  const int R = (nrows + RS - 1) / RS;
  RS = (nrows + R - 1) / R;
  hipLaunchKernelGGL(colsum_split_k, dim3(tiles, RS), dim3(256), 0, st, part, nrows, ncols, R);
  MAMBA_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(colsum_k, dim3(tiles), dim3(1024), 0, st, part, RS, ncols, (int64_t)R * ncols, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Batched late column sums (ops/grad_accum.py::late_colsum): at the sync micro-step every deferred parameter-gradient
// partial block of the backward (norm weights, conv taps + bias, A_log / D / dt_bias) is reduced by ONE pair of
// launches after the backward instead of two launches per block inside it -- at one micro-batch per optimizer step
// (the 8-GPU per-rank regime) those ~4 small launch pairs per layer were 1.6% of the step.  The column sums go
// straight into the parameters' .grad storage.  Host table row (ops/grad_accum.py _LATE_DTYPE, 64 bytes):
struct LateCol {
  float* part;               // (nrows, ncols) fp32 partial rows (stage 1 overwrites the first row of each split)
  float* dst[3];             // destinations (see mode)
  int nrows, ncols, R, RS;   // rows per split, splits
  int G, mode, acc, pad0;    // mode 0: dst0[j]; 1: j = o G + i -> i < G - 1 ? dst0[o (G - 1) + i] : dst1[o]
                             // (conv taps | bias); 2: j = o G + i -> dst[o][i] (A | D | bias); acc bit k: dst k +=
  int blk0, tile0;           // first stage-1 block / stage-2 tile of this entry
  int pad1, pad2;
};
static_assert(sizeof(LateCol) == 80, "late column-sum table row layout is shared with the host");

__device__ __forceinline__ int late_find(const LateCol* __restrict__ t, int n, int key, bool by_tile) {
  int lo = 0, hi = n - 1;  // last entry whose first index <= key
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((by_tile ? t[mid].tile0 : t[mid].blk0) <= key) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// stage 1: block = (entry, column tile, split): the split's R rows of 64 columns, summed in a fixed order, written
// over the split's first row
__global__ __launch_bounds__(256) void late_colsum_split_k(const LateCol* __restrict__ tab, int n) {
  __shared__ float red[4][65];
  __shared__ int ent;
  if (threadIdx.x == 0) ent = late_find(tab, n, blockIdx.x, false);
  __syncthreads();
  const LateCol e = tab[ent];
  const int tiles = (e.ncols + 63) / 64, rel = blockIdx.x - e.blk0;
  const int tile = rel % tiles, sp = rel / tiles;
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = tile * 64 + cl;
  const int r0 = sp * e.R, r1 = min(r0 + e.R, e.nrows);
  float s0 = 0.f, s1 = 0.f;
  if (c < e.ncols) {
    int r = r0 + rg;
    for (; r + 4 < r1; r += 8) {
      s0 += e.part[(int64_t)r * e.ncols + c];
      s1 += e.part[(int64_t)(r + 4) * e.ncols + c];
    }
    if (r < r1) s0 += e.part[(int64_t)r * e.ncols + c];
  }
  red[rg][cl] = s0 + s1;
  __syncthreads();
  if (rg == 0 && c < e.ncols) e.part[(int64_t)r0 * e.ncols + c] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

// stage 2: block = (entry, column tile): the RS split sums in order, then the destination mapping
__global__ __launch_bounds__(256) void late_colsum_final_k(const LateCol* __restrict__ tab, int n) {
  __shared__ float red[4][65];
  __shared__ int ent;
  if (threadIdx.x == 0) ent = late_find(tab, n, blockIdx.x, true);
  __syncthreads();
  const LateCol e = tab[ent];
  const int tile = blockIdx.x - e.tile0;
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = tile * 64 + cl;
  float s = 0.f;
  if (c < e.ncols)
    for (int k = rg; k < e.RS; k += 4) s += e.part[(int64_t)k * e.R * e.ncols + c];
  red[rg][cl] = s;
  __syncthreads();
  if (rg != 0 || c >= e.ncols) return;
  const float t = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
  int k = 0;
  int64_t off = c;
  if (e.mode == 1) {
    const int o = c / e.G, i = c % e.G;
    if (i < e.G - 1) { k = 0; off = (int64_t)o * (e.G - 1) + i; } else { k = 1; off = o; }
  } else if (e.mode == 2) {
    k = c / e.G;
    off = c % e.G;
  }
  float* d = e.dst[k];
  if (d == nullptr) return;
  d[off] = ((e.acc >> k) & 1) ? d[off] + t : t;
}

hipError_t launch_late_colsum(const void* tab, int n, int nblk, int ntile, hipStream_t st) {
  if (n <= 0 || nblk <= 0 || ntile <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(late_colsum_split_k, dim3(nblk), dim3(256), 0, st, (const LateCol*)tab, n);
  MAMBA_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(late_colsum_final_k, dim3(ntile), dim3(256), 0, st, (const LateCol*)tab, n);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// gated RMSNorm: y = RMSNorm_group(x * silu(z)) * w   (NBG = norm_before_gate=false)
//                y = RMSNorm_group(x) * w * silu(z)    (NBG = true)
template <int NCH, bool NBG>
__global__ __launch_bounds__(256) void gated_rmsnorm_fwd_k(
    const void* __restrict__ x, int xdt, int64_t sx, const void* __restrict__ z, int zdt, int64_t sz,
    const float* __restrict__ w, void* __restrict__ y, int ydt, float* __restrict__ rstd, int64_t M, int D,
    int G, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int ngroups = D / G;
  float v[NCH][4], sz4[NCH][4], sq[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4;
    sq[c] = 0.f;
    if (col < D) {
      float zz[4];
      ld4_dyn(x, xdt, row * sx + col, v[c]);
      ld4_dyn(z, zdt, row * sz + col, zz);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sz4[c][k] = siluf_(zz[k]);
        if (!NBG) v[c][k] *= sz4[c][k];
        sq[c] += v[c][k] * v[c][k];
      }
    }
  }
  float rsc[NCH];
  for (int g = 0; g < ngroups; ++g) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      if (col < D && col / G == g) s += sq[c];
    }
    s = wave_sum(s);
    const float rs = rsqrtf(s / (float)G + eps);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      if (col / G == g) rsc[c] = rs;
    }
    if (lane == 0) rstd[row * ngroups + g] = rs;
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4;
    if (col < D) {
      float wv[4], o[4];
      ld4<float>(w + col, wv);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[k] = v[c][k] * rsc[c] * wv[k];
        if (NBG) o[k] *= sz4[c][k];
      }
      st4_dyn(y, ydt, row * D + col, o);
    }
  }
}

template <int NCH, bool NBG>
__global__ __launch_bounds__(256) void gated_rmsnorm_bwd_k(
    const void* __restrict__ dy, int ydt, const void* __restrict__ x, int xdt, int64_t sx,
    const void* __restrict__ z, int zdt, int64_t sz, const float* __restrict__ w,
    const float* __restrict__ rstd, void* __restrict__ dx, int64_t sdx, void* __restrict__ dz, int64_t sdz,
    float* __restrict__ part, bool pacc, int64_t M, int D, int G) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  const int ngroups = D / G;
  float acc[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[c][k] = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += (int64_t)gridDim.x * 4) {
    float xv[NCH][4], zv[NCH][4], dyw[NCH][4], xh[NCH][4], rsc[NCH], dotc[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      rsc[c] = 0.f;
      dotc[c] = 0.f;
      if (col < D) {
        float g[4], wv[4];
        ld4_dyn(x, xdt, row * sx + col, xv[c]);
        ld4_dyn(z, zdt, row * sz + col, zv[c]);
        ld4_dyn(dy, ydt, row * D + col, g);
        ld4<float>(w + col, wv);
        rsc[c] = rstd[row * ngroups + col / G];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float s = siluf_(zv[c][k]);
          const float base = NBG ? xv[c][k] : xv[c][k] * s;
          xh[c][k] = base * rsc[c];
          const float dyn = NBG ? g[k] * s : g[k];
          dyw[c][k] = dyn * wv[k];
          dotc[c] += dyw[c][k] * xh[c][k];
          acc[c][k] += dyn * xh[c][k];
        }
      }
    }
    float dotg[NCH];
    for (int gi = 0; gi < ngroups; ++gi) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = (lane + 64 * c) * 4;
        if (col < D && col / G == gi) s += dotc[c];
      }
      s = wave_sum(s) / (float)G;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = (lane + 64 * c) * 4;
        if (col / G == gi) dotg[c] = s;
      }
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      if (col < D) {
        float ox[4], oz[4], g[4], wv[4];
        if (NBG) {
          ld4_dyn(dy, ydt, row * D + col, g);
          ld4<float>(w + col, wv);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float sg = sigmoidf_(zv[c][k]);
          const float s = zv[c][k] * sg;
          const float dsilu = sg * (1.f + zv[c][k] * (1.f - sg));
          const float dbase = (dyw[c][k] - xh[c][k] * dotg[c]) * rsc[c];
          if (NBG) {
            ox[k] = dbase;
            oz[k] = g[k] * xh[c][k] * wv[k] * dsilu;
          } else {
            ox[k] = dbase * s;
            oz[k] = dbase * xv[c][k] * dsilu;
          }
        }
        st4_dyn(dx, xdt, row * sdx + col, ox);
        st4_dyn(dz, zdt, row * sdz + col, oz);
      }
    }
  }
  block_dw_partial<NCH>(acc, part, D, lds, pacc);
}

// bf16 fast path of the gated backward: x / z / dy stay PACKED (4 bf16 = 2 VGPRs per chunk) between
// the statistics pass and the output pass and every derived value is recomputed -> ~1/2 the VGPRs of
// the generic kernel, 2x the resident waves for this HBM-bound kernel.
__device__ __forceinline__ void unpack4(uint2 v, float (&o)[4]) {
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
}
template <int NCH, bool NBG>
__global__ __launch_bounds__(256) void gated_rmsnorm_bwd_bf16_k(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, int64_t sx, const bf16_t* __restrict__ z,
    int64_t sz, const float* __restrict__ w, const float* __restrict__ rstd, bf16_t* __restrict__ dx, int64_t sdx,
    bf16_t* __restrict__ dz, int64_t sdz, float* __restrict__ part, bool pacc, int64_t M, int D, int G) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  const int ngroups = D / G;
  float acc[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[c][k] = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += (int64_t)gridDim.x * 4) {
    uint2 px[NCH], pz[NCH], pg[NCH];
    float dotc[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      dotc[c] = 0.f;
      if (col < D) {
        px[c] = *reinterpret_cast<const uint2*>(x + row * sx + col);
        pz[c] = *reinterpret_cast<const uint2*>(z + row * sz + col);
        pg[c] = *reinterpret_cast<const uint2*>(dy + row * D + col);
      }
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      if (col < D) {
        float xv[4], zv[4], g[4], wv[4];
        unpack4(px[c], xv); unpack4(pz[c], zv); unpack4(pg[c], g);
        ld4<float>(w + col, wv);
        const float rs = rstd[row * ngroups + col / G];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float s = siluf_(zv[k]);
          const float xh = (NBG ? xv[k] : xv[k] * s) * rs;
          const float dyn = NBG ? g[k] * s : g[k];
          dotc[c] += dyn * wv[k] * xh;
          acc[c][k] += dyn * xh;
        }
      }
    }
    // make the packed inputs opaque here so the compiler recomputes pass-1 values in pass 2 instead of
    // keeping ~6 unpacked fp32 copies per element live across the reduction (register pressure)
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("" : "+v"(px[c].x), "+v"(px[c].y), "+v"(pz[c].x), "+v"(pz[c].y), "+v"(pg[c].x), "+v"(pg[c].y));
    float dotg[NCH];
    for (int gi = 0; gi < ngroups; ++gi) {
      float sacc = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = (lane + 64 * c) * 4;
        if (col < D && col / G == gi) sacc += dotc[c];
      }
      sacc = wave_sum(sacc) / (float)G;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = (lane + 64 * c) * 4;
        if (col / G == gi) dotg[c] = sacc;
      }
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      if (col < D) {
        float xv[4], zv[4], g[4], wv[4], ox[4], oz[4];
        unpack4(px[c], xv); unpack4(pz[c], zv); unpack4(pg[c], g);
        ld4<float>(w + col, wv);
        const float rs = rstd[row * ngroups + col / G];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float sg = sigmoidf_(zv[k]);
          const float s = zv[k] * sg;
          const float dsilu = sg * (1.f + zv[k] * (1.f - sg));
          const float xh = (NBG ? xv[k] : xv[k] * s) * rs;
          const float dyn = NBG ? g[k] * s : g[k];
          const float dbase = (dyn * wv[k] - xh * dotg[c]) * rs;
          if (NBG) {
            ox[k] = dbase;
            oz[k] = g[k] * xh * wv[k] * dsilu;
          } else {
            ox[k] = dbase * s;
            oz[k] = dbase * xv[k] * dsilu;
          }
        }
        st4<bf16_t>(dx + row * sdx + col, ox);
        st4<bf16_t>(dz + row * sdz + col, oz);
      }
    }
  }
  block_dw_partial<NCH>(acc, part, D, lds, pacc);
}

// ------------------------------------------------------------------------------------------
// 16-byte fast path of the gated norm (bf16 x / z / y, one norm group per row, norm_before_gate=False,
// D % 512 == 0, 16-B aligned rows): each lane owns NCH chunks of 8 consecutive columns
// (col = 8 (lane + 64 c)), so every load / store is one dwordx4 per lane and a wave instruction moves
// 1 KiB of a row.  The Mamba-2 shape (D = 1536, z a strided slice of zxbcdt) runs here.
__device__ __forceinline__ void unpack8f(uint4 v, float (&o)[8]) {
  const unsigned q[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[2 * j] = __uint_as_float(q[j] << 16);
    o[2 * j + 1] = __uint_as_float(q[j] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8f(const float (&o)[8]) {
  return make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
}

template <int NCH>
__global__ __launch_bounds__(256) void gated_rmsnorm_fwd_v8_k(const bf16_t* __restrict__ x, int64_t sx,
                                                              const bf16_t* __restrict__ z, int64_t sz,
                                                              const float* __restrict__ w, bf16_t* __restrict__ y,
                                                              float* __restrict__ rstd, int64_t M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  uint4 px[NCH], pz[NCH];
  float4 w0[NCH], w1[NCH];  // w issued with the row, not after the reduction (an L2 round trip per chunk)
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 8;
    px[c] = *reinterpret_cast<const uint4*>(x + row * sx + col);
    pz[c] = *reinterpret_cast<const uint4*>(z + row * sz + col);
    w0[c] = *reinterpret_cast<const float4*>(w + col);
    w1[c] = *reinterpret_cast<const float4*>(w + col + 4);
  }
  float g[NCH][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    float xv[8], zv[8];
    unpack8f(px[c], xv);
    unpack8f(pz[c], zv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[c][j] = xv[j] * siluf_(zv[j]);
      ss = fmaf(g[c][j], g[c][j], ss);
    }
  }
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 8;
    const float wv[8] = {w0[c].x, w0[c].y, w0[c].z, w0[c].w, w1[c].x, w1[c].y, w1[c].z, w1[c].w};
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[c][j] * rs * wv[j];
    *reinterpret_cast<uint4*>(y + row * D + col) = pack8f(o);
  }
  if (lane == 0) rstd[row] = rs;
}

template <int NCH>
__global__ __launch_bounds__(256) void gated_rmsnorm_bwd_v8_k(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, int64_t sx, const bf16_t* __restrict__ z,
    int64_t sz, const float* __restrict__ w, const float* __restrict__ rstd, bf16_t* __restrict__ dx, int64_t sdx,
    bf16_t* __restrict__ dz, int64_t sdz, float* __restrict__ part, bool pacc, int64_t M, int D) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // w staged once per block in LDS behind the dw-partial area: both passes read it per row, and from
  // global memory the compiler rematerialised those reads (to save VGPRs) as L2 round trips with a
  // vmcnt(0) each in the output pass
  float* wl = lds + 4 * D;
  for (int i = threadIdx.x * 4; i < D; i += 1024) *reinterpret_cast<float4*>(wl + i) = *reinterpret_cast<const float4*>(w + i);
  __syncthreads();
  float acc[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < M; row += (int64_t)gridDim.x * 4) {
    uint4 pg[NCH], px[NCH], pz[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 8;
      pg[c] = *reinterpret_cast<const uint4*>(dy + row * D + col);
      px[c] = *reinterpret_cast<const uint4*>(x + row * sx + col);
      pz[c] = *reinterpret_cast<const uint4*>(z + row * sz + col);
    }
    const float rs = rstd[row];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 8;
      const float4 w0 = *reinterpret_cast<const float4*>(wl + col), w1 = *reinterpret_cast<const float4*>(wl + col + 4);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      float gv[8], xv[8], zv[8];
      unpack8f(pg[c], gv);
      unpack8f(px[c], xv);
      unpack8f(pz[c], zv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = xv[j] * siluf_(zv[j]) * rs;
        dot = fmaf(gv[j] * wv[j], xh, dot);
        acc[c][j] = fmaf(gv[j], xh, acc[c][j]);
      }
    }
    // keep the packed inputs opaque across the reduction so pass 2 recomputes from them instead of
    // holding ~3 unpacked fp32 copies of every element (register pressure -> occupancy)
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("" : "+v"(pg[c].x), "+v"(pg[c].y), "+v"(pg[c].z), "+v"(pg[c].w), "+v"(px[c].x), "+v"(px[c].y),
                   "+v"(px[c].z), "+v"(px[c].w), "+v"(pz[c].x), "+v"(pz[c].y), "+v"(pz[c].z), "+v"(pz[c].w));
    dot = wave_sum(dot) / (float)D;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 8;
      const float4 w0 = *reinterpret_cast<const float4*>(wl + col), w1 = *reinterpret_cast<const float4*>(wl + col + 4);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      float gv[8], xv[8], zv[8], ox[8], oz[8];
      unpack8f(pg[c], gv);
      unpack8f(px[c], xv);
      unpack8f(pz[c], zv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float sg = sigmoidf_(zv[j]);
        const float sl = zv[j] * sg;
        const float dsilu = sg * (1.f + zv[j] * (1.f - sg));
        const float xh = xv[j] * sl * rs;
        const float dbase = (gv[j] * wv[j] - xh * dot) * rs;
        ox[j] = dbase * sl;
        oz[j] = dbase * xv[j] * dsilu;
      }
      *reinterpret_cast<uint4*>(dx + row * sdx + col) = pack8f(ox);
      *reinterpret_cast<uint4*>(dz + row * sdz + col) = pack8f(oz);
    }
  }
  // per-block dw partial: the 4 waves' accumulators summed through LDS in wave order
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) lds[wave * D + col + j] = acc[c][j];
  }
  __syncthreads();
  for (int col = threadIdx.x; col < D; col += blockDim.x) {
    const int64_t i = (int64_t)blockIdx.x * D + col;
    const float v = lds[col] + lds[D + col] + lds[2 * D + col] + lds[3 * D + col];
    part[i] = pacc ? part[i] + v : v;
  }
}

#define NCH8_SWITCH(D, ...)                                         \
  do {                                                              \
    switch ((D) / 512) {                                            \
      case 1: { constexpr int NCH = 1; __VA_ARGS__; break; }        \
      case 2: { constexpr int NCH = 2; __VA_ARGS__; break; }        \
      case 3: { constexpr int NCH = 3; __VA_ARGS__; break; }        \
      case 4: { constexpr int NCH = 4; __VA_ARGS__; break; }        \
      case 6: { constexpr int NCH = 6; __VA_ARGS__; break; }        \
      case 8: { constexpr int NCH = 8; __VA_ARGS__; break; }        \
      case 10: { constexpr int NCH = 10; __VA_ARGS__; break; }      \
      default: return hipErrorInvalidValue;                         \
    }                                                               \
  } while (0)

static bool gated_v8_ok(int D, int G, bool nbg, int xdt, int zdt, int64_t sx, int64_t sz, const void* x,
                        const void* z) {
  const int q = D / 512;
  return !nbg && G == D && D % 512 == 0 && (q <= 4 || q == 6 || q == 8 || q == 10) && xdt == kBF16 &&
         zdt == kBF16 && sx % 8 == 0 && sz % 8 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)z % 16 == 0;
}

// ------------------------------------------------------------------------------------------
// host launchers
#define NCH_SWITCH(D, ...)                                               \
  do {                                                                   \
    int _nch = ((D) + 255) / 256;                                        \
    if (_nch <= 1) { constexpr int NCH = 1; __VA_ARGS__; }               \
    else if (_nch <= 2) { constexpr int NCH = 2; __VA_ARGS__; }          \
    else if (_nch <= 3) { constexpr int NCH = 3; __VA_ARGS__; }          \
    else if (_nch <= 4) { constexpr int NCH = 4; __VA_ARGS__; }          \
    else if (_nch <= 6) { constexpr int NCH = 6; __VA_ARGS__; }          \
    else if (_nch <= 8) { constexpr int NCH = 8; __VA_ARGS__; }          \
    else if (_nch <= 10) { constexpr int NCH = 10; __VA_ARGS__; }        \
    else if (_nch <= 12) { constexpr int NCH = 12; __VA_ARGS__; }        \
    else if (_nch <= 16) { constexpr int NCH = 16; __VA_ARGS__; }        \
    else if (_nch <= 20) { constexpr int NCH = 20; __VA_ARGS__; }        \
    else return hipErrorInvalidValue;                                    \
  } while (0)

static int bwd_grid(int64_t M) {
  constexpr int cap = 2048;  // partial rows of the weight-gradient column sums (1024 / 4096 measured equal or slower)
  int64_t g = (M + 3) / 4;
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

hipError_t launch_add_rmsnorm_fwd(const void* x, int xdt, int64_t sx, const void* res, int rdt, int64_t sr,
                                  const float* w, void* y, int ydt, void* ro, int rodt, float* rstd, int64_t M,
                                  int D, float eps, hipStream_t st) {
  if (M == 0) return hipSuccess;
  dim3 grid((unsigned)((M + 3) / 4)), block(256);
  if (xdt == kBF16 && ydt == kBF16 && rodt == kF32 && (!res || rdt == kF32)) {
    const bf16_t* xb = (const bf16_t*)x;
    if (res) {
      NCH_SWITCH(D, hipLaunchKernelGGL((add_rmsnorm_fwd_t_k<NCH, bf16_t, float, true>), grid, block, 0, st, xb, sx,
                                       (const float*)res, sr, w, (bf16_t*)y, (float*)ro, rstd, M, D, eps));
    } else {
      NCH_SWITCH(D, hipLaunchKernelGGL((add_rmsnorm_fwd_t_k<NCH, bf16_t, float, false>), grid, block, 0, st, xb, sx,
                                       (const float*)nullptr, sr, w, (bf16_t*)y, (float*)ro, rstd, M, D, eps));
    }
    return hipGetLastError();
  }
  NCH_SWITCH(D, hipLaunchKernelGGL((add_rmsnorm_fwd_k<NCH>), grid, block, 0, st, x, xdt, sx, res, rdt, sr, w, y,
                                   ydt, ro, rodt, rstd, M, D, eps));
  return hipGetLastError();
}

int add_rmsnorm_bwd_partial_rows(int64_t M) { return bwd_grid(M); }

hipError_t launch_add_rmsnorm_bwd(const void* dy, int ydt, const void* dro, int drodt, const void* ro, int rodt,
                                  const float* w, const float* rstd, void* dx, int xdt, void* dres, int rdt,
                                  float* part, float* dw, bool pacc, int64_t M, int D, hipStream_t st) {
  const int g = bwd_grid(M);
  const size_t lds = 4 * (size_t)D * sizeof(float);
  if (ydt == kBF16 && xdt == kBF16 && rodt == kF32 && (!dro || drodt == kF32) && (!dres || rdt == kF32)) {
    const bf16_t* dyb = (const bf16_t*)dy;
    if (dro) {
      NCH_SWITCH(D, hipLaunchKernelGGL((add_rmsnorm_bwd_t_k<NCH, bf16_t, float, true>), dim3(g), dim3(256), lds, st,
                                       dyb, (const float*)dro, (const float*)ro, w, rstd, (bf16_t*)dx, (float*)dres,
                                       part, pacc, M, D));
    } else {
      NCH_SWITCH(D, hipLaunchKernelGGL((add_rmsnorm_bwd_t_k<NCH, bf16_t, float, false>), dim3(g), dim3(256), lds, st,
                                       dyb, (const float*)nullptr, (const float*)ro, w, rstd, (bf16_t*)dx,
                                       (float*)dres, part, pacc, M, D));
    }
  } else {
    NCH_SWITCH(D, hipLaunchKernelGGL((add_rmsnorm_bwd_k<NCH>), dim3(g), dim3(256), lds, st, dy, ydt, dro, drodt, ro,
                                     rodt, w, rstd, dx, xdt, dres, rdt, part, pacc, M, D));
  }
  MAMBA_HIP_CHECK(hipGetLastError());
  return dw ? launch_colsum(part, g, D, dw, st) : hipSuccess;
}

hipError_t launch_gated_rmsnorm_fwd(const void* x, int xdt, int64_t sx, const void* z, int zdt, int64_t sz,
                                    const float* w, void* y, int ydt, float* rstd, int64_t M, int D, int G,
                                    float eps, bool nbg, hipStream_t st) {
  if (M == 0) return hipSuccess;
  dim3 grid((unsigned)((M + 3) / 4)), block(256);
  if (ydt == kBF16 && gated_v8_ok(D, G, nbg, xdt, zdt, sx, sz, x, z) && (uintptr_t)y % 16 == 0) {
    NCH8_SWITCH(D, hipLaunchKernelGGL((gated_rmsnorm_fwd_v8_k<NCH>), grid, block, 0, st, (const bf16_t*)x, sx,
                                      (const bf16_t*)z, sz, w, (bf16_t*)y, rstd, M, D, eps));
    return hipGetLastError();
  }
  if (nbg) {
    NCH_SWITCH(D, hipLaunchKernelGGL((gated_rmsnorm_fwd_k<NCH, true>), grid, block, 0, st, x, xdt, sx, z, zdt, sz,
                                     w, y, ydt, rstd, M, D, G, eps));
  } else {
    NCH_SWITCH(D, hipLaunchKernelGGL((gated_rmsnorm_fwd_k<NCH, false>), grid, block, 0, st, x, xdt, sx, z, zdt,
                                     sz, w, y, ydt, rstd, M, D, G, eps));
  }
  return hipGetLastError();
}

hipError_t launch_gated_rmsnorm_bwd(const void* dy, int ydt, const void* x, int xdt, int64_t sx, const void* z,
                                    int zdt, int64_t sz, const float* w, const float* rstd, void* dx, int64_t sdx,
                                    void* dz, int64_t sdz, float* part, float* dw, bool pacc, int64_t M, int D, int G,
                                    bool nbg, hipStream_t st) {
  const int g = bwd_grid(M);
  const size_t lds = 4 * (size_t)D * sizeof(float);
  const bool fast = ydt == kBF16 && xdt == kBF16 && zdt == kBF16;
  if (fast && gated_v8_ok(D, G, nbg, xdt, zdt, sx, sz, x, z) && sdx % 8 == 0 && sdz % 8 == 0 &&
      (uintptr_t)dx % 16 == 0 && (uintptr_t)dz % 16 == 0 && (uintptr_t)dy % 16 == 0) {
    NCH8_SWITCH(D, hipLaunchKernelGGL((gated_rmsnorm_bwd_v8_k<NCH>), dim3(g), dim3(256), lds + D * sizeof(float), st, (const bf16_t*)dy,
                                      (const bf16_t*)x, sx, (const bf16_t*)z, sz, w, rstd, (bf16_t*)dx, sdx,
                                      (bf16_t*)dz, sdz, part, pacc, M, D));
  } else if (fast && nbg) {
    NCH_SWITCH(D, hipLaunchKernelGGL((gated_rmsnorm_bwd_bf16_k<NCH, true>), dim3(g), dim3(256), lds, st,
                                     (const bf16_t*)dy, (const bf16_t*)x, sx, (const bf16_t*)z, sz, w, rstd,
                                     (bf16_t*)dx, sdx, (bf16_t*)dz, sdz, part, pacc, M, D, G));
  } else if (fast) {
    NCH_SWITCH(D, hipLaunchKernelGGL((gated_rmsnorm_bwd_bf16_k<NCH, false>), dim3(g), dim3(256), lds, st,
                                     (const bf16_t*)dy, (const bf16_t*)x, sx, (const bf16_t*)z, sz, w, rstd,
                                     (bf16_t*)dx, sdx, (bf16_t*)dz, sdz, part, pacc, M, D, G));
  } else if (nbg) {
    NCH_SWITCH(D, hipLaunchKernelGGL((gated_rmsnorm_bwd_k<NCH, true>), dim3(g), dim3(256), lds, st, dy, ydt, x,
                                     xdt, sx, z, zdt, sz, w, rstd, dx, sdx, dz, sdz, part, pacc, M, D, G));
  } else {
    NCH_SWITCH(D, hipLaunchKernelGGL((gated_rmsnorm_bwd_k<NCH, false>), dim3(g), dim3(256), lds, st, dy, ydt, x,
                                     xdt, sx, z, zdt, sz, w, rstd, dx, sdx, dz, sdz, part, pacc, M, D, G));
  }
  MAMBA_HIP_CHECK(hipGetLastError());
  return dw ? launch_colsum(part, g, D, dw, st) : hipSuccess;
}

int norm_bwd_partial_rows(int64_t M) { return bwd_grid(M); }

}  // namespace mamba_amd
