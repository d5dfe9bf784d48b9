// Causal depthwise conv1d (+ optional SiLU), both memory layouts, for gfx950.
//   out[b,c,t] = act(bias_c + sum_{k<W} w[c,k] * x[b,c,t-(W-1)+k])      (zero left padding)
// Reference semantics: causal-conv1d.
//
// Channel-first (Mamba-1; x is (b, d, l) with unit time stride):
//   one wavefront per (b, d) row walks time in 512-step chunks; lane i owns 8 consecutive steps
//   (one 16-B bf16 load).  The W-1 halo comes from lane i-1 by __shfl_up; lane 0 takes it from the
//   previous chunk's lane 63 (carried in registers) — every x element is read from HBM once.
//   Backward walks the chunks in reverse and carries the next chunk's first W-1 dpre values the
//   same way; dw/db are wave-reduced per row and summed over the batch in a second, fixed-order
//   pass (deterministic; no float atomics).  Rows are numbered in the input's memory order (cf_row), so the waves
//   running together stream neighbouring rows.
// Channel-last (Mamba-2; xBC is a column slice of the token-major in_proj output):
//   lane = 8 consecutive channels (16-B), a wave = 512 channels of one time tile, each lane slides
//   a W-row register window down its T_TILE timesteps.  dw/db: per-lane registers -> the block's
//   4 waves (4 time tiles) summed through LDS -> one partial row per block -> fixed-order sum.
#include "common.h"
#include "launchers.h"
#include <cstdlib>
#include <type_traits>

namespace mamba_amd {

template <typename T> struct Vec8 {
  static __device__ __forceinline__ void load(const T* p, float (&o)[8]);
  static __device__ __forceinline__ void store(T* p, const float (&o)[8]);
};
template <> struct Vec8<bf16_t> {
  static __device__ __forceinline__ void load(const bf16_t* p, float (&o)[8]) { ld8bf(p, o); }
  static __device__ __forceinline__ void store(bf16_t* p, const float (&o)[8]) { st8bf(p, o); }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&o)[8]) {
    float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&o)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(o[0], o[1], o[2], o[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
};

// load 8 consecutive elements starting at p (index t0..t0+7 of a row of length L), zero beyond L
template <typename T, bool VEC>
__device__ __forceinline__ void load_run(const T* p, int t0, int L, float (&o)[8]) {
  if (VEC && t0 + 8 <= L) {
    Vec8<T>::load(p, o);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (t0 + j < L) ? ld(p + j) : 0.f;
  }
}
template <typename T, bool VEC>
__device__ __forceinline__ void store_run(T* p, int t0, int L, const float (&o)[8]) {
  if (VEC && t0 + 8 <= L) {
    Vec8<T>::store(p, o);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (t0 + j < L) st(p + j, o[j]);
  }
}

__device__ __forceinline__ float act_fwd(float a, bool silu) { return silu ? siluf_(a) : a; }
__device__ __forceinline__ float act_bwd(float a, float g, bool silu) {
  if (!silu) return g;
  const float s = sigmoidf_(a);
  return g * s * (1.f + a * (1.f - s));
}

// 8 consecutive elements of a VEC row (wholly inside or wholly past L) as raw 16-B pieces, unpacked at use:
// half the registers of the fp32 form for bf16 while the load is in flight
template <typename T> struct Raw8 {
  static constexpr int NV = sizeof(T) / 2;
  uint4 v[NV];
  __device__ __forceinline__ void load(const T* p) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = reinterpret_cast<const uint4*>(p)[i];
  }
  __device__ __forceinline__ void unpack(float (&o)[8], bool valid) const {
    if constexpr (sizeof(T) == 2) {
      const uint32_t u[4] = {v[0].x, v[0].y, v[0].z, v[0].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o[2 * i] = __uint_as_float(u[i] << 16);
        o[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        o[4 * i] = __uint_as_float(v[i].x); o[4 * i + 1] = __uint_as_float(v[i].y);
        o[4 * i + 2] = __uint_as_float(v[i].z); o[4 * i + 3] = __uint_as_float(v[i].w);
      }
    }
    if (!valid) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = 0.f;
    }
  }
};

// =========================== channel-first ===============================================
// A wave walks its row in PAIRS of 512-step chunks whose loads are all issued before the first is used: with one
// 1-KB load per wave in flight the kernels ran at ~3.9 TB/s (bytes in flight per CU, not HBM, set the rate).

// (b, d) of row r: rows are numbered in memory order, b fastest when the batch stride is the smaller one (Mamba-1's
// (d, b, l) buffers), so neighbouring waves read neighbouring 2-KB rows instead of rows a whole (b, l) plane apart
__device__ __forceinline__ void cf_row(int64_t r, int Bn, int Dn, bool binner, int& b, int& d) {
  if (binner) { b = (int)(r % Bn); d = (int)(r / Bn); }
  else { b = (int)(r / Dn); d = (int)(r % Dn); }
}

// one 512-step chunk of the forward: cur = x[t0 .. t0 + 7] of this lane; carry = lane 0's halo, advanced to this
// chunk's last W-1 steps for the next chunk
template <typename T, int W, bool VEC>
__device__ __forceinline__ void cf_fwd_chunk(const float (&cur)[8], int t0, const float (&wk)[W], float bs,
                                             float (&carry)[3], T* orow, int L, bool silu, int lane) {
  float prev[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float v = __shfl_up(cur[5 + j], 1, 64);
    prev[j] = lane == 0 ? carry[j] : v;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) carry[j] = __shfl(cur[5 + j], 63, 64);
  float win[11];
#pragma unroll
  for (int j = 0; j < 3; ++j) win[j] = prev[j];
#pragma unroll
  for (int j = 0; j < 8; ++j) win[3 + j] = cur[j];
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = bs;
#pragma unroll
    for (int k = 0; k < W; ++k) a += wk[k] * win[3 + j - (W - 1) + k];
    o[j] = act_fwd(a, silu);
  }
  if (t0 < L) store_run<T, VEC>(orow + t0, t0, L, o);
}

// one chunk of the backward: cur / g its x and dout, halo = x[t0-3 .. t0-1] for lane 0; nextd = dpre of the 3 steps
// after the chunk (lane 63's), advanced to this chunk's first 3
template <typename T, int W, bool VEC>
__device__ __forceinline__ void cf_bwd_chunk(const float (&cur)[8], const float (&g)[8], const float (&halo)[3], int t0,
                                             const float (&wk)[W], float bs, float (&nextd)[3], float (&accw)[W],
                                             float& accb, T* dxr, int L, bool silu, int lane) {
  float prev[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float v = __shfl_up(cur[5 + j], 1, 64);
    prev[j] = lane == 0 ? halo[j] : v;
  }
  float win[11];
#pragma unroll
  for (int j = 0; j < 3; ++j) win[j] = prev[j];
#pragma unroll
  for (int j = 0; j < 8; ++j) win[3 + j] = cur[j];
  float dp[11];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = bs;
#pragma unroll
    for (int k = 0; k < W; ++k) a += wk[k] * win[3 + j - (W - 1) + k];
    dp[j] = (t0 + j < L) ? act_bwd(a, g[j], silu) : 0.f;
  }
  // dpre of the next 3 steps: from lane+1, lane 63 from the carried next chunk
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float v = __shfl_down(dp[j], 1, 64);
    dp[8 + j] = lane == 63 ? nextd[j] : v;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) nextd[j] = __shfl(dp[j], 0, 64);
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < W; ++k) s += wk[k] * dp[j + (W - 1) - k];
    o[j] = s;
#pragma unroll
    for (int k = 0; k < W; ++k) accw[k] += dp[j] * win[3 + j - (W - 1) + k];
    accb += dp[j];
  }
  if (t0 < L) store_run<T, VEC>(dxr + t0, t0, L, o);
}

// the loads of one backward chunk pair (VEC rows): x / dout of the lo (tl) and hi (tl + 512) chunks, clamped to legal
// runs and kept packed, and lane 0's halo of the lo chunk
template <typename T> struct CfBwdPair {
  Raw8<T> xl, gl, xh, gh;
  float hl[3];
  __device__ __forceinline__ void load(const T* xr, const T* gr, int tl, int L, int lane) {
    xl.load(xr + min(tl, L - 8));
    gl.load(gr + min(tl, L - 8));
    xh.load(xr + min(tl + 512, L - 8));
    gh.load(gr + min(tl + 512, L - 8));
#pragma unroll
    for (int j = 0; j < 3; ++j) hl[j] = 0.f;
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j) hl[j] = (tl - 3 + j >= 0) ? ld(xr + tl - 3 + j) : 0.f;
    }
  }
  // hi chunk first (reverse time), its halo is the lo chunk's last lane
  template <int W>
  __device__ __forceinline__ void run(int p0, const float (&wk)[W], float bs, float (&nextd)[3], float (&accw)[W],
                                      float& accb, T* dxr, int L, bool silu, int lane) const {
    const int tl = p0 + lane * 8, th = tl + 512;
    float x0[8], g0[8], hh[3];
    xl.unpack(x0, tl < L);
#pragma unroll
    for (int j = 0; j < 3; ++j) hh[j] = __shfl(x0[5 + j], 63, 64);
    if (p0 + 512 < L) {
      float x1[8], g1[8];
      xh.unpack(x1, th < L);
      gh.unpack(g1, th < L);
      cf_bwd_chunk<T, W, true>(x1, g1, hh, th, wk, bs, nextd, accw, accb, dxr, L, silu, lane);
    }
    gl.unpack(g0, tl < L);
    cf_bwd_chunk<T, W, true>(x0, g0, hl, tl, wk, bs, nextd, accw, accb, dxr, L, silu, lane);
  }
};

template <typename T, int W, bool VEC>
__global__ __launch_bounds__(256) void conv_cf_fwd_k(const T* __restrict__ x, int64_t sxb, int64_t sxd,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     T* __restrict__ out, int64_t sob, int64_t sod, int Bn, int Dn,
                                                     int L, bool silu, bool binner) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)Bn * Dn) return;  // whole wave exits together
  int b, d;
  cf_row(row, Bn, Dn, binner, b, d);
  const T* xr = x + b * sxb + d * sxd;
  T* orow = out + b * sob + d * sod;
  float wk[W];
#pragma unroll
  for (int k = 0; k < W; ++k) wk[k] = w[d * W + k];
  const float bs = bias ? bias[d] : 0.f;
  float carry[3] = {0.f, 0.f, 0.f};  // x[t0-3..t0-1] for lane 0 of the current chunk
  for (int c0 = 0; c0 < L; c0 += 1024) {
    const int ta = c0 + lane * 8, tb = ta + 512;
    float ca[8], cb[8];
    if constexpr (VEC) {  // both loads in flight (clamped to a legal run), unpacked at use
      Raw8<T> ra, rb;
      ra.load(xr + min(ta, L - 8));
      rb.load(xr + min(tb, L - 8));
      ra.unpack(ca, ta < L);
      cf_fwd_chunk<T, W, VEC>(ca, ta, wk, bs, carry, orow, L, silu, lane);
      if (c0 + 512 < L) {
        rb.unpack(cb, tb < L);
        cf_fwd_chunk<T, W, VEC>(cb, tb, wk, bs, carry, orow, L, silu, lane);
      }
    } else {
      load_run<T, VEC>(xr + ta, ta, L, ca);
      load_run<T, VEC>(xr + tb, tb, L, cb);
      cf_fwd_chunk<T, W, VEC>(ca, ta, wk, bs, carry, orow, L, silu, lane);
      if (c0 + 512 < L) cf_fwd_chunk<T, W, VEC>(cb, tb, wk, bs, carry, orow, L, silu, lane);
    }
  }
}

template <typename T, int W, bool VEC>
__global__ __launch_bounds__(256) void conv_cf_bwd_k(const T* __restrict__ x, int64_t sxb, int64_t sxd,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     const T* __restrict__ dout, int64_t sgb, int64_t sgd,
                                                     T* __restrict__ dx, int64_t sdb, int64_t sdd,
                                                     float* __restrict__ part, bool pacc, int Bn, int Dn, int L, bool silu,
                                                     bool binner) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)Bn * Dn) return;
  int b, d;
  cf_row(row, Bn, Dn, binner, b, d);
  const T* xr = x + b * sxb + d * sxd;
  const T* gr = dout + b * sgb + d * sgd;
  T* dxr = dx + b * sdb + d * sdd;
  float wk[W];
#pragma unroll
  for (int k = 0; k < W; ++k) wk[k] = w[d * W + k];
  const float bs = bias ? bias[d] : 0.f;
  float accw[W], accb = 0.f;
#pragma unroll
  for (int k = 0; k < W; ++k) accw[k] = 0.f;
  float nextd[3] = {0.f, 0.f, 0.f};  // dpre[t_end .. t_end+2] of the chunk after this one
  // pairs of chunks from the last: (lo, hi) = chunks (2p, 2p + 1); every load of the pair, and lane 0's halo of
  // the lo chunk, issued first; the hi chunk's halo is the lo chunk's last lane
  const int npairs = (L + 1023) / 1024;
  for (int pi = npairs - 1; pi >= 0; --pi) {
    const int tl = pi * 1024 + lane * 8, th = tl + 512;
    if constexpr (VEC) {  // the four loads in flight, unpacked at use
      CfBwdPair<T> pr;
      pr.load(xr, gr, tl, L, lane);
      pr.template run<W>(pi * 1024, wk, bs, nextd, accw, accb, dxr, L, silu, lane);
    } else {
      float xl[8], gl[8], xh[8], gh[8], hl[3] = {0.f, 0.f, 0.f}, hh[3];
      load_run<T, VEC>(xr + tl, tl, L, xl);
      load_run<T, VEC>(gr + tl, tl, L, gl);
      load_run<T, VEC>(xr + th, th, L, xh);
      load_run<T, VEC>(gr + th, th, L, gh);
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < 3; ++j) hl[j] = (tl - 3 + j >= 0) ? ld(xr + tl - 3 + j) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) hh[j] = __shfl(xl[5 + j], 63, 64);
      if (pi * 1024 + 512 < L) cf_bwd_chunk<T, W, VEC>(xh, gh, hh, th, wk, bs, nextd, accw, accb, dxr, L, silu, lane);
      cf_bwd_chunk<T, W, VEC>(xl, gl, hl, tl, wk, bs, nextd, accw, accb, dxr, L, silu, lane);
    }
  }
#pragma unroll
  for (int k = 0; k < W; ++k) accw[k] = wave_sum(accw[k]);
  accb = wave_sum(accb);
  if (lane == 0) {
    float* pr = part + ((int64_t)b * Dn + d) * (W + 1);
#pragma unroll
    for (int k = 0; k < W; ++k) pr[k] = pacc ? pr[k] + accw[k] : accw[k];
    pr[W] = pacc ? pr[W] + accb : accb;
  }
}

// =========================== channel-last ================================================
constexpr int CL_T = 16;  // timesteps per wave tile

template <typename T, int W, bool VEC>
__global__ __launch_bounds__(256) void conv_cl_fwd_k(const T* __restrict__ x, int64_t sxb, int64_t sxl,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     T* __restrict__ out, int64_t sob, int64_t sol, int Bn, int L,
                                                     int C, bool silu) {
  // grid: x = channel groups of 512, y = time tiles (4 per block), z = batch
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 8;
  const int t0 = (blockIdx.y * 4 + wave) * CL_T;
  const int b = blockIdx.z;
  if (c >= C || t0 >= L) return;
  const int nc = min(8, C - c);
  float wk[W][8], bs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int cc = j < nc ? c + j : c;
#pragma unroll
    for (int k = 0; k < W; ++k) wk[k][j] = w[cc * W + k];
    bs[j] = bias ? bias[cc] : 0.f;
  }
  const T* xb = x + b * sxb + c;
  T* ob = out + b * sob + c;
  auto loadrow = [&](int t, float (&o)[8]) {
    if (t < 0 || t >= L) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = 0.f;
    } else if (VEC && nc == 8) {
      Vec8<T>::load(xb + t * sxl, o);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = j < nc ? ld(xb + t * sxl + j) : 0.f;
    }
  };
  float win[W][8];
#pragma unroll
  for (int k = 0; k < W - 1; ++k) loadrow(t0 - (W - 1) + k, win[k]);
  for (int t = t0; t < min(t0 + CL_T, L); ++t) {
    loadrow(t, win[W - 1]);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = bs[j];
#pragma unroll
      for (int k = 0; k < W; ++k) a += wk[k][j] * win[k][j];
      o[j] = act_fwd(a, silu);
    }
    if (VEC && nc == 8) {
      Vec8<T>::store(ob + t * sol, o);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < nc) st(ob + t * sol + j, o[j]);
    }
#pragma unroll
    for (int k = 0; k < W - 1; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) win[k][j] = win[k + 1][j];
  }
}

constexpr int CLB_T = 32;  // backward time tile per wave

template <typename T, int W, bool VEC>
__global__ __launch_bounds__(256) void conv_cl_bwd_k(const T* __restrict__ x, int64_t sxb, int64_t sxl,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     const T* __restrict__ dout, int64_t sgb, int64_t sgl,
                                                     T* __restrict__ dx, int64_t sdb, int64_t sdl,
                                                     float* __restrict__ part, bool pacc, int Bn, int L, int C, bool silu) {
  __shared__ float red[4][64 * 8 * (W + 1)];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 8;
  const int t0 = (blockIdx.y * 4 + wave) * CLB_T;
  const int b = blockIdx.z;
  float acc[W + 1][8];
#pragma unroll
  for (int k = 0; k < W + 1; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  if (c < C && t0 < L) {
    const int nc = min(8, C - c);
    float wk[W][8], bs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int cc = j < nc ? c + j : c;
#pragma unroll
      for (int k = 0; k < W; ++k) wk[k][j] = w[cc * W + k];
      bs[j] = bias ? bias[cc] : 0.f;
    }
    const T* xb = x + b * sxb + c;
    const T* gb = dout + b * sgb + c;
    T* db_ = dx + b * sdb + c;
    auto loadv = [&](const T* base, int64_t stride, int t, float (&o)[8]) {
      if (t < 0 || t >= L) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = 0.f;
      } else if (VEC && nc == 8) {
        Vec8<T>::load(base + t * stride, o);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = j < nc ? ld(base + t * stride + j) : 0.f;
      }
    };
    float xw[W][8];   // x[t-W+1 .. t]
    float dpw[W][8];  // dpre[t-W+1 .. t]
#pragma unroll
    for (int k = 0; k < W - 1; ++k) {
      loadv(xb, sxl, t0 - (W - 1) + k, xw[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) dpw[k][j] = 0.f;
    }
    const int tend = min(t0 + CLB_T, L);
    for (int t = t0; t < tend + W - 1; ++t) {
      loadv(xb, sxl, t, xw[W - 1]);
      float g[8];
      loadv(gb, sgl, t, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = bs[j];
#pragma unroll
        for (int k = 0; k < W; ++k) a += wk[k][j] * xw[k][j];
        dpw[W - 1][j] = (t < L) ? act_bwd(a, g[j], silu) : 0.f;
      }
      if (t < tend) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
          for (int k = 0; k < W; ++k) acc[k][j] += dpw[W - 1][j] * xw[k][j];
          acc[W][j] += dpw[W - 1][j];
        }
      }
      const int s = t - (W - 1);
      if (s >= t0) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = 0.f;
#pragma unroll
          for (int k = 0; k < W; ++k) v += wk[k][j] * dpw[W - 1 - k][j];
          o[j] = v;
        }
        if (VEC && nc == 8) {
          Vec8<T>::store(db_ + s * sdl, o);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < nc) st(db_ + s * sdl + j, o[j]);
        }
      }
#pragma unroll
      for (int k = 0; k < W - 1; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xw[k][j] = xw[k + 1][j];
          dpw[k][j] = dpw[k + 1][j];
        }
    }
  }
  // block reduction over the 4 time tiles, then one partial row per block
#pragma unroll
  for (int k = 0; k < W + 1; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wave][(lane * 8 + j) * (W + 1) + k] = acc[k][j];
  __syncthreads();
  const int64_t prow = (int64_t)blockIdx.z * gridDim.y + blockIdx.y;
  for (int i = threadIdx.x; i < 64 * 8 * (W + 1); i += 256) {
    const int ch = blockIdx.x * 512 + i / (W + 1);
    if (ch < C) {
      float* pp = part + prow * (int64_t)C * (W + 1) + (int64_t)ch * (W + 1) + i % (W + 1);
      const float v = red[0][i] + red[1][i] + red[2][i] + red[3][i];
      *pp = pacc ? *pp + v : v;  // pacc: accumulate across micro-steps (reduced once per optimizer step)
    }
  }
}

// ---- bf16 fast path (16-B aligned rows, C % 8 == 0): the headline Mamba-2 shape -------------------
// Same math as conv_cl_bwd_k, restructured for CDNA4 issue:
//  * the W-row windows of x and dpre are register RINGS whose slots are compile-time indices of the
//    W-step unrolled loop body, so advancing the window costs no moves;
//  * each group of W steps issues its 2W 16-B row loads up front (kept packed as bf16 until used),
//    so a wave waits for memory once per group instead of once per step;
//  * channel pairs run on packed FP32 (v_pk_fma_f32 / v_pk_mul_f32).
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void unpack8(const uint4 v, f2v (&o)[4]) {
  const unsigned u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = f2v{__uint_as_float(u[q] << 16), __uint_as_float(u[q] & 0xffff0000u)};
}
// CV channels of one row as CV/2 packed pairs: CV = 8 -> one 16-B load, CV = 4 -> one 8-B load
template <int CV> struct RowV;
template <> struct RowV<8> {
  uint4 v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void zero() { v = make_uint4(0, 0, 0, 0); }
  __device__ __forceinline__ void unpack(f2v (&o)[4]) const { unpack8(v, o); }
};
template <> struct RowV<4> {
  uint2 v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const uint2*>(p); }
  __device__ __forceinline__ void zero() { v = make_uint2(0, 0); }
  __device__ __forceinline__ void unpack(f2v (&o)[2]) const {
    o[0] = f2v{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u)};
    o[1] = f2v{__uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u)};
  }
};
__device__ __forceinline__ unsigned pack2(const f2v v) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf2v));
}
__device__ __forceinline__ uint4 pack8(const f2v (&o)[4]) {
  return make_uint4(pack2(o[0]), pack2(o[1]), pack2(o[2]), pack2(o[3]));
}
__device__ __forceinline__ void store_row(bf16_t* p, const f2v (&o)[4]) { *reinterpret_cast<uint4*>(p) = pack8(o); }
__device__ __forceinline__ void store_row(bf16_t* p, const f2v (&o)[2]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2(o[0]), pack2(o[1]));
}

// CV = channels per lane (8: 16-B rows, 4: 8-B rows -- half the registers, twice the waves in flight and
// no idle lanes when C % 512 != 0, e.g. the 280M conv width 1792)
template <int W, int TT, int CV, bool SILU>
__global__ __launch_bounds__(256) void conv_cl_fwd_bf16_k(const bf16_t* __restrict__ x, int64_t sxb, int64_t sxl,
                                                          const float* __restrict__ w, const float* __restrict__ bias,
                                                          bf16_t* __restrict__ out, int64_t sob, int64_t sol, int L,
                                                          int C) {
  constexpr int NQ = CV / 2;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: row guards are scalar branches
  const int c = (blockIdx.x * 64 + lane) * CV;
  const int t0 = (blockIdx.y * 4 + wave) * TT;
  const int b = blockIdx.z;
  if (c >= C || t0 >= L) return;
  f2v wk[W][NQ], bs[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
#pragma unroll
    for (int k = 0; k < W; ++k) wk[k][q] = f2v{w[(c + 2 * q) * W + k], w[(c + 2 * q + 1) * W + k]};
    bs[q] = bias ? f2v{bias[c + 2 * q], bias[c + 2 * q + 1]} : f2v{0.f, 0.f};
  }
  const bf16_t* xb = x + b * sxb + c;
  bf16_t* ob = out + b * sob + c;
  const int tend = min(t0 + TT, L);
  auto ldrow = [&](int t) {
    RowV<CV> r;
    if (t >= 0 && t < tend) r.load(xb + t * sxl);
    else r.zero();
    return r;
  };
  f2v xr[W][NQ];
#pragma unroll
  for (int k = 0; k < W - 1; ++k) ldrow(t0 - (W - 1) + k).unpack(xr[k]);
  const int nsteps = tend - t0;
  // each group of W rows is requested one group ahead (two groups of loads in flight per wave)
  RowV<CV> rx[W];
#pragma unroll
  for (int u = 0; u < W; ++u) rx[u] = ldrow(t0 + u);
  for (int i0 = 0; i0 < nsteps; i0 += W) {
    RowV<CV> nx[W];
#pragma unroll
    for (int u = 0; u < W; ++u) nx[u] = ldrow(t0 + i0 + W + u);
#pragma unroll
    for (int u = 0; u < W; ++u) {
      const int i = i0 + u;
      if (i < nsteps) {
        const int sl = (u + W - 1) % W;
        rx[u].unpack(xr[sl]);
        f2v o[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          f2v a = bs[q];
#pragma unroll
          for (int k = 0; k < W; ++k) a += wk[k][q] * xr[(u + k) % W][q];
          if (SILU) a = a * f2v{sigmoidf_(a.x), sigmoidf_(a.y)};
          o[q] = a;
        }
        store_row(ob + (t0 + i) * sol, o);
      }
    }
#pragma unroll
    for (int u = 0; u < W; ++u) rx[u] = nx[u];
  }
}

template <int W, int TT, int CV, bool SILU>
__global__ __launch_bounds__(256) void conv_cl_bwd_bf16_k(const bf16_t* __restrict__ x, int64_t sxb, int64_t sxl,
                                                          const float* __restrict__ w, const float* __restrict__ bias,
                                                          const bf16_t* __restrict__ dout, int64_t sgb, int64_t sgl,
                                                          bf16_t* __restrict__ dx, int64_t sdb, int64_t sdl,
                                                          float* __restrict__ part, bool pacc, int L, int C) {
  constexpr int NQ = CV / 2;
  __shared__ float red[4][64 * CV * (W + 1)];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: row guards are scalar branches
  const int c = (blockIdx.x * 64 + lane) * CV;
  const int t0 = (blockIdx.y * 4 + wave) * TT;
  const int b = blockIdx.z;
  f2v acc[W + 1][NQ];
#pragma unroll
  for (int k = 0; k < W + 1; ++k)
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[k][q] = f2v{0.f, 0.f};
  if (c < C && t0 < L) {
    f2v wk[W][NQ], bs[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
#pragma unroll
      for (int k = 0; k < W; ++k) wk[k][q] = f2v{w[(c + 2 * q) * W + k], w[(c + 2 * q + 1) * W + k]};
      bs[q] = bias ? f2v{bias[c + 2 * q], bias[c + 2 * q + 1]} : f2v{0.f, 0.f};
    }
    const bf16_t* xb = x + b * sxb + c;
    const bf16_t* gb = dout + b * sgb + c;
    bf16_t* db_ = dx + b * sdb + c;
    const int tend = min(t0 + TT, L);
    const int nsteps = tend + W - 1 - t0;  // main steps t = t0 .. t0+nsteps-1
    const int tlim = min(L, t0 + nsteps);
    auto ldrow = [&](const bf16_t* base, int64_t stride, int t) {
      RowV<CV> r;
      if (t >= 0 && t < tlim) r.load(base + t * stride);
      else r.zero();
      return r;
    };
    f2v xr[W][NQ], dp[W][NQ];
#pragma unroll
    for (int k = 0; k < W; ++k) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) dp[k][q] = f2v{0.f, 0.f};
      if (k < W - 1) ldrow(xb, sxl, t0 - (W - 1) + k).unpack(xr[k]);
    }
    // each group of W rows of x and dout is requested one group ahead (two groups in flight per wave)
    RowV<CV> rx[W], rg[W];
#pragma unroll
    for (int u = 0; u < W; ++u) {
      rx[u] = ldrow(xb, sxl, t0 + u);
      rg[u] = ldrow(gb, sgl, t0 + u);
    }
    for (int i0 = 0; i0 < nsteps; i0 += W) {
      RowV<CV> nx[W], ng[W];
#pragma unroll
      for (int u = 0; u < W; ++u) {
        nx[u] = ldrow(xb, sxl, t0 + i0 + W + u);
        ng[u] = ldrow(gb, sgl, t0 + i0 + W + u);
      }
#pragma unroll
      for (int u = 0; u < W; ++u) {
        const int i = i0 + u, t = t0 + i;
        if (i < nsteps) {
          const int sl = (u + W - 1) % W;  // slot of step t (compile-time after unrolling)
          rx[u].unpack(xr[sl]);
          f2v g[NQ];
          rg[u].unpack(g);
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            f2v a = bs[q];
#pragma unroll
            for (int k = 0; k < W; ++k) a += wk[k][q] * xr[(u + k) % W][q];
            f2v d = g[q];
            if (SILU) {
              const float s0 = sigmoidf_(a.x), s1 = sigmoidf_(a.y);
              const f2v sv = f2v{s0, s1};
              d = g[q] * sv * (1.f + a * (1.f - sv));
            }
            dp[sl][q] = (t < L) ? d : f2v{0.f, 0.f};
          }
          if (t < tend) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
#pragma unroll
              for (int k = 0; k < W; ++k) acc[k][q] += dp[sl][q] * xr[(u + k) % W][q];
              acc[W][q] += dp[sl][q];
            }
          }
          if (i >= W - 1) {  // dx[s], s = t-(W-1) >= t0
            f2v o[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
              f2v v = f2v{0.f, 0.f};
#pragma unroll
              for (int m = 0; m < W; ++m) v += wk[W - 1 - m][q] * dp[(u + m) % W][q];
              o[q] = v;
            }
            store_row(db_ + (t - (W - 1)) * sdl, o);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < W; ++u) {
        rx[u] = nx[u];
        rg[u] = ng[u];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < W + 1; ++k)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      red[wave][(lane * CV + 2 * q) * (W + 1) + k] = acc[k][q].x;
      red[wave][(lane * CV + 2 * q + 1) * (W + 1) + k] = acc[k][q].y;
    }
  __syncthreads();
  const int64_t prow = (int64_t)blockIdx.z * gridDim.y + blockIdx.y;
  for (int i = threadIdx.x; i < 64 * CV * (W + 1); i += 256) {
    const int ch = blockIdx.x * 64 * CV + i / (W + 1);
    if (ch < C) {
      float* pp = part + prow * (int64_t)C * (W + 1) + (int64_t)ch * (W + 1) + i % (W + 1);
      const float v = red[0][i] + red[1][i] + red[2][i] + red[3][i];
      *pp = pacc ? *pp + v : v;  // pacc: accumulate across micro-steps (reduced once per optimizer step)
    }
  }
}

// =========================== varlen / state hand-off (channel-last) =========================
// causal-conv1d >= 1.4 interface: seq_idx (b, l) int32 -- a tap never reads a token of another
// sequence; initial_states (b, c, W-1) -- the inputs before t = 0; final_states (b, c, W-1) -- the last
// W-1 inputs (for decode or the next context-parallel shard).  Used only when one of them is given (the
// dense kernels above stay the hot path): thread = one channel, wave = CV_T steps, fp32 math.
constexpr int CV_T = 16;

template <typename T, int W>
struct VarIO {
  const T* x; int64_t sxb, sxl;
  const int* seq; int64_t sqb;
  const T* init; int64_t sib, sic;
  int b, c, L;
  __device__ __forceinline__ int sq(int t) const { return seq ? seq[b * sqb + t] : 0; }
  // input at time s as seen by an output of sequence sqt (s < 0: initial state slot W-1+s)
  __device__ __forceinline__ float in(int s, int sqt) const {
    // the initial states precede the first sequence of the row only
    if (s < 0) return init && (!seq || seq[b * sqb] == sqt) ? ld(init + b * sib + (int64_t)c * sic + (W - 1) + s) : 0.f;
    if (seq && seq[b * sqb + s] != sqt) return 0.f;
    return ld(x + b * sxb + (int64_t)s * sxl + c);
  }
};

template <typename T, int W>
__global__ __launch_bounds__(256) void conv_cl_fwd_var_k(VarIO<T, W> io, const float* __restrict__ w,
                                                         const float* __restrict__ bias, T* __restrict__ out,
                                                         int64_t sob, int64_t sol, T* __restrict__ fin, int64_t sfb,
                                                         int64_t sfc, int C, bool silu) {
  io.c = blockIdx.x * 64 + (threadIdx.x & 63);
  io.b = blockIdx.z;
  const int t0 = (blockIdx.y * 4 + (threadIdx.x >> 6)) * CV_T;
  if (io.c >= C) return;
  float wk[W];
#pragma unroll
  for (int k = 0; k < W; ++k) wk[k] = w[io.c * W + k];
  const float bs = bias ? bias[io.c] : 0.f;
  for (int t = t0; t < min(t0 + CV_T, io.L); ++t) {
    const int sqt = io.sq(t);
    float a = bs;
#pragma unroll
    for (int k = 0; k < W; ++k) a += wk[k] * io.in(t - (W - 1) + k, sqt);
    st(out + io.b * sob + (int64_t)t * sol + io.c, act_fwd(a, silu));
  }
  if (fin && t0 == 0) {  // the last W-1 inputs, initial states in front when L < W-1
#pragma unroll
    for (int j = 0; j < W - 1; ++j) {
      const int s = io.L - (W - 1) + j;
      const float v = s >= 0 ? ld(io.x + io.b * io.sxb + (int64_t)s * io.sxl + io.c) : io.in(s, io.sq(0));
      st(fin + io.b * sfb + (int64_t)io.c * sfc + j, v);
    }
  }
}

// dx, d(initial_states), per-block (W taps + bias) partial rows; dfin: gradient of final_states (or null)
template <typename T, int W>
__global__ __launch_bounds__(256) void conv_cl_bwd_var_k(VarIO<T, W> io, const float* __restrict__ w,
                                                         const float* __restrict__ bias, const T* __restrict__ g,
                                                         int64_t sgb, int64_t sgl, const T* __restrict__ dfin,
                                                         int64_t sdfb, int64_t sdfc, T* __restrict__ dx, int64_t sdb,
                                                         int64_t sdl, T* __restrict__ dinit, int64_t sdib,
                                                         int64_t sdic, float* __restrict__ part, bool pacc, int C,
                                                         bool silu) {
  __shared__ float red[4][64][W + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  io.c = blockIdx.x * 64 + lane;
  io.b = blockIdx.z;
  const int t0 = (blockIdx.y * 4 + wave) * CV_T;
  const bool on = io.c < C;
  float accw[W + 1];
#pragma unroll
  for (int k = 0; k < W + 1; ++k) accw[k] = 0.f;
  if (on) {
    float wk[W];
#pragma unroll
    for (int k = 0; k < W; ++k) wk[k] = w[io.c * W + k];
    const float bs = bias ? bias[io.c] : 0.f;
    // g'(t) = dout(t) act'(pre(t)) for the outputs this tile's inputs feed: t in [t0, t0 + CV_T + W - 1)
    auto gp = [&](int t) -> float {
      if (t < 0 || t >= io.L) return 0.f;
      const int sqt = io.sq(t);
      float a = bs;
#pragma unroll
      for (int k = 0; k < W; ++k) a += wk[k] * io.in(t - (W - 1) + k, sqt);
      return act_bwd(a, ld(g + io.b * sgb + (int64_t)t * sgl + io.c), silu);
    };
    float gw[CV_T + W - 1];
#pragma unroll
    for (int i = 0; i < CV_T + W - 1; ++i) gw[i] = gp(t0 + i);
    // weight / bias partials over this tile's outputs
#pragma unroll
    for (int i = 0; i < CV_T; ++i) {
      const int t = t0 + i;
      if (t < io.L) {
        const int sqt = io.sq(t);
#pragma unroll
        for (int k = 0; k < W; ++k) accw[k] += gw[i] * io.in(t - (W - 1) + k, sqt);
        accw[W] += gw[i];
      }
    }
    // dx(s) = sum_k w_k g'(s + W-1-k) [same sequence]  (+ d final_states for the last W-1 inputs)
    for (int i = 0; i < CV_T && t0 + i < io.L; ++i) {
      const int s = t0 + i, sqs = io.sq(s);
      float d = 0.f;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int t = s + (W - 1) - k;
        if (t < io.L && (!io.seq || io.sq(t) == sqs)) d += wk[k] * gw[i + (W - 1) - k];
      }
      const int j = s - (io.L - (W - 1));
      if (dfin && j >= 0) d += ld(dfin + io.b * sdfb + (int64_t)io.c * sdfc + j);
      st(dx + io.b * sdb + (int64_t)s * sdl + io.c, d);
    }
    if (dinit && t0 == 0) {  // initial-state slot j = W-1+s (s < 0) feeds output t = s + (W-1) - k
#pragma unroll
      for (int j = 0; j < W - 1; ++j) {
        const int s = j - (W - 1);
        float d = 0.f;
#pragma unroll
        for (int k = 0; k < W; ++k) {
          const int t = s + (W - 1) - k;
          if (t >= 0 && t < io.L && (!io.seq || io.sq(t) == io.sq(0))) d += wk[k] * gp(t);
        }
        const int jf = s - (io.L - (W - 1));  // final_states may reach back into the initial states
        if (dfin && jf >= 0) d += ld(dfin + io.b * sdfb + (int64_t)io.c * sdfc + jf);
        st(dinit + io.b * sdib + (int64_t)io.c * sdic + j, d);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < W + 1; ++k) red[wave][lane][k] = accw[k];
  __syncthreads();
  const int64_t prow = (int64_t)blockIdx.z * gridDim.y + blockIdx.y;
  for (int i = threadIdx.x; i < 64 * (W + 1); i += 256) {
    const int ch = blockIdx.x * 64 + i / (W + 1), k = i % (W + 1);
    if (ch < C) {
      float* pp = part + prow * (int64_t)C * (W + 1) + (int64_t)ch * (W + 1) + k;
      const float v = red[0][i / (W + 1)][k] + red[1][i / (W + 1)][k] + red[2][i / (W + 1)][k] + red[3][i / (W + 1)][k];
      *pp = pacc ? *pp + v : v;
    }
  }
}

// =========================== decode update ===============================================
template <typename T, int W>
__global__ void conv_update_k(const T* __restrict__ x, int64_t sxb, T* __restrict__ state, int64_t ssb,
                              int64_t ssc, const float* __restrict__ w, const float* __restrict__ bias,
                              T* __restrict__ out, int Bn, int C, int SL, bool silu) {
  // state (SL >= W-1 columns, oldest first; causal-conv1d >= 1.4 semantics): the output uses its last W-1
  // entries and x; afterwards the state holds the last SL inputs (shifted by one, x appended)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Bn * C) return;
  const int b = i / C, c = i % C;
  T* sp = state + b * ssb + c * ssc;
  const float xv = ld(x + b * sxb + c);
  float a = bias ? bias[c] : 0.f;
#pragma unroll
  for (int k = 0; k < W - 1; ++k) a += w[c * W + k] * ld(sp + SL - (W - 1) + k);
  a += w[c * W + W - 1] * xv;
  for (int k = 0; k + 1 < SL; ++k) st(sp + k, ld(sp + k + 1));
  if (SL > 0) st(sp + SL - 1, xv);
  st(out + (int64_t)b * C + c, act_fwd(a, silu));
}

// =========================== launchers ===================================================
#define W_SWITCH(Wv, ...)                                         \
  do {                                                            \
    if ((Wv) == 2) { constexpr int WW = 2; __VA_ARGS__; }         \
    else if ((Wv) == 3) { constexpr int WW = 3; __VA_ARGS__; }    \
    else if ((Wv) == 4) { constexpr int WW = 4; __VA_ARGS__; }    \
    else return hipErrorInvalidValue;                             \
  } while (0)

// row order of the channel-first kernels: 1 = memory order of the input (default), 0 = b-major;
// MAMBA_AMD_CONV_CF_ORDER sets the process default, set_conv_cf_order overrides it
static int g_cf_order = -1;
int conv_cf_order() {
  if (g_cf_order < 0) {
    const char* e = getenv("MAMBA_AMD_CONV_CF_ORDER");
    g_cf_order = (e && atoi(e) == 0) ? 0 : 1;
  }
  return g_cf_order;
}
void set_conv_cf_order(int v) { g_cf_order = v == 0 ? 0 : 1; }
static bool cf_batch_inner(int64_t sxb, int64_t sxd) { return conv_cf_order() != 0 && sxb < sxd; }

template <typename T>
static hipError_t cf_fwd(const T* x, int64_t sxb, int64_t sxd, const float* w, const float* bias, T* out,
                         int64_t sob, int64_t sod, int Bn, int Dn, int L, int Wd, bool silu, hipStream_t st) {
  const bool vec = (L % 8 == 0) && (sxb % 8 == 0) && (sxd % 8 == 0) && (sob % 8 == 0) && (sod % 8 == 0) &&
                   ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0);
  dim3 grid((unsigned)(((int64_t)Bn * Dn + 3) / 4)), block(256);
  const bool binner = cf_batch_inner(sxb, sxd);
  W_SWITCH(Wd, {
    if (vec) hipLaunchKernelGGL((conv_cf_fwd_k<T, WW, true>), grid, block, 0, st, x, sxb, sxd, w, bias, out, sob,
                                sod, Bn, Dn, L, silu, binner);
    else hipLaunchKernelGGL((conv_cf_fwd_k<T, WW, false>), grid, block, 0, st, x, sxb, sxd, w, bias, out, sob, sod,
                            Bn, Dn, L, silu, binner);
  });
  return hipGetLastError();
}

hipError_t launch_conv_cf_fwd(const void* x, int dt, int64_t sxb, int64_t sxd, const float* w, const float* bias,
                              void* out, int64_t sob, int64_t sod, int Bn, int Dn, int L, int Wd, bool silu,
                              hipStream_t st) {
  if (dt == kBF16)
    return cf_fwd<bf16_t>((const bf16_t*)x, sxb, sxd, w, bias, (bf16_t*)out, sob, sod, Bn, Dn, L, Wd, silu, st);
  if (dt == kF32)
    return cf_fwd<float>((const float*)x, sxb, sxd, w, bias, (float*)out, sob, sod, Bn, Dn, L, Wd, silu, st);
  return hipErrorInvalidValue;
}

template <typename T>
static hipError_t cf_bwd(const T* x, int64_t sxb, int64_t sxd, const float* w, const float* bias, const T* g,
                         int64_t sgb, int64_t sgd, T* dx, int64_t sdb, int64_t sdd, float* part, float* dw, float* db,
                         bool pacc, int Bn, int Dn, int L, int Wd, bool silu, hipStream_t st) {
  const bool vec = (L % 8 == 0) && (sxb % 8 == 0) && (sxd % 8 == 0) && (sgb % 8 == 0) && (sgd % 8 == 0) &&
                   (sdb % 8 == 0) && (sdd % 8 == 0) && ((uintptr_t)x % 16 == 0) && ((uintptr_t)g % 16 == 0) &&
                   ((uintptr_t)dx % 16 == 0);
  dim3 grid((unsigned)(((int64_t)Bn * Dn + 3) / 4)), block(256);
  const bool binner = cf_batch_inner(sxb, sxd);
  W_SWITCH(Wd, {
    if (vec) hipLaunchKernelGGL((conv_cf_bwd_k<T, WW, true>), grid, block, 0, st, x, sxb, sxd, w, bias, g, sgb, sgd,
                                dx, sdb, sdd, part, pacc, Bn, Dn, L, silu, binner);
    else hipLaunchKernelGGL((conv_cf_bwd_k<T, WW, false>), grid, block, 0, st, x, sxb, sxd, w, bias, g, sgb, sgd, dx,
                            sdb, sdd, part, pacc, Bn, Dn, L, silu, binner);
  });
  MAMBA_HIP_CHECK(hipGetLastError());
  return dw ? launch_colsum(part, Bn, Dn * (Wd + 1), dw, st) : hipSuccess;  // dw buffer holds (D, W+1): [w taps | bias]
}

hipError_t launch_conv_cf_bwd(const void* x, int dt, int64_t sxb, int64_t sxd, const float* w, const float* bias,
                              const void* g, int64_t sgb, int64_t sgd, void* dx, int64_t sdb, int64_t sdd,
                              float* part, float* dw, float* db, bool pacc, int Bn, int Dn, int L, int Wd, bool silu,
                              hipStream_t st) {
  if (dt == kBF16)
    return cf_bwd<bf16_t>((const bf16_t*)x, sxb, sxd, w, bias, (const bf16_t*)g, sgb, sgd, (bf16_t*)dx, sdb, sdd,
                          part, dw, db, pacc, Bn, Dn, L, Wd, silu, st);
  if (dt == kF32)
    return cf_bwd<float>((const float*)x, sxb, sxd, w, bias, (const float*)g, sgb, sgd, (float*)dx, sdb, sdd, part,
                         dw, db, pacc, Bn, Dn, L, Wd, silu, st);
  return hipErrorInvalidValue;
}

// channels per lane of the bf16 channel-last kernels: 4 (8-B rows; measured faster than 8)
static int conv_cl_cv(int C) { return (C % 4 == 0) ? 4 : 8; }

template <typename T>
static hipError_t cl_fwd(const T* x, int64_t sxb, int64_t sxl, const float* w, const float* bias, T* out,
                         int64_t sob, int64_t sol, int Bn, int L, int C, int Wd, bool silu, hipStream_t st) {
  const bool vec = (C % 8 == 0) && (sxb % 8 == 0) && (sxl % 8 == 0) && (sob % 8 == 0) && (sol % 8 == 0) &&
                   ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0);
  if constexpr (std::is_same<T, bf16_t>::value) {
    if (vec) {
      constexpr int TF = 32;
      if (conv_cl_cv(C) == 4) {
        dim3 g2((C + 255) / 256, (L + 4 * TF - 1) / (4 * TF), Bn);
        if (silu) W_SWITCH(Wd, hipLaunchKernelGGL((conv_cl_fwd_bf16_k<WW, TF, 4, true>), g2, dim3(256), 0, st, x, sxb,
                                                  sxl, w, bias, out, sob, sol, L, C));
        else W_SWITCH(Wd, hipLaunchKernelGGL((conv_cl_fwd_bf16_k<WW, TF, 4, false>), g2, dim3(256), 0, st, x, sxb, sxl,
                                             w, bias, out, sob, sol, L, C));
      } else {
        dim3 g2((C + 511) / 512, (L + 4 * TF - 1) / (4 * TF), Bn);
        if (silu) W_SWITCH(Wd, hipLaunchKernelGGL((conv_cl_fwd_bf16_k<WW, TF, 8, true>), g2, dim3(256), 0, st, x, sxb,
                                                  sxl, w, bias, out, sob, sol, L, C));
        else W_SWITCH(Wd, hipLaunchKernelGGL((conv_cl_fwd_bf16_k<WW, TF, 8, false>), g2, dim3(256), 0, st, x, sxb, sxl,
                                             w, bias, out, sob, sol, L, C));
      }
      return hipGetLastError();
    }
  }
  dim3 grid((C + 511) / 512, (L + 4 * CL_T - 1) / (4 * CL_T), Bn), block(256);
  W_SWITCH(Wd, {
    if (vec) hipLaunchKernelGGL((conv_cl_fwd_k<T, WW, true>), grid, block, 0, st, x, sxb, sxl, w, bias, out, sob,
                                sol, Bn, L, C, silu);
    else hipLaunchKernelGGL((conv_cl_fwd_k<T, WW, false>), grid, block, 0, st, x, sxb, sxl, w, bias, out, sob, sol,
                            Bn, L, C, silu);
  });
  return hipGetLastError();
}

hipError_t launch_conv_cl_fwd(const void* x, int dt, int64_t sxb, int64_t sxl, const float* w, const float* bias,
                              void* out, int64_t sob, int64_t sol, int Bn, int L, int C, int Wd, bool silu,
                              hipStream_t st) {
  if (dt == kBF16)
    return cl_fwd<bf16_t>((const bf16_t*)x, sxb, sxl, w, bias, (bf16_t*)out, sob, sol, Bn, L, C, Wd, silu, st);
  if (dt == kF32)
    return cl_fwd<float>((const float*)x, sxb, sxl, w, bias, (float*)out, sob, sol, Bn, L, C, Wd, silu, st);
  return hipErrorInvalidValue;
}

int conv_cl_bwd_partial_rows(int Bn, int L) { return Bn * ((L + 4 * CLB_T - 1) / (4 * CLB_T)); }

template <typename T>
static hipError_t cl_bwd(const T* x, int64_t sxb, int64_t sxl, const float* w, const float* bias, const T* g,
                         int64_t sgb, int64_t sgl, T* dx, int64_t sdb, int64_t sdl, float* part, float* dw, float* db,
                         bool pacc, int Bn, int L, int C, int Wd, bool silu, hipStream_t st) {
  const bool vec = (C % 8 == 0) && (sxb % 8 == 0) && (sxl % 8 == 0) && (sgb % 8 == 0) && (sgl % 8 == 0) &&
                   (sdb % 8 == 0) && (sdl % 8 == 0) && ((uintptr_t)x % 16 == 0) && ((uintptr_t)g % 16 == 0) &&
                   ((uintptr_t)dx % 16 == 0);
  dim3 grid((C + 511) / 512, (L + 4 * CLB_T - 1) / (4 * CLB_T), Bn), block(256);
  if constexpr (std::is_same<T, bf16_t>::value) {
    if (vec) {
      if (conv_cl_cv(C) == 4) {
        dim3 g4((C + 255) / 256, grid.y, grid.z);
        if (silu) W_SWITCH(Wd, hipLaunchKernelGGL((conv_cl_bwd_bf16_k<WW, CLB_T, 4, true>), g4, block, 0, st, x, sxb,
                                                  sxl, w, bias, g, sgb, sgl, dx, sdb, sdl, part, pacc, L, C));
        else W_SWITCH(Wd, hipLaunchKernelGGL((conv_cl_bwd_bf16_k<WW, CLB_T, 4, false>), g4, block, 0, st, x, sxb, sxl,
                                             w, bias, g, sgb, sgl, dx, sdb, sdl, part, pacc, L, C));
      } else {
        if (silu) W_SWITCH(Wd, hipLaunchKernelGGL((conv_cl_bwd_bf16_k<WW, CLB_T, 8, true>), grid, block, 0, st, x, sxb,
                                                  sxl, w, bias, g, sgb, sgl, dx, sdb, sdl, part, pacc, L, C));
        else W_SWITCH(Wd, hipLaunchKernelGGL((conv_cl_bwd_bf16_k<WW, CLB_T, 8, false>), grid, block, 0, st, x, sxb,
                                             sxl, w, bias, g, sgb, sgl, dx, sdb, sdl, part, pacc, L, C));
      }
      MAMBA_HIP_CHECK(hipGetLastError());
      return dw ? launch_colsum(part, conv_cl_bwd_partial_rows(Bn, L), C * (Wd + 1), dw, st) : hipSuccess;
    }
  }
  W_SWITCH(Wd, {
    if (vec) hipLaunchKernelGGL((conv_cl_bwd_k<T, WW, true>), grid, block, 0, st, x, sxb, sxl, w, bias, g, sgb, sgl,
                                dx, sdb, sdl, part, pacc, Bn, L, C, silu);
    else hipLaunchKernelGGL((conv_cl_bwd_k<T, WW, false>), grid, block, 0, st, x, sxb, sxl, w, bias, g, sgb, sgl, dx,
                            sdb, sdl, part, pacc, Bn, L, C, silu);
  });
  MAMBA_HIP_CHECK(hipGetLastError());
  return dw ? launch_colsum(part, conv_cl_bwd_partial_rows(Bn, L), C * (Wd + 1), dw, st) : hipSuccess;  // (C, W+1)
}

hipError_t launch_conv_cl_bwd(const void* x, int dt, int64_t sxb, int64_t sxl, const float* w, const float* bias,
                              const void* g, int64_t sgb, int64_t sgl, void* dx, int64_t sdb, int64_t sdl,
                              float* part, float* dw, float* db, bool pacc, int Bn, int L, int C, int Wd, bool silu,
                              hipStream_t st) {
  if (dt == kBF16)
    return cl_bwd<bf16_t>((const bf16_t*)x, sxb, sxl, w, bias, (const bf16_t*)g, sgb, sgl, (bf16_t*)dx, sdb, sdl,
                          part, dw, db, pacc, Bn, L, C, Wd, silu, st);
  if (dt == kF32)
    return cl_bwd<float>((const float*)x, sxb, sxl, w, bias, (const float*)g, sgb, sgl, (float*)dx, sdb, sdl, part,
                         dw, db, pacc, Bn, L, C, Wd, silu, st);
  return hipErrorInvalidValue;
}

hipError_t launch_conv_update(const void* x, int dt, int64_t sxb, void* state, int64_t ssb, int64_t ssc,
                              const float* w, const float* bias, void* out, int Bn, int C, int Wd, int SL, bool silu,
                              hipStream_t st) {
  if (SL < Wd - 1) return hipErrorInvalidValue;
  const int n = Bn * C;
  dim3 grid((n + 255) / 256), block(256);
  if (dt == kBF16) {
    W_SWITCH(Wd, hipLaunchKernelGGL((conv_update_k<bf16_t, WW>), grid, block, 0, st, (const bf16_t*)x, sxb,
                                    (bf16_t*)state, ssb, ssc, w, bias, (bf16_t*)out, Bn, C, SL, silu));
  } else if (dt == kF32) {
    W_SWITCH(Wd, hipLaunchKernelGGL((conv_update_k<float, WW>), grid, block, 0, st, (const float*)x, sxb,
                                    (float*)state, ssb, ssc, w, bias, (float*)out, Bn, C, SL, silu));
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

int conv_cl_var_partial_rows(int Bn, int L) { return Bn * ((L + 4 * CV_T - 1) / (4 * CV_T)); }

template <typename T>
static hipError_t cl_var(const T* x, int64_t sxb, int64_t sxl, const int* seq, int64_t sqb, const T* init,
                         int64_t sib, int64_t sic, const float* w, const float* bias, T* out, int64_t sob, int64_t sol,
                         T* fin, int64_t sfb, int64_t sfc, const T* g, int64_t sgb, int64_t sgl, const T* dfin,
                         int64_t sdfb, int64_t sdfc, T* dx, int64_t sdb, int64_t sdl, T* dinit, int64_t sdib,
                         int64_t sdic, float* part, float* dw, bool pacc, int Bn, int L, int C, int Wd, bool silu,
                         bool backward, hipStream_t st) {
  dim3 grid((C + 63) / 64, (L + 4 * CV_T - 1) / (4 * CV_T), Bn), block(256);
  W_SWITCH(Wd, {
    VarIO<T, WW> io{x, sxb, sxl, seq, sqb, init, sib, sic, 0, 0, L};
    if (!backward)
      hipLaunchKernelGGL((conv_cl_fwd_var_k<T, WW>), grid, block, 0, st, io, w, bias, out, sob, sol, fin, sfb, sfc, C,
                         silu);
    else
      hipLaunchKernelGGL((conv_cl_bwd_var_k<T, WW>), grid, block, 0, st, io, w, bias, g, sgb, sgl, dfin, sdfb, sdfc,
                         dx, sdb, sdl, dinit, sdib, sdic, part, pacc, C, silu);
  });
  MAMBA_HIP_CHECK(hipGetLastError());
  if (backward && dw) return launch_colsum(part, conv_cl_var_partial_rows(Bn, L), C * (Wd + 1), dw, st);
  return hipSuccess;
}

hipError_t launch_conv_cl_var(const ConvVarArgs& a, hipStream_t st) {
  if (a.dt == kBF16)
    return cl_var<bf16_t>((const bf16_t*)a.x, a.sxb, a.sxl, a.seq, a.sqb, (const bf16_t*)a.init, a.sib, a.sic, a.w,
                          a.bias, (bf16_t*)a.out, a.sob, a.sol, (bf16_t*)a.fin, a.sfb, a.sfc, (const bf16_t*)a.g,
                          a.sgb, a.sgl, (const bf16_t*)a.dfin, a.sdfb, a.sdfc, (bf16_t*)a.dx, a.sdb, a.sdl,
                          (bf16_t*)a.dinit, a.sdib, a.sdic, a.part, a.dw, a.pacc, a.Bn, a.L, a.C, a.Wd, a.silu,
                          a.backward, st);
  if (a.dt == kF32)
    return cl_var<float>((const float*)a.x, a.sxb, a.sxl, a.seq, a.sqb, (const float*)a.init, a.sib, a.sic, a.w,
                         a.bias, (float*)a.out, a.sob, a.sol, (float*)a.fin, a.sfb, a.sfc, (const float*)a.g, a.sgb,
                         a.sgl, (const float*)a.dfin, a.sdfb, a.sdfc, (float*)a.dx, a.sdb, a.sdl, (float*)a.dinit,
                         a.sdib, a.sdic, a.part, a.dw, a.pacc, a.Bn, a.L, a.C, a.Wd, a.silu, a.backward, st);
  return hipErrorInvalidValue;
}

}  // namespace mamba_amd
