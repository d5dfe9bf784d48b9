// Cross-entropy over the LM vocabulary for gfx950.
//
// One 512-thread workgroup (8 waves) per logit row.  The row (V = 50304 bf16 = 98 KiB) is read
// from HBM exactly once with 16-byte loads and kept in registers as packed bf16 pairs
// (<= 13 x uint4 per lane), so
//   pass 1 (max), pass 2 (sum exp), pass 3 (gradient) all run from registers;
// the gradient (softmax - onehot) * scale is written in the same launch (optionally in place
// over the logits).  HBM traffic = 1 read + 1 write of the logits, vs. the reference's
// bf16 -> fp32 upcast + log_softmax + fp32 grad + cast chain (~5x the bytes).
#include "common.h"
#include "launchers.h"

namespace mamba_amd {

constexpr int CE_THREADS = 512;
constexpr int CE_MAXV = 16;  // uint4 (8 x bf16) vectors cached per lane: V <= 16*8*512 = 65536

__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = is_max ? wave_max(v) : wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  float r = sh[0];
#pragma unroll
  for (int i = 1; i < CE_THREADS / 64; ++i) r = is_max ? fmaxf(r, sh[i]) : r + sh[i];
  return r;
}

// bf16 rows, V % 8 == 0, 16-B aligned rows
__global__ __launch_bounds__(CE_THREADS) void ce_fwd_bf16_k(const bf16_t* __restrict__ logits, int64_t ld,
                                                            const int64_t* __restrict__ tgt, int V,
                                                            int64_t ignore_index,
                                                            const float* __restrict__ scale,
                                                            float* __restrict__ loss, bf16_t* __restrict__ grad,
                                                            int64_t ldg) {
  __shared__ float sh[CE_THREADS / 64];
  const int64_t row = blockIdx.x;
  const bf16_t* p = logits + row * ld;
  const int nvec = V / 8;
  uint4 cache[CE_MAXV];
  float m = -INFINITY;
  // the row's loads all in flight before the first use: a per-lane guard around each load made the compiler
  // wait for every one of them on the spot (16 serialized HBM round trips per row); the guard is uniform per
  // slot here and lanes past the row re-read its last vector
#pragma unroll
  for (int i = 0; i < CE_MAXV; ++i)
    if (i * CE_THREADS < nvec) cache[i] = reinterpret_cast<const uint4*>(p)[min((int)threadIdx.x + i * CE_THREADS, nvec - 1)];
#pragma unroll
  for (int i = 0; i < CE_MAXV; ++i) {
    const int vi = threadIdx.x + i * CE_THREADS;
    if (vi < nvec) {
      unsigned wv[4] = {cache[i].x, cache[i].y, cache[i].z, cache[i].w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        m = fmaxf(m, fmaxf(__uint_as_float(wv[k] << 16), __uint_as_float(wv[k] & 0xffff0000u)));
    }
  }
  m = block_reduce(m, sh, true);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CE_MAXV; ++i) {
    const int vi = threadIdx.x + i * CE_THREADS;
    if (vi < nvec) {
      unsigned wv[4] = {cache[i].x, cache[i].y, cache[i].z, cache[i].w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        s += __expf(__uint_as_float(wv[k] << 16) - m) + __expf(__uint_as_float(wv[k] & 0xffff0000u) - m);
    }
  }
  s = block_reduce(s, sh, false);
  const float lse = m + __logf(s);
  const int64_t t = tgt[row];
  const bool valid = t != ignore_index;
  if (threadIdx.x == 0) loss[row] = valid ? lse - bf2f(p[t]) : 0.f;
  if (grad) {
    const float sc = valid ? *scale : 0.f;
    bf16_t* g = grad + row * ldg;
    __syncthreads();  // in-place: every lane has read its cache before anyone overwrites
#pragma unroll
    for (int i = 0; i < CE_MAXV; ++i) {
      const int vi = threadIdx.x + i * CE_THREADS;
      if (vi < nvec) {
        unsigned wv[4] = {cache[i].x, cache[i].y, cache[i].z, cache[i].w};
        float o[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o[2 * k] = __expf(__uint_as_float(wv[k] << 16) - lse) * sc;
          o[2 * k + 1] = __expf(__uint_as_float(wv[k] & 0xffff0000u) - lse) * sc;
        }
        const int base = vi * 8;
        if (t >= base && t < base + 8) o[t - base] -= sc;
        st8bf(g + base, o);
      }
    }
  }
}

// generic path (fp32 or unaligned / large V): three passes over global memory (L2-resident row)
template <typename T>
__global__ __launch_bounds__(CE_THREADS) void ce_fwd_generic_k(const T* __restrict__ logits, int64_t ldl,
                                                               const int64_t* __restrict__ tgt, int V,
                                                               int64_t ignore_index, const float* __restrict__ scale,
                                                               float* __restrict__ loss, T* __restrict__ grad,
                                                               int64_t ldg) {
  __shared__ float sh[CE_THREADS / 64];
  const int64_t row = blockIdx.x;
  const T* p = logits + row * ldl;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < V; i += CE_THREADS) m = fmaxf(m, ld(p + i));
  m = block_reduce(m, sh, true);
  float s = 0.f;
  for (int i = threadIdx.x; i < V; i += CE_THREADS) s += __expf(ld(p + i) - m);
  s = block_reduce(s, sh, false);
  const float lse = m + __logf(s);
  const int64_t t = tgt[row];
  const bool valid = t != ignore_index;
  const float tl = valid ? ld(p + t) : 0.f;
  if (threadIdx.x == 0) loss[row] = valid ? lse - tl : 0.f;
  if (grad) {
    const float sc = valid ? *scale : 0.f;
    T* g = grad + row * ldg;
    __syncthreads();
    // in place is safe: each element is read then written by the same thread
    for (int i = threadIdx.x; i < V; i += CE_THREADS) {
      float v = __expf(ld(p + i) - lse) * sc;
      if (i == t) v -= sc;
      st(g + i, v);
    }
  }
}

hipError_t launch_ce_fwd(const void* logits, int dt, int64_t ld, const int64_t* tgt, int64_t M, int V,
                         int64_t ignore_index, const float* scale, float* loss, void* grad, int64_t ldg,
                         hipStream_t st) {
  if (M == 0) return hipSuccess;
  const bool aligned = ((uintptr_t)logits % 16 == 0) && (ld % 8 == 0) && (V % 8 == 0) &&
                       (grad == nullptr || (((uintptr_t)grad % 16 == 0) && ldg % 8 == 0));
  if (dt == kBF16 && aligned && V / 8 <= CE_MAXV * CE_THREADS) {
    hipLaunchKernelGGL(ce_fwd_bf16_k, dim3((unsigned)M), dim3(CE_THREADS), 0, st, (const bf16_t*)logits, ld, tgt,
                       V, ignore_index, scale, loss, (bf16_t*)grad, ldg);
  } else if (dt == kBF16) {
    hipLaunchKernelGGL(ce_fwd_generic_k<bf16_t>, dim3((unsigned)M), dim3(CE_THREADS), 0, st, (const bf16_t*)logits,
                       ld, tgt, V, ignore_index, scale, loss, (bf16_t*)grad, ldg);
  } else if (dt == kF32) {
    hipLaunchKernelGGL(ce_fwd_generic_k<float>, dim3((unsigned)M), dim3(CE_THREADS), 0, st, (const float*)logits,
                       ld, tgt, V, ignore_index, scale, loss, (float*)grad, ldg);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace mamba_amd
