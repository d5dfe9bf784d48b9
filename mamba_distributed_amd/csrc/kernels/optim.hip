// Native optimizer step for gfx950: multi-tensor AdamW (decoupled weight decay, torch.optim.AdamW semantics) with
// the gradient-clipping coefficient and the data-parallel 1/world average folded into its gradient read, and the
// bf16 weight images the next step's GEMMs consume written by the same pass.
//
// Reference: /root/reference/model.py:146-148 (configure_optimizers -> torch.optim.AdamW(fused=True)),
// /root/reference/train.py:222 (clip_grad_norm_(1.0)), :227 (optimizer.step()); SURVEY.md G8 / G9.
//
// Why native: at one micro-batch per optimizer step (8 ranks x 65,536 tokens) every per-step pass over the
// 280M-parameter state is paid per 64k tokens: torch's fused AdamW (one read of p, g, m, v and one write of p, m, v),
// the clip (a norm pass and a scale pass over every gradient), the reducer's 1/world pass, and the per-step bf16
// casts / zero-padded copies of the projection weights.  Here: ONE sum-of-squares pass over the gradients, ONE
// tiny launch that turns it into the clip scale, ONE update pass that also emits the bf16 images.
//
// Work decomposition: the host packs a segment table (one row per parameter: pointers, length, the per-parameter
// step size / bias correction / decay factor) and a block table (one row per 4096-element chunk: segment, offset),
// so one launch covers every parameter whatever its size; chunks never straddle two parameters.  Deterministic:
// each element has one writer, and the gradient norm is a fixed-order reduction (per-block partials in block
// order, summed in fp64 by one block).
#include "common.h"
#include "launchers.h"

namespace mamba_amd {

// one row of the segment table (host layout: ops/optim.py _SEG_DTYPE, 64 bytes)
struct OptSeg {
  float* p;          // fp32 parameter (master)
  const float* g;    // fp32 gradient
  float* m;          // exp_avg
  float* v;          // exp_avg_sq
  bf16_t* img;       // bf16 image of the updated parameter, same row-major layout (nullptr: none)
  int64_t n;         // elements
  float step_size;   // lr / (1 - beta1^step)
  float bc2_rsqrt;   // 1 / sqrt(1 - beta2^step)
  float decay;       // 1 - lr * weight_decay
  int vec;           // p, g, m, v (and img) 16-B / 8-B aligned and n % 4 == 0: float4 path
};
static_assert(sizeof(OptSeg) == 64, "segment table row layout is shared with the host");

constexpr int OPT_CHUNK = 4096;  // elements per block (256 threads x 16)

// per-block partial sums of g^2 over the block's chunk (fp32 within the block, fixed order)
__global__ __launch_bounds__(256) void grad_sumsq_k(const OptSeg* __restrict__ segs, const int64_t* __restrict__ blk,
                                                    float* __restrict__ partial) {
  __shared__ float red[4];
  const OptSeg s = segs[blk[2 * blockIdx.x]];
  const int64_t o = blk[2 * blockIdx.x + 1];
  const int64_t e = min(o + OPT_CHUNK, s.n);
  float acc = 0.f;
  if (s.vec) {
    for (int64_t i = o + 4 * threadIdx.x; i < e; i += 4 * 256) {
      const float4 g = *reinterpret_cast<const float4*>(s.g + i);
      acc = fmaf(g.x, g.x, acc); acc = fmaf(g.y, g.y, acc); acc = fmaf(g.z, g.z, acc); acc = fmaf(g.w, g.w, acc);
    }
  } else {
    for (int64_t i = o + threadIdx.x; i < e; i += 256) acc = fmaf(s.g[i], s.g[i], acc);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out[0] = || g / divisor ||_2 ; out[1] = min(1, max_norm / (out[0] + 1e-6)) / divisor  (max_norm <= 0: no clip)
__global__ __launch_bounds__(1024) void clip_scale_k(const float* __restrict__ partial, int nblk, float max_norm,
                                                     float divisor, float* __restrict__ out) {
  __shared__ double red[1024];
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;  // 4 independent loads in flight per thread
  int i = threadIdx.x;
  for (; i + 3 * 1024 < nblk; i += 4 * 1024) {
    a0 += (double)partial[i];
    a1 += (double)partial[i + 1024];
    a2 += (double)partial[i + 2 * 1024];
    a3 += (double)partial[i + 3 * 1024];
  }
  for (; i < nblk; i += 1024) a0 += (double)partial[i];
  red[threadIdx.x] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float norm = (float)(sqrt(red[0]) / (double)divisor);
    // torch.nn.utils.clip_grad_norm_: clamp(max_norm / (norm + 1e-6), max=1) -- a NaN norm gives a NaN coefficient
    // (poisoning every parameter, as torch does; fminf would return 1 and drop it)
    const float c = max_norm / (norm + 1e-6f);
    const float coef = max_norm > 0.f ? (c > 1.f ? 1.f : c) : 1.f;
    out[0] = norm;
    out[1] = coef / divisor;
  }
}

// the update, torch.optim.AdamW (fused) order of operations:
//   p *= 1 - lr wd;  m += (1 - b1) (g - m);  v = b2 v + (1 - b2) g^2;  p -= step_size m / (sqrt(v) / sqrt(bc2) + eps)
__device__ __forceinline__ float adamw1(float& p, float g, float& m, float& v, const OptSeg& s, float b1c, float b2,
                                        float b2c, float eps) {
  p *= s.decay;
  m = fmaf(b1c, g - m, m);
  v = fmaf(b2, v, b2c * g * g);
  p = fmaf(-s.step_size, m / fmaf(sqrtf(v), s.bc2_rsqrt, eps), p);
  return p;
}

__global__ __launch_bounds__(256) void adamw_k(const OptSeg* __restrict__ segs, const int64_t* __restrict__ blk,
                                               const float* __restrict__ gscale, float b1, float b2, float eps) {
  const OptSeg s = segs[blk[2 * blockIdx.x]];
  const int64_t o = blk[2 * blockIdx.x + 1];
  const int64_t e = min(o + OPT_CHUNK, s.n);
  const float sc = gscale ? gscale[1] : 1.f;
  const float b1c = 1.f - b1, b2c = 1.f - b2;
  if (s.vec) {
    for (int64_t i = o + 4 * threadIdx.x; i < e; i += 4 * 256) {
      float4 p = *reinterpret_cast<const float4*>(s.p + i);
      const float4 g = *reinterpret_cast<const float4*>(s.g + i);
      float4 m = *reinterpret_cast<const float4*>(s.m + i);
      float4 v = *reinterpret_cast<const float4*>(s.v + i);
      adamw1(p.x, g.x * sc, m.x, v.x, s, b1c, b2, b2c, eps);
      adamw1(p.y, g.y * sc, m.y, v.y, s, b1c, b2, b2c, eps);
      adamw1(p.z, g.z * sc, m.z, v.z, s, b1c, b2, b2c, eps);
      adamw1(p.w, g.w * sc, m.w, v.w, s, b1c, b2, b2c, eps);
      *reinterpret_cast<float4*>(s.p + i) = p;
      *reinterpret_cast<float4*>(s.m + i) = m;
      *reinterpret_cast<float4*>(s.v + i) = v;
      if (s.img) *reinterpret_cast<uint2*>(s.img + i) = make_uint2(pack2(p.x, p.y), pack2(p.z, p.w));
    }
  } else {
    for (int64_t i = o + threadIdx.x; i < e; i += 256) {
      float p = s.p[i], m = s.m[i], v = s.v[i];
      adamw1(p, s.g[i] * sc, m, v, s, b1c, b2, b2c, eps);
      s.p[i] = p;
      s.m[i] = m;
      s.v[i] = v;
      if (s.img) s.img[i] = f2bf(p);
    }
  }
}

hipError_t launch_grad_norm(const void* segs, const int64_t* blk, int nblk, float* partial, float max_norm,
                            float divisor, float* out, hipStream_t st) {
  if (nblk <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(grad_sumsq_k, dim3(nblk), dim3(256), 0, st, (const OptSeg*)segs, blk, partial);
  MAMBA_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(clip_scale_k, dim3(1), dim3(1024), 0, st, partial, nblk, max_norm, divisor, out);
  return hipGetLastError();
}

hipError_t launch_adamw(const void* segs, const int64_t* blk, int nblk, const float* gscale, float b1, float b2,
                        float eps, hipStream_t st) {
  if (nblk <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(adamw_k, dim3(nblk), dim3(256), 0, st, (const OptSeg*)segs, blk, gscale, b1, b2, eps);
  return hipGetLastError();
}

int opt_chunk() { return OPT_CHUNK; }

}  // namespace mamba_amd
