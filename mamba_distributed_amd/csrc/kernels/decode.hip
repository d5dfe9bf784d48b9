// Fused single-token decode step of a Mamba-2 layer for gfx950: 4 kernels per layer instead of ~7
// library/elementwise launches plus the per-call parameter casts (the
// reference has no cached decode at all: its generate() re-runs the whole prefix, model.py:49-75).
//
// A decode step is latency-bound: per layer it streams the in_proj / out_proj weights once
// (~7.5 MB bf16 at 280M) and touches 1-2 small vectors per sequence.  What costs time is the number
// of dependent launches (each a HIP-graph node, ~2-4 us), so each kernel below fuses everything up to
// the next point where every workgroup needs a value that a different workgroup produced:
//
//   (the block's residual add + RMSNorm runs first: the native add_rmsnorm kernel, one row per wave)
//   K1 dec_inproj_k    zxbcdt = hn W_in^T (4 output rows per wave, 16-B weight loads issued before hn
//                      is staged in LDS, every batch row per weight load), and for the xBC rows the
//                      causal-conv window update + SiLU in the epilogue.
//   K2 dec_ssm_k       per (batch, head, 16-row slice of P): dt = softplus(dt + bias),
//                      S = e^{dt A} S + dt x B^T, y = S C + D x, g = y * silu(z), and the slice's
//                      sum of g^2 (the gated norm's statistics, finished by K3).
//   K3 dec_outproj_k   rstd from the partial sums, out = rstd * (g (W_out diag(w))^T): the gate-norm
//                      weight folded into the weight once, rstd applied in the epilogue.
// GEMVs: bf16 weight and activation pairs straight into v_dot2c_f32_bf16.
//
// Shapes are validated on the host (bindings.cpp: decode_* ops); every kernel has a fixed grid and
// no inter-workgroup waiting, so it is HIP-graph capturable.
#include "common.h"
#include "launchers.h"

namespace mamba_amd {

namespace {
constexpr int DEC_MAXB = 16;  // batch rows per launch (host splits larger batches)

__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// Reduce M per-lane partials over the wave at once (transpose-reduce: M-1 shuffles instead of
// 6 M): lane l ends with the wave total of entry idx(l); lanes 0..M-1 cover every entry once.
template <int M>
__device__ __forceinline__ float multi_wave_sum(float (&v)[M], int lane, int& idx) {
  idx = 0;
#pragma unroll
  for (int m = 1, h = M / 2; h >= 1; m <<= 1, h >>= 1) {
    const bool up = (lane & m) != 0;
#pragma unroll
    for (int j = 0; j < h; ++j) {
      const float send = up ? v[j] : v[j + h];
      const float keep = up ? v[j + h] : v[j];
      v[j] = keep + __shfl_xor(send, m, 64);
    }
    idx += up ? h : 0;
  }
  float s = v[0];
#pragma unroll
  for (int m = M; m < 64; m <<= 1) s += __shfl_xor(s, m, 64);
  return s;
}
}  // namespace

// ---------------------------------------------------------------------------------------------
// Shared GEMV core: out[r][o] = sum_k W[o][k] x[r][k] for the RPW rows o of this wave, every batch row r
// (x staged in LDS as bf16).  The wave's weight chunks are loaded before the caller stages x, so the HBM latency
// of the weight stream overlaps the staging.
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));

template <int RPW, int MB>
struct GemvRows {
  // The first KC 512-element chunks of every row (K <= 2048 at 280M-2.8B widths) are all loaded before the caller
  // stages x: one HBM round trip per kernel instead of one per chunk (a decode step streams ~560 MB of cold
  // weights; with one wave per SIMD nothing else hides a per-chunk wait).  Chunks past KC load in the loop.
  static constexpr int KC = 4;
  uint4 w0[KC][RPW];
  __device__ __forceinline__ void prefetch(const bf16_t* W, int o0, int n_out, int K, int lane) {
#pragma unroll
    for (int c = 0; c < KC; ++c)
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const int k = lane * 8 + 512 * c;
        w0[c][q] = (o0 + q < n_out && k < K) ? *reinterpret_cast<const uint4*>(W + (int64_t)(o0 + q) * K + k)
                                             : make_uint4(0, 0, 0, 0);
      }
  }
  // acc[q * MB + r]: row o0 + q, batch row r (rows r >= b stay zero).  bf16 pairs go straight into
  // v_dot2c_f32_bf16 (2 products per instruction, no unpacking of weights or activations).
  __device__ __forceinline__ void chunk(const uint4 (&u)[RPW], int k, int K, const bf16_t* xs, int b,
                                        float (&acc)[RPW * MB]) {
    bf2v wv[RPW][4];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      wv[q][0] = __builtin_bit_cast(bf2v, u[q].x);
      wv[q][1] = __builtin_bit_cast(bf2v, u[q].y);
      wv[q][2] = __builtin_bit_cast(bf2v, u[q].z);
      wv[q][3] = __builtin_bit_cast(bf2v, u[q].w);
    }
#pragma unroll
    for (int r = 0; r < MB; ++r) {
      if (r < b) {
        const uint4 xu = *reinterpret_cast<const uint4*>(xs + r * K + k);
        const bf2v x0 = __builtin_bit_cast(bf2v, xu.x), x1 = __builtin_bit_cast(bf2v, xu.y);
        const bf2v x2 = __builtin_bit_cast(bf2v, xu.z), x3 = __builtin_bit_cast(bf2v, xu.w);
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
          float a = acc[q * MB + r];
          a = __builtin_amdgcn_fdot2_f32_bf16(wv[q][0], x0, a, false);
          a = __builtin_amdgcn_fdot2_f32_bf16(wv[q][1], x1, a, false);
          a = __builtin_amdgcn_fdot2_f32_bf16(wv[q][2], x2, a, false);
          a = __builtin_amdgcn_fdot2_f32_bf16(wv[q][3], x3, a, false);
          acc[q * MB + r] = a;
        }
      }
    }
  }
  __device__ __forceinline__ void run(const bf16_t* W, int o0, int n_out, int K, int lane, const bf16_t* xs, int b,
                                      float (&acc)[RPW * MB]) {
#pragma unroll
    for (int i = 0; i < RPW * MB; ++i) acc[i] = 0.f;
#pragma unroll
    for (int c = 0; c < KC; ++c) {  // K % 8 == 0
      const int k = lane * 8 + 512 * c;
      if (k < K) chunk(w0[c], k, K, xs, b, acc);
    }
    for (int k = lane * 8 + 512 * KC; k < K; k += 512) {
      uint4 u[RPW];
#pragma unroll
      for (int q = 0; q < RPW; ++q)
        u[q] = (o0 + q < n_out) ? *reinterpret_cast<const uint4*>(W + (int64_t)(o0 + q) * K + k) : make_uint4(0, 0, 0, 0);
      chunk(u, k, K, xs, b, acc);
    }
  }
};

// K1.  hn (b, d) bf16 = RMSNorm(residual + h) * w from the add+RMSNorm kernel; grid ceil(n_out / (4 RPW)).
// LDS: hn staged (b * d * 2 <= 64 KiB, host-checked).
// Output rows per wave: 4, or 2 at 16 batch rows -- 4 x 16 accumulators went to scratch (272 B per lane) and a
// narrower wave also doubles the grid (3392 in_proj rows: 212 -> 424 workgroups for 256 CUs).
constexpr int k1_rpw(int mb) { return mb >= 16 ? 2 : 4; }
template <int MB>  // batch-row capacity (1, 4 or 16); the transpose-reduce leaves one (row, batch) per lane
__global__ __launch_bounds__(256) void dec_inproj_k(const bf16_t* __restrict__ hn, const bf16_t* __restrict__ W,
                                                    int n_out, int d, int b, float* __restrict__ zxbcdt, int conv_lo,
                                                    int conv_hi, bf16_t* __restrict__ conv_state, int64_t csb,
                                                    int64_t csc, int SL, const float* __restrict__ cw,
                                                    const float* __restrict__ cb, int Wd) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem);  // [b][d]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int K1_RPW = k1_rpw(MB);
  const int o0 = (blockIdx.x * 4 + wave) * K1_RPW;
  GemvRows<K1_RPW, MB> gv;
  gv.prefetch(W, o0, n_out, d, lane);
  // stage hn: 8 independent 16-B loads in flight per thread before the first LDS store
  for (int base = threadIdx.x * 8; base < b * d; base += 8 * 256 * 8) {
    uint4 t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * 256 * 8;
      t[u] = i < b * d ? *reinterpret_cast<const uint4*>(hn + i) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * 256 * 8;
      if (i < b * d) *reinterpret_cast<uint4*>(xs + i) = t[u];
    }
  }
  __syncthreads();
  if (o0 >= n_out) return;
  float acc[K1_RPW * MB];
  gv.run(W, o0, n_out, d, lane, xs, b, acc);
  int idx;
  float v = multi_wave_sum<K1_RPW * MB>(acc, lane, idx);
  // epilogue: one (output row, batch row) per lane, all in parallel
  const int q = idx / MB, r = idx % MB, o = o0 + q;
  if (lane < K1_RPW * MB && r < b && o < n_out) {
    if (o >= conv_lo && o < conv_hi) {
      // causal conv window: the state holds the last SL >= Wd-1 inputs of channel c (oldest first); the
      // output uses its last Wd-1 entries and v, then the state shifts by one and takes v
      const int c = o - conv_lo;
      bf16_t* st = conv_state + (int64_t)r * csb + (int64_t)c * csc;
      float a = cb ? cb[c] : 0.f;
      for (int k = 0; k < Wd - 1; ++k) a = fmaf(cw[c * Wd + k], bf2f(st[SL - (Wd - 1) + k]), a);
      a = fmaf(cw[c * Wd + Wd - 1], v, a);
      for (int k = 0; k + 1 < SL; ++k) st[k] = st[k + 1];
      if (SL > 0) st[SL - 1] = f2bf(v);
      v = a * sigmoidf_(a);
    }
    zxbcdt[(int64_t)r * n_out + o] = v;
  }
}

// ---------------------------------------------------------------------------------------------
// K2.  grid (H * P/16, b), 256 threads: thread t -> row p = p0 + t/16, states n = (t%16)*NPT ..
// zxbcdt row layout: [z (di) | x (di) | B (G N) | C (G N) | dt (H)], conv already applied to x/B/C.
template <int NPT>  // states per thread (N / 16)
__global__ __launch_bounds__(256) void dec_ssm_k(const float* __restrict__ zxbcdt, int n_out, float* __restrict__ state,
                                                 const float* __restrict__ A, const float* __restrict__ Dp,
                                                 const float* __restrict__ dt_bias, int H, int P, int G,
                                                 bf16_t* __restrict__ g_out, float* __restrict__ part) {
  constexpr int N = NPT * 16;
  __shared__ float red[16];
  const int slices = P / 16;
  const int h = blockIdx.x / slices, ps = blockIdx.x % slices, r = blockIdx.y;
  const int t = threadIdx.x, p = ps * 16 + (t >> 4), n0 = (t & 15) * NPT;
  const int di = H * P, gi = h / (H / G);
  const float* row = zxbcdt + (int64_t)r * n_out;
  float dt = row[2 * di + 2 * G * N + h] + (dt_bias ? dt_bias[h] : 0.f);
  dt = softplusf_(dt);
  const float dA = __expf(dt * A[h]);
  const float x = row[di + h * P + p];
  const float* Bv = row + 2 * di + gi * N;
  const float* Cv = row + 2 * di + G * N + gi * N;
  float* S = state + (((int64_t)r * H + h) * P + p) * N + n0;
  float y = 0.f;
#pragma unroll
  for (int j = 0; j < NPT; j += 4) {
    float4 s4 = *reinterpret_cast<const float4*>(S + j);
    float sv[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = n0 + j + q;
      sv[q] = fmaf(sv[q], dA, dt * x * Bv[n]);
      y = fmaf(sv[q], Cv[n], y);
    }
    *reinterpret_cast<float4*>(S + j) = make_float4(sv[0], sv[1], sv[2], sv[3]);
  }
  // sum over the 16 threads of row p (a DPP row)
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) y += __shfl_xor(y, m, 64);
  float g2 = 0.f;
  if ((t & 15) == 0) {
    y = fmaf(Dp ? Dp[h] : 0.f, x, y);
    const float z = row[h * P + p];
    const float g = y * (z * sigmoidf_(z));
    g_out[(int64_t)r * di + h * P + p] = f2bf(g);
    g2 = g * g;
  }
  g2 = wave_sum64(g2);
  if ((t & 63) == 0) red[t >> 6] = g2;
  __syncthreads();
  if (t == 0) part[(int64_t)r * (H * slices) + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// ---------------------------------------------------------------------------------------------
// K3.  grid: ceil(d_model / (4 RPW)) workgroups; LDS xn[b][di] bf16 (host-checked <= 64 KiB).
// Output rows per wave: 2, or 1 at 16 batch rows (d_model 768: 96 -> 192 workgroups for 256 CUs).
constexpr int k3_rpw(int mb) { return mb >= 16 ? 1 : 2; }
// The gate-norm weight is folded into the weight on the host (W' = W diag(w), static during decode)
// and rstd is a per-row scalar, so the GEMV runs on g as produced by K2 and the epilogue scales by
// rstd:  out = rstd * (g W'^T)  ==  (g * rstd * w) W^T.
template <int MB>
__global__ __launch_bounds__(256) void dec_outproj_k(const bf16_t* __restrict__ g, const float* __restrict__ part,
                                                     int nparts, float eps, const bf16_t* __restrict__ W, int d_out,
                                                     int di, int b, bf16_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem);
  __shared__ float rstd_s[DEC_MAXB];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int K3_RPW = k3_rpw(MB);
  const int o0 = (blockIdx.x * 4 + wave) * K3_RPW;
  GemvRows<K3_RPW, MB> gv;
  gv.prefetch(W, o0, d_out, di, lane);
  {  // rstd per batch row: 16 threads per row, every partial load issued up front
    const int r = threadIdx.x >> 4, j = threadIdx.x & 15;
    float s = 0.f;
    if (r < b)
      for (int i = j; i < nparts; i += 16) s += part[(int64_t)r * nparts + i];
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
    if (r < b && j == 0) rstd_s[r] = rsqrtf(s / (float)di + eps);
  }
  for (int base = threadIdx.x * 8; base < b * di; base += 8 * 256 * 8) {
    uint4 t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * 256 * 8;
      t[u] = i < b * di ? *reinterpret_cast<const uint4*>(g + i) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * 256 * 8;
      if (i < b * di) *reinterpret_cast<uint4*>(xs + i) = t[u];
    }
  }
  __syncthreads();
  if (o0 >= d_out) return;
  float acc[K3_RPW * MB];
  gv.run(W, o0, d_out, di, lane, xs, b, acc);
  int idx;
  const float v = multi_wave_sum<K3_RPW * MB>(acc, lane, idx);
  const int q = idx / MB, r = idx % MB;
  if (lane < K3_RPW * MB && r < b && o0 + q < d_out) out[(int64_t)r * d_out + o0 + q] = f2bf(v * rstd_s[r]);
}

// ---------------------------------------------------------------------------------------------
int decode_max_batch() { return DEC_MAXB; }

hipError_t launch_decode_inproj(const void* hn, const void* W, int n_out, int d, int b, float* zxbcdt, int conv_lo,
                                int conv_hi, void* conv_state, int64_t csb, int64_t csc, int SL, const float* cw,
                                const float* cb, int Wd, hipStream_t st) {
  if (b < 1 || b > DEC_MAXB || d % 8 || (size_t)b * d * 2 > 65536 || SL < Wd - 1) return hipErrorInvalidValue;
  const size_t lds = (size_t)b * d * 2;
#define DEC_K1(MB) hipLaunchKernelGGL(dec_inproj_k<MB>, dim3((n_out + 4 * k1_rpw(MB) - 1) / (4 * k1_rpw(MB))), dim3(256), lds, st, (const bf16_t*)hn, (const bf16_t*)W, \
                                      n_out, d, b, zxbcdt, conv_lo, conv_hi, (bf16_t*)conv_state, csb, csc, SL, cw, cb, Wd)
  if (b == 1) DEC_K1(1);
  else if (b <= 4) DEC_K1(4);
  else DEC_K1(16);
#undef DEC_K1
  return hipGetLastError();
}

hipError_t launch_decode_ssm(const float* zxbcdt, int n_out, float* state, const float* A, const float* D,
                             const float* dt_bias, int H, int P, int G, int N, int b, void* g_out_, float* part,
                             hipStream_t st) {
  bf16_t* g_out = (bf16_t*)g_out_;
  if (P % 16 || b < 1) return hipErrorInvalidValue;
  dim3 grid(H * (P / 16), b);
  switch (N) {
    case 64: hipLaunchKernelGGL(dec_ssm_k<4>, grid, dim3(256), 0, st, zxbcdt, n_out, state, A, D, dt_bias, H, P, G, g_out, part); break;
    case 128: hipLaunchKernelGGL(dec_ssm_k<8>, grid, dim3(256), 0, st, zxbcdt, n_out, state, A, D, dt_bias, H, P, G, g_out, part); break;
    case 256: hipLaunchKernelGGL(dec_ssm_k<16>, grid, dim3(256), 0, st, zxbcdt, n_out, state, A, D, dt_bias, H, P, G, g_out, part); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_decode_outproj(const void* g, const float* part, int nparts, float eps, const void* W, int d_out,
                                 int di, int b, void* out, hipStream_t st) {
  if (b < 1 || b > DEC_MAXB || di % 8 || (size_t)b * di * 2 > 65536) return hipErrorInvalidValue;
  const size_t lds = (size_t)b * di * 2;
#define DEC_K3(MB) hipLaunchKernelGGL(dec_outproj_k<MB>, dim3((d_out + 4 * k3_rpw(MB) - 1) / (4 * k3_rpw(MB))), dim3(256), lds, st, (const bf16_t*)g, part, nparts, \
                                      eps, (const bf16_t*)W, d_out, di, b, (bf16_t*)out)
  if (b == 1) DEC_K3(1);
  else if (b <= 4) DEC_K3(4);
  else DEC_K3(16);
#undef DEC_K3
  return hipGetLastError();
}

}  // namespace mamba_amd
