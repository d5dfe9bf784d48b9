// Mamba-2 SSD (state-space duality) chunked scan, forward + backward, for gfx950 (MI355X).
//
// Math (per batch b, head h with group g, chunk of Q = 64 steps, local step i):
//   dt_i  = clamp(softplus(dt_raw_i + dt_bias_h))      a_i = dt_i * A_h    cum = cumsum_in_chunk(a)
//   y_i   = sum_{j<=i} (C_i.B_j) e^{cum_i-cum_j} dt_j x_j  +  e^{cum_i} C_i . S_in  +  D_h x_i
//   S_out = e^{cum_last} S_in + sum_j e^{cum_last-cum_j} dt_j x_j B_j^T          (S: P x N, fp32)
// (upstream ops/triton/ssd_*.py; the chunk length is an implementation detail)
//
// Kernels (all MFMA work on v_mfma_f32_16x16x32_bf16; operand layouts in mfma.h):
//   ssd_cumsum      wave per (b,h,chunk): dt transform + wave64 inclusive scan of dt*A.
//   ssd_state_fwd   WG per (n-slice of 64, h, b), walks the chunks in order with the running state
//                   in MFMA accumulators: stores S_in (bf16) per chunk, then S = e^{cum_last} S +
//                   (w.X)^T B as 16x16x32 MFMAs whose operands come through ds_read_b64_tr_b16
//                   (token-major tiles contracted over time need the hardware transpose).
//   ssd_scan_fwd    WG per (chunk, head-group, b): CB^T tiles computed once and kept in registers
//                   for all heads of the group; per head y = e^{cum} C S_in^T  +  (CB o L)^T-as-A x
//                   (the masked CB^T accumulator feeds the next MFMA directly, PERM k order) + D x.
//   ssd_dstate_bwd  reverse-time twin of ssd_state_fwd: dS_out per chunk (bf16), dS_init.
//   ssd_chunk_bwd   WG per (chunk, head-group, b): dM, M, dX, ddt (incl. the in-chunk reverse cumsum
//                   of dcum), dA/dD/dbias partials; head-summed dCB, dB_off, dC_off accumulators
//                   stay in registers across the heads of the group (no per-head HBM round trip).
//   ssd_dbc_bwd     WG per (chunk, group, b): dC = sum dC_off + dCB B ; dB = sum dB_off + dCB^T C.
// No float atomics on global memory: every cross-workgroup sum goes through fixed-order partials.
#include "mfma.h"
#include "ssd.h"

namespace mamba_amd {

constexpr int Q = 64;
constexpr int P = 64;
constexpr int LD64 = 72;  // padded LDS row (elements) for 64-wide bf16 tiles

__device__ __forceinline__ float ld_any(const void* p, int dt, int64_t i) {
  return dt == kF32 ? reinterpret_cast<const float*>(p)[i] : bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
}
__device__ __forceinline__ void st_any(void* p, int dt, int64_t i, float v) {
  if (dt == kF32) reinterpret_cast<float*>(p)[i] = v;
  else reinterpret_cast<bf16_t*>(p)[i] = f2bf(v);
}

// ============================== K0: dt transform + cumsum ====================================
__global__ __launch_bounds__(256) void ssd_cumsum_k(SSDArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= (int64_t)a.B * a.H * a.nc) return;
  const int c = wid % a.nc, h = (wid / a.nc) % a.H, b = wid / ((int64_t)a.nc * a.H);
  const int t = c * Q + lane;
  float v = 0.f;
  if (t < a.L) {
    float raw = ld_any(a.dt, a.dt_dtype, (int64_t)b * a.sdtb + (int64_t)t * a.sdtl + (int64_t)h * a.sdth);
    if (a.dt_bias) raw += a.dt_bias[h];
    v = a.softplus ? softplusf_(raw) : raw;
    v = fminf(fmaxf(v, a.dt_min), a.dt_max);
  }
  float x = v * a.A[h];
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  const int64_t o = ((int64_t)b * a.H + h) * a.Lp + t;
  a.dtp[o] = v;
  a.cum[o] = x;
}

// ============================== K1: chunk states + state passing (forward) =================
template <int N>
__global__ __launch_bounds__(256) void ssd_state_fwd_k(SSDArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t Xs[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t Os[P * LD64];
  __shared__ float wrow[Q];
  const int ns = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int g = h / (a.H / a.G);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const float* cumbh = a.cum + ((int64_t)b * a.H + h) * a.Lp;
  const float* dtbh = a.dtp + ((int64_t)b * a.H + h) * a.Lp;
  f32x4 acc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    acc[nt] = zero4();
    if (a.init) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * w + 4 * (l >> 4) + r, n = ns * 64 + 16 * nt + (l & 15);
        acc[nt][r] = a.init[(((int64_t)b * a.H + h) * P + p) * N + n];
      }
    }
  }
  for (int c = 0; c < a.nc; ++c) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc_to_lds(Os, LD64, 16 * w, 16 * nt, acc[nt]);
    if (threadIdx.x < Q) {
      const int t = c * Q + threadIdx.x;
      wrow[threadIdx.x] = __expf(cumbh[c * Q + Q - 1] - cumbh[t]) * dtbh[t];
    }
    __syncthreads();
    store_tile<P, 64>(a.states + ((((int64_t)b * a.nc + c) * a.H + h) * P) * N + ns * 64, N, Os, LD64, P);
    const int valid = min(Q, a.L - c * Q);
    stage_tile<Q, 64>(Xs, LD64, a.x + (int64_t)b * a.sxb + (int64_t)c * Q * a.sxl + (int64_t)h * a.sxh, a.sxl, valid,
                      wrow);
    stage_tile<Q, 64>(Bs, LD64, a.Bm + (int64_t)b * a.sBb + (int64_t)c * Q * a.sBl + (int64_t)g * a.sBg + ns * 64,
                      a.sBl, valid);
    __syncthreads();
    const float decay = __expf(cumbh[c * Q + Q - 1]);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] *= decay;
#pragma unroll
    for (int ks = 0; ks < Q / 32; ++ks) {
      const bf16x8 A = frag_tr(Xs, LD64, 32 * ks, 16 * w);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma16(A, frag_tr(Bs, LD64, 32 * ks, 16 * nt), acc[nt]);
    }
    __syncthreads();
  }
  if (a.final_state) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * w + 4 * (l >> 4) + r, n = ns * 64 + 16 * nt + (l & 15);
        a.final_state[(((int64_t)b * a.H + h) * P + p) * N + n] = acc[nt][r];
      }
  }
}

// ============================== K2: chunk output (forward) ==================================
template <int N>
__global__ __launch_bounds__(256) void ssd_scan_fwd_k(SSDArgs a) {
  constexpr int LDN = N + 8;
  __shared__ __attribute__((aligned(16))) bf16_t Cs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Ss[P * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Xs[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t XDs[Q * LD64];  // also the output staging tile
  __shared__ float cumr[Q], dtr[Q];
  bf16_t* Os = XDs;
  const int c = blockIdx.x, hgi = blockIdx.y, b = blockIdx.z;
  const int h0 = hgi * a.HG, g = h0 / (a.H / a.G);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int valid = min(Q, a.L - c * Q);
  stage_tile<Q, N>(Cs, LDN, a.Cm + (int64_t)b * a.sCb + (int64_t)c * Q * a.sCl + (int64_t)g * a.sCg, a.sCl, valid);
  stage_tile<Q, N>(Bs, LDN, a.Bm + (int64_t)b * a.sBb + (int64_t)c * Q * a.sBl + (int64_t)g * a.sBg, a.sBl, valid);
  __syncthreads();
  // CB^T tiles: rows j (tile jt), cols i (tile w); only jt <= w is ever non-zero (causal)
  f32x4 cbt[4];
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    cbt[jt] = zero4();
    if (jt <= w) {
#pragma unroll
      for (int ks = 0; ks < N / 32; ++ks)
        cbt[jt] = mfma16(frag_kc(Bs, LDN, 16 * jt, 32 * ks), frag_kc(Cs, LDN, 16 * w, 32 * ks), cbt[jt]);
    }
  }
  for (int hh = 0; hh < a.HG; ++hh) {
    const int h = h0 + hh;
    const int64_t bh = ((int64_t)b * a.H + h) * a.Lp + (int64_t)c * Q;
    if (threadIdx.x < Q) {
      cumr[threadIdx.x] = a.cum[bh + threadIdx.x];
      dtr[threadIdx.x] = a.dtp[bh + threadIdx.x];
    }
    __syncthreads();
    const bf16_t* xg = a.x + (int64_t)b * a.sxb + (int64_t)c * Q * a.sxl + (int64_t)h * a.sxh;
    stage_tile<Q, 64>(Xs, LD64, xg, a.sxl, valid);
    stage_tile<Q, 64>(XDs, LD64, xg, a.sxl, valid, dtr);
    stage_tile<P, N>(Ss, LDN, a.states + ((((int64_t)b * a.nc + c) * a.H + h) * P) * N, N, P);
    __syncthreads();
    f32x4 acc[4];
    // y_off = e^{cum_i} C_i . S^T
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      acc[pt] = zero4();
#pragma unroll
      for (int ks = 0; ks < N / 32; ++ks)
        acc[pt] = mfma16(frag_kc(Cs, LDN, 16 * w, 32 * ks), frag_kc(Ss, LDN, 16 * pt, 32 * ks), acc[pt]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = __expf(cumr[16 * w + 4 * (l >> 4) + r]);
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) acc[pt][r] *= e;
    }
    // y_diag: masked CB^T (rows j, cols i) used as A = (M^T)^T in PERM order
    const int i_col = 16 * w + (l & 15);
    const float cum_i = cumr[i_col];
    f32x4 mt[4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 16 * jt + 4 * (l >> 4) + r;
        mt[jt][r] = (jt <= w && j <= i_col) ? cbt[jt][r] * __expf(cum_i - cumr[j]) : 0.f;
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (2 * ks <= w) {
        const bf16x8 A = acc_frag(mt[2 * ks], mt[2 * ks + 1]);
#pragma unroll
        for (int pt = 0; pt < 4; ++pt) acc[pt] = mfma16(A, frag_tr_perm(XDs, LD64, 32 * ks, 16 * pt), acc[pt]);
      }
    }
    const float Dh = a.D ? a.D[h] : 0.f;
    __syncthreads();  // every wave is done reading XDs before it becomes the output tile
#pragma unroll
    for (int pt = 0; pt < 4; ++pt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * w + 4 * (l >> 4) + r, p = 16 * pt + (l & 15);
        Os[i * LD64 + p] = f2bf(acc[pt][r] + Dh * bf2f(Xs[i * LD64 + p]));
      }
    __syncthreads();
    store_tile<Q, 64>(a.y + (int64_t)b * a.syb + (int64_t)c * Q * a.syl + (int64_t)h * a.syh, a.syl, Os, LD64, valid);
    __syncthreads();
  }
}

// ============================== K3: reverse state pass (backward) ===========================
template <int N>
__global__ __launch_bounds__(256) void ssd_dstate_bwd_k(SSDArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t Ys[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t Cs[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t Os[P * LD64];
  __shared__ float er[Q];
  const int ns = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int g = h / (a.H / a.G);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const float* cumbh = a.cum + ((int64_t)b * a.H + h) * a.Lp;
  f32x4 acc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    acc[nt] = zero4();
    if (a.dfinal) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * w + 4 * (l >> 4) + r, n = ns * 64 + 16 * nt + (l & 15);
        acc[nt][r] = a.dfinal[(((int64_t)b * a.H + h) * P + p) * N + n];
      }
    }
  }
  for (int c = a.nc - 1; c >= 0; --c) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc_to_lds(Os, LD64, 16 * w, 16 * nt, acc[nt]);
    if (threadIdx.x < Q) er[threadIdx.x] = __expf(cumbh[c * Q + threadIdx.x]);
    __syncthreads();
    store_tile<P, 64>(a.dstates + ((((int64_t)b * a.nc + c) * a.H + h) * P) * N + ns * 64, N, Os, LD64, P);
    const int valid = min(Q, a.L - c * Q);
    stage_tile<Q, 64>(Ys, LD64, a.dy + (int64_t)b * a.sdyb + (int64_t)c * Q * a.sdyl + (int64_t)h * a.sdyh, a.sdyl,
                      valid, er);
    stage_tile<Q, 64>(Cs, LD64, a.Cm + (int64_t)b * a.sCb + (int64_t)c * Q * a.sCl + (int64_t)g * a.sCg + ns * 64,
                      a.sCl, valid);
    __syncthreads();
    const float decay = __expf(cumbh[c * Q + Q - 1]);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] *= decay;
#pragma unroll
    for (int ks = 0; ks < Q / 32; ++ks) {
      const bf16x8 A = frag_tr(Ys, LD64, 32 * ks, 16 * w);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma16(A, frag_tr(Cs, LD64, 32 * ks, 16 * nt), acc[nt]);
    }
    __syncthreads();
  }
  if (a.dinit) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * w + 4 * (l >> 4) + r, n = ns * 64 + 16 * nt + (l & 15);
        a.dinit[(((int64_t)b * a.H + h) * P + p) * N + n] = acc[nt][r];
      }
  }
}

// ============================== K4: per-chunk backward =======================================
__device__ __forceinline__ float sum16(float v) {  // over the 16 lanes l&15 of a lane group
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}
__device__ __forceinline__ float sum_groups(float v) {  // over the 4 lane groups l>>4
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

template <int N>
__global__ __launch_bounds__(256) void ssd_chunk_bwd_k(SSDArgs a) {
  constexpr int LDN = N + 8;
  constexpr int NT = N / 16;
  __shared__ __attribute__((aligned(16))) bf16_t Cs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Ss[P * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t dSs[P * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Xs[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t dYs[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t Os[Q * LD64];
  __shared__ float cumr[Q], dtr[Q], dcum[Q], ddtd[Q], red[4];
  const int c = blockIdx.x, hgi = blockIdx.y, b = blockIdx.z;
  const int h0 = hgi * a.HG, g = h0 / (a.H / a.G);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int valid = min(Q, a.L - c * Q);
  stage_tile<Q, N>(Cs, LDN, a.Cm + (int64_t)b * a.sCb + (int64_t)c * Q * a.sCl + (int64_t)g * a.sCg, a.sCl, valid);
  stage_tile<Q, N>(Bs, LDN, a.Bm + (int64_t)b * a.sBb + (int64_t)c * Q * a.sBl + (int64_t)g * a.sBg, a.sBl, valid);
  __syncthreads();
  // CB tiles for the wave's column tile (j in tile w): rows i in tile I >= w
  f32x4 cb[4], dcb[4], dBa[NT], dCa[NT];
#pragma unroll
  for (int I = 0; I < 4; ++I) {
    cb[I] = zero4();
    dcb[I] = zero4();
    if (I >= w) {
#pragma unroll
      for (int ks = 0; ks < N / 32; ++ks)
        cb[I] = mfma16(frag_kc(Cs, LDN, 16 * I, 32 * ks), frag_kc(Bs, LDN, 16 * w, 32 * ks), cb[I]);
    }
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    dBa[nt] = zero4();
    dCa[nt] = zero4();
  }
  const int jl = 16 * w + (l & 15);  // this lane's column index in the M / dM tiles
  for (int hh = 0; hh < a.HG; ++hh) {
    const int h = h0 + hh;
    const int64_t bh = ((int64_t)b * a.H + h) * a.Lp + (int64_t)c * Q;
    if (threadIdx.x < Q) {
      cumr[threadIdx.x] = a.cum[bh + threadIdx.x];
      dtr[threadIdx.x] = a.dtp[bh + threadIdx.x];
      dcum[threadIdx.x] = 0.f;
      ddtd[threadIdx.x] = 0.f;
    }
    if (threadIdx.x < 4) red[threadIdx.x] = 0.f;
    stage_tile<Q, 64>(Xs, LD64, a.x + (int64_t)b * a.sxb + (int64_t)c * Q * a.sxl + (int64_t)h * a.sxh, a.sxl, valid);
    stage_tile<Q, 64>(dYs, LD64, a.dy + (int64_t)b * a.sdyb + (int64_t)c * Q * a.sdyl + (int64_t)h * a.sdyh, a.sdyl,
                      valid);
    const int64_t soff = ((((int64_t)b * a.nc + c) * a.H + h) * P) * N;
    stage_tile<P, N>(Ss, LDN, a.states + soff, N, P);
    stage_tile<P, N>(dSs, LDN, a.dstates + soff, N, P);
    __syncthreads();
    const float cl = cumr[Q - 1];
    const float Ah = a.A[h];
    const float Dh = a.D ? a.D[h] : 0.f;
    const float dtj = dtr[jl], cumj = cumr[jl];
    // ---- (1)(2) dM, M, dCB, G row/col sums
    f32x4 m[4];
    float colG = 0.f;
#pragma unroll
    for (int I = 0; I < 4; ++I) {
      m[I] = zero4();
      if (I >= w) {
        f32x4 dm = zero4();
#pragma unroll
        for (int ks = 0; ks < P / 32; ++ks)
          dm = mfma16(frag_kc(dYs, LD64, 16 * I, 32 * ks), frag_kc(Xs, LD64, 16 * w, 32 * ks), dm);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * I + 4 * (l >> 4) + r;
          const float Lij = (jl <= i) ? __expf(cumr[i] - cumj) : 0.f;
          const float dmv = dm[r] * dtj;
          const float mv = cb[I][r] * Lij;
          m[I][r] = mv;
          dcb[I][r] += dmv * Lij;
          const float G = dmv * mv;
          colG += G;
          const float rs = sum16(G);
          if ((l & 15) == 0) atomicAdd(&dcum[i], rs);
        }
      }
    }
    colG = sum_groups(colG);
    if (l < 16) atomicAdd(&dcum[jl], -colG);
    // ---- (3) dXdt = M^T dY   and (4) BdS = B dS^T     (rows j of tile w, cols p)
    f32x4 dxd[4], bds[4];
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      dxd[pt] = zero4();
      bds[pt] = zero4();
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (2 * ks + 1 >= w) {
        const bf16x8 Af = acc_frag(m[2 * ks], m[2 * ks + 1]);
#pragma unroll
        for (int pt = 0; pt < 4; ++pt) dxd[pt] = mfma16(Af, frag_tr_perm(dYs, LD64, 32 * ks, 16 * pt), dxd[pt]);
      }
    }
#pragma unroll
    for (int ks = 0; ks < N / 32; ++ks) {
      const bf16x8 Af = frag_kc(Bs, LDN, 16 * w, 32 * ks);
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) bds[pt] = mfma16(Af, frag_kc(dSs, LDN, 16 * pt, 32 * ks), bds[pt]);
    }
    // ---- (5) dX, ddt_direct, U, dD
    float ddp[4] = {0.f, 0.f, 0.f, 0.f}, up[4] = {0.f, 0.f, 0.f, 0.f}, dDp = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * w + 4 * (l >> 4) + r;
      const float dt_ = dtr[j];
      const float ej = __expf(cl - cumr[j]);
      const float wj = ej * dt_;
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) {
        const int p = 16 * pt + (l & 15);
        const float xv = bf2f(Xs[j * LD64 + p]);
        const float dyv = bf2f(dYs[j * LD64 + p]);
        Os[j * LD64 + p] = f2bf(dt_ * dxd[pt][r] + wj * bds[pt][r] + Dh * dyv);
        ddp[r] += xv * (dxd[pt][r] + ej * bds[pt][r]);
        up[r] += wj * xv * bds[pt][r];
        dDp += xv * dyv;
      }
    }
    float usum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * w + 4 * (l >> 4) + r;
      const float dd = sum16(ddp[r]);
      const float uu = sum16(up[r]);
      if ((l & 15) == 0) {
        ddtd[j] = dd;
        atomicAdd(&dcum[j], -uu);
      }
      usum += uu;
    }
    usum = sum_groups(usum);  // every lane now holds the wave's total U over its 16 rows
    if (l == 0) atomicAdd(&dcum[Q - 1], usum);
    dDp = wave_sum(dDp);
    if (l == 0) atomicAdd(&red[0], dDp);
    // ---- (6) Yoff term of dcum: rows i of tile w
    {
      float yp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) {
        f32x4 yo = zero4();
#pragma unroll
        for (int ks = 0; ks < N / 32; ++ks)
          yo = mfma16(frag_kc(Cs, LDN, 16 * w, 32 * ks), frag_kc(Ss, LDN, 16 * pt, 32 * ks), yo);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * w + 4 * (l >> 4) + r, p = 16 * pt + (l & 15);
          yp[r] += yo[r] * bf2f(dYs[i * LD64 + p]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * w + 4 * (l >> 4) + r;
        const float s = sum16(yp[r]);
        if ((l & 15) == 0) atomicAdd(&dcum[i], s * __expf(cumr[i]));
      }
    }
    // ---- (7) dC_off += (e^{cum_i} dY) S     (8) dB_off += (w_j x) dS
    {
      const float ei = __expf(cumr[jl]);  // A-operand row index = 16w + (l&15)
      const float wl = __expf(cl - cumr[jl]) * dtr[jl];
#pragma unroll
      for (int ks = 0; ks < P / 32; ++ks) {
        const bf16x8 Ay = scale_frag(frag_kc(dYs, LD64, 16 * w, 32 * ks), ei);
        const bf16x8 Ax = scale_frag(frag_kc(Xs, LD64, 16 * w, 32 * ks), wl);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          dCa[nt] = mfma16(Ay, frag_tr(Ss, LDN, 32 * ks, 16 * nt), dCa[nt]);
          dBa[nt] = mfma16(Ax, frag_tr(dSs, LDN, 32 * ks, 16 * nt), dBa[nt]);
        }
      }
    }
    // ---- (9) e^{cl} sum(dS o S) -> dcum[last]
    {
      float s = 0.f;
      for (int v = threadIdx.x; v < P * N; v += 256) {
        const int p = v / N, n = v % N;
        s += bf2f(Ss[p * LDN + n]) * bf2f(dSs[p * LDN + n]);
      }
      s = wave_sum(s);
      if (l == 0) atomicAdd(&dcum[Q - 1], s * __expf(cl));
    }
    __syncthreads();
    store_tile<Q, 64>(a.dx + (int64_t)b * a.sdxb + (int64_t)c * Q * a.sdxl + (int64_t)h * a.sdxh, a.sdxl, Os, LD64,
                      valid);
    // ---- (10) dt gradients for this head (wave 0; lane = local step)
    if (w == 0) {
      float da = dcum[l];
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {  // reverse inclusive scan: da_i = sum_{t>=i} dcum_t
        const float y = __shfl_down(da, off, 64);
        if (l + off < 64) da += y;
      }
      const float ddt = ddtd[l] + da * Ah;
      const float dAp = wave_sum(da * dtr[l]);
      const int t = c * Q + l;
      float gdt = 0.f;
      if (t < a.L) {
        float raw = ld_any(a.dt, a.dt_dtype, (int64_t)b * a.sdtb + (int64_t)t * a.sdtl + (int64_t)h * a.sdth);
        if (a.dt_bias) raw += a.dt_bias[h];
        const float v = a.softplus ? softplusf_(raw) : raw;
        const bool inside = (v >= a.dt_min) && (v <= a.dt_max);
        gdt = inside ? ddt * (a.softplus ? sigmoidf_(raw) : 1.f) : 0.f;
        st_any(a.ddt, a.ddt_dtype, (int64_t)b * a.sddtb + (int64_t)t * a.sddtl + (int64_t)h * a.sddth, gdt);
      }
      const float dbp = wave_sum(gdt);
      if (l == 0) {
        const int64_t pi = ((int64_t)b * a.nc + c) * a.H + h;
        a.part_dA[pi] = dAp;
        a.part_dbias[pi] = dbp;
        a.part_dD[pi] = red[0];
      }
    }
    __syncthreads();
  }
  // ---- head-group partials
  const int64_t pbase = ((int64_t)b * a.nc + c) * a.nhg + hgi;
#pragma unroll
  for (int I = 0; I < 4; ++I)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * I + 4 * (l >> 4) + r;
      a.part_dcb[(pbase * Q + i) * Q + jl] = dcb[I][r];
    }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * w + 4 * (l >> 4) + r, n = 16 * nt + (l & 15);
      a.part_db[(pbase * Q + row) * N + n] = dBa[nt][r];
      a.part_dc[(pbase * Q + row) * N + n] = dCa[nt][r];
    }
}

// ============================== K5: dB / dC (backward) =======================================
template <int N>
__global__ __launch_bounds__(256) void ssd_dbc_bwd_k(SSDArgs a) {
  constexpr int LDN = N + 8;
  constexpr int NT = N / 16;
  __shared__ __attribute__((aligned(16))) bf16_t Cs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Os[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t dCBs[Q * LD64];
  const int c = blockIdx.x, g = blockIdx.y, b = blockIdx.z;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int valid = min(Q, a.L - c * Q);
  const int hpg = a.H / a.G;
  const int hg0 = g * hpg / a.HG, hg1 = (g + 1) * hpg / a.HG;
  stage_tile<Q, N>(Cs, LDN, a.Cm + (int64_t)b * a.sCb + (int64_t)c * Q * a.sCl + (int64_t)g * a.sCg, a.sCl, valid);
  stage_tile<Q, N>(Bs, LDN, a.Bm + (int64_t)b * a.sBb + (int64_t)c * Q * a.sBl + (int64_t)g * a.sBg, a.sBl, valid);
  for (int v = threadIdx.x; v < Q * Q; v += 256) {
    float s = 0.f;
    for (int hg = hg0; hg < hg1; ++hg) s += a.part_dcb[((((int64_t)b * a.nc + c) * a.nhg + hg) * Q) * Q + v];
    dCBs[(v / Q) * LD64 + v % Q] = f2bf(s);
  }
  __syncthreads();
  f32x4 dc[NT], db[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * w + 4 * (l >> 4) + r, n = 16 * nt + (l & 15);
      float sc = 0.f, sb = 0.f;
      for (int hg = hg0; hg < hg1; ++hg) {
        const int64_t o = (((((int64_t)b * a.nc + c) * a.nhg + hg) * Q) + row) * N + n;
        sc += a.part_dc[o];
        sb += a.part_db[o];
      }
      dc[nt][r] = sc;
      db[nt][r] = sb;
    }
#pragma unroll
  for (int ks = 0; ks < Q / 32; ++ks) {
    const bf16x8 Ac = frag_kc(dCBs, LD64, 16 * w, 32 * ks);  // dCB rows i, k = j
    const bf16x8 Ab = frag_tr(dCBs, LD64, 32 * ks, 16 * w);  // dCB^T rows j, k = i
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      dc[nt] = mfma16(Ac, frag_tr(Bs, LDN, 32 * ks, 16 * nt), dc[nt]);
      db[nt] = mfma16(Ab, frag_tr(Cs, LDN, 32 * ks, 16 * nt), db[nt]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc_to_lds(Os, LDN, 16 * w, 16 * nt, dc[nt]);
  __syncthreads();
  store_tile<Q, N>(a.dC + (int64_t)b * a.sdCb + (int64_t)c * Q * a.sdCl + (int64_t)g * a.sdCg, a.sdCl, Os, LDN, valid);
  __syncthreads();
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc_to_lds(Os, LDN, 16 * w, 16 * nt, db[nt]);
  __syncthreads();
  store_tile<Q, N>(a.dB + (int64_t)b * a.sdBb + (int64_t)c * Q * a.sdBl + (int64_t)g * a.sdBg, a.sdBl, Os, LDN, valid);
}

// ============================== launchers =====================================================
#define N_SWITCH(Nv, ...)                                       \
  do {                                                          \
    if ((Nv) == 128) { constexpr int NN = 128; __VA_ARGS__; }   \
    else if ((Nv) == 64) { constexpr int NN = 64; __VA_ARGS__; } \
    else return hipErrorInvalidValue;                           \
  } while (0)

hipError_t launch_ssd_fwd(const SSDArgs& a, hipStream_t st) {
  const int64_t waves = (int64_t)a.B * a.H * a.nc;
  hipLaunchKernelGGL(ssd_cumsum_k, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, a);
  MAMBA_HIP_CHECK(hipGetLastError());
  N_SWITCH(a.N, hipLaunchKernelGGL(ssd_state_fwd_k<NN>, dim3(NN / 64, a.H, a.B), dim3(256), 0, st, a));
  MAMBA_HIP_CHECK(hipGetLastError());
  N_SWITCH(a.N, hipLaunchKernelGGL(ssd_scan_fwd_k<NN>, dim3(a.nc, a.nhg, a.B), dim3(256), 0, st, a));
  return hipGetLastError();
}

hipError_t launch_ssd_bwd(const SSDArgs& a, hipStream_t st) {
  N_SWITCH(a.N, hipLaunchKernelGGL(ssd_dstate_bwd_k<NN>, dim3(NN / 64, a.H, a.B), dim3(256), 0, st, a));
  MAMBA_HIP_CHECK(hipGetLastError());
  N_SWITCH(a.N, hipLaunchKernelGGL(ssd_chunk_bwd_k<NN>, dim3(a.nc, a.nhg, a.B), dim3(256), 0, st, a));
  MAMBA_HIP_CHECK(hipGetLastError());
  N_SWITCH(a.N, hipLaunchKernelGGL(ssd_dbc_bwd_k<NN>, dim3(a.nc, a.G, a.B), dim3(256), 0, st, a));
  return hipGetLastError();
}

}  // namespace mamba_amd
