// Mamba-1 selective scan (S6), forward + backward, for gfx950.
//
//   delta = softplus(delta_raw + delta_bias)            (per channel d, step t)
//   h_t[n] = exp(delta_t A[d,n]) h_{t-1}[n] + delta_t B_t[n] u_t
//   y_t    = sum_n C_t[n] h_t[n] + D[d] u_t ;  out_t = y_t * silu(z_t)
// (upstream csrc/selective_scan)
//
// Work decomposition (MI355X-first):
//  * a 256-thread workgroup owns Kc channels of one batch row and walks them one channel at a time;
//    its 4 wavefronts split the N states (N/4 each), so every (channel, state) recurrence lives in
//    exactly one wave and the per-state cross-channel sums dB[t,n], dC[t,n] accumulate in that
//    wave's REGISTERS over the Kc channels — deterministic, no float atomics.  Sums over n (y, du,
//    ddelta) are the only cross-wave traffic: one LDS partial row per wave, one barrier.
//  * time is cut into tiles of 64 lanes x ITEMS steps; each lane composes its ITEMS steps into an
//    affine map (a, b), a wave64 Hillis-Steele scan over lanes combines the maps, and the state at
//    the tile boundary is carried in LDS per (channel, state) across tiles.
//  * backward replays the forward inside the tile from the saved tile-start states, then runs the
//    adjoint recurrence lambda_t = dy_t C_t + a_{t+1} lambda_{t+1} as a reverse wave scan.
//  * loads along time are 16-B vectors (8 x bf16) whenever the row is aligned.
#include "common.h"
#include "selective_scan.h"

namespace mamba_amd {

constexpr int SS_ITEMS = 8;
constexpr int SS_T = 64 * SS_ITEMS;

template <typename T>
__device__ __forceinline__ void load_items(const T* row, int t0, int L, bool vec, float (&o)[SS_ITEMS]) {
  if (vec && t0 + SS_ITEMS <= L) {
    ld8bf(reinterpret_cast<const bf16_t*>(row + t0), o);
  } else {
#pragma unroll
    for (int i = 0; i < SS_ITEMS; ++i) o[i] = (t0 + i < L) ? ld(row + t0 + i) : 0.f;
  }
}
template <>
__device__ __forceinline__ void load_items<float>(const float* row, int t0, int L, bool vec, float (&o)[SS_ITEMS]) {
#pragma unroll
  for (int i = 0; i < SS_ITEMS; ++i) o[i] = (t0 + i < L) ? row[t0 + i] : 0.f;
}

// inclusive scan of affine maps over the 64 lanes: (a1,b1) then (a2,b2) = (a1 a2, a2 b1 + b2)
__device__ __forceinline__ void wave_affine_scan(float& a, float& b) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float pa = __shfl_up(a, off, 64), pb = __shfl_up(b, off, 64);
    if (lane >= off) {
      b = a * pb + b;
      a = a * pa;
    }
  }
}
// reverse inclusive scan: lane i composes lanes i..63 in reverse order:
//   (a_i, b_i) after (a_{i+1}, b_{i+1}):  lambda_i = b_i + a_i * lambda_{i+1}
__device__ __forceinline__ void wave_affine_rscan(float& a, float& b) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float na = __shfl_down(a, off, 64), nb = __shfl_down(b, off, 64);
    if (lane + off < 64) {
      b = b + a * nb;
      a = a * na;
    }
  }
}

template <typename T, int N>
__global__ __launch_bounds__(256) void selscan_fwd_k(SelScanArgs a) {
  constexpr int NW = N / 4;
  __shared__ float ypart[4][SS_T];
  __shared__ float carry_s[64][N];
  const int dg = blockIdx.x, b = blockIdx.y;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int d0 = dg * a.Kc, nch = min(a.Kc, a.D - d0);
  const int ntiles = (a.L + SS_T - 1) / SS_T;
  for (int v = threadIdx.x; v < 64 * N; v += 256) carry_s[v / N][v % N] = 0.f;
  __syncthreads();
  for (int tile = 0; tile < ntiles; ++tile) {
    const int t0 = tile * SS_T;
    const int tl = t0 + lane * SS_ITEMS;
    for (int ci = 0; ci < nch; ++ci) {
      const int d = d0 + ci;
      const int g = d / (a.D / a.G);
      const T* urow = ((const T*)a.u_) + (int64_t)b * a.sub + (int64_t)d * a.sud;
      const T* drow = ((const T*)a.delta_) + (int64_t)b * a.sdb + (int64_t)d * a.sdd;
      float u[SS_ITEMS], dl[SS_ITEMS], yp[SS_ITEMS];
      load_items<T>(urow, tl, a.L, a.vec, u);
      load_items<T>(drow, tl, a.L, a.vec, dl);
      const float bias = a.delta_bias ? a.delta_bias[d] : 0.f;
#pragma unroll
      for (int i = 0; i < SS_ITEMS; ++i) {
        float v = dl[i] + bias;
        v = a.softplus ? softplusf_(v) : v;
        dl[i] = (tl + i < a.L) ? v : 0.f;
        yp[i] = 0.f;
      }
#pragma unroll
      for (int nn = 0; nn < NW; ++nn) {
        const int n = w * NW + nn;
        const float An = a.A[d * N + n];
        float Bv[SS_ITEMS], Cv[SS_ITEMS];
        load_items<T>(((const T*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g * a.sBg + (int64_t)n * a.sBn, tl, a.L, a.vecbc, Bv);
        load_items<T>(((const T*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g * a.sCg + (int64_t)n * a.sCn, tl, a.L, a.vecbc, Cv);
        float Ac[SS_ITEMS], Bc[SS_ITEMS];
        float ca = 1.f, cb = 0.f;
#pragma unroll
        for (int i = 0; i < SS_ITEMS; ++i) {
          const float ai = __expf(dl[i] * An);
          cb = ai * cb + dl[i] * Bv[i] * u[i];
          ca = ca * ai;
          Ac[i] = ca;
          Bc[i] = cb;
        }
        float sa = ca, sb = cb;
        wave_affine_scan(sa, sb);
        float ea = __shfl_up(sa, 1, 64), eb = __shfl_up(sb, 1, 64);
        if (lane == 0) { ea = 1.f; eb = 0.f; }
        const float c0 = carry_s[ci][n];
        const float hs = ea * c0 + eb;
        float hlast = 0.f;
#pragma unroll
        for (int i = 0; i < SS_ITEMS; ++i) {
          const float hi = Ac[i] * hs + Bc[i];
          yp[i] += Cv[i] * hi;
          hlast = hi;
        }
        const float cnew = __shfl(hlast, 63, 64);
        if (lane == 0) {
          if (a.carries) a.carries[(((int64_t)b * a.D + d) * ntiles + tile) * N + n] = c0;
          carry_s[ci][n] = cnew;
          if (tile == ntiles - 1 && a.last_state) a.last_state[((int64_t)b * a.D + d) * N + n] = cnew;
        }
      }
#pragma unroll
      for (int i = 0; i < SS_ITEMS; ++i) ypart[w][lane * SS_ITEMS + i] = yp[i];
      __syncthreads();
      const float Dd = a.D_ ? a.D_[d] : 0.f;
      T* orow = ((T*)a.out_) + (int64_t)b * a.sob + (int64_t)d * a.sod;
      const T* zrow = a.z_ ? ((const T*)a.z_) + (int64_t)b * a.szb + (int64_t)d * a.szd : nullptr;
      for (int k = threadIdx.x; k < SS_T; k += 256) {
        const int t = t0 + k;
        if (t < a.L) {
          float y = ypart[0][k] + ypart[1][k] + ypart[2][k] + ypart[3][k] + Dd * ld(urow + t);
          if (zrow) y *= siluf_(ld(zrow + t));
          st(orow + t, y);
        }
      }
      __syncthreads();
    }
  }
}

template <typename T, int N>
__global__ __launch_bounds__(256) void selscan_bwd_k(SelScanArgs a) {
  constexpr int NW = N / 4;
  __shared__ float ypart[4][SS_T];
  __shared__ float upart[4][SS_T];
  __shared__ float dpart[4][SS_T];
  __shared__ float lam_s[64][N];
  const int dg = blockIdx.x, b = blockIdx.y;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int d0 = dg * a.Kc, nch = min(a.Kc, a.D - d0);
  const int ntiles = (a.L + SS_T - 1) / SS_T;
  const int ndg = (a.D + a.Kc - 1) / a.Kc;
  for (int v = threadIdx.x; v < 64 * N; v += 256) lam_s[v / N][v % N] = 0.f;
  __syncthreads();
  for (int tile = ntiles - 1; tile >= 0; --tile) {
    const int t0 = tile * SS_T;
    const int tl = t0 + lane * SS_ITEMS;
    float dBa[NW][SS_ITEMS], dCa[NW][SS_ITEMS];
#pragma unroll
    for (int nn = 0; nn < NW; ++nn)
#pragma unroll
      for (int i = 0; i < SS_ITEMS; ++i) dBa[nn][i] = dCa[nn][i] = 0.f;
    for (int ci = 0; ci < nch; ++ci) {
      const int d = d0 + ci;
      const int g = d / (a.D / a.G);
      const T* urow = ((const T*)a.u_) + (int64_t)b * a.sub + (int64_t)d * a.sud;
      const T* drow = ((const T*)a.delta_) + (int64_t)b * a.sdb + (int64_t)d * a.sdd;
      const T* grow = ((const T*)a.dout_) + (int64_t)b * a.sgb + (int64_t)d * a.sgd;
      const T* zrow = a.z_ ? ((const T*)a.z_) + (int64_t)b * a.szb + (int64_t)d * a.szd : nullptr;
      float u[SS_ITEMS], dl[SS_ITEMS], dlraw[SS_ITEMS], go[SS_ITEMS], zz[SS_ITEMS];
      load_items<T>(urow, tl, a.L, a.vec, u);
      load_items<T>(drow, tl, a.L, a.vec, dlraw);
      load_items<T>(grow, tl, a.L, a.vecg, go);
      if (zrow) load_items<T>(zrow, tl, a.L, a.vecz, zz);
      const float bias = a.delta_bias ? a.delta_bias[d] : 0.f;
#pragma unroll
      for (int i = 0; i < SS_ITEMS; ++i) {
        const float v0 = dlraw[i] + bias;
        dl[i] = (tl + i < a.L) ? (a.softplus ? softplusf_(v0) : v0) : 0.f;
      }
      // ---- phase 1: replay the forward for this wave's states, keep h_{t-1}
      float hprev[NW][SS_ITEMS];
      float yp[SS_ITEMS];
#pragma unroll
      for (int i = 0; i < SS_ITEMS; ++i) yp[i] = 0.f;
#pragma unroll
      for (int nn = 0; nn < NW; ++nn) {
        const int n = w * NW + nn;
        const float An = a.A[d * N + n];
        float Bv[SS_ITEMS], Cv[SS_ITEMS];
        load_items<T>(((const T*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g * a.sBg + (int64_t)n * a.sBn, tl, a.L, a.vecbc, Bv);
        load_items<T>(((const T*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g * a.sCg + (int64_t)n * a.sCn, tl, a.L, a.vecbc, Cv);
        float Ac[SS_ITEMS], Bc[SS_ITEMS];
        float ca = 1.f, cb = 0.f;
#pragma unroll
        for (int i = 0; i < SS_ITEMS; ++i) {
          const float ai = __expf(dl[i] * An);
          cb = ai * cb + dl[i] * Bv[i] * u[i];
          ca = ca * ai;
          Ac[i] = ca;
          Bc[i] = cb;
        }
        float sa = ca, sb = cb;
        wave_affine_scan(sa, sb);
        float ea = __shfl_up(sa, 1, 64), eb = __shfl_up(sb, 1, 64);
        if (lane == 0) { ea = 1.f; eb = 0.f; }
        const float c0 = a.carries[(((int64_t)b * a.D + d) * ntiles + tile) * N + n];
        const float hs = ea * c0 + eb;
        float hp = hs;
#pragma unroll
        for (int i = 0; i < SS_ITEMS; ++i) {
          hprev[nn][i] = hp;
          const float hi = Ac[i] * hs + Bc[i];
          yp[i] += Cv[i] * hi;
          hp = hi;
        }
      }
#pragma unroll
      for (int i = 0; i < SS_ITEMS; ++i) ypart[w][lane * SS_ITEMS + i] = yp[i];
      __syncthreads();
      const float Dd = a.D_ ? a.D_[d] : 0.f;
      float dy[SS_ITEMS];
#pragma unroll
      for (int i = 0; i < SS_ITEMS; ++i) dy[i] = zrow ? go[i] * siluf_(zz[i]) : go[i];
      // ---- phase 2: adjoint recurrence per state
      float dup[SS_ITEMS], ddp[SS_ITEMS];
#pragma unroll
      for (int i = 0; i < SS_ITEMS; ++i) dup[i] = ddp[i] = 0.f;
#pragma unroll
      for (int nn = 0; nn < NW; ++nn) {
        const int n = w * NW + nn;
        const float An = a.A[d * N + n];
        float Bv[SS_ITEMS], Cv[SS_ITEMS], av[SS_ITEMS];
        load_items<T>(((const T*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g * a.sBg + (int64_t)n * a.sBn, tl, a.L, a.vecbc, Bv);
        load_items<T>(((const T*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g * a.sCg + (int64_t)n * a.sCn, tl, a.L, a.vecbc, Cv);
#pragma unroll
        for (int i = 0; i < SS_ITEMS; ++i) av[i] = __expf(dl[i] * An);
        // lane-local reverse composition: lambda_i = dyC_i + a_{i+1} lambda_{i+1}
        // map over the lane's items from the right: (A_i, B_i) with lambda_i = B_i + A_i * lambda_next
        float ra = 1.f, rb = 0.f;  // composed map of items i..ITEMS-1 wrt lambda after the lane
        float RA[SS_ITEMS], RB[SS_ITEMS];
#pragma unroll
        for (int i = SS_ITEMS - 1; i >= 0; --i) {
          const float anext = (i + 1 < SS_ITEMS) ? av[i + 1] : 1.f;  // a of the following step (in-lane)
          // lambda_i = dy_i C_i + anext * lambda_{i+1};  lambda_{i+1} = RB_{i+1} + RA_{i+1} * lam_out
          rb = dy[i] * Cv[i] + anext * rb;
          ra = anext * ra;
          RA[i] = ra;
          RB[i] = rb;
        }
        // across lanes: lam_out of lane L = a_first(L+1) * lambda_first(L+1)
        // lane map: lambda_0 = RB_0 + RA_0 * lam_out; contribution to previous lane: a0 * lambda_0
        float ma = av[0] * RA[0], mb = av[0] * RB[0];
        wave_affine_rscan(ma, mb);  // lane i: composed map for lanes i..63 (input: carry from next tile)
        float na = __shfl_down(ma, 1, 64), nb = __shfl_down(mb, 1, 64);
        if (lane == 63) { na = 1.f; nb = 0.f; }
        const float cin = lam_s[ci][n];  // a_T * lambda_T from the following tile
        const float lam_out = nb + na * cin;
        float dAp = 0.f;
#pragma unroll
        for (int i = 0; i < SS_ITEMS; ++i) {
          const float lam = RB[i] + RA[i] * lam_out;
          const float dlu = dl[i] * u[i];
          dBa[nn][i] += lam * dlu;
          const float hcur = av[i] * hprev[nn][i] + dl[i] * Bv[i] * u[i];
          dCa[nn][i] += dy[i] * hcur;
          dup[i] += lam * dl[i] * Bv[i];
          const float t1 = lam * av[i] * hprev[nn][i];
          ddp[i] += lam * u[i] * Bv[i] + An * t1;
          dAp += dl[i] * t1;
        }
        const float cnew = __shfl(mb + ma * cin, 0, 64);  // a_0 * lambda_0 of this tile (lane 0)
        dAp = wave_sum(dAp);
        if (lane == 0) {
          lam_s[ci][n] = cnew;
          a.part_dA[((int64_t)b * a.D + d) * N + n] += dAp;
        }
      }
      __syncthreads();  // ypart reads done before the partial rows are reused
#pragma unroll
      for (int i = 0; i < SS_ITEMS; ++i) {
        upart[w][lane * SS_ITEMS + i] = dup[i];
        dpart[w][lane * SS_ITEMS + i] = ddp[i];
      }
      __syncthreads();
      T* durow = ((T*)a.du_) + (int64_t)b * a.sdub + (int64_t)d * a.sdud;
      T* ddrow = ((T*)a.ddelta_) + (int64_t)b * a.sddb + (int64_t)d * a.sddd;
      T* dzrow = a.dz_ ? ((T*)a.dz_) + (int64_t)b * a.sdzb + (int64_t)d * a.sdzd : nullptr;
      float dDp = 0.f, dbp = 0.f;
      for (int k = threadIdx.x; k < SS_T; k += 256) {
        const int t = t0 + k;
        if (t < a.L) {
          const float uu = ld(urow + t);
          const float g = ld(grow + t);
          float dyv = g, y = ypart[0][k] + ypart[1][k] + ypart[2][k] + ypart[3][k] + Dd * uu;
          if (zrow) {
            const float zv = ld(zrow + t);
            const float sg = sigmoidf_(zv);
            dyv = g * zv * sg;
            if (dzrow) st(dzrow + t, g * y * sg * (1.f + zv * (1.f - sg)));
          }
          st(durow + t, upart[0][k] + upart[1][k] + upart[2][k] + upart[3][k] + Dd * dyv);
          const float raw = ld(drow + t) + bias;
          const float ddl = (dpart[0][k] + dpart[1][k] + dpart[2][k] + dpart[3][k]) *
                            (a.softplus ? sigmoidf_(raw) : 1.f);
          st(ddrow + t, ddl);
          dDp += dyv * uu;
          dbp += ddl;
        }
      }
      dDp = wave_sum(dDp);
      dbp = wave_sum(dbp);
      // per-channel partials summed over the 4 waves in a fixed order through LDS
      __syncthreads();
      if (lane == 0) {
        upart[w][0] = dDp;
        dpart[w][0] = dbp;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        a.part_dD[(int64_t)b * a.D + d] += upart[0][0] + upart[1][0] + upart[2][0] + upart[3][0];
        a.part_dbias[(int64_t)b * a.D + d] += dpart[0][0] + dpart[1][0] + dpart[2][0] + dpart[3][0];
      }
      __syncthreads();
    }
    // tile partials of dB / dC for this channel group
#pragma unroll
    for (int nn = 0; nn < NW; ++nn) {
      const int n = w * NW + nn;
      float* pb = a.part_dB + (((int64_t)b * ndg + dg) * N + n) * a.L;
      float* pc = a.part_dC + (((int64_t)b * ndg + dg) * N + n) * a.L;
#pragma unroll
      for (int i = 0; i < SS_ITEMS; ++i) {
        const int t = tl + i;
        if (t < a.L) {
          pb[t] = dBa[nn][i];
          pc[t] = dCa[nn][i];
        }
      }
    }
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

hipError_t launch_selscan_fwd(const SelScanArgs& a, hipStream_t st) {
  if (a.Kc > 64) return hipErrorInvalidValue;
  dim3 grid((a.D + a.Kc - 1) / a.Kc, a.B), block(256);
  SS_DISPATCH(hipLaunchKernelGGL((selscan_fwd_k<TT, NN>), grid, block, 0, st, a));
  return hipGetLastError();
}

int selscan_ntiles(int L) { return (L + SS_T - 1) / SS_T; }

hipError_t launch_selscan_bwd(const SelScanArgs& a, hipStream_t st) {
  if (a.Kc > 64) return hipErrorInvalidValue;
  dim3 grid((a.D + a.Kc - 1) / a.Kc, a.B), block(256);
  SS_DISPATCH(hipLaunchKernelGGL((selscan_bwd_k<TT, NN>), grid, block, 0, st, a));
  MAMBA_HIP_CHECK(hipGetLastError());
  const int64_t total = (int64_t)a.B * a.G * a.N * a.L;
  if (a.dtype == kBF16)
    hipLaunchKernelGGL(selscan_reduce_bc_k<bf16_t>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(selscan_reduce_bc_k<float>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ---- single-token state update (decode), Mamba-1 and Mamba-2 forms -------------------------
// state (b, H, P, N) fp32 [Mamba-1: H = d, P = 1]; x, z (b, H, P); dt (b, H) [Mamba-1: dt per d]
template <typename T>
__global__ void ssm_update_k(SSMUpdateArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over B*H*P
  if (i >= (int64_t)a.B * a.H * a.P) return;
  const int p = i % a.P, h = (i / a.P) % a.H, b = i / ((int64_t)a.P * a.H);
  const int g = h / (a.H / a.G);
  float dt = ld((const T*)a.dt_ + (int64_t)b * a.sdtb + (int64_t)h * a.sdth + (int64_t)p * a.sdtp);
  if (a.dt_bias) dt += a.dt_bias[a.dt_bias_per_p ? h * a.P + p : h];
  if (a.softplus) dt = softplusf_(dt);
  const float xv = ld((const T*)a.x_ + (int64_t)b * a.sxb + (int64_t)h * a.sxh + p);
  float* s = a.state + (((int64_t)b * a.H + h) * a.P + p) * a.N;
  const T* Bp = ((const T*)a.Bm_) + (int64_t)b * a.sBb + (int64_t)g * a.sBg;
  const T* Cp = ((const T*)a.Cm_) + (int64_t)b * a.sCb + (int64_t)g * a.sCg;
  float y = 0.f;
  for (int n = 0; n < a.N; ++n) {
    const float An = a.A_per_n ? a.A[(h * a.P + p) * a.N + n] : a.A[h];
    const float nv = s[n] * __expf(dt * An) + dt * xv * ld(Bp + n);
    s[n] = nv;
    y += nv * ld(Cp + n);
  }
  if (a.D) y += xv * a.D[a.D_per_p ? h * a.P + p : h];
  if (a.z_) y *= siluf_(ld(((const T*)a.z_) + (int64_t)b * a.szb + (int64_t)h * a.szh + p));
  st(((T*)a.out_) + (int64_t)b * a.H * a.P + (int64_t)h * a.P + p, y);
}

hipError_t launch_ssm_update(const SSMUpdateArgs& a, hipStream_t st) {
  const int64_t n = (int64_t)a.B * a.H * a.P;
  dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (a.dtype == kBF16) hipLaunchKernelGGL(ssm_update_k<bf16_t>, grid, block, 0, st, a);
  else if (a.dtype == kF32) hipLaunchKernelGGL(ssm_update_k<float>, grid, block, 0, st, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace mamba_amd
