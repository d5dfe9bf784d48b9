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
//   ssd_fused_fwd   WG per (h, b) walks the chunks in order with the running state in MFMA
//                   accumulators; per chunk: S_in -> HBM (saved for the backward), y = e^{cum} C S_in^T
//                   + (CB^T o L o dt)-as-A x (the masked CB^T accumulator feeds the next MFMA directly,
//                   PERM k order) + D x, then S = e^{cum_last} S + (w.X)^T B with operands through
//                   ds_read_b64_tr_b16 (token-major tiles contracted over time need the transpose).
//   ssd_dstate_bwd  reverse-time state pass: dS_out per chunk (bf16), dS_init.
//   ssd_chunk_bwd   WG per (chunk, head-group, b): dM, M, dX, ddt (incl. the in-chunk reverse cumsum
//                   of dcum), dA/dD/dbias partials; head-summed dCB, dB_off, dC_off accumulators
//                   stay in registers across the heads of the group (no per-head HBM round trip).
//   ssd_dbc_bwd     WG per (chunk, group, b): dC = sum dC_off + dCB B ; dB = sum dB_off + dCB^T C.
// No float atomics on global memory: every cross-workgroup sum goes through fixed-order partials.
#include <algorithm>
#include <cstdlib>

#include "mfma.h"
#include "ssd.h"

namespace mamba_amd {

constexpr int Q = 64;
constexpr int P = 64;
constexpr int LD64 = 80;  // padded LDS row (elements) for 64-wide bf16 tiles: conflict-free b128 / tr_perm fragment reads
constexpr float kSeqBreak = -256.f;  // e^{-256 + O(10)} == 0 in fp32

__device__ __forceinline__ float ld_any(const void* p, int dt, int64_t i) {
  return dt == kF32 ? reinterpret_cast<const float*>(p)[i] : bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
}
// Prefetch form of ld_any: two unconditional 16-bit loads (the same instruction for either dtype, no
// branch, no use of the value) so a register prefetch never forces an early s_waitcnt; raw_f()
// combines them at the point of use.
struct RawF { uint32_t lo, hi; };
__device__ __forceinline__ RawF ld_raw(const void* p, int dt, int64_t i) {
  const uint16_t* q = reinterpret_cast<const uint16_t*>(p);
  const int64_t e = dt == kF32 ? 2 * i : i;
  return {q[e], q[e + (dt == kF32 ? 1 : 0)]};
}
__device__ __forceinline__ float raw_f(RawF r, int dt) {
  return __uint_as_float(dt == kF32 ? ((r.hi << 16) | r.lo) : (r.lo << 16));
}
__device__ __forceinline__ void st_any(void* p, int dt, int64_t i, float v) {
  if (dt == kF32) reinterpret_cast<float*>(p)[i] = v;
  else reinterpret_cast<bf16_t*>(p)[i] = f2bf(v);
}

// ---- diagnostic phase timing (ssd_stamps): one wave of every workgroup (MAMBA_AMD_SSD_STAMP_WAVE, default 0)
// accumulates s_memtime deltas per phase of its
// loop and writes them (vector stores) to a host-provided buffer; the STAMPS = false kernels compile it away.
static unsigned long long* g_ssd_stamps = nullptr;  // host: (blocks, 8) u64 per stamped kernel, or null
static int64_t g_ssd_stamps_n = 0;                   // its capacity in u64; a launch that needs more runs unstamped
static int g_ssd_stamp_wave = 0;                     // the stamped wave (MAMBA_AMD_SSD_STAMP_WAVE, default 0)
void set_ssd_stamps(void* p, int64_t n) {
  g_ssd_stamps = reinterpret_cast<unsigned long long*>(p);
  g_ssd_stamps_n = p ? n : 0;
  const char* e = getenv("MAMBA_AMD_SSD_STAMP_WAVE");
  g_ssd_stamp_wave = e ? atoi(e) : 0;
}
#define SSD_STAMP(k)                                                                   \
  if constexpr (STAMPS) {                                                              \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    if (threadIdx.x == 64 * swave) {                                                   \
      const unsigned long long _n = __builtin_amdgcn_s_memtime();                      \
      st_acc[k] += _n - st_prev;                                                       \
      st_prev = _n;                                                                    \
    }                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  }
#define SSD_STAMP_INIT                                                                 \
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev = 0;               \
  if constexpr (STAMPS) { if (threadIdx.x == 64 * swave) st_prev = __builtin_amdgcn_s_memtime(); }
#define SSD_STAMP_FLUSH(blk)                                                           \
  if constexpr (STAMPS) {                                                              \
    if (threadIdx.x == 64 * swave && stamps) {                                         \
      for (int _k = 0; _k < 8; ++_k) stamps[(int64_t)(blk) * 8 + _k] = st_acc[_k];     \
    }                                                                                  \
  }

// ============================== K0: dt transform + cumsum ====================================
// One 256-thread workgroup per (b, chunk) stages the chunk's dt rows (64 steps x H heads, each step's heads
// contiguous in the in_proj output) through LDS with the threads walking the rows in order, then every wave scans
// heads w, w+4, ... (lane = step) and writes dt / cumsum rows (b, h, Lp) contiguously.  (A wave per (b, h, chunk)
// read its 64 dt values 64 row strides apart: one 128-B line per element, ~20 us per layer at 64k tokens.)
constexpr int CS_HMAX = 32;  // heads staged per pass
__global__ __launch_bounds__(256) void ssd_cumsum_k(SSDArgs a) {
  __shared__ float raw_s[Q][CS_HMAX + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x % a.nc, b = blockIdx.x / a.nc;
  const int t = c * Q + lane;
  // seq_idx: a sequence start is a decay to zero.  Adding kSeqBreak to the in-chunk cumsum makes every
  // e^{cum_i - cum_j} across the break (intra-chunk L, the decay of the carried state, the state inputs
  // of earlier tokens) underflow to exactly 0 in fp32, i.e. upstream's seq_idx masks, with no change to
  // any other term or to the backward (the offset is a constant: d cum / d dt is unchanged).
  const bool brk = a.seq && t > 0 && t < a.L &&
                   a.seq[(int64_t)b * a.sqb + (int64_t)t * a.sql] != a.seq[(int64_t)b * a.sqb + (int64_t)(t - 1) * a.sql];
  for (int h0 = 0; h0 < a.H; h0 += CS_HMAX) {
    const int nh = min(CS_HMAX, a.H - h0);
    if (h0 > 0) __syncthreads();  // the previous pass's readers are done
    {  // every element's load in flight before the first LDS store (ld_raw: branch-free, clamped row)
      constexpr int NE = (Q * CS_HMAX + 255) / 256;
      RawF rv[NE];
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        const int e = min((int)threadIdx.x + 256 * k, Q * nh - 1), r = e / nh, hh = e - r * nh;
        const int tr = min(c * Q + r, a.L - 1);
        rv[k] = ld_raw(a.dt, a.dt_dtype, (int64_t)b * a.sdtb + (int64_t)tr * a.sdtl + (int64_t)(h0 + hh) * a.sdth);
      }
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        const int e = threadIdx.x + 256 * k;
        if (e >= Q * nh) break;
        const int r = e / nh, hh = e - r * nh;
        raw_s[r][hh] = c * Q + r < a.L ? raw_f(rv[k], a.dt_dtype) : 0.f;
      }
    }
    __syncthreads();
    for (int hh = w; hh < nh; hh += 4) {
      const int h = h0 + hh;
      float v = 0.f;
      if (t < a.L) {
        float raw = raw_s[lane][hh];
        if (a.dt_bias) raw += a.dt_bias[h];
        v = a.softplus ? softplusf_(raw) : raw;
        v = fminf(fmaxf(v, a.dt_min), a.dt_max);
      }
      float x = v * (a.a_log ? -__expf(a.A[h]) : a.A[h]);
      if (brk) x += kSeqBreak;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const float y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      const int64_t o = ((int64_t)b * a.H + h) * a.Lp + t;
      a.dtp[o] = v;
      a.cum[o] = x;
    }
  }
}

// ---- register-staged tile loads (issue early, write to LDS late: latency hides under the MFMAs) ----
// one 64 x 64 bf16 tile = 512 16-B chunks; with NT threads each thread owns 512/NT chunks
template <int NT>
struct Tile64 {
  static constexpr int K = 512 / NT;
  uint4 v[K];
  int nv;  // rows >= nv are zero-filled at store time
  // Branch-free: rows past the end re-read the last valid row (always a legal address) and are
  // zeroed in store().  A `valid ? load : 0` select here makes the compiler wait for the load on
  // the spot (s_waitcnt vmcnt(0) right after issue), which serialises the whole prefetch.
  __device__ __forceinline__ void load(const bf16_t* g, int64_t gs, int valid) {
    nv = valid;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int idx = threadIdx.x + k * NT, r = min(idx >> 3, valid - 1), c = (idx & 7) * 8;
      v[k] = *reinterpret_cast<const uint4*>(g + (int64_t)r * gs + c);
    }
  }
  __device__ __forceinline__ void store(bf16_t* lds, int ld, const float* rowscale = nullptr) const {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int idx = threadIdx.x + k * NT, r = idx >> 3, c = (idx & 7) * 8;
      uint4 d = v[k];
      if (nv < 64 && r >= nv) d = make_uint4(0, 0, 0, 0);  // uniform test first: full tiles skip the selects
      if (rowscale) {
        float f[8];
        ld8bf(reinterpret_cast<const bf16_t*>(&d), f);
        const float s = rowscale[r];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= s;
        st8bf(reinterpret_cast<bf16_t*>(&d), f);
      }
      *reinterpret_cast<uint4*>(lds + r * ld + c) = d;
    }
  }
};
// a 64 x N bf16 state tile (P x N) as N/64 column blocks of Tile64
template <int NT, int N>
struct TileState {
  Tile64<NT> t[N / 64];
  __device__ __forceinline__ void load(const bf16_t* g) {
#pragma unroll
    for (int i = 0; i < N / 64; ++i) t[i].load(g + 64 * i, N, 64);
  }
  __device__ __forceinline__ void store(bf16_t* lds, int ld) const {
#pragma unroll
    for (int i = 0; i < N / 64; ++i) t[i].store(lds + 64 * i, ld);
  }
};

// ============================== K1+K2 fused: sequential chunk walk (forward) =================
// One 256-thread workgroup per (b, h) walks the chunks in order with the running state S (P x N) in
// MFMA accumulators: wave w owns state rows p in [16w, 16w+16) and output rows i in [16w, 16w+16).
// Per chunk (two barriers):
//   S_c -> LDS (bf16) and -> HBM (saved for the backward);
//   Y = e^{cum_i} C S_c^T + (CB^T o L o dt_j) X + D X        (Y rows stored by the wave that owns them)
//   S_{c+1} = e^{cl} S_c + (X o w)^T B,  w_j = e^{cl - cum_j} dt_j (applied to the X fragments in VGPRs)
// X, B, C, cum, dt of chunk c+1 are register-prefetched while chunk c computes.  Against the split
// state/scan kernels this reads X once, never re-reads the 2x-larger state tensor, and needs no
// per-head-group CB^T staging: HBM traffic ~ x + y + states instead of 2x + y + 2 states.
template <int N, bool STAMPS = false>
__global__ __launch_bounds__(256) void ssd_fused_fwd_k(SSDArgs a, unsigned long long* stamps = nullptr, int swave = 0) {
  constexpr int LDN = N + 16;  // conflict-free ds_read_b128 fragments (see LD64)
  constexpr int NTS = N / 16;  // state n-tiles per wave
  __shared__ __attribute__((aligned(16))) bf16_t Cs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Ss[P * LDN];
  constexpr int LDY = P + 8;  // Y staging: written as column pairs (acc_to_lds_pk), read as 16-B rows only
  __shared__ __attribute__((aligned(16))) bf16_t Xs[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t Os[Q * LDY];
  __shared__ __attribute__((aligned(16))) float cumr[Q], dtr[Q], wjr[Q];  // wjr = e^{cl-cum_j} dt_j
  const int h = blockIdx.x, b = blockIdx.y, sg = blockIdx.z;  // segment sg: chunks [c0, c1)
  const int c0 = sg * a.cps, c1 = min(a.nc, c0 + a.cps);
  const int g = h / (a.H / a.G);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;  // wave-uniform: scalar branches
  const int li = l & 15, lg = l >> 4;
  const int64_t bh = (int64_t)b * a.H + h;
  // the state entering the segment: initial_states for the first, the combined carry (ssd_seg_combine_k) after
  const float* ini = sg == 0 ? (a.init ? a.init + bh * P * N : nullptr)
                             : a.seg + (bh * (a.nseg - 1) + sg - 1) * P * N;
  const float* cumbh = a.cum + ((int64_t)b * a.H + h) * a.Lp;
  const float* dtbh = a.dtp + ((int64_t)b * a.H + h) * a.Lp;
  const bf16_t* xg = a.x + (int64_t)b * a.sxb + (int64_t)h * a.sxh;
  const bf16_t* bg = a.Bm + (int64_t)b * a.sBb + (int64_t)g * a.sBg;
  const bf16_t* cg = a.Cm + (int64_t)b * a.sCb + (int64_t)g * a.sCg;
  const float Dh = a.D ? a.D[h] : 0.f;
  f32x4 st[NTS];  // S rows 16w + 4lg + r, cols 16nt + li
#pragma unroll
  for (int nt = 0; nt < NTS; ++nt) {
    st[nt] = zero4();
    if (ini) {
#pragma unroll
      for (int r = 0; r < 4; ++r) st[nt][r] = ini[(16 * w + 4 * lg + r) * N + 16 * nt + li];
    }
  }
  Tile64<256> px;
  TileState<256, N> pb, pc;
  float pcum = 0.f, pdt = 0.f;
  auto prefetch = [&](int c) {
    const int valid = min(Q, a.L - c * Q);
    px.load(xg + (int64_t)c * Q * a.sxl, a.sxl, valid);
#pragma unroll
    for (int i = 0; i < N / 64; ++i) {
      pb.t[i].load(bg + (int64_t)c * Q * a.sBl + 64 * i, a.sBl, valid);
      pc.t[i].load(cg + (int64_t)c * Q * a.sCl + 64 * i, a.sCl, valid);
    }
    if (w == 0) {  // only the staging wave uses them (a wave-uniform branch: no load in the other three)
      pcum = cumbh[c * Q + l];
      pdt = dtbh[c * Q + l];
    }
  };
  // Y rows of one chunk, staged in Os by the wave that owns them (no block barrier needed)
  auto store_y_rows = [&](int cc) {
    const int row = 16 * w + (l >> 2), col = 16 * (l & 3);
    if (row < min(Q, a.L - cc * Q)) {
      bf16_t* yg = a.y + (int64_t)b * a.syb + (int64_t)(cc * Q + row) * a.syl + (int64_t)h * a.syh + col;
      *reinterpret_cast<uint4*>(yg) = *reinterpret_cast<const uint4*>(Os + row * LDY + col);
      *reinterpret_cast<uint4*>(yg + 8) = *reinterpret_cast<const uint4*>(Os + row * LDY + col + 8);
    }
  };
  prefetch(c0);
  SSD_STAMP_INIT
  for (int c = c0; c < c1; ++c) {
    __syncthreads();  // chunk c-1 is fully consumed
    SSD_STAMP(0)
    px.store(Xs, LD64);
    pb.store(Bs, LDN);
    pc.store(Cs, LDN);
    if (threadIdx.x < Q) {  // wave 0: lane = local step
      cumr[threadIdx.x] = pcum;
      dtr[threadIdx.x] = pdt;
      wjr[threadIdx.x] = __expf(__shfl(pcum, Q - 1, 64) - pcum) * pdt;
    }
#pragma unroll
    for (int nt = 0; nt < NTS; ++nt) acc_to_lds(Ss, LDN, 16 * w, 16 * nt, st[nt]);
    SSD_STAMP(1)
    __syncthreads();
    SSD_STAMP(2)
    // ---- global stores BEFORE the prefetch loads: vmcnt counts stores too and completes in order,
    // so the wait for chunk c+1's operands at the next loop top must not also wait for stores issued
    // at the end of this chunk.  Y rows of chunk c-1 (staged in Os by this same wave), then S_c.
    if (c > c0) store_y_rows(c - 1);
    {
      bf16_t* sgp = a.states + ((((int64_t)b * a.nc + c) * a.H + h) * P) * N;
#pragma unroll
      for (int q = 0; q < N / 64; ++q) {
        const int row = 16 * w + (l >> 2), col = 64 * q + 16 * (l & 3);
        *reinterpret_cast<uint4*>(sgp + (int64_t)row * N + col) = *reinterpret_cast<const uint4*>(Ss + row * LDN + col);
        *reinterpret_cast<uint4*>(sgp + (int64_t)row * N + col + 8) =
            *reinterpret_cast<const uint4*>(Ss + row * LDN + col + 8);
      }
    }
    if (c + 1 < c1) prefetch(c + 1);
    SSD_STAMP(3)
    const float cl = cumr[Q - 1];
    // ---- Y_off = e^{cum_i} C_i . S_c^T   (rows i of tile w, 4 p-tiles)
    f32x4 acc[4];
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      acc[pt] = zero4();
#pragma unroll
      for (int ks = 0; ks < N / 32; ++ks)
        acc[pt] = mfma16(frag_kc(Cs, LDN, 16 * w, 32 * ks), frag_kc(Ss, LDN, 16 * pt, 32 * ks), acc[pt]);
    }
    {
      const float4 ci = *reinterpret_cast<const float4*>(&cumr[16 * w + 4 * lg]);
      const float e[4] = {__expf(ci.x), __expf(ci.y), __expf(ci.z), __expf(ci.w)};
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int pt = 0; pt < 4; ++pt) acc[pt][r] *= e[r];
    }
    SSD_STAMP(4)
    // ---- Y_diag: CB^T tiles (rows j of tile jt <= w, cols i of tile w), masked, decayed, x dt_j
    const int i_col = 16 * w + li;
    const float cum_i = cumr[i_col];
    f32x4 mt[4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      mt[jt] = zero4();
      if (jt <= w) {
        f32x4 cb = zero4();
#pragma unroll
        for (int ks = 0; ks < N / 32; ++ks)
          cb = mfma16(frag_kc(Bs, LDN, 16 * jt, 32 * ks), frag_kc(Cs, LDN, 16 * w, 32 * ks), cb);
        const float4 cj4 = *reinterpret_cast<const float4*>(&cumr[16 * jt + 4 * lg]);
        const float4 dj4 = *reinterpret_cast<const float4*>(&dtr[16 * jt + 4 * lg]);
        const float cj[4] = {cj4.x, cj4.y, cj4.z, cj4.w}, dj[4] = {dj4.x, dj4.y, dj4.z, dj4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = 16 * jt + 4 * lg + r;
          mt[jt][r] = (j <= i_col) ? cb[r] * __expf(cum_i - cj[r]) * dj[r] : 0.f;
        }
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (2 * ks <= w) {
        const bf16x8 A = acc_frag(mt[2 * ks], mt[2 * ks + 1]);
#pragma unroll
        for (int pt = 0; pt < 4; ++pt) acc[pt] = mfma16(A, frag_tr_perm(Xs, LD64, 32 * ks, 16 * pt), acc[pt]);
      }
    }
    SSD_STAMP(5)
    // ---- + D x, stage this wave's 16 rows, store them (no block barrier: same-wave LDS order)
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const bf16x4 xr = acc_rows4(Xs, LD64, 16 * w, 16 * pt);
      f32x4 yv;
#pragma unroll
      for (int r = 0; r < 4; ++r) yv[r] = acc[pt][r] + Dh * (float)xr[r];
      acc_to_lds_pk(Os, LDY, 16 * w, 16 * pt, yv);
    }
    SSD_STAMP(6)
    // ---- S_{c+1} = e^{cl} S_c + (X o w)^T B
    const float decay = __expf(cl);
#pragma unroll
    for (int nt = 0; nt < NTS; ++nt) st[nt] *= decay;
#pragma unroll
    for (int ks = 0; ks < Q / 32; ++ks) {
      bf16x8 A = frag_tr(Xs, LD64, 32 * ks, 16 * w);  // A[p][k=j], j = 32ks + 8lg + jj
      const float4 w0 = *reinterpret_cast<const float4*>(&wjr[32 * ks + 8 * lg]);
      const float4 w1 = *reinterpret_cast<const float4*>(&wjr[32 * ks + 8 * lg + 4]);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) A[jj] = (__bf16)((float)A[jj] * wv[jj]);
#pragma unroll
      for (int nt = 0; nt < NTS; ++nt) st[nt] = mfma16(A, frag_tr(Bs, LDN, 32 * ks, 16 * nt), st[nt]);
    }
    SSD_STAMP(7)
  }
  SSD_STAMP_FLUSH(blockIdx.y * gridDim.x + blockIdx.x)
  store_y_rows(c1 - 1);
  if (a.final_state && sg == a.nseg - 1) {
#pragma unroll
    for (int nt = 0; nt < NTS; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        a.final_state[(((int64_t)b * a.H + h) * P + 16 * w + 4 * lg + r) * N + 16 * nt + li] = st[nt][r];
  }
}

// ============================== K3: reverse state pass (backward) ===========================
// WG per (h, b) walks the chunks from the last: dS_out(c) -> HBM (bf16), then
// dS = e^{cum_last} dS + (e^{cum} dY)^T C.  All N columns per workgroup, so each dY tile is read once.
template <int N>
__global__ __launch_bounds__(256) void ssd_dstate_bwd_k(SSDArgs a) {
  constexpr int LDN = N + 16;
  constexpr int LDO = N + 8;  // dS staging: written as column pairs (acc_to_lds_pk), read as 16-B rows only
  constexpr int NTS = N / 16;
  __shared__ __attribute__((aligned(16))) bf16_t Ys[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t Cs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Os[P * LDO];
  __shared__ float er[Q];
  const int h = blockIdx.x, b = blockIdx.y, sg = blockIdx.z;  // segment sg: chunks [c0, c1), walked from c1 - 1
  const int c0 = sg * a.cps, c1 = min(a.nc, c0 + a.cps);
  const int g = h / (a.H / a.G);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;  // wave-uniform: scalar branches
  const int64_t bh = (int64_t)b * a.H + h;
  const float* cumbh = a.cum + ((int64_t)b * a.H + h) * a.Lp;
  const bf16_t* yg = a.dy + (int64_t)b * a.sdyb + (int64_t)h * a.sdyh;
  const bf16_t* cg = a.Cm + (int64_t)b * a.sCb + (int64_t)g * a.sCg;
  // the gradient entering the segment from the right: dfinal for the last, the combined carry before
  const float* ini = sg == a.nseg - 1 ? (a.dfinal ? a.dfinal + bh * P * N : nullptr)
                                      : a.seg + (bh * (a.nseg - 1) + sg) * P * N;
  f32x4 acc[NTS];
#pragma unroll
  for (int nt = 0; nt < NTS; ++nt) {
    acc[nt] = zero4();
    if (ini) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * w + 4 * (l >> 4) + r, n = 16 * nt + (l & 15);
        acc[nt][r] = ini[p * N + n];
      }
    }
  }
  Tile64<256> py;
  TileState<256, N> pcs;
  float pe = 0.f, pl = 0.f;
  auto prefetch = [&](int c) {
    pl = cumbh[c * Q + Q - 1];
    const int valid = min(Q, a.L - c * Q);
    py.load(yg + (int64_t)c * Q * a.sdyl, a.sdyl, valid);
#pragma unroll
    for (int i = 0; i < N / 64; ++i) pcs.t[i].load(cg + (int64_t)c * Q * a.sCl + 64 * i, a.sCl, valid);
    pe = cumbh[c * Q + (threadIdx.x & 63)];  // exp at use: no ALU on a value still in flight
  };
  prefetch(c1 - 1);
  for (int c = c1 - 1; c >= c0; --c) {
#pragma unroll
    for (int nt = 0; nt < NTS; ++nt) acc_to_lds_pk(Os, LDO, 16 * w, 16 * nt, acc[nt]);
    if (threadIdx.x < Q) er[threadIdx.x] = __expf(pe);
    const float decay = __expf(pl);
    __syncthreads();
    // operands first (waits for the loads issued last chunk), then this chunk's stores, then the next
    // loads: vmcnt completes in order, so stores issued before a wait would be waited for too
    py.store(Ys, LD64, er);
    pcs.store(Cs, LDN);
    store_tile<P, N>(a.dstates + ((((int64_t)b * a.nc + c) * a.H + h) * P) * N, N, Os, LDO, P);
    if (c > c0) prefetch(c - 1);
    __syncthreads();
#pragma unroll
    for (int nt = 0; nt < NTS; ++nt) acc[nt] *= decay;
#pragma unroll
    for (int ks = 0; ks < Q / 32; ++ks) {
      const bf16x8 A = frag_tr(Ys, LD64, 32 * ks, 16 * w);
#pragma unroll
      for (int nt = 0; nt < NTS; ++nt) acc[nt] = mfma16(A, frag_tr(Cs, LDN, 32 * ks, 16 * nt), acc[nt]);
    }
  }
  if (a.dinit && sg == 0) {
#pragma unroll
    for (int nt = 0; nt < NTS; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * w + 4 * (l >> 4) + r, n = 16 * nt + (l & 15);
        a.dinit[(((int64_t)b * a.H + h) * P + p) * N + n] = acc[nt][r];
      }
  }
}

// ============================== segment-parallel state walks (small b * H) ====================
// At 2.8B / T = 8192 (b = 4, H = 80) the forward and reverse walks are 320 workgroups of 128 chunks on 256 CUs that
// hold two of them each: the kernel time is one workgroup's serial walk.  With nseg segments of cps chunks:
//   ssd_seg_state_k    (h, b, segment < nseg - 1): the segment's state contribution from a zero state,
//                      S = e^{cl} S + (X o w)^T B per chunk (no y, no C, no per-chunk stores), and its summed
//                      log-decay D = sum cl;
//   ssd_seg_combine_k  (h, b): S_in(s + 1) = e^{D_s} S_in(s) + L_s carried through the segments (fp32, in place);
//   ssd_fused_fwd_k    (h, b, segment): the full walk over the segment's chunks from S_in(segment).
// The backward mirrors it: ssd_seg_dstate_k walks segments 1 .. nseg - 1 in reverse from zero, the combine carries
// right to left, and ssd_dstate_bwd_k walks every segment from its carried-in gradient.  Exact in real arithmetic:
// both recurrences are linear in the carried state and a segment's decay is the scalar e^{D} (A is per head).
template <int N>
__global__ __launch_bounds__(256) void ssd_seg_state_k(SSDArgs a) {
  constexpr int LDN = N + 16, NTS = N / 16;
  __shared__ __attribute__((aligned(16))) bf16_t Bs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Xs[Q * LD64];
  __shared__ __attribute__((aligned(16))) float wjr[Q];
  const int h = blockIdx.x, b = blockIdx.y, sg = blockIdx.z;
  const int c0 = sg * a.cps, c1 = min(a.nc, c0 + a.cps);
  const int g = h / (a.H / a.G);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  const int li = l & 15, lg = l >> 4;
  const int64_t bh = (int64_t)b * a.H + h;
  const float* cumbh = a.cum + bh * a.Lp;
  const float* dtbh = a.dtp + bh * a.Lp;
  const bf16_t* xg = a.x + (int64_t)b * a.sxb + (int64_t)h * a.sxh;
  const bf16_t* bg = a.Bm + (int64_t)b * a.sBb + (int64_t)g * a.sBg;
  f32x4 st[NTS];
#pragma unroll
  for (int nt = 0; nt < NTS; ++nt) st[nt] = zero4();
  Tile64<256> px;
  TileState<256, N> pb;
  float pcum = 0.f, pdt = 0.f;
  auto prefetch = [&](int c) {
    const int valid = min(Q, a.L - c * Q);
    px.load(xg + (int64_t)c * Q * a.sxl, a.sxl, valid);
#pragma unroll
    for (int i = 0; i < N / 64; ++i) pb.t[i].load(bg + (int64_t)c * Q * a.sBl + 64 * i, a.sBl, valid);
    pcum = cumbh[c * Q + l];
    pdt = dtbh[c * Q + l];
  };
  float dsum = 0.f;
  prefetch(c0);
  for (int c = c0; c < c1; ++c) {
    __syncthreads();  // chunk c-1 is consumed
    px.store(Xs, LD64);
    pb.store(Bs, LDN);
    const float cl = __shfl(pcum, Q - 1, 64);
    if (w == 0) wjr[l] = __expf(cl - pcum) * pdt;
    __syncthreads();
    if (c + 1 < c1) prefetch(c + 1);
    dsum += cl;
    const float decay = __expf(cl);
#pragma unroll
    for (int nt = 0; nt < NTS; ++nt) st[nt] *= decay;
#pragma unroll
    for (int ks = 0; ks < Q / 32; ++ks) {
      bf16x8 A = frag_tr(Xs, LD64, 32 * ks, 16 * w);
      const float4 w0 = *reinterpret_cast<const float4*>(&wjr[32 * ks + 8 * lg]);
      const float4 w1 = *reinterpret_cast<const float4*>(&wjr[32 * ks + 8 * lg + 4]);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) A[jj] = (__bf16)((float)A[jj] * wv[jj]);
#pragma unroll
      for (int nt = 0; nt < NTS; ++nt) st[nt] = mfma16(A, frag_tr(Bs, LDN, 32 * ks, 16 * nt), st[nt]);
    }
  }
  float* out = a.seg + (bh * (a.nseg - 1) + sg) * P * N;
#pragma unroll
  for (int nt = 0; nt < NTS; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(16 * w + 4 * lg + r) * N + 16 * nt + li] = st[nt][r];
  if (threadIdx.x == 0) a.segd[bh * (a.nseg - 1) + sg] = dsum;
}

// reverse walk of segment blockIdx.z + 1 from a zero gradient: dS = e^{cl} dS + (e^{cum} dY)^T C per chunk
template <int N>
__global__ __launch_bounds__(256) void ssd_seg_dstate_k(SSDArgs a) {
  constexpr int LDN = N + 16, NTS = N / 16;
  __shared__ __attribute__((aligned(16))) bf16_t Ys[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t Cs[Q * LDN];
  __shared__ float er[Q];
  const int h = blockIdx.x, b = blockIdx.y, sg = blockIdx.z + 1;
  const int c0 = sg * a.cps, c1 = min(a.nc, c0 + a.cps);
  const int g = h / (a.H / a.G);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  const int64_t bh = (int64_t)b * a.H + h;
  const float* cumbh = a.cum + bh * a.Lp;
  const bf16_t* yg = a.dy + (int64_t)b * a.sdyb + (int64_t)h * a.sdyh;
  const bf16_t* cg = a.Cm + (int64_t)b * a.sCb + (int64_t)g * a.sCg;
  f32x4 acc[NTS];
#pragma unroll
  for (int nt = 0; nt < NTS; ++nt) acc[nt] = zero4();
  Tile64<256> py;
  TileState<256, N> pcs;
  float pe = 0.f, pl = 0.f;
  auto prefetch = [&](int c) {
    pl = cumbh[c * Q + Q - 1];
    const int valid = min(Q, a.L - c * Q);
    py.load(yg + (int64_t)c * Q * a.sdyl, a.sdyl, valid);
#pragma unroll
    for (int i = 0; i < N / 64; ++i) pcs.t[i].load(cg + (int64_t)c * Q * a.sCl + 64 * i, a.sCl, valid);
    pe = cumbh[c * Q + l];
  };
  float dsum = 0.f;
  prefetch(c1 - 1);
  for (int c = c1 - 1; c >= c0; --c) {
    __syncthreads();  // chunk c+1 is consumed (Ys, Cs and er)
    if (threadIdx.x < Q) er[threadIdx.x] = __expf(pe);
    const float cl = pl;
    __syncthreads();
    py.store(Ys, LD64, er);
    pcs.store(Cs, LDN);
    if (c > c0) prefetch(c - 1);
    __syncthreads();
    dsum += cl;
    const float decay = __expf(cl);
#pragma unroll
    for (int nt = 0; nt < NTS; ++nt) acc[nt] *= decay;
#pragma unroll
    for (int ks = 0; ks < Q / 32; ++ks) {
      const bf16x8 A = frag_tr(Ys, LD64, 32 * ks, 16 * w);
#pragma unroll
      for (int nt = 0; nt < NTS; ++nt) acc[nt] = mfma16(A, frag_tr(Cs, LDN, 32 * ks, 16 * nt), acc[nt]);
    }
  }
  float* out = a.seg + (bh * (a.nseg - 1) + sg - 1) * P * N;
#pragma unroll
  for (int nt = 0; nt < NTS; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(16 * w + 4 * (l >> 4) + r) * N + 16 * nt + (l & 15)] = acc[nt][r];
  if (threadIdx.x == 0) a.segd[bh * (a.nseg - 1) + sg - 1] = dsum;
}

// (h, b): carry the segment states through the segments in place.  fwd: slot s holds L_s (segment s's local state,
// decay D_s) and becomes S_in(s + 1), starting from initial_states; bwd: slot s holds segment s + 1's local gradient
// (decay D_{s+1}) and becomes the gradient entering segment s from the right, starting from dfinal.
constexpr int SEG_MAX = 16;
__global__ __launch_bounds__(256) void ssd_seg_combine_k(SSDArgs a, int fwd) {
  const int h = blockIdx.x, b = blockIdx.y;
  const int64_t bh = (int64_t)b * a.H + h;
  const int ns = a.nseg - 1, PN = P * a.N;
  float* base = a.seg + bh * ns * PN;
  const float* dec = a.segd + bh * ns;
  const float* first = fwd ? a.init : a.dfinal;
  float d[SEG_MAX];
#pragma unroll
  for (int k = 0; k < SEG_MAX; ++k) d[k] = k < ns ? __expf(dec[fwd ? k : ns - 1 - k]) : 0.f;
  for (int e = 4 * threadIdx.x; e < PN; e += 4 * 256) {
    float4 v[SEG_MAX];
#pragma unroll
    for (int k = 0; k < SEG_MAX; ++k)
      if (k < ns) v[k] = *reinterpret_cast<const float4*>(base + (int64_t)(fwd ? k : ns - 1 - k) * PN + e);
    float4 cy = first ? *reinterpret_cast<const float4*>(first + bh * PN + e) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < SEG_MAX; ++k) {
      if (k < ns) {
        cy = make_float4(fmaf(d[k], cy.x, v[k].x), fmaf(d[k], cy.y, v[k].y), fmaf(d[k], cy.z, v[k].z),
                         fmaf(d[k], cy.w, v[k].w));
        *reinterpret_cast<float4*>(base + (int64_t)(fwd ? k : ns - 1 - k) * PN + e) = cy;
      }
    }
  }
}

// ============================== K4: per-chunk backward =======================================
// 512 threads: wave w4 = wid & 3 owns row/column tile w4 of the 64x64 chunk matrices; the two
// halves (wid >> 2) split the p-tiles (dX, BdS, Yoff) and the n-tiles (dB/dC accumulators).  The
// M / dM tiles of column w4 are computed by both halves (cheap: 2 MFMAs per tile) so neither has to
// wait for the other; only half 0 accumulates dCB and the G row/col sums.
template <int N, bool STAMPS = false>
__global__ __launch_bounds__(512) void ssd_chunk_bwd_k(SSDArgs a, unsigned long long* stamps = nullptr, int swave = 0) {
  constexpr int LDN = N + 16;  // conflict-free ds_read_b128 fragments (see LD64)
  constexpr int NT = N / 16;
  constexpr int NTH = NT / 2;
  __shared__ __attribute__((aligned(16))) bf16_t Cs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Ss[P * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t dSs[P * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Xs[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t dYs[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t Os[Q * LD64];
  __shared__ __attribute__((aligned(16))) bf16_t MsT[Q * LD64];  // M^T [j][i] of the current head
  // per-head dt-gradient inputs, kept for all heads of the group so step (10) runs once at the end
  // with one wave per head instead of serialising wave 0 inside the head loop
  // Every cross-lane partial goes to a slot owned by ONE wave (plain read-modify-write in program
  // order) and the slots are summed in a fixed order in (10): deterministic, no LDS float atomics.
  __shared__ __attribute__((aligned(16))) float cumr[Q], dtr[8][Q], rawl[8][Q];
  // per-step decay factors of the current head, computed once by the staging lanes instead of by all 16 lanes of
  // every row group: eir = e^{cum_t}, ejr = e^{cl - cum_t}
  __shared__ __attribute__((aligned(16))) float eir[Q], ejr[Q];
  __shared__ __attribute__((aligned(16))) float dcw[8][8][Q];   // [head][wave][step]  dcum contributions
  __shared__ __attribute__((aligned(16))) float ddw[8][2][Q];   // [head][half][step]  direct ddt contributions
  __shared__ float redw[8][8];     // [head][wave]        dD
  const int c = blockIdx.x, hgi = blockIdx.y, b = blockIdx.z;
  const int h0 = hgi * a.HG, g = h0 / (a.H / a.G);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;  // wave-uniform: scalar branches
  const int w = wid & 3, half = wid >> 2;
  const int li = l & 15, lg = l >> 4;
  const int valid = min(Q, a.L - c * Q);
  Tile64<512> px, py;
  TileState<512, N> ps, pds;
  float pc = 0.f, pd = 0.f;
  RawF praw;
  const int tl = min(c * Q + (int)(threadIdx.x & 63), a.L - 1);  // clamped: the loads below never branch
  // the next head's operands in three groups (x / dY / dt rows, S, dS): issued together, the 8 waves' 10 loads each
  // queue behind one another in the vector-memory pipe and the younger half (waves 4-7) stalled ~1.2k cycles per
  // head issuing them (per-wave s_memtime stamps); spread over the compute phases they issue under the MFMAs
  auto prefetch_a = [&](int h) {
    px.load(a.x + (int64_t)b * a.sxb + (int64_t)c * Q * a.sxl + (int64_t)h * a.sxh, a.sxl, valid);
    praw = ld_raw(a.dt, a.dt_dtype, (int64_t)b * a.sdtb + (int64_t)tl * a.sdtl + (int64_t)h * a.sdth);
    py.load(a.dy + (int64_t)b * a.sdyb + (int64_t)c * Q * a.sdyl + (int64_t)h * a.sdyh, a.sdyl, valid);
    {
      const int64_t bh = ((int64_t)b * a.H + h) * a.Lp + (int64_t)c * Q + (threadIdx.x & 63);
      pc = a.cum[bh];
      pd = a.dtp[bh];
    }
  };
  auto prefetch_s = [&](int h) { ps.load(a.states + ((((int64_t)b * a.nc + c) * a.H + h) * P) * N); };
  auto prefetch_ds = [&](int h) { pds.load(a.dstates + ((((int64_t)b * a.nc + c) * a.H + h) * P) * N); };
  prefetch_a(h0);
  prefetch_s(h0);
  prefetch_ds(h0);
  for (int v = threadIdx.x; v < 8 * 8 * Q; v += 512) (&dcw[0][0][0])[v] = 0.f;
  for (int v = threadIdx.x; v < 8 * 2 * Q; v += 512) (&ddw[0][0][0])[v] = 0.f;
  {  // both tiles' loads in flight before the first LDS store
    StageRegs<Q, N, 512> sc, sb;
    sc.load(a.Cm + (int64_t)b * a.sCb + (int64_t)c * Q * a.sCl + (int64_t)g * a.sCg, a.sCl, valid);
    sb.load(a.Bm + (int64_t)b * a.sBb + (int64_t)c * Q * a.sBl + (int64_t)g * a.sBg, a.sBl, valid);
    sc.store(Cs, LDN);
    sb.store(Bs, LDN);
  }
  // (1)(2) tile ownership: the 10 lower-triangular 16x16 tiles (I >= J) of M / dM go to the 8 waves
  // (waves 0 and 1 take two diagonal tiles each) -- no tile is computed twice and the busiest wave has
  // 2 tiles (a column-tile split gives 4:3:2:1).  M^T goes through LDS to the waves that need it in (3).
  // Waves 2..7 also own one of the 6 all-zero upper tiles (zeroed in MsT once, written to part_dcb).
  // wid:   0          1          2     3     4     5     6     7
  // owns:  (0,0)(3,3) (1,1)(2,2) (1,0) (2,0) (3,0) (2,1) (3,1) (3,2);  zero tile of wid 2..7:
  //                               (0,1) (0,2) (0,3) (1,2) (1,3) (2,3)      (nibble tables, no scratch)
  const int own = wid < 2 ? 2 : 1;
  const int tI[2] = {(0x33232110 >> (4 * wid)) & 15, wid == 0 ? 3 : 2};
  const int tJ[2] = {(0x21100010 >> (4 * wid)) & 15, wid == 0 ? 3 : 2};
  const int zI = (0x21100000 >> (4 * wid)) & 15, zJ = (0x33232100 >> (4 * wid)) & 15;
  if (wid >= 2)
    *reinterpret_cast<uint2*>(MsT + (16 * zJ + li) * LD64 + 16 * zI + 4 * lg) = make_uint2(0u, 0u);
  __syncthreads();
  f32x4 cbo[2], dcbo[2], dBa[NTH], dCa[NTH];  // C.B^T and the dCB accumulators of the owned tiles
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    cbo[k] = zero4();
    dcbo[k] = zero4();
    if (k < own) {
#pragma unroll
      for (int ks = 0; ks < N / 32; ++ks)
        cbo[k] = mfma16(frag_kc(Cs, LDN, 16 * tI[k], 32 * ks), frag_kc(Bs, LDN, 16 * tJ[k], 32 * ks), cbo[k]);
    }
  }
#pragma unroll
  for (int nt = 0; nt < NTH; ++nt) {
    dBa[nt] = zero4();
    dCa[nt] = zero4();
  }
  // ---- (10) dt gradients for a batch of up to 8 heads, one wave per head (lane = local step);
  // the per-head slots form a ring of 8 so any head-group size fits in LDS
  auto flush = [&](int first, int cnt) {
    __syncthreads();  // every wave's slot contributions for these heads are written
    if (wid < cnt) {
      const int hh = first + wid, h = h0 + hh, sl = hh & 7;
      const float Ah = a.a_log ? -__expf(a.A[h]) : a.A[h];
      float da = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) da += dcw[sl][v][l];
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {  // reverse inclusive scan: da_i = sum_{t>=i} dcum_t
        const float y = __shfl_down(da, off, 64);
        if (l + off < 64) da += y;
      }
      const float ddt = (ddw[sl][0][l] + ddw[sl][1][l]) + da * Ah;
      const float dAp = wave_sum(da * dtr[sl][l]);
      const int t = c * Q + l;
      float gdt = 0.f;
      if (t < a.L) {
        float raw = rawl[sl][l];
        if (a.dt_bias) raw += a.dt_bias[h];
        const float v = a.softplus ? softplusf_(raw) : raw;
        const bool inside = (v >= a.dt_min) && (v <= a.dt_max);
        gdt = inside ? ddt * (a.softplus ? sigmoidf_(raw) : 1.f) : 0.f;
        st_any(a.ddt, a.ddt_dtype, (int64_t)b * a.sddtb + (int64_t)t * a.sddtl + (int64_t)h * a.sddth, gdt);
        if (a.ddt_zero_pad && h == 0) {  // the row's pad columns past the H dt columns: 16-B stores (host-checked)
          bf16_t* pr = reinterpret_cast<bf16_t*>(a.ddt) + (int64_t)b * a.sddtb + (int64_t)t * a.sddtl + a.H;
          for (int k = 0; k < a.ddt_zero_pad; k += 8) *reinterpret_cast<uint4*>(pr + k) = make_uint4(0u, 0u, 0u, 0u);
        }
      }
      const float dbp = wave_sum(gdt);
      if (l == 0) {
        const int64_t pi = ((int64_t)b * a.nc + c) * a.psl + h;
        const float pa = a.a_log ? dAp * Ah : dAp;  // d/dA_log = dA * A
        float dd = 0.f;
#pragma unroll
        for (int v = 0; v < 8; ++v) dd += redw[sl][v];
        if (a.pacc) {
          a.part_dA[pi] += pa; a.part_dbias[pi] += dbp; a.part_dD[pi] += dd;
        } else {
          a.part_dA[pi] = pa; a.part_dbias[pi] = dbp; a.part_dD[pi] = dd;
        }
      }
      // recycle this head's slots for head hh + 8 (the next head's top barrier orders it)
#pragma unroll
      for (int v = 0; v < 8; ++v) dcw[sl][v][l] = 0.f;
      ddw[sl][0][l] = 0.f;
      ddw[sl][1][l] = 0.f;
    }
  };
  const int jl = 16 * w + li;  // this lane's column index in the M / dM tiles
  // causal mask of the owned tiles as an additive exponent offset (0 or -inf: e^{d - inf} = 0 for any finite d):
  // a select on (jt <= i) is loop-invariant, so hipcc hoists its 64-bit lane masks out of the head loop, runs out
  // of SGPRs and spills them to VGPR lanes; the offsets come from one VGPR of mask bits instead
  // bit 4k + r set: element (row 4 lg + r, column li) of owned tile k is above the diagonal (one VGPR for all 8)
  unsigned mbits = 0u;
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      mbits |= (16 * tJ[k] + li <= 16 * tI[k] + 4 * lg + r) ? 0u : (1u << (4 * k + r));
  SSD_STAMP_INIT
  for (int hh = 0; hh < a.HG; ++hh) {
    const int h = h0 + hh;
    __syncthreads();  // previous head fully consumed (LDS tiles, dcum, Os)
    SSD_STAMP(0)
    if (threadIdx.x < Q) {
      cumr[threadIdx.x] = pc;
      dtr[hh & 7][threadIdx.x] = pd;
      rawl[hh & 7][threadIdx.x] = raw_f(praw, a.dt_dtype);
      eir[threadIdx.x] = __expf(pc);
      ejr[threadIdx.x] = __expf(__shfl(pc, Q - 1, 64) - pc);
    }
    px.store(Xs, LD64);
    py.store(dYs, LD64);
    ps.store(Ss, LDN);
    pds.store(dSs, LDN);
    SSD_STAMP(1)
    __syncthreads();
    if (hh + 1 < a.HG) prefetch_a(h + 1);
    SSD_STAMP(2)
    const float cl = cumr[Q - 1];
    const float Ah = a.a_log ? -__expf(a.A[h]) : a.A[h];
    const float Dh = a.D ? a.D[h] : 0.f;
    // ---- (1)(2) dM, M of the owned tiles: dCB, the G row/col sums, M^T -> LDS
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k < own) {
        const int I = tI[k], jt = 16 * tJ[k] + li;
        const float dtj = dtr[hh & 7][jt], cumj = cumr[jt];
        f32x4 dm = zero4();
#pragma unroll
        for (int ks = 0; ks < P / 32; ++ks)
          dm = mfma16(frag_kc(dYs, LD64, 16 * I, 32 * ks), frag_kc(Xs, LD64, 16 * tJ[k], 32 * ks), dm);
        float gr[4], mv[4], colG = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * I + 4 * lg + r;
          const float moff = __uint_as_float((0u - ((mbits >> (4 * k + r)) & 1u)) & 0xFF800000u);  // 0 or -inf
          const float Lij = __expf(cumr[i] - cumj + moff);
          const float dmv = dm[r] * dtj;
          mv[r] = cbo[k][r] * Lij;
          dcbo[k][r] += dmv * Lij;
          gr[r] = dmv * mv[r];
          colG += gr[r];
        }
        // the 4 row sums of this lane group's rows as ONE 16-B read-modify-write (4 scalar ones serialise:
        // hipcc cannot tell the slots apart and waits for each read before the next)
        float rs[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) rs[r] = row_sum16(gr[r]);
        if (li == 0) {
          float4* pr = reinterpret_cast<float4*>(&dcw[hh & 7][wid][16 * I + 4 * lg]);
          float4 o = *pr;
          o.x += rs[0]; o.y += rs[1]; o.z += rs[2]; o.w += rs[3];
          *pr = o;
        }
        colG = rows_sum4(colG);
        if (l < 16) dcw[hh & 7][wid][jt] -= colG;
        *reinterpret_cast<uint2*>(MsT + jt * LD64 + 16 * I + 4 * lg) = make_uint2(pack2(mv[0], mv[1]), pack2(mv[2], mv[3]));
      }
    }
    if (hh + 1 < a.HG) prefetch_s(h + 1);
    SSD_STAMP(3)
    // ---- (4) BdS = B dS^T, (6) Yoff = C S^T for this half's p-tiles (independent of M: they fill the
    // wait for the M^T barrier), then (3) dXdt = M^T dY
    f32x4 dxd[2], bds[2], yo[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      dxd[q] = zero4();
      bds[q] = zero4();
      yo[q] = zero4();
    }
#pragma unroll
    for (int ks = 0; ks < N / 32; ++ks) {
      const bf16x8 Ab = frag_kc(Bs, LDN, 16 * w, 32 * ks);
      const bf16x8 Ac = frag_kc(Cs, LDN, 16 * w, 32 * ks);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        bds[q] = mfma16(Ab, frag_kc(dSs, LDN, 16 * (2 * half + q), 32 * ks), bds[q]);
        yo[q] = mfma16(Ac, frag_kc(Ss, LDN, 16 * (2 * half + q), 32 * ks), yo[q]);
      }
    }
    if (hh + 1 < a.HG) prefetch_ds(h + 1);
    SSD_STAMP(4)
    __syncthreads();  // M^T complete
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (2 * ks + 1 >= w) {
        const bf16x8 Af = frag_kc(MsT, LD64, 16 * w, 32 * ks);
#pragma unroll
        for (int q = 0; q < 2; ++q)
          dxd[q] = mfma16(Af, frag_tr(dYs, LD64, 32 * ks, 16 * (2 * half + q)), dxd[q]);
      }
    }
    SSD_STAMP(5)
    // ---- (5) dX, ddt_direct, U, dD ; (6) dcum Yoff term   (rows j = i = 16w + 4lg + r)
    bf16x4 xr[2], yr[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      xr[q] = acc_rows4(Xs, LD64, 16 * w, 16 * (2 * half + q));
      yr[q] = acc_rows4(dYs, LD64, 16 * w, 16 * (2 * half + q));
    }
    float dDp = 0.f, usum = 0.f;
    float ddv[4], dcv[4];  // this lane group's rows: direct ddt and dcum contributions (one 16-B RMW each below)
    f32x4 ov[2];  // dX tile values, staged to Os as 4-byte column pairs after the row loop
    const float4 dt4 = *reinterpret_cast<const float4*>(&dtr[hh & 7][16 * w + 4 * lg]);
    const float4 ej4 = *reinterpret_cast<const float4*>(&ejr[16 * w + 4 * lg]);
    const float4 ei4 = *reinterpret_cast<const float4*>(&eir[16 * w + 4 * lg]);
    const float dtv[4] = {dt4.x, dt4.y, dt4.z, dt4.w}, ejv[4] = {ej4.x, ej4.y, ej4.z, ej4.w};
    const float eiv[4] = {ei4.x, ei4.y, ei4.z, ei4.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * w + 4 * lg + r;
      const float dt_ = dtv[r];
      const float ej = ejv[r];
      const float wj = ej * dt_;
      const float ei = eiv[r];
      float ddp = 0.f, up = 0.f, yp = 0.f;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float xv = (float)xr[q][r];
        const float dyv = (float)yr[q][r];
        ov[q][r] = dt_ * dxd[q][r] + wj * bds[q][r] + Dh * dyv;
        ddp += xv * (dxd[q][r] + ej * bds[q][r]);
        up += xv * bds[q][r];
        yp += yo[q][r] * dyv;
        dDp += xv * dyv;
      }
      ddv[r] = row_sum16(ddp);
      up = row_sum16(up) * wj;
      yp = row_sum16(yp) * ei;
      dcv[r] = yp - up;
      usum += up;
    }
    if (li == 0) {
      float4* pd = reinterpret_cast<float4*>(&ddw[hh & 7][half][16 * w + 4 * lg]);
      float4* pc = reinterpret_cast<float4*>(&dcw[hh & 7][wid][16 * w + 4 * lg]);
      float4 od = *pd, oc = *pc;
      od.x += ddv[0]; od.y += ddv[1]; od.z += ddv[2]; od.w += ddv[3];
      oc.x += dcv[0]; oc.y += dcv[1]; oc.z += dcv[2]; oc.w += dcv[3];
      *pd = od;
      *pc = oc;
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) acc_to_lds_pk(Os, LD64, 16 * w, 16 * (2 * half + q), ov[q]);
    usum = rows_sum4(usum);  // the wave's U total over its 16 rows (x its p-half)
    if (l == 0) dcw[hh & 7][wid][Q - 1] += usum;
    dDp = wave_sum(dDp);
    if (l == 0) redw[hh & 7][wid] = dDp;
    // ---- (7) dC_off += (e^{cum_i} dY) S , (8) dB_off += (w_j x) dS   for this half's n-tiles
    {
      const float ei = eir[jl];
      const float wl = ejr[jl] * dtr[hh & 7][jl];
#pragma unroll
      for (int ks = 0; ks < P / 32; ++ks) {
        const bf16x8 Ay = scale_frag(frag_kc(dYs, LD64, 16 * w, 32 * ks), ei);
        const bf16x8 Ax = scale_frag(frag_kc(Xs, LD64, 16 * w, 32 * ks), wl);
#pragma unroll
        for (int nt = 0; nt < NTH; ++nt) {
          const int n0 = 16 * (half * NTH + nt);
          dCa[nt] = mfma16(Ay, frag_tr(Ss, LDN, 32 * ks, n0), dCa[nt]);
          dBa[nt] = mfma16(Ax, frag_tr(dSs, LDN, 32 * ks, n0), dBa[nt]);
        }
      }
    }
    SSD_STAMP(6)
    // ---- (9) e^{cl} sum(dS o S) -> dcum[last]   (16-B LDS reads)
    {
      float s = 0.f;
      for (int v = threadIdx.x; v < P * N / 8; v += 512) {
        const int p = v / (N / 8), n = (v % (N / 8)) * 8;
        float fa[8], fb[8];
        ld8bf(Ss + p * LDN + n, fa);
        ld8bf(dSs + p * LDN + n, fb);
#pragma unroll
        for (int k = 0; k < 8; ++k) s += fa[k] * fb[k];
      }
      s = wave_sum(s);
      if (l == 0) dcw[hh & 7][wid][Q - 1] += s * __expf(cl);
    }
    // dX: each wave stores the 16x32 sub-tile of Os it wrote itself (same-wave LDS ops are in order,
    // so no block barrier is needed)
    {
      const int row = 16 * w + (l >> 2), col = 32 * half + 8 * (l & 3);
      if (row < valid)
        *reinterpret_cast<uint4*>(a.dx + (int64_t)b * a.sdxb + (int64_t)(c * Q + row) * a.sdxl +
                                  (int64_t)h * a.sdxh + col) = *reinterpret_cast<const uint4*>(Os + row * LD64 + col);
    }
    if ((hh & 7) == 7 || hh == a.HG - 1) flush(hh & ~7, (hh & 7) + 1);
    SSD_STAMP(7)
  }
  SSD_STAMP_FLUSH((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x)
  if (a.fuse_dbc) {
    // ---- this workgroup holds every head of group g (HG == H / G): finish dC = dC_off + dCB B and
    // dB = dB_off + dCB^T C here (ssd_dbc_bwd's math in the same order, so bitwise the same result) instead of
    // writing the head-group partials and re-reading them in a fourth kernel.  dCB goes to LDS as bf16 [i][j]
    // in MsT (all 16 tiles: the 10 owned ones and the 6 zero ones), dC / dB are staged in Ss / dSs.
    __syncthreads();  // every wave is done with MsT / Ss / dSs and the last flush
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k < own) {
#pragma unroll
        for (int r = 0; r < 4; ++r) MsT[(16 * tI[k] + 4 * lg + r) * LD64 + 16 * tJ[k] + li] = f2bf(dcbo[k][r]);
      }
    }
    if (wid >= 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) MsT[(16 * zI + 4 * lg + r) * LD64 + 16 * zJ + li] = f2bf(0.f);
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < Q / 32; ++ks) {
      const bf16x8 Ac = frag_kc(MsT, LD64, 16 * w, 32 * ks);  // dCB rows i, k = j
      const bf16x8 Ab = frag_tr(MsT, LD64, 32 * ks, 16 * w);  // dCB^T rows j, k = i
#pragma unroll
      for (int nt = 0; nt < NTH; ++nt) {
        const int n0 = 16 * (half * NTH + nt);
        dCa[nt] = mfma16(Ac, frag_tr(Bs, LDN, 32 * ks, n0), dCa[nt]);
        dBa[nt] = mfma16(Ab, frag_tr(Cs, LDN, 32 * ks, n0), dBa[nt]);
      }
    }
#pragma unroll
    for (int nt = 0; nt < NTH; ++nt) {
      acc_to_lds(Ss, LDN, 16 * w, 16 * (half * NTH + nt), dCa[nt]);
      acc_to_lds(dSs, LDN, 16 * w, 16 * (half * NTH + nt), dBa[nt]);
    }
    __syncthreads();
    store_tile<Q, N>(a.dC + (int64_t)b * a.sdCb + (int64_t)c * Q * a.sdCl + (int64_t)g * a.sdCg, a.sdCl, Ss, LDN, valid);
    store_tile<Q, N>(a.dB + (int64_t)b * a.sdBb + (int64_t)c * Q * a.sdBl + (int64_t)g * a.sdBg, a.sdBl, dSs, LDN, valid);
    return;
  }
  // ---- head-group partials
  const int64_t pbase = ((int64_t)b * a.nc + c) * a.nhg + hgi;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (k < own) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        a.part_dcb[(pbase * Q + 16 * tI[k] + 4 * lg + r) * Q + 16 * tJ[k] + li] = dcbo[k][r];
    }
  }
  if (wid >= 2) {
#pragma unroll
    for (int r = 0; r < 4; ++r) a.part_dcb[(pbase * Q + 16 * zI + 4 * lg + r) * Q + 16 * zJ + li] = 0.f;
  }
#pragma unroll
  for (int nt = 0; nt < NTH; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * w + 4 * lg + r, n = 16 * (half * NTH + nt) + li;
      a.part_db[(pbase * Q + row) * N + n] = dBa[nt][r];
      a.part_dc[(pbase * Q + row) * N + n] = dCa[nt][r];
    }
}

// ============================== K5: dB / dC (backward) =======================================
template <int N>
__global__ __launch_bounds__(256) void ssd_dbc_bwd_k(SSDArgs a) {
  constexpr int LDN = N + 16;  // conflict-free ds_read_b128 fragments (see LD64)
  constexpr int NT = N / 16;
  __shared__ __attribute__((aligned(16))) bf16_t Cs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t Os[Q * LDN];
  __shared__ __attribute__((aligned(16))) bf16_t dCBs[Q * LD64];
  const int c = blockIdx.x, g = blockIdx.y, b = blockIdx.z;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;  // wave-uniform: scalar branches
  const int valid = min(Q, a.L - c * Q);
  const int hpg = a.H / a.G;
  const int hg0 = g * hpg / a.HG, hg1 = (g + 1) * hpg / a.HG;
  {  // both tiles' loads in flight before the first LDS store
    StageRegs<Q, N, 256> sc, sb;
    sc.load(a.Cm + (int64_t)b * a.sCb + (int64_t)c * Q * a.sCl + (int64_t)g * a.sCg, a.sCl, valid);
    sb.load(a.Bm + (int64_t)b * a.sBb + (int64_t)c * Q * a.sBl + (int64_t)g * a.sBg, a.sBl, valid);
    sc.store(Cs, LDN);
    sb.store(Bs, LDN);
  }
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

// ============================== fp32 sequential forward (evaluation) =========================
// The reference evaluates HellaSwag in fp32 (eval.py); the MFMA kernels above are bf16.  This path keeps
// every operand fp32 and runs the recurrence itself, step by step (S_t = e^{dt A} S_{t-1} + dt x_t B_t^T,
// y_t = S_t C_t + D x_t): one 256-thread workgroup per (b, h), thread = (row p = tid / 4, a quarter of
// the N states), 16 steps of B / C / x / dt staged in LDS at a time, y summed over the quad by DPP.
// Not a training path (no backward); throughput is irrelevant next to the eval's GEMMs.
template <int N>
__global__ __launch_bounds__(256) void ssd_fwd_f32_k(SSDF32Args a) {
  constexpr int NS = N / 4, TS = 16;
  __shared__ float Bs[TS][N], Cs[TS][N], Xs[TS][P], dts[TS];
  const int h = blockIdx.x, b = blockIdx.y, g = h / (a.H / a.G);
  const int p = threadIdx.x >> 2, nq = threadIdx.x & 3;
  const float Ah = a.A[h], Dh = a.D ? a.D[h] : 0.f, bias = a.dt_bias ? a.dt_bias[h] : 0.f;
  const int64_t srow = (((int64_t)b * a.H + h) * P + p) * N + nq * NS;
  float S[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) S[j] = a.init ? a.init[srow + j] : 0.f;
  for (int t0 = 0; t0 < a.L; t0 += TS) {
    const int nt = min(TS, a.L - t0);
    __syncthreads();  // the previous block of steps is consumed
    for (int i = threadIdx.x; i < nt * N; i += 256) {
      const int tt = i / N, n = i % N;
      Bs[tt][n] = a.Bm[(int64_t)b * a.sBb + (int64_t)(t0 + tt) * a.sBl + (int64_t)g * a.sBg + n];
      Cs[tt][n] = a.Cm[(int64_t)b * a.sCb + (int64_t)(t0 + tt) * a.sCl + (int64_t)g * a.sCg + n];
    }
    for (int i = threadIdx.x; i < nt * P; i += 256) {
      const int tt = i / P, pp = i % P;
      Xs[tt][pp] = a.x[(int64_t)b * a.sxb + (int64_t)(t0 + tt) * a.sxl + (int64_t)h * a.sxh + pp];
    }
    if (threadIdx.x < nt) {
      float v = a.dt[(int64_t)b * a.sdtb + (int64_t)(t0 + threadIdx.x) * a.sdtl + (int64_t)h * a.sdth] + bias;
      if (a.softplus) v = v > 20.f ? v : log1pf(expf(v));  // torch.nn.functional.softplus (threshold 20)
      if (a.clamp) v = fminf(fmaxf(v, a.dt_min), a.dt_max);
      dts[threadIdx.x] = v;
    }
    __syncthreads();
    for (int tt = 0; tt < nt; ++tt) {
      const float d = dts[tt], dA = expf(d * Ah), xv = Xs[tt][p], dx = d * xv;
      float yp = 0.f;
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        S[j] = fmaf(dA, S[j], dx * Bs[tt][nq * NS + j]);
        yp = fmaf(S[j], Cs[tt][nq * NS + j], yp);
      }
      yp += __shfl_xor(yp, 1, 4);
      yp += __shfl_xor(yp, 2, 4);
      if (nq == 0) a.y[(int64_t)b * a.syb + (int64_t)(t0 + tt) * a.syl + (int64_t)h * a.syh + p] = fmaf(Dh, xv, yp);
    }
  }
  if (a.final_state) {
#pragma unroll
    for (int j = 0; j < NS; ++j) a.final_state[srow + j] = S[j];
  }
}

hipError_t launch_ssd_fwd_f32(const SSDF32Args& a, hipStream_t st) {
  if (a.H % a.G != 0 || (a.N != 64 && a.N != 128)) return hipErrorInvalidValue;
  N_SWITCH(a.N, hipLaunchKernelGGL(ssd_fwd_f32_k<NN>, dim3(a.H, a.B), dim3(256), 0, st, a));
  return hipGetLastError();
}

static int g_ssd_nseg = -1;  // < 0: read MAMBA_AMD_SSD_SEG once; 0: automatic; n: forced
void set_ssd_segments(int n) { g_ssd_nseg = n < 0 ? 0 : n; }

int ssd_pick_segments(int B, int H, int nc) {
  if (g_ssd_nseg < 0) {
    const char* e = getenv("MAMBA_AMD_SSD_SEG");
    g_ssd_nseg = e ? std::max(0, atoi(e)) : 0;
  }
  if (g_ssd_nseg > 0) return std::max(1, std::min({g_ssd_nseg, nc, SEG_MAX}));
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
  }
  // Measured on MI355X (profiles/r6/ssd_segments.txt): with b * H >= the CU count every CU already runs a walk and
  // splitting does not pay (2.8B at T = 8192, b * H = 320: forward -6% at 4 segments, reverse walk +2%, worse beyond);
  // with fewer walks than CUs the chip idles and segments pay almost linearly (batch-1 prefill of 32k tokens at
  // H = 24: forward 1552 -> 237 us, backward 1056 -> 406 us at 16 segments).  So: segments only below one walk per
  // CU, as many as keep b * H * segments within two workgroups per CU and >= 4 chunks per segment.
  const int64_t bh = (int64_t)B * H;
  if (bh >= ncu) return 1;
  int best = 1;
  for (int s = 2; s <= SEG_MAX; ++s) {
    const int cps = (nc + s - 1) / s, se = (nc + cps - 1) / cps;
    if (cps < 4 || bh * se > 2LL * ncu) break;
    best = se;
  }
  return best;
}

static hipError_t launch_seg_pass(const SSDArgs& a, bool fwd, hipStream_t st) {
  if (a.nseg < 2) return hipSuccess;
  if (a.nseg > SEG_MAX || !a.seg || !a.segd || (int64_t)(a.nseg - 1) * a.cps >= a.nc) return hipErrorInvalidValue;
  const dim3 grid(a.H, a.B, a.nseg - 1);
  if (fwd) N_SWITCH(a.N, hipLaunchKernelGGL(ssd_seg_state_k<NN>, grid, dim3(256), 0, st, a));
  else N_SWITCH(a.N, hipLaunchKernelGGL(ssd_seg_dstate_k<NN>, grid, dim3(256), 0, st, a));
  MAMBA_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(ssd_seg_combine_k, dim3(a.H, a.B), dim3(256), 0, st, a, fwd ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_ssd_fwd(const SSDArgs& a, hipStream_t st) {
  if (a.nseg < 1 || a.cps < 1 || (int64_t)a.nseg * a.cps < a.nc) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ssd_cumsum_k, dim3((unsigned)((int64_t)a.B * a.nc)), dim3(256), 0, st, a);
  MAMBA_HIP_CHECK(hipGetLastError());
  MAMBA_HIP_CHECK(launch_seg_pass(a, true, st));
  if (a.nseg > 1) {
    N_SWITCH(a.N, hipLaunchKernelGGL(ssd_fused_fwd_k<NN>, dim3(a.H, a.B, a.nseg), dim3(256), 0, st, a, nullptr));
    return hipGetLastError();
  }
  if (g_ssd_stamps && a.N == 128 && (int64_t)a.H * a.B * 8 <= g_ssd_stamps_n) {
    hipLaunchKernelGGL((ssd_fused_fwd_k<128, true>), dim3(a.H, a.B), dim3(256), 0, st, a, g_ssd_stamps,
                       g_ssd_stamp_wave & 3);
    return hipGetLastError();
  }
  N_SWITCH(a.N, hipLaunchKernelGGL(ssd_fused_fwd_k<NN>, dim3(a.H, a.B), dim3(256), 0, st, a, nullptr));
  return hipGetLastError();
}

hipError_t launch_ssd_bwd(const SSDArgs& a, hipStream_t st) {
  if (a.nseg < 1 || a.cps < 1 || (int64_t)a.nseg * a.cps < a.nc) return hipErrorInvalidValue;
  MAMBA_HIP_CHECK(launch_seg_pass(a, false, st));
  N_SWITCH(a.N, hipLaunchKernelGGL(ssd_dstate_bwd_k<NN>, dim3(a.H, a.B, a.nseg), dim3(256), 0, st, a));
  MAMBA_HIP_CHECK(hipGetLastError());
  if (a.fuse_dbc && a.HG != a.H / a.G) return hipErrorInvalidValue;  // the fused finish needs the whole group
  if (g_ssd_stamps && a.N == 128 && ((int64_t)a.H * a.B + (int64_t)a.nc * a.nhg * a.B) * 8 <= g_ssd_stamps_n) {
    // the stamp buffer holds the forward's (H * B) rows first, then the chunk backward's (nc * nhg * B)
    hipLaunchKernelGGL((ssd_chunk_bwd_k<128, true>), dim3(a.nc, a.nhg, a.B), dim3(512), 0, st, a,
                       g_ssd_stamps + (int64_t)a.H * a.B * 8, g_ssd_stamp_wave & 7);
  } else {
    N_SWITCH(a.N, hipLaunchKernelGGL(ssd_chunk_bwd_k<NN>, dim3(a.nc, a.nhg, a.B), dim3(512), 0, st, a, nullptr, 0));
  }
  MAMBA_HIP_CHECK(hipGetLastError());
  if (a.fuse_dbc) return hipSuccess;
  N_SWITCH(a.N, hipLaunchKernelGGL(ssd_dbc_bwd_k<NN>, dim3(a.nc, a.G, a.B), dim3(256), 0, st, a));
  return hipGetLastError();
}

}  // namespace mamba_amd
