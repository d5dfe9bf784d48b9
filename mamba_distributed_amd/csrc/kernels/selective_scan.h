// Argument blocks for kernels/selective_scan.hip (Mamba-1 scan + decode state update).
#pragma once
#include "types.h"

namespace mamba_amd {

// saved-state (carry) granularities: every 16 steps for the wave-per-state-group kernels, else every
// backward tile of the time-parallel kernels
constexpr int kSelScanCarrySG = 16, kSelScanCarryTile = 512;

struct SelScanArgs {
  int B, D, L, N, G, Kc;  // Kc = channels per workgroup (<= 64)
  int dtype;              // dtype of u / delta / z / B / C / out (kBF16 or kF32)
  bool softplus, vec, vecbc, vecg, vecz;
  const void* u_; const void* delta_;
  int64_t sub, sud, sdb, sdd;                       // (b, d, l) strides, unit l
  const float* A;                                   // (D, N)
  const void* Bm_; int64_t sBb, sBg, sBn;           // (b, g, n, l)
  const void* Cm_; int64_t sCb, sCg, sCn;
  const float* D_; const float* delta_bias;
  const void* z_; int64_t szb, szd;
  void* out_; int64_t sob, sod;
  float* carries;                                   // (B, D, nct, N) state at every carry_t-th step
  int carry_t, nct;                                 // steps between saved states, nct = ceil(L / carry_t)
  float* last_state;                                // (B, D, N) or null
  // backward
  const void* dout_; int64_t sgb, sgd;
  void* du_; int64_t sdub, sdud;
  void* ddelta_; int64_t sddb, sddd;
  void* dz_; int64_t sdzb, sdzd;
  void* dB_; int64_t sdBb, sdBg, sdBn;
  void* dC_; int64_t sdCb, sdCg, sdCn;
  float* part_dB; float* part_dC;                   // (B, ndg, N, L)
  float* part_dA;                                   // (B, D, N)   zero-initialised
  float* part_dD; float* part_dbias;                // (B, D)      zero-initialised
  bool pacc;  // sequential backward only: add into part_dA / part_dD / part_dbias (deferred reduction)
  // fused dt_proj (Mamba-1, wave-per-state-group kernels only): delta_raw[b, d, t] = sum_r dtw[d, r] dtx[r, b L + t],
  // computed per 16-step tile with MFMA inside the scan (delta_ unused, never materialised).  dtw (D, R) bf16
  // contiguous, dtx (R, B L) bf16 rows (row stride sdtx, unit column stride); R % 8 == 0, R <= 128.
  const void* dtw_; const void* dtx_; int64_t sdtx; int R;
  // workgroup order of the wave-per-state-group kernels: b fastest (set by the launchers for (d, b, l) memory)
  bool binner;
};

struct SSMUpdateArgs {
  int B, H, P, N, G, dtype;
  bool softplus, A_per_n, D_per_p, dt_bias_per_p;
  float* state;                                     // (B, H, P, N) fp32, updated in place
  const void* x_; int64_t sxb, sxh;                 // (B, H, P) unit p
  const void* dt_; int64_t sdtb, sdth, sdtp;
  const float* A; const float* D; const float* dt_bias;
  const void* Bm_; int64_t sBb, sBg;                // (B, G, N) unit n
  const void* Cm_; int64_t sCb, sCg;
  const void* z_; int64_t szb, szh;
  void* out_;                                       // (B, H, P) contiguous
};

hipError_t launch_selscan_fwd(const SelScanArgs& a, hipStream_t st);
hipError_t launch_selscan_bwd(const SelScanArgs& a, hipStream_t st);
// carry granularity the forward will use for these args (16 with the wave-per-state-group kernels, else 512)
int selscan_carry_t(const SelScanArgs& a);
// channels per backward workgroup (SelScanArgs::Kc; sizes the dB / dC partials); needs carry_t set
int selscan_bwd_kc(const SelScanArgs& a);
bool selscan_dt_fusable(const SelScanArgs& a);  // fused dt_proj (dtw_ / dtx_) supported for this shape
bool selscan_bwd_sequential(const SelScanArgs& a);  // the wave-per-state-group kernel runs (supports pacc)
hipError_t launch_ssm_update(const SSMUpdateArgs& a, hipStream_t st);
int selscan_order();
void set_selscan_order(int v);

}  // namespace mamba_amd
