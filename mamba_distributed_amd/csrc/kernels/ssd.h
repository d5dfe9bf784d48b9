// Argument block shared by the SSD kernels (kernels/ssd.hip) and the torch binding.
#pragma once
#include "types.h"

namespace mamba_amd {

struct SSDArgs {
  int B, L, H, G, N, nc, Lp;  // Lp = nc * 64
  int HG, nhg;                // heads per workgroup in the chunk kernels, nhg = H / HG
  // forward inputs
  const bf16_t* x; int64_t sxb, sxl, sxh;  // (b, l, h, p) unit p stride
  const void* dt; int dt_dtype; int64_t sdtb, sdtl, sdth;
  const float* A; const float* D; const float* dt_bias;
  const bf16_t* Bm; int64_t sBb, sBl, sBg;  // (b, l, g, n) unit n stride
  const bf16_t* Cm; int64_t sCb, sCl, sCg;
  bool softplus; float dt_min, dt_max;
  bool a_log;                 // A holds A_log: kernels use A = -exp(A_log), dA partials become dA_log
  int psl;                    // row stride of the (b*nc, 3, H) small-partials block (= 3H)
  bool pacc;                  // add into the small partials (deferred reduction across micro-steps)
  const int* seq; int64_t sqb, sql;  // seq_idx (b, l) int32 or null: packed variable-length sequences
  const float* init;      // (b, h, p, n) or null
  // forward outputs / saved
  float* dtp; float* cum; // (b, h, Lp)
  bf16_t* states;         // (b, nc, h, p, n) state entering each chunk
  float* final_state;     // (b, h, p, n) or null
  bf16_t* y; int64_t syb, syl, syh;
  // backward
  const bf16_t* dy; int64_t sdyb, sdyl, sdyh;
  const float* dfinal;    // (b, h, p, n) or null
  bf16_t* dstates;        // (b, nc, h, p, n) workspace
  float* dinit;           // or null
  bf16_t* dx; int64_t sdxb, sdxl, sdxh;
  void* ddt; int ddt_dtype; int64_t sddtb, sddtl, sddth;
  int ddt_zero_pad;       // bf16 ddt rows (sddth == 1): zero this many columns after the H dt columns (the padded
                          // in_proj gradient's pad, ops/linear.py), written by the chunk kernel's first head flush
  bf16_t* dB; int64_t sdBb, sdBl, sdBg;
  bf16_t* dC; int64_t sdCb, sdCl, sdCg;
  bool fuse_dbc;          // HG == H / G: ssd_chunk_bwd finishes dB / dC itself (no partials, no ssd_dbc_bwd)
  float* part_dcb;        // (b, nc, nhg, 64, 64)
  float* part_db;         // (b, nc, nhg, 64, N)
  float* part_dc;         // (b, nc, nhg, 64, N)
  float* part_dA; float* part_dD; float* part_dbias;  // (b, nc, h)
  // segment-parallel state walks (small b * H): the chunks split into nseg segments of cps chunks; the forward's
  // and the reverse walk's workgroups run one (h, b, segment) each from a carried-in state that a state-only pass
  // per segment plus a (b, h) combine produced.  nseg = 1, cps = nc: one walk per (h, b) over every chunk.
  int nseg, cps;
  float* seg;             // (b, h, nseg - 1, p, n) fp32: per-segment local states, then the carried-in states
  float* segd;            // (b, h, nseg - 1): the summed log-decay of each segment
};

// segments for a state walk over nc chunks at B * H (h, b) pairs: 1 unless a split fills the CUs better
// (set_ssd_segments(n > 0) forces n, clamped to nc; 0 = automatic)
int ssd_pick_segments(int B, int H, int nc);
void set_ssd_segments(int n);

// fp32 sequential SSD forward (evaluation in fp32, e.g. the reference's HellaSwag protocol); P = 64,
// N = 64 / 128, no varlen.  Outputs y (b, l, h, p) and optionally the final state (b, h, p, n).
struct SSDF32Args {
  int B, L, H, G, N;
  const float* x; int64_t sxb, sxl, sxh;       // unit p
  const float* dt; int64_t sdtb, sdtl, sdth;   // raw dt
  const float* A; const float* D; const float* dt_bias;
  const float* Bm; int64_t sBb, sBl, sBg;      // unit n
  const float* Cm; int64_t sCb, sCl, sCg;
  const float* init;                           // (B, H, 64, N) contiguous or null
  float* y; int64_t syb, syl, syh;             // unit p
  float* final_state;                          // (B, H, 64, N) contiguous or null
  bool softplus, clamp; float dt_min, dt_max;
};
hipError_t launch_ssd_fwd_f32(const SSDF32Args& a, hipStream_t st);

hipError_t launch_ssd_fwd(const SSDArgs& a, hipStream_t st);
// diagnostic: non-null = the next forward / chunk-backward launches record per-phase s_memtime sums (8 x u64 per
// workgroup: the forward's H*B rows, then the chunk backward's nc*nhg*B rows); N = 128 only
void set_ssd_stamps(void* p, int64_t n);  // n: capacity in u64 (stamped launches that need more run unstamped)
hipError_t launch_ssd_bwd(const SSDArgs& a, hipStream_t st);

}  // namespace mamba_amd
