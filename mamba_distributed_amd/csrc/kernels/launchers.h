// Host-side launchers exported by kernels/*.hip (pure HIP; no torch types) and called by
// ../bindings.cpp.  All take raw device pointers + element strides + the caller's stream,
// never allocate and never synchronise (graph-capturable).  dtype codes: see common.h DType.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mamba_amd {

// Split-K count of a weight-gradient GEMM with `tiles` 256x256 output tiles of a (P, Q) fp32 result over K
// tokens, one workgroup per CU (256 CUs): minimise ceil(tiles S / 256) / S -- the time in full-K tile units,
// so a grid just past a round (272 tiles: 2 rounds at S = 1) is split until the last round is nearly full --
// plus the fp32 slab round trip of each extra split (P Q x 8 B at ~5 TB/s against 256 x 256 x 2K flop per CU
// at ~3.5 TF/s: P Q / (23405 K) tile units), keeping >= min_k tokens per split.
inline int split_k_count(int64_t tiles, int64_t P, int64_t Q, int64_t K, int64_t min_k) {
  // up to 64 slices: a narrow output (the Mamba-1 x_proj / dt_proj weight gradients: 6 tiles) at the old cap of 16
  // ran 96 workgroups on 256 CUs (profiles/r6/narrow_wgrad_splits.txt)
  int best = 1;
  double bc = 1e30;
  for (int S = 1; S <= 64; ++S) {
    if (S > 1 && K / S < min_k) break;
    const double c = (double)((tiles * S + 255) / 256) / S + (double)S * P * Q / (23405.0 * K);
    if (c < bc - 1e-9) { bc = c; best = S; }
  }
  return best;
}

// Backward kernels with a `part` buffer write one fp32 partial row per workgroup for a parameter
// gradient; pacc = true ADDS into the rows instead (accumulation across the no-sync micro-steps of one
// optimizer step), and dw == nullptr skips the final column sum (deferred to the sync micro-step).
// deterministic column sum of a (nrows, ncols) fp32 partial matrix (norm.hip)
hipError_t launch_colsum(float* part, int nrows, int ncols, float* out, hipStream_t st);  // clobbers part
// batched column sums into parameter gradients (kernels/norm.hip LateCol table rows, 80 bytes each)
hipError_t launch_late_colsum(const void* tab, int n, int nblk, int ntile, hipStream_t st);

// ---- norm.hip -------------------------------------------------------------------------------
hipError_t launch_add_rmsnorm_fwd(const void* x, int xdt, int64_t sx, const void* res, int rdt, int64_t sr,
                                  const float* w, void* y, int ydt, void* ro, int rodt, float* rstd, int64_t M,
                                  int D, float eps, hipStream_t st);
int add_rmsnorm_bwd_partial_rows(int64_t M);
hipError_t launch_add_rmsnorm_bwd(const void* dy, int ydt, const void* dro, int drodt, const void* ro, int rodt,
                                  const float* w, const float* rstd, void* dx, int xdt, void* dres, int rdt,
                                  float* part, float* dw, bool pacc, int64_t M, int D, hipStream_t st);
hipError_t launch_gated_rmsnorm_fwd(const void* x, int xdt, int64_t sx, const void* z, int zdt, int64_t sz,
                                    const float* w, void* y, int ydt, float* rstd, int64_t M, int D, int G,
                                    float eps, bool nbg, hipStream_t st);
int norm_bwd_partial_rows(int64_t M);
hipError_t launch_gated_rmsnorm_bwd(const void* dy, int ydt, const void* x, int xdt, int64_t sx, const void* z,
                                    int zdt, int64_t sz, const float* w, const float* rstd, void* dx, int64_t sdx,
                                    void* dz, int64_t sdz, float* part, float* dw, bool pacc, int64_t M, int D, int G,
                                    bool nbg, hipStream_t st);

// ---- cross_entropy.hip ------------------------------------------------------------------------
hipError_t launch_ce_fwd(const void* logits, int dt, int64_t ld, const int64_t* tgt, int64_t M, int V,
                         int64_t ignore_index, const float* scale, float* loss, void* grad, int64_t ldg,
                         hipStream_t st);

// ---- conv1d.hip ---------------------------------------------------------------------------------
hipError_t launch_conv_cf_fwd(const void* x, int dt, int64_t sxb, int64_t sxd, const float* w, const float* bias,
                              void* out, int64_t sob, int64_t sod, int Bn, int Dn, int L, int Wd, bool silu,
                              hipStream_t st);
hipError_t launch_conv_cf_bwd(const void* x, int dt, int64_t sxb, int64_t sxd, const float* w, const float* bias,
                              const void* g, int64_t sgb, int64_t sgd, void* dx, int64_t sdb, int64_t sdd,
                              float* part, float* dw, float* db, bool pacc, int Bn, int Dn, int L, int Wd, bool silu,
                              hipStream_t st);
hipError_t launch_conv_cl_fwd(const void* x, int dt, int64_t sxb, int64_t sxl, const float* w, const float* bias,
                              void* out, int64_t sob, int64_t sol, int Bn, int L, int C, int Wd, bool silu,
                              hipStream_t st);
int conv_cl_bwd_partial_rows(int Bn, int L);
hipError_t launch_conv_cl_bwd(const void* x, int dt, int64_t sxb, int64_t sxl, const float* w, const float* bias,
                              const void* g, int64_t sgb, int64_t sgl, void* dx, int64_t sdb, int64_t sdl,
                              float* part, float* dw, float* db, bool pacc, int Bn, int L, int C, int Wd, bool silu,
                              hipStream_t st);
hipError_t launch_conv_update(const void* x, int dt, int64_t sxb, void* state, int64_t ssb, int64_t ssc,
                              const float* w, const float* bias, void* out, int Bn, int C, int Wd, int SL, bool silu,
                              hipStream_t st);  // state: (Bn, C, SL >= Wd-1), upstream layout SL = Wd

// varlen / state hand-off channel-last conv (seq_idx, initial_states, final_states), fwd or bwd
struct ConvVarArgs {
  int dt;                                   // dtype of x / out / g / dx / states
  const void* x; int64_t sxb, sxl;          // (b, l, c), unit channel stride
  const int* seq; int64_t sqb;              // (b, l) int32, unit time stride; null = one sequence per row
  const void* init; int64_t sib, sic;       // (b, c, W-1), unit last stride; null = zeros
  const float* w; const float* bias;        // (c, W) fp32, (c) or null
  void* out; int64_t sob, sol;              // fwd output
  void* fin; int64_t sfb, sfc;              // fwd: (b, c, W-1) final states or null
  const void* g; int64_t sgb, sgl;          // bwd: d out
  const void* dfin; int64_t sdfb, sdfc;     // bwd: d final_states or null
  void* dx; int64_t sdb, sdl;               // bwd: d x
  void* dinit; int64_t sdib, sdic;          // bwd: d initial_states or null
  float* part; float* dw; bool pacc;        // bwd: partial rows (conv_cl_var_partial_rows, c, W+1), dw (c, W+1) or null
  int Bn, L, C, Wd;
  bool silu, backward;
};
int conv_cl_var_partial_rows(int Bn, int L);
hipError_t launch_conv_cl_var(const ConvVarArgs& a, hipStream_t st);

// ---- gemm.hip ---------------------------------------------------------------------------------
// C[M, N] = A[M, K] . B[N, K]^T, bf16 in/out, fp32 accumulate (K % 64 == 0, N % 8 == 0)
bool gemm_tn_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc);
// C[N, M] (+)= A[N, K] . B[K, M], bf16, rows of B / C contiguous along M (channel-major activations)
bool gemm_skinny_supported(int N, int K, int M, int64_t lda, int64_t ldb, int64_t ldc);
hipError_t launch_gemm_skinny(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int N,
                              int K, int M, bool accumulate, hipStream_t st);
hipError_t launch_gemm_tn_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                               int N, int K, hipStream_t st);
// fp32 C[P, Q] (+)= dY[M, P]^T . X[M, Q] (bf16 token-major operands), split over M into
// gemm_wgrad_splits() fp32 partials (part: splits * P * Q floats) summed in fixed order
int gemm_wgrad_splits(int M, int P, int Q);
bool gemm_wgrad_cm_supported(int M, int P, int Q, int64_t ldy, int64_t ldx);
hipError_t launch_gemm_wgrad_cm(const void* dY, int64_t ldy, const void* X, int64_t ldx, float* part, float* out,
                                int M, int P, int Q, bool accumulate, bool dy_cm, bool x_cm, hipStream_t st,
                                bool pacc = false, bool reduce = true);
hipError_t launch_gemm_wgrad(const void* dY, int64_t ldy, const void* X, int64_t ldx, float* part, float* out,
                             int M, int P, int Q, bool accumulate, hipStream_t st);

// ---- gemm_pipe.hip: pipelined 256x256 MFMA GEMM engine, C[M,N] (op)= A . B^T ----------------------------
// la / lb: 0 = operand stored [rows][K] (K contiguous), 1 = stored [K][rows]; epi: 0 = bf16 C, 1 = fp32 C
// (K split `splits` ways into slabs split_stride elements apart), 2 = fp32 C +=; bm: 256 (the only tile)
bool gemm_pipe_supported(int la, int lb, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc);
int gemm_pipe_splits(int M, int N, int K);
hipError_t launch_gemm_pipe(int la, int lb, const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                            int64_t ldc, int M, int N, int K, int splits, int64_t split_stride, int epi, int bm,
                            hipStream_t st);
// persistent variant (one workgroup per CU walking the output tiles; KC . KC, bf16 output (epi 0) only,
// staged through LDS into whole-row stores; rowscale (epi 0, nullable): C[m, :] *= rowscale[m])
bool gemm_pk_supported(int la, int lb, int epi, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc);
hipError_t launch_gemm_pk(int la, int lb, const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                          int64_t ldc, int M, int N, int K, int epi, const float* rowscale, hipStream_t st);
// launches that may ever be captured into HIP graphs per process (their counter pairs are never recycled; a
// launch past it returns hipErrorNotReady)
int gemm_pk_graph_counter_capacity();
// the split-K engine's workgroup shape: 8 waves (128 x 64 per wave) or 4 waves (128 x 128 per wave)
int gemm_pipe_waves();
void set_gemm_pipe_waves(int w);
// LDS slots (4 or 5) of the XC . XC fp32 weight-gradient engine gemm_wg_k, or 0: those products on gemm_pipe_k
int gemm_wg_nb();
void set_gemm_wg_nb(int nb);
// paired 64-deep KC operand images in the staged-ring engine: 0 never, 1 KC operands of >= 1536 rows over K >= 16384
// (default), 2 always
int gemm_wg_kcpair();
int conv_cf_order();
void set_conv_cf_order(int v);
void set_gemm_wg_kcpair(int v);
// out[i] (+)= sum_s part[s * stride + i], fixed order
hipError_t launch_transpose_bf16(const void* x, int64_t ldx, void* y, int64_t ldy, int R, int C, hipStream_t st);
// native optimizer step (optim.hip): segs = OptSeg table (64 B per parameter), blk = (segment, offset) per chunk
int opt_chunk();
hipError_t launch_grad_norm(const void* segs, const int64_t* blk, int nblk, float* partial, float max_norm,
                            float divisor, float* out, hipStream_t st);
hipError_t launch_adamw(const void* segs, const int64_t* blk, int nblk, const float* gscale, float b1, float b2,
                        float eps, hipStream_t st);
hipError_t launch_gp_reduce(const float* part, int S, int64_t stride, int64_t n, float* out, bool accumulate,
                            hipStream_t st);

// ---- decode.hip (fused single-token Mamba-2 layer step; buffers preallocated, graph-capturable) --------
int decode_max_batch();
hipError_t launch_decode_inproj(const void* hn, const void* W, int n_out, int d, int b, float* zxbcdt, int conv_lo,
                                int conv_hi, void* conv_state, int64_t csb, int64_t csc, int SL, const float* cw,
                                const float* cb, int Wd, hipStream_t st);
hipError_t launch_decode_ssm(const float* zxbcdt, int n_out, float* state, const float* A, const float* D,
                             const float* dt_bias, int H, int P, int G, int N, int b, void* g_out, float* part,
                             hipStream_t st);  // g_out bf16
hipError_t launch_decode_outproj(const void* g, const float* part, int nparts, float eps, const void* W, int d_out,
                                 int di, int b, void* out, hipStream_t st);  // W = W_out diag(gate-norm weight)

}  // namespace mamba_amd
