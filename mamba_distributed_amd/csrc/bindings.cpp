// PyTorch operator registrations for the gfx950 kernels: torch.ops.mamba_amd.*
//
// Every op: validates device / dtype / shape / stride assumptions of its kernel with TORCH_CHECK
// (a kernel is never launched on operands whose layout it does not handle), allocates outputs
// with the caching allocator, launches on the current torch HIP stream, and checks the launch.
#include <ATen/ATen.h>
#include <cstdlib>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "kernels/launchers.h"
#include "kernels/selective_scan.h"
#include "kernels/ssd.h"

using at::Tensor;
using c10::optional;

namespace {

hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

int dcode(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return mamba_amd::kF32;
    case at::kBFloat16: return mamba_amd::kBF16;
    default: TORCH_CHECK(false, "mamba_amd: unsupported dtype ", t);
  }
  return -1;
}

#define HIPCHK(e)                                                                              \
  do {                                                                                         \
    hipError_t _e = (e);                                                                       \
    TORCH_CHECK(_e == hipSuccess, "mamba_amd HIP launch failed: ", hipGetErrorString(_e));     \
  } while (0)

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "mamba_amd: ", name, " must be a GPU tensor");
}
void check_same_device(const Tensor& a, const Tensor& b) {
  TORCH_CHECK(a.device() == b.device(), "mamba_amd: tensors on different devices");
}
Tensor f32c(const Tensor& t) { return t.to(at::kFloat).contiguous(); }
Tensor f32c_opt(const optional<Tensor>& t) { return t.has_value() && t->defined() ? f32c(*t) : Tensor(); }
const float* fptr(const Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }

// ---------------------------------------------------------------------------------------------
// norms
std::tuple<Tensor, Tensor, Tensor> add_rmsnorm_fwd(Tensor x, optional<Tensor> residual, Tensor weight, double eps,
                                                   at::ScalarType out_dtype, at::ScalarType res_dtype) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be (M, D) with unit column stride");
  const int64_t M = x.size(0), D = x.size(1);
  TORCH_CHECK(D % 4 == 0 && D <= 20 * 256 && x.stride(0) % 4 == 0, "D must be a multiple of 4 and <= 5120");
  Tensor res;
  if (residual.has_value() && residual->defined()) {
    res = *residual;
    TORCH_CHECK(res.dim() == 2 && res.size(0) == M && res.size(1) == D && res.stride(1) == 1 && res.stride(0) % 4 == 0,
                "residual shape/stride mismatch");
    check_same_device(x, res);
  }
  Tensor w = f32c(weight);
  TORCH_CHECK(w.numel() == D, "weight size mismatch");
  auto y = at::empty({M, D}, x.options().dtype(out_dtype));
  auto ro = at::empty({M, D}, x.options().dtype(res_dtype));
  auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
  HIPCHK(mamba_amd::launch_add_rmsnorm_fwd(x.data_ptr(), dcode(x.scalar_type()), x.stride(0),
                                           res.defined() ? res.data_ptr() : nullptr,
                                           res.defined() ? dcode(res.scalar_type()) : 0, res.defined() ? res.stride(0) : 0,
                                           w.data_ptr<float>(), y.data_ptr(), dcode(out_dtype), ro.data_ptr(),
                                           dcode(res_dtype), rstd.data_ptr<float>(), M, (int)D, (float)eps, cur_stream()));
  return {y, ro, rstd};
}

// Deferred parameter-gradient reductions: part_mode 0 = transient partials + column sum (plain call);
// 1 / 2 = store / ADD this call's partial rows into the caller-kept buffer `part_buf` and skip the sum
// (no-sync micro-steps); 3 / 4 = store / add, then sum (the sync micro-step).  Without the sum the returned
// parameter gradients are empty (0-element) tensors.
struct PartMode {
  bool pacc, reduce;
};
static PartMode part_mode(int64_t m) {
  TORCH_CHECK(m >= 0 && m <= 4, "part_mode must be 0..4");
  return {m == 2 || m == 4, m == 0 || m == 3 || m == 4};
}
static Tensor part_tensor(const optional<Tensor>& buf, int64_t mode, at::IntArrayRef shape, const at::TensorOptions& o) {
  if (mode == 0) return at::empty(shape, o.dtype(at::kFloat));
  TORCH_CHECK(buf.has_value() && buf->defined(), "part_mode > 0 needs part_buf");
  TORCH_CHECK(buf->scalar_type() == at::kFloat && buf->is_contiguous() && buf->sizes() == shape,
              "part_buf must be contiguous fp32 of shape ", shape, " (got ", buf->sizes(), ")");
  return *buf;
}
int64_t part_rows(std::string kind, int64_t a, int64_t b) {
  if (kind == "add_rmsnorm") return mamba_amd::add_rmsnorm_bwd_partial_rows(a);
  if (kind == "gated_rmsnorm") return mamba_amd::norm_bwd_partial_rows(a);
  if (kind == "conv_cl") return mamba_amd::conv_cl_bwd_partial_rows((int)a, (int)b);
  if (kind == "conv_cl_var") return mamba_amd::conv_cl_var_partial_rows((int)a, (int)b);
  TORCH_CHECK(false, "part_rows: unknown kind ", kind);
}

std::tuple<Tensor, Tensor, Tensor> add_rmsnorm_bwd(Tensor dy, optional<Tensor> dres_out, Tensor res_out, Tensor weight,
                                                   Tensor rstd, at::ScalarType dx_dtype, at::ScalarType dres_dtype,
                                                   bool write_dres, optional<Tensor> part_buf, int64_t part_mode_) {
  check_cuda(dy, "dy");
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  dy = dy.contiguous();
  res_out = res_out.contiguous();
  const int64_t M = res_out.size(0), D = res_out.size(1);
  TORCH_CHECK(dy.size(0) == M && dy.size(1) == D, "dy shape mismatch");
  Tensor dro;
  if (dres_out.has_value() && dres_out->defined()) {
    dro = dres_out->contiguous();
    TORCH_CHECK(dro.size(0) == M && dro.size(1) == D, "dres_out shape mismatch");
  }
  Tensor w = f32c(weight);
  auto dx = at::empty({M, D}, dy.options().dtype(dx_dtype));
  Tensor dres = write_dres ? at::empty({M, D}, dy.options().dtype(dres_dtype)) : at::empty({0}, dy.options());
  const int rows = mamba_amd::add_rmsnorm_bwd_partial_rows(M);
  const PartMode pm = part_mode(part_mode_);
  Tensor part = part_tensor(part_buf, part_mode_, {rows, D}, dy.options());
  auto dw = at::empty({pm.reduce ? D : 0}, dy.options().dtype(at::kFloat));
  HIPCHK(mamba_amd::launch_add_rmsnorm_bwd(dy.data_ptr(), dcode(dy.scalar_type()), dro.defined() ? dro.data_ptr() : nullptr,
                                           dro.defined() ? dcode(dro.scalar_type()) : 0, res_out.data_ptr(),
                                           dcode(res_out.scalar_type()), w.data_ptr<float>(), rstd.data_ptr<float>(),
                                           dx.data_ptr(), dcode(dx_dtype), write_dres ? dres.data_ptr() : nullptr,
                                           dcode(dres_dtype), part.data_ptr<float>(),
                                           pm.reduce ? dw.data_ptr<float>() : nullptr, pm.pacc, M, (int)D, cur_stream()));
  return {dx, dres, dw.to(weight.scalar_type())};
}

std::tuple<Tensor, Tensor> gated_rmsnorm_fwd(Tensor x, Tensor z, Tensor weight, double eps, int64_t group_size,
                                             bool norm_before_gate) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 2 && z.dim() == 2 && x.stride(1) == 1 && z.stride(1) == 1, "x, z must be (M, D), unit col stride");
  const int64_t M = x.size(0), D = x.size(1);
  TORCH_CHECK(z.size(0) == M && z.size(1) == D, "z shape mismatch");
  TORCH_CHECK(D % 4 == 0 && D <= 20 * 256 && group_size % 4 == 0 && D % group_size == 0 && D / group_size <= 64,
              "unsupported D / group_size");
  TORCH_CHECK(x.stride(0) % 4 == 0 && z.stride(0) % 4 == 0, "row strides must be multiples of 4");
  Tensor w = f32c(weight);
  auto y = at::empty({M, D}, x.options());
  auto rstd = at::empty({M, D / group_size}, x.options().dtype(at::kFloat));
  HIPCHK(mamba_amd::launch_gated_rmsnorm_fwd(x.data_ptr(), dcode(x.scalar_type()), x.stride(0), z.data_ptr(),
                                             dcode(z.scalar_type()), z.stride(0), w.data_ptr<float>(), y.data_ptr(),
                                             dcode(x.scalar_type()), rstd.data_ptr<float>(), M, (int)D, (int)group_size,
                                             (float)eps, norm_before_gate, cur_stream()));
  return {y, rstd};
}

std::tuple<Tensor, Tensor, Tensor> gated_rmsnorm_bwd(Tensor dy, Tensor x, Tensor z, Tensor weight, Tensor rstd,
                                                     int64_t group_size, bool norm_before_gate, optional<Tensor> dx_out,
                                                     optional<Tensor> dz_out, optional<Tensor> part_buf,
                                                     int64_t part_mode_) {
  check_cuda(dy, "dy");
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  dy = dy.contiguous();
  const int64_t M = x.size(0), D = x.size(1);
  TORCH_CHECK(x.stride(1) == 1 && z.stride(1) == 1 && x.stride(0) % 4 == 0 && z.stride(0) % 4 == 0, "x/z layout");
  Tensor dx = dx_out.has_value() && dx_out->defined() ? *dx_out : at::empty({M, D}, x.options());
  Tensor dz = dz_out.has_value() && dz_out->defined() ? *dz_out : at::empty({M, D}, z.options());
  TORCH_CHECK(dx.size(0) == M && dx.size(1) == D && dx.stride(1) == 1 && dx.stride(0) % 4 == 0 &&
                  dx.scalar_type() == x.scalar_type(), "dx_out layout");
  TORCH_CHECK(dz.size(0) == M && dz.size(1) == D && dz.stride(1) == 1 && dz.stride(0) % 4 == 0 &&
                  dz.scalar_type() == z.scalar_type(), "dz_out layout");
  Tensor w = f32c(weight);
  const int rows = mamba_amd::norm_bwd_partial_rows(M);
  const PartMode pm = part_mode(part_mode_);
  Tensor part = part_tensor(part_buf, part_mode_, {rows, D}, dy.options());
  auto dw = at::empty({pm.reduce ? D : 0}, dy.options().dtype(at::kFloat));
  HIPCHK(mamba_amd::launch_gated_rmsnorm_bwd(dy.data_ptr(), dcode(dy.scalar_type()), x.data_ptr(), dcode(x.scalar_type()),
                                             x.stride(0), z.data_ptr(), dcode(z.scalar_type()), z.stride(0),
                                             w.data_ptr<float>(), rstd.data_ptr<float>(), dx.data_ptr(), dx.stride(0),
                                             dz.data_ptr(), dz.stride(0), part.data_ptr<float>(),
                                             pm.reduce ? dw.data_ptr<float>() : nullptr, pm.pacc, M, (int)D,
                                             (int)group_size, norm_before_gate, cur_stream()));
  return {dx, dz, dw.to(weight.scalar_type())};
}

// ---------------------------------------------------------------------------------------------
// cross entropy
Tensor ce_fwd(Tensor logits, Tensor targets, int64_t ignore_index, Tensor scale, optional<Tensor> grad) {
  check_cuda(logits, "logits");
  at::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be (M, V) with unit col stride");
  const int64_t M = logits.size(0), V = logits.size(1);
  auto t = targets.to(at::kLong).contiguous();
  TORCH_CHECK(t.numel() == M, "targets size mismatch");
  auto sc = scale.to(at::kFloat).contiguous();
  auto loss = at::empty({M}, logits.options().dtype(at::kFloat));
  void* g = nullptr;
  int64_t ldg = 0;
  if (grad.has_value() && grad->defined()) {
    TORCH_CHECK(grad->size(0) == M && grad->size(1) == V && grad->stride(1) == 1 &&
                grad->scalar_type() == logits.scalar_type(), "grad layout");
    g = grad->data_ptr();
    ldg = grad->stride(0);
  }
  HIPCHK(mamba_amd::launch_ce_fwd(logits.data_ptr(), dcode(logits.scalar_type()), logits.stride(0), t.data_ptr<int64_t>(),
                                  M, (int)V, ignore_index, sc.data_ptr<float>(), loss.data_ptr<float>(), g, ldg,
                                  cur_stream()));
  return loss;
}

// ---------------------------------------------------------------------------------------------
// causal conv1d
Tensor conv1d_cf_fwd(Tensor x, Tensor weight, optional<Tensor> bias, bool silu) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "x must be (b, d, l) with unit time stride");
  const int64_t B = x.size(0), D = x.size(1), L = x.size(2);
  Tensor w = f32c(weight);
  TORCH_CHECK(w.dim() == 2 && w.size(0) == D && w.size(1) >= 2 && w.size(1) <= 4, "weight must be (d, w), 2<=w<=4");
  Tensor bb = f32c_opt(bias);
  auto out = at::empty({D, B, L}, x.options()).permute({1, 0, 2});
  HIPCHK(mamba_amd::launch_conv_cf_fwd(x.data_ptr(), dcode(x.scalar_type()), x.stride(0), x.stride(1), w.data_ptr<float>(),
                                       fptr(bb), out.data_ptr(), out.stride(0), out.stride(1), (int)B, (int)D, (int)L,
                                       (int)w.size(1), silu, cur_stream()));
  return out;
}

std::tuple<Tensor, Tensor, Tensor> conv1d_cf_bwd(Tensor x, Tensor weight, optional<Tensor> bias, Tensor dout, bool silu,
                                                 optional<Tensor> dx_out, optional<Tensor> part_buf,
                                                 int64_t part_mode_) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "x must be (b, d, l) with unit time stride");
  if (dout.stride(2) != 1) dout = dout.contiguous();
  const int64_t B = x.size(0), D = x.size(1), L = x.size(2);
  TORCH_CHECK(dout.size(0) == B && dout.size(1) == D && dout.size(2) == L && dout.scalar_type() == x.scalar_type(),
              "dout mismatch");
  Tensor w = f32c(weight);
  Tensor bb = f32c_opt(bias);
  Tensor dx = dx_out.has_value() && dx_out->defined() ? *dx_out : at::empty({D, B, L}, x.options()).permute({1, 0, 2});
  TORCH_CHECK(dx.size(0) == B && dx.size(1) == D && dx.size(2) == L && dx.stride(2) == 1 &&
              dx.scalar_type() == x.scalar_type(), "dx_out layout");
  const int W = (int)w.size(1);
  const PartMode pm = part_mode(part_mode_);
  Tensor part = part_tensor(part_buf, part_mode_, {B, D, W + 1}, x.options());
  auto dwb = at::empty({pm.reduce ? D : 0, W + 1}, x.options().dtype(at::kFloat));  // [taps | bias] per channel
  HIPCHK(mamba_amd::launch_conv_cf_bwd(x.data_ptr(), dcode(x.scalar_type()), x.stride(0), x.stride(1), w.data_ptr<float>(),
                                       fptr(bb), dout.data_ptr(), dout.stride(0), dout.stride(1), dx.data_ptr(),
                                       dx.stride(0), dx.stride(1), part.data_ptr<float>(),
                                       pm.reduce ? dwb.data_ptr<float>() : nullptr, nullptr, pm.pacc, (int)B, (int)D,
                                       (int)L, W, silu, cur_stream()));
  return {dx, dwb.narrow(1, 0, W), dwb.select(1, W)};
}

Tensor conv1d_cl_fwd(Tensor x, Tensor weight, optional<Tensor> bias, bool silu) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "x must be (b, l, c) with unit channel stride");
  const int64_t B = x.size(0), L = x.size(1), C = x.size(2);
  Tensor w = f32c(weight);
  TORCH_CHECK(w.dim() == 2 && w.size(0) == C && w.size(1) >= 2 && w.size(1) <= 4, "weight must be (c, w), 2<=w<=4");
  Tensor bb = f32c_opt(bias);
  auto out = at::empty({B, L, C}, x.options());
  HIPCHK(mamba_amd::launch_conv_cl_fwd(x.data_ptr(), dcode(x.scalar_type()), x.stride(0), x.stride(1), w.data_ptr<float>(),
                                       fptr(bb), out.data_ptr(), out.stride(0), out.stride(1), (int)B, (int)L, (int)C,
                                       (int)w.size(1), silu, cur_stream()));
  return out;
}

std::tuple<Tensor, Tensor, Tensor> conv1d_cl_bwd(Tensor x, Tensor weight, optional<Tensor> bias, Tensor dout, bool silu,
                                                 optional<Tensor> dx_out, optional<Tensor> part_buf,
                                                 int64_t part_mode_) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "x must be (b, l, c) with unit channel stride");
  if (dout.stride(2) != 1) dout = dout.contiguous();
  const int64_t B = x.size(0), L = x.size(1), C = x.size(2);
  TORCH_CHECK(dout.size(0) == B && dout.size(1) == L && dout.size(2) == C && dout.scalar_type() == x.scalar_type(),
              "dout mismatch");
  Tensor w = f32c(weight);
  Tensor bb = f32c_opt(bias);
  Tensor dx = dx_out.has_value() && dx_out->defined() ? *dx_out : at::empty({B, L, C}, x.options());
  TORCH_CHECK(dx.size(0) == B && dx.size(1) == L && dx.size(2) == C && dx.stride(2) == 1 &&
              dx.scalar_type() == x.scalar_type(), "dx_out layout");
  const int W = (int)w.size(1);
  const PartMode pm = part_mode(part_mode_);
  Tensor part = part_tensor(part_buf, part_mode_, {mamba_amd::conv_cl_bwd_partial_rows((int)B, (int)L), C, W + 1},
                            x.options());
  auto dwb = at::empty({pm.reduce ? C : 0, W + 1}, x.options().dtype(at::kFloat));  // [taps | bias] per channel
  HIPCHK(mamba_amd::launch_conv_cl_bwd(x.data_ptr(), dcode(x.scalar_type()), x.stride(0), x.stride(1), w.data_ptr<float>(),
                                       fptr(bb), dout.data_ptr(), dout.stride(0), dout.stride(1), dx.data_ptr(),
                                       dx.stride(0), dx.stride(1), part.data_ptr<float>(),
                                       pm.reduce ? dwb.data_ptr<float>() : nullptr, nullptr, pm.pacc, (int)B, (int)L,
                                       (int)C, W, silu, cur_stream()));
  return {dx, dwb.narrow(1, 0, W), dwb.select(1, W)};
}

// varlen / state hand-off conv (kernels/conv1d.hip ConvVarArgs), channel-last x (b, l, c):
// seq_idx (b, l) int, initial_states (b, c, W-1), final states returned when want_final.
static void conv_var_common(mamba_amd::ConvVarArgs& a, const Tensor& x, const Tensor& w, const Tensor& bb,
                            const optional<Tensor>& seq_idx, const optional<Tensor>& init, Tensor& sq, Tensor& ini) {
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "x must be (b, l, c) with unit channel stride");
  a.Bn = (int)x.size(0); a.L = (int)x.size(1); a.C = (int)x.size(2); a.Wd = (int)w.size(1);
  TORCH_CHECK(w.dim() == 2 && w.size(0) == a.C && a.Wd >= 2 && a.Wd <= 4, "weight must be (c, w), 2<=w<=4");
  a.dt = dcode(x.scalar_type());
  a.x = x.data_ptr(); a.sxb = x.stride(0); a.sxl = x.stride(1);
  a.w = w.data_ptr<float>(); a.bias = fptr(bb);
  if (seq_idx.has_value() && seq_idx->defined()) {
    sq = seq_idx->to(at::kInt).contiguous();
    TORCH_CHECK(sq.dim() == 2 && sq.size(0) == a.Bn && sq.size(1) == a.L, "seq_idx must be (b, l)");
    a.seq = sq.data_ptr<int>(); a.sqb = sq.stride(0);
  }
  if (init.has_value() && init->defined()) {
    ini = *init;
    if (ini.stride(2) != 1) ini = ini.contiguous();
    TORCH_CHECK(ini.dim() == 3 && ini.size(0) == a.Bn && ini.size(1) == a.C && ini.size(2) == a.Wd - 1 &&
                ini.scalar_type() == x.scalar_type(), "initial_states must be (b, c, w-1), x's dtype");
    a.init = ini.data_ptr(); a.sib = ini.stride(0); a.sic = ini.stride(1);
  }
}

std::tuple<Tensor, Tensor> conv1d_cl_var_fwd(Tensor x, Tensor weight, optional<Tensor> bias, bool silu,
                                            optional<Tensor> seq_idx, optional<Tensor> initial_states, bool want_final) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  mamba_amd::ConvVarArgs a{};
  Tensor w = f32c(weight), bb = f32c_opt(bias), sq, ini;
  conv_var_common(a, x, w, bb, seq_idx, initial_states, sq, ini);
  auto out = at::empty({a.Bn, a.L, a.C}, x.options());
  a.out = out.data_ptr(); a.sob = out.stride(0); a.sol = out.stride(1);
  Tensor fin = want_final ? at::empty({a.Bn, a.C, a.Wd - 1}, x.options()) : at::empty({0}, x.options());
  if (want_final) { a.fin = fin.data_ptr(); a.sfb = fin.stride(0); a.sfc = fin.stride(1); }
  a.silu = silu; a.backward = false;
  HIPCHK(mamba_amd::launch_conv_cl_var(a, cur_stream()));
  return {out, fin};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> conv1d_cl_var_bwd(Tensor x, Tensor weight, optional<Tensor> bias,
                                                             Tensor dout, bool silu, optional<Tensor> seq_idx,
                                                             optional<Tensor> initial_states, optional<Tensor> dfinal,
                                                             optional<Tensor> dx_out, optional<Tensor> part_buf,
                                                             int64_t part_mode_) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  mamba_amd::ConvVarArgs a{};
  Tensor w = f32c(weight), bb = f32c_opt(bias), sq, ini;
  conv_var_common(a, x, w, bb, seq_idx, initial_states, sq, ini);
  if (dout.stride(2) != 1) dout = dout.contiguous();
  TORCH_CHECK(dout.sizes() == x.sizes() && dout.scalar_type() == x.scalar_type(), "dout mismatch");
  a.g = dout.data_ptr(); a.sgb = dout.stride(0); a.sgl = dout.stride(1);
  Tensor dfin;
  if (dfinal.has_value() && dfinal->defined()) {
    dfin = dfinal->to(x.scalar_type());
    if (dfin.stride(2) != 1) dfin = dfin.contiguous();
    TORCH_CHECK(dfin.dim() == 3 && dfin.size(0) == a.Bn && dfin.size(1) == a.C && dfin.size(2) == a.Wd - 1,
                "dfinal must be (b, c, w-1)");
    a.dfin = dfin.data_ptr(); a.sdfb = dfin.stride(0); a.sdfc = dfin.stride(1);
  }
  Tensor dx = dx_out.has_value() && dx_out->defined() ? *dx_out : at::empty({a.Bn, a.L, a.C}, x.options());
  TORCH_CHECK(dx.sizes() == x.sizes() && dx.stride(2) == 1 && dx.scalar_type() == x.scalar_type(), "dx_out layout");
  a.dx = dx.data_ptr(); a.sdb = dx.stride(0); a.sdl = dx.stride(1);
  Tensor dinit = a.init ? at::empty({a.Bn, a.C, a.Wd - 1}, x.options()) : at::empty({0}, x.options());
  if (a.init) { a.dinit = dinit.data_ptr(); a.sdib = dinit.stride(0); a.sdic = dinit.stride(1); }
  const PartMode pm = part_mode(part_mode_);
  Tensor part = part_tensor(part_buf, part_mode_, {mamba_amd::conv_cl_var_partial_rows(a.Bn, a.L), a.C, a.Wd + 1},
                            x.options());
  auto dwb = at::empty({pm.reduce ? a.C : 0, a.Wd + 1}, x.options().dtype(at::kFloat));
  a.part = part.data_ptr<float>(); a.dw = pm.reduce ? dwb.data_ptr<float>() : nullptr; a.pacc = pm.pacc;
  a.silu = silu; a.backward = true;
  HIPCHK(mamba_amd::launch_conv_cl_var(a, cur_stream()));
  return {dx, dwb.narrow(1, 0, a.Wd), dwb.select(1, a.Wd), dinit};
}

Tensor conv1d_update(Tensor x, Tensor conv_state, Tensor weight, optional<Tensor> bias, bool silu) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be (b, c)");
  const int64_t B = x.size(0), C = x.size(1);
  Tensor w = f32c(weight);
  TORCH_CHECK(w.size(0) == C && conv_state.size(0) == B && conv_state.size(1) == C && conv_state.size(2) >= w.size(1) - 1 &&
              conv_state.size(2) <= 16 && conv_state.stride(2) == 1 && conv_state.scalar_type() == x.scalar_type(),
              "conv_state must be (b, c, state_len >= w-1) with unit last stride");
  Tensor bb = f32c_opt(bias);
  auto out = at::empty({B, C}, x.options());
  HIPCHK(mamba_amd::launch_conv_update(x.data_ptr(), dcode(x.scalar_type()), x.stride(0), conv_state.data_ptr(),
                                       conv_state.stride(0), conv_state.stride(1), w.data_ptr<float>(), fptr(bb),
                                       out.data_ptr(), (int)B, (int)C, (int)w.size(1), (int)conv_state.size(2), silu,
                                       cur_stream()));
  return out;
}

// ---------------------------------------------------------------------------------------------
// SSD
int pick_hg(int B, int nc, int H, int G) {
  const int hpg = H / G;
  if (const char* e = std::getenv("MAMBA_AMD_SSD_HG")) {  // tuning override (must divide H/G, <= 32)
    const int v = std::atoi(e);
    if (v >= 1 && v <= 32 && hpg % v == 0) return v;
  }
  // largest head group (<= 32) that still leaves >= 512 workgroups (2 per CU): measured on MI355X
  // at the 280M shape, 8 -> 24 heads per workgroup is -12% chunk-bwd time (CB^T and the B/C staging
  // are amortised over more heads)
  int best = 1;
  for (int d = 1; d <= 32 && d <= hpg; ++d)
    if (hpg % d == 0 && (int64_t)B * nc * (H / d) >= 512) best = d;
  return best;
}

void ssd_common(mamba_amd::SSDArgs& a, const Tensor& x, const Tensor& dt, const Tensor& A, const Tensor& Bm,
                const Tensor& Cm, int64_t chunk, bool softplus, double dt_min, double dt_max) {
  TORCH_CHECK(chunk == 64, "native SSD chunk must be 64");
  TORCH_CHECK(x.dim() == 4 && x.stride(3) == 1 && x.scalar_type() == at::kBFloat16, "x must be bf16 (b,l,h,p), unit p");
  TORCH_CHECK(x.size(3) == 64, "native SSD supports headdim 64");
  TORCH_CHECK(Bm.dim() == 4 && Cm.dim() == 4 && Bm.stride(3) == 1 && Cm.stride(3) == 1 &&
              Bm.scalar_type() == at::kBFloat16 && Cm.scalar_type() == at::kBFloat16, "B/C must be bf16 (b,l,g,n)");
  a.B = x.size(0); a.L = x.size(1); a.H = x.size(2); a.G = Bm.size(2); a.N = Bm.size(3);
  TORCH_CHECK(a.N == 64 || a.N == 128, "native SSD supports d_state 64 or 128");
  TORCH_CHECK(a.H % a.G == 0 && Bm.size(0) == a.B && Bm.size(1) == a.L && Cm.sizes() == Bm.sizes(), "B/C shape");
  TORCH_CHECK(dt.dim() == 3 && dt.size(0) == a.B && dt.size(1) == a.L && dt.size(2) == a.H, "dt shape");
  TORCH_CHECK(A.numel() == a.H, "A shape");
  // 16-B aligned rows for the tile loads
  auto al = [](const Tensor& t, int64_t s) { return ((uintptr_t)t.data_ptr() % 16 == 0) && (s % 8 == 0); };
  TORCH_CHECK(al(x, x.stride(1)) && x.stride(2) % 8 == 0 && x.stride(0) % 8 == 0, "x rows must be 16-B aligned");
  TORCH_CHECK(al(Bm, Bm.stride(1)) && al(Cm, Cm.stride(1)) && Bm.stride(0) % 8 == 0 && Cm.stride(0) % 8 == 0 &&
              Bm.stride(2) % 8 == 0 && Cm.stride(2) % 8 == 0, "B/C rows must be 16-B aligned");
  a.nc = (a.L + 63) / 64; a.Lp = a.nc * 64;
  a.HG = pick_hg(a.B, a.nc, a.H, a.G); a.nhg = a.H / a.HG;
  a.nseg = mamba_amd::ssd_pick_segments(a.B, a.H, a.nc);
  a.cps = (a.nc + a.nseg - 1) / a.nseg;
  a.nseg = (a.nc + a.cps - 1) / a.cps;  // no empty segment
  a.x = (const mamba_amd::bf16_t*)x.data_ptr(); a.sxb = x.stride(0); a.sxl = x.stride(1); a.sxh = x.stride(2);
  a.dt = dt.data_ptr(); a.dt_dtype = dcode(dt.scalar_type());
  a.sdtb = dt.stride(0); a.sdtl = dt.stride(1); a.sdth = dt.stride(2);
  a.Bm = (const mamba_amd::bf16_t*)Bm.data_ptr(); a.sBb = Bm.stride(0); a.sBl = Bm.stride(1); a.sBg = Bm.stride(2);
  a.Cm = (const mamba_amd::bf16_t*)Cm.data_ptr(); a.sCb = Cm.stride(0); a.sCl = Cm.stride(1); a.sCg = Cm.stride(2);
  a.softplus = softplus; a.dt_min = (float)dt_min; a.dt_max = (float)dt_max;
}

// the segment-parallel walks' workspace: (b, h, nseg - 1) fp32 states and their decays (none for one segment)
Tensor ssd_seg_workspace(mamba_amd::SSDArgs& a, const Tensor& like) {
  if (a.nseg < 2) return Tensor();
  const int64_t n = (int64_t)a.B * a.H * (a.nseg - 1);
  auto ws = at::empty({n * 64 * a.N + n}, like.options().dtype(at::kFloat));
  a.seg = ws.data_ptr<float>();
  a.segd = a.seg + n * 64 * a.N;
  return ws;
}

// fp32 sequential SSD forward (evaluation in fp32): x (b,l,h,64), dt (b,l,h), B/C (b,l,g,n) fp32
std::tuple<Tensor, Tensor> ssd_fwd_f32(Tensor x, Tensor dt, Tensor A, Tensor Bm, Tensor Cm, optional<Tensor> D,
                                       optional<Tensor> dt_bias, optional<Tensor> init, bool softplus,
                                       double dt_min, double dt_max, bool want_final) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto f32 = [](const Tensor& t) { return t.scalar_type() == at::kFloat; };
  TORCH_CHECK(f32(x) && f32(dt) && f32(Bm) && f32(Cm), "ssd_fwd_f32: fp32 operands");
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 64 && x.stride(3) == 1, "x must be (b,l,h,64), unit p");
  TORCH_CHECK(Bm.dim() == 4 && Cm.sizes() == Bm.sizes() && Bm.stride(3) == 1 && Cm.stride(3) == 1, "B/C (b,l,g,n)");
  mamba_amd::SSDF32Args a{};
  a.B = x.size(0); a.L = x.size(1); a.H = x.size(2); a.G = Bm.size(2); a.N = Bm.size(3);
  TORCH_CHECK(a.N == 64 || a.N == 128, "d_state 64 or 128");
  TORCH_CHECK(a.H % a.G == 0 && Bm.size(0) == a.B && Bm.size(1) == a.L, "B/C shape");
  TORCH_CHECK(dt.dim() == 3 && dt.size(0) == a.B && dt.size(1) == a.L && dt.size(2) == a.H, "dt shape");
  Tensor Af = f32c(A), Df = f32c_opt(D), bf = f32c_opt(dt_bias);
  TORCH_CHECK(Af.numel() == a.H && (!Df.defined() || Df.numel() == a.H), "A / D per head");
  a.x = x.data_ptr<float>(); a.sxb = x.stride(0); a.sxl = x.stride(1); a.sxh = x.stride(2);
  a.dt = dt.data_ptr<float>(); a.sdtb = dt.stride(0); a.sdtl = dt.stride(1); a.sdth = dt.stride(2);
  a.A = Af.data_ptr<float>(); a.D = fptr(Df); a.dt_bias = fptr(bf);
  a.Bm = Bm.data_ptr<float>(); a.sBb = Bm.stride(0); a.sBl = Bm.stride(1); a.sBg = Bm.stride(2);
  a.Cm = Cm.data_ptr<float>(); a.sCb = Cm.stride(0); a.sCl = Cm.stride(1); a.sCg = Cm.stride(2);
  Tensor initc;
  if (init.has_value() && init->defined()) {
    initc = init->to(at::kFloat).contiguous();
    TORCH_CHECK(initc.numel() == (int64_t)a.B * a.H * 64 * a.N, "initial states (b,h,p,n)");
    a.init = initc.data_ptr<float>();
  }
  auto y = at::empty({a.B, a.L, a.H, 64}, x.options());
  a.y = y.data_ptr<float>(); a.syb = y.stride(0); a.syl = y.stride(1); a.syh = y.stride(2);
  Tensor fin = want_final ? at::empty({a.B, a.H, 64, a.N}, x.options()) : at::empty({0}, x.options());
  a.final_state = want_final ? fin.data_ptr<float>() : nullptr;
  a.softplus = softplus;
  a.clamp = !(dt_min == 0.0 && std::isinf(dt_max));
  a.dt_min = (float)dt_min; a.dt_max = (float)dt_max;
  HIPCHK(mamba_amd::launch_ssd_fwd_f32(a, cur_stream()));
  return {y, fin};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> ssd_fwd(Tensor x, Tensor dt, Tensor A, Tensor Bm, Tensor Cm,
                                                           optional<Tensor> D, optional<Tensor> dt_bias,
                                                           optional<Tensor> init, int64_t chunk, bool softplus,
                                                           double dt_min, double dt_max, bool A_is_log,
                                                           optional<Tensor> seq_idx) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  mamba_amd::SSDArgs a{};
  ssd_common(a, x, dt, A, Bm, Cm, chunk, softplus, dt_min, dt_max);
  a.a_log = A_is_log;
  Tensor Af = f32c(A), Df = f32c_opt(D), bf = f32c_opt(dt_bias), If = f32c_opt(init);
  if (Df.defined()) TORCH_CHECK(Df.numel() == a.H, "D must be (h,)");
  if (bf.defined()) TORCH_CHECK(bf.numel() == a.H, "dt_bias must be (h,)");
  if (If.defined()) TORCH_CHECK(If.numel() == (int64_t)a.B * a.H * 64 * a.N, "initial_states must be (b,h,p,n)");
  a.A = Af.data_ptr<float>(); a.D = fptr(Df); a.dt_bias = fptr(bf); a.init = fptr(If);
  Tensor sq;
  if (seq_idx.has_value() && seq_idx->defined()) {
    sq = seq_idx->to(at::kInt);
    TORCH_CHECK(sq.dim() == 2 && sq.size(0) == a.B && sq.size(1) == a.L && sq.is_cuda(), "seq_idx must be (b, l)");
    a.seq = sq.data_ptr<int>(); a.sqb = sq.stride(0); a.sql = sq.stride(1);
  }
  auto fo = x.options().dtype(at::kFloat);
  auto dtp = at::empty({a.B, a.H, a.Lp}, fo);
  auto cum = at::empty({a.B, a.H, a.Lp}, fo);
  auto states = at::empty({a.B, a.nc, a.H, 64, a.N}, x.options());
  auto final_ = at::empty({a.B, a.H, 64, a.N}, fo);
  auto y = at::empty({a.B, a.L, a.H, 64}, x.options());
  a.dtp = dtp.data_ptr<float>(); a.cum = cum.data_ptr<float>();
  a.states = (mamba_amd::bf16_t*)states.data_ptr(); a.final_state = final_.data_ptr<float>();
  a.y = (mamba_amd::bf16_t*)y.data_ptr(); a.syb = y.stride(0); a.syl = y.stride(1); a.syh = y.stride(2);
  Tensor seg_ws = ssd_seg_workspace(a, x);
  HIPCHK(mamba_amd::launch_ssd_fwd(a, cur_stream()));
  return {y, cum, dtp, states, final_};
}

std::vector<Tensor> ssd_bwd(Tensor dy, Tensor x, Tensor dt, Tensor A, Tensor Bm, Tensor Cm, optional<Tensor> D,
                            optional<Tensor> dt_bias, optional<Tensor> init, Tensor cum, Tensor dtp, Tensor states,
                            optional<Tensor> dfinal, int64_t chunk, bool softplus, double dt_min, double dt_max,
                            optional<Tensor> dx_out, optional<Tensor> ddt_out, optional<Tensor> dB_out,
                            optional<Tensor> dC_out, bool A_is_log, optional<Tensor> part_buf, int64_t part_mode_,
                            int64_t ddt_zero_pad) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  mamba_amd::SSDArgs a{};
  ssd_common(a, x, dt, A, Bm, Cm, chunk, softplus, dt_min, dt_max);
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.stride(3) == 1 && dy.scalar_type() == at::kBFloat16, "dy layout");
  if (!(((uintptr_t)dy.data_ptr() % 16 == 0) && dy.stride(1) % 8 == 0 && dy.stride(2) % 8 == 0 && dy.stride(0) % 8 == 0))
    dy = dy.contiguous();
  Tensor Af = f32c(A), Df = f32c_opt(D), bf = f32c_opt(dt_bias), If = f32c_opt(init), dF = f32c_opt(dfinal);
  a.A = Af.data_ptr<float>(); a.D = fptr(Df); a.dt_bias = fptr(bf); a.init = fptr(If);
  TORCH_CHECK(cum.is_contiguous() && dtp.is_contiguous() && states.is_contiguous(), "saved tensors must be contiguous");
  a.cum = cum.data_ptr<float>(); a.dtp = dtp.data_ptr<float>(); a.states = (mamba_amd::bf16_t*)states.data_ptr();
  a.dy = (const mamba_amd::bf16_t*)dy.data_ptr(); a.sdyb = dy.stride(0); a.sdyl = dy.stride(1); a.sdyh = dy.stride(2);
  a.dfinal = fptr(dF);
  auto fo = x.options().dtype(at::kFloat);
  auto dstates = at::empty_like(states);
  a.dstates = (mamba_amd::bf16_t*)dstates.data_ptr();
  Tensor dinit = If.defined() ? at::empty({a.B, a.H, 64, a.N}, fo) : at::empty({0}, fo);
  a.dinit = If.defined() ? dinit.data_ptr<float>() : nullptr;
  Tensor dx = dx_out.has_value() && dx_out->defined() ? *dx_out : at::empty_like(x, at::MemoryFormat::Contiguous);
  TORCH_CHECK(dx.sizes() == x.sizes() && dx.stride(3) == 1 && dx.scalar_type() == at::kBFloat16 &&
              (uintptr_t)dx.data_ptr() % 16 == 0 && dx.stride(1) % 8 == 0 && dx.stride(0) % 8 == 0 &&
              dx.stride(2) % 8 == 0, "dx layout");
  Tensor ddt = ddt_out.has_value() && ddt_out->defined() ? *ddt_out : at::empty(dt.sizes(), dt.options());
  TORCH_CHECK(ddt.sizes() == dt.sizes(), "ddt shape");
  Tensor dB = dB_out.has_value() && dB_out->defined() ? *dB_out : at::empty(Bm.sizes(), Bm.options());
  Tensor dC = dC_out.has_value() && dC_out->defined() ? *dC_out : at::empty(Cm.sizes(), Cm.options());
  auto chk = [](const Tensor& t) {
    TORCH_CHECK(t.stride(3) == 1 && t.scalar_type() == at::kBFloat16 && (uintptr_t)t.data_ptr() % 16 == 0 &&
                t.stride(1) % 8 == 0 && t.stride(0) % 8 == 0 && t.stride(2) % 8 == 0, "dB/dC layout");
  };
  chk(dB);
  chk(dC);
  a.dx = (mamba_amd::bf16_t*)dx.data_ptr(); a.sdxb = dx.stride(0); a.sdxl = dx.stride(1); a.sdxh = dx.stride(2);
  a.ddt = ddt.data_ptr(); a.ddt_dtype = dcode(ddt.scalar_type());
  a.sddtb = ddt.stride(0); a.sddtl = ddt.stride(1); a.sddth = ddt.stride(2);
  if (ddt_zero_pad > 0) {
    // the pad columns [H, H + pad) of every ddt row are part of the same allocation (the caller's padded row);
    // zeroed with 16-B stores: bf16, unit column stride, pad a multiple of 8, 16-B aligned pad start and rows
    TORCH_CHECK(ddt.scalar_type() == at::kBFloat16 && ddt.stride(2) == 1 && ddt_zero_pad % 8 == 0 &&
                ddt.stride(1) >= a.H + ddt_zero_pad && ddt.stride(1) % 8 == 0 && ddt.stride(0) % 8 == 0 &&
                ((uintptr_t)ddt.data_ptr() + 2 * (uintptr_t)a.H) % 16 == 0,
                "ssd_bwd: ddt_zero_pad needs bf16 rows with 16-B aligned pad columns");
    a.ddt_zero_pad = (int)ddt_zero_pad;
  }
  a.dB = (mamba_amd::bf16_t*)dB.data_ptr(); a.sdBb = dB.stride(0); a.sdBl = dB.stride(1); a.sdBg = dB.stride(2);
  a.dC = (mamba_amd::bf16_t*)dC.data_ptr(); a.sdCb = dC.stride(0); a.sdCl = dC.stride(1); a.sdCg = dC.stride(2);
  // one head group per B/C group: the chunk kernel finishes dB / dC itself (no head-group partials)
  a.fuse_dbc = a.HG == a.H / a.G;
  const int64_t pn = a.fuse_dbc ? 0 : 1;
  auto part_dcb = at::empty({pn * a.B, a.nc, a.nhg, 64, 64}, fo);
  auto part_db = at::empty({pn * a.B, a.nc, a.nhg, 64, a.N}, fo);
  auto part_dc = at::empty({pn * a.B, a.nc, a.nhg, 64, a.N}, fo);
  const PartMode pm = part_mode(part_mode_);
  Tensor part_small = part_tensor(part_buf, part_mode_, {a.B * a.nc, 3, a.H}, x.options());
  a.pacc = pm.pacc;
  a.part_dcb = part_dcb.data_ptr<float>(); a.part_db = part_db.data_ptr<float>(); a.part_dc = part_dc.data_ptr<float>();
  a.psl = 3 * a.H;
  a.part_dA = part_small.data_ptr<float>(); a.part_dD = a.part_dA + a.H; a.part_dbias = a.part_dA + 2 * a.H;
  a.a_log = A_is_log;
  Tensor seg_ws = ssd_seg_workspace(a, x);
  HIPCHK(mamba_amd::launch_ssd_bwd(a, cur_stream()));
  if (!pm.reduce) return {dx, ddt, at::empty({0}, fo), dB, dC, at::empty({0}, fo), at::empty({0}, fo), dinit};
  auto sums = at::empty({3, a.H}, fo);  // deterministic column sums over the (b, chunk) rows
  HIPCHK(mamba_amd::launch_colsum(part_small.data_ptr<float>(), a.B * a.nc, 3 * a.H, sums.data_ptr<float>(), cur_stream()));
  Tensor dA = sums[0].to(A.scalar_type());
  Tensor dD = D.has_value() && D->defined() ? sums[1].to(D->scalar_type()) : at::empty({0}, fo);
  Tensor dbias = dt_bias.has_value() && dt_bias->defined() ? sums[2].to(dt_bias->scalar_type()) : at::empty({0}, fo);
  return {dx, ddt, dA, dB, dC, dD, dbias, dinit};
}

// ---------------------------------------------------------------------------------------------
// selective scan (Mamba-1)
void selscan_common(mamba_amd::SelScanArgs& a, const Tensor& u, const Tensor& delta, const Tensor& A, const Tensor& Bm,
                    const Tensor& Cm, const Tensor& z, bool softplus) {
  TORCH_CHECK(u.dim() == 3 && u.stride(2) == 1 && delta.stride(2) == 1, "u/delta must be (b,d,l) with unit time stride");
  TORCH_CHECK(delta.sizes() == u.sizes() && delta.scalar_type() == u.scalar_type(), "delta mismatch");
  TORCH_CHECK(Bm.dim() == 4 && Cm.dim() == 4 && Bm.stride(3) == 1 && Cm.stride(3) == 1, "B/C must be (b,g,n,l), unit l");
  TORCH_CHECK(Bm.scalar_type() == u.scalar_type() && Cm.scalar_type() == u.scalar_type(), "B/C dtype must match u");
  a.B = u.size(0); a.D = u.size(1); a.L = u.size(2); a.G = Bm.size(1); a.N = Bm.size(2);
  TORCH_CHECK(A.dim() == 2 && A.size(0) == a.D && A.size(1) == a.N, "A must be (d, n)");
  TORCH_CHECK(a.N == 16 || a.N == 8 || a.N == 4, "native selective scan supports d_state 4/8/16");
  TORCH_CHECK(a.D % a.G == 0 && Bm.size(3) == a.L && Cm.sizes() == Bm.sizes(), "B/C shape");
  a.dtype = dcode(u.scalar_type());
  a.softplus = softplus;
  auto v8 = [&](const Tensor& t, int64_t s0, int64_t s1) {
    return a.dtype == mamba_amd::kBF16 && (uintptr_t)t.data_ptr() % 16 == 0 && s0 % 8 == 0 && s1 % 8 == 0;
  };
  a.vec = v8(u, u.stride(0), u.stride(1)) && v8(delta, delta.stride(0), delta.stride(1));
  a.vecbc = v8(Bm, Bm.stride(0), Bm.stride(2)) && v8(Cm, Cm.stride(0), Cm.stride(2)) && Bm.stride(1) % 8 == 0 &&
            Cm.stride(1) % 8 == 0;
  a.vecz = z.defined() && v8(z, z.stride(0), z.stride(1));
  a.u_ = u.data_ptr(); a.sub = u.stride(0); a.sud = u.stride(1);
  a.delta_ = delta.data_ptr(); a.sdb = delta.stride(0); a.sdd = delta.stride(1);
  a.Bm_ = Bm.data_ptr(); a.sBb = Bm.stride(0); a.sBg = Bm.stride(1); a.sBn = Bm.stride(2);
  a.Cm_ = Cm.data_ptr(); a.sCb = Cm.stride(0); a.sCg = Cm.stride(1); a.sCn = Cm.stride(2);
  if (z.defined()) {
    TORCH_CHECK(z.sizes() == u.sizes() && z.stride(2) == 1 && z.scalar_type() == u.scalar_type(), "z layout");
    a.z_ = z.data_ptr(); a.szb = z.stride(0); a.szd = z.stride(1);
  }
}

// fused dt_proj (kernels/selective_scan.hip DTF): delta_raw = dtw (D, R) . dtx (R, B L) is computed inside the scan
// kernels; the (b, d, l) delta tensor is never formed.  u stands in for delta in the shared layout checks.
void selscan_dt_args(mamba_amd::SelScanArgs& a, const Tensor& dtw, const Tensor& dtx) {
  TORCH_CHECK(dtw.dim() == 2 && dtw.is_contiguous() && dtw.scalar_type() == at::kBFloat16 && dtw.size(0) == a.D,
              "dtw must be a contiguous bf16 (D, R) weight");
  TORCH_CHECK(dtx.dim() == 2 && dtx.size(0) == dtw.size(1) && dtx.size(1) == (int64_t)a.B * a.L && dtx.stride(1) == 1 &&
              dtx.scalar_type() == at::kBFloat16, "dtx must be (R, B L) bf16 rows with unit column stride");
  a.delta_ = nullptr;
  a.dtw_ = dtw.data_ptr(); a.dtx_ = dtx.data_ptr(); a.sdtx = dtx.stride(0); a.R = (int)dtw.size(1);
}

std::tuple<Tensor, Tensor, Tensor> selscan_fwd_impl(Tensor u, Tensor delta, Tensor A, Tensor Bm, Tensor Cm,
                                                    optional<Tensor> D, optional<Tensor> z, optional<Tensor> delta_bias,
                                                    bool softplus, optional<Tensor> dtw = c10::nullopt,
                                                    optional<Tensor> dtx = c10::nullopt) {
  check_cuda(u, "u");
  at::hip::HIPGuardMasqueradingAsCUDA guard(u.device());
  mamba_amd::SelScanArgs a{};
  Tensor zz = z.has_value() && z->defined() ? *z : Tensor();
  selscan_common(a, u, delta, A, Bm, Cm, zz, softplus);
  if (dtw.has_value()) selscan_dt_args(a, *dtw, *dtx);
  Tensor Af = f32c(A), Df = f32c_opt(D), bf = f32c_opt(delta_bias);
  a.A = Af.data_ptr<float>(); a.D_ = fptr(Df); a.delta_bias = fptr(bf);
  auto out = at::empty({a.D, a.B, a.L}, u.options()).permute({1, 0, 2});
  a.out_ = out.data_ptr(); a.sob = out.stride(0); a.sod = out.stride(1);
  a.carry_t = mamba_amd::selscan_carry_t(a);
  a.nct = (a.L + a.carry_t - 1) / a.carry_t;
  auto fo = u.options().dtype(at::kFloat);
  // (B, D, nct, N) view; 16-step carries are laid out (B, nct, D, N) (kernels: carry_index)
  auto carries = a.carry_t == mamba_amd::kSelScanCarryTile ? at::empty({a.B, a.D, a.nct, a.N}, fo)
                                                           : at::empty({a.B, a.nct, a.D, a.N}, fo).permute({0, 2, 1, 3});
  auto last = at::empty({a.B, a.D, a.N}, fo);
  a.carries = carries.data_ptr<float>(); a.last_state = last.data_ptr<float>();
  TORCH_CHECK(!a.dtw_ || mamba_amd::selscan_dt_fusable(a), "selscan_fwd_dt: shape not supported by the fused walk "
              "(bf16, d_state 16, D % 64 == 0, L % 16 == 0, B D >= 32768, dt_rank % 8 == 0 and <= 128)");
  HIPCHK(mamba_amd::launch_selscan_fwd(a, cur_stream()));
  return {out, carries, last};
}

std::tuple<Tensor, Tensor, Tensor> selscan_fwd(Tensor u, Tensor delta, Tensor A, Tensor Bm, Tensor Cm,
                                               optional<Tensor> D, optional<Tensor> z, optional<Tensor> delta_bias,
                                               bool softplus) {
  return selscan_fwd_impl(u, delta, A, Bm, Cm, D, z, delta_bias, softplus);
}

std::tuple<Tensor, Tensor, Tensor> selscan_fwd_dt(Tensor u, Tensor dtw, Tensor dtx, Tensor A, Tensor Bm, Tensor Cm,
                                                  optional<Tensor> D, optional<Tensor> z, optional<Tensor> delta_bias,
                                                  bool softplus) {
  return selscan_fwd_impl(u, u, A, Bm, Cm, D, z, delta_bias, softplus, dtw, dtx);
}

std::vector<Tensor> selscan_bwd_impl(Tensor dout, Tensor u, Tensor delta, Tensor A, Tensor Bm, Tensor Cm,
                                     optional<Tensor> D, optional<Tensor> z, optional<Tensor> delta_bias, Tensor carries,
                                     bool softplus, optional<Tensor> dz_out, optional<Tensor> dB_out,
                                     optional<Tensor> dC_out, optional<Tensor> part_buf = c10::nullopt,
                                     int64_t part_mode_ = 0, optional<Tensor> dtw = c10::nullopt,
                                     optional<Tensor> dtx = c10::nullopt) {
  check_cuda(u, "u");
  at::hip::HIPGuardMasqueradingAsCUDA guard(u.device());
  mamba_amd::SelScanArgs a{};
  Tensor zz = z.has_value() && z->defined() ? *z : Tensor();
  selscan_common(a, u, delta, A, Bm, Cm, zz, softplus);
  if (dtw.has_value()) selscan_dt_args(a, *dtw, *dtx);
  if (dout.stride(2) != 1 || dout.scalar_type() != u.scalar_type()) dout = dout.to(u.scalar_type()).contiguous();
  TORCH_CHECK(dout.sizes() == u.sizes(), "dout shape");
  // the carry granularity is the forward's choice: 16 steps (wave-per-state-group kernels) or 512
  a.nct = carries.size(2);
  a.carry_t = a.nct == (a.L + mamba_amd::kSelScanCarrySG - 1) / mamba_amd::kSelScanCarrySG
                  ? mamba_amd::kSelScanCarrySG : mamba_amd::kSelScanCarryTile;
  TORCH_CHECK(carries.dim() == 4 && carries.size(0) == a.B && carries.size(1) == a.D && carries.size(3) == a.N &&
              a.nct == (a.L + a.carry_t - 1) / a.carry_t, "carries shape");
  TORCH_CHECK(a.carry_t == mamba_amd::kSelScanCarryTile ? carries.is_contiguous()
                                                        : carries.permute({0, 2, 1, 3}).is_contiguous(),
              "carries layout (selscan_fwd's output)");
  Tensor Af = f32c(A), Df = f32c_opt(D), bf = f32c_opt(delta_bias);
  a.A = Af.data_ptr<float>(); a.D_ = fptr(Df); a.delta_bias = fptr(bf);
  a.carries = carries.data_ptr<float>();
  a.dout_ = dout.data_ptr(); a.sgb = dout.stride(0); a.sgd = dout.stride(1);
  a.vecg = a.dtype == mamba_amd::kBF16 && (uintptr_t)dout.data_ptr() % 16 == 0 && dout.stride(0) % 8 == 0 &&
           dout.stride(1) % 8 == 0;
  auto mk = [&]() { return at::empty({a.D, a.B, a.L}, u.options()).permute({1, 0, 2}); };
  Tensor du = mk(), ddelta = mk();
  a.du_ = du.data_ptr(); a.sdub = du.stride(0); a.sdud = du.stride(1);
  a.ddelta_ = ddelta.data_ptr(); a.sddb = ddelta.stride(0); a.sddd = ddelta.stride(1);
  Tensor dz;
  if (zz.defined()) {
    dz = dz_out.has_value() && dz_out->defined() ? *dz_out : mk();
    TORCH_CHECK(dz.sizes() == u.sizes() && dz.stride(2) == 1 && dz.scalar_type() == u.scalar_type(), "dz layout");
    a.dz_ = dz.data_ptr(); a.sdzb = dz.stride(0); a.sdzd = dz.stride(1);
  }
  Tensor dB = dB_out.has_value() && dB_out->defined() ? *dB_out : at::empty(Bm.sizes(), Bm.options());
  Tensor dC = dC_out.has_value() && dC_out->defined() ? *dC_out : at::empty(Cm.sizes(), Cm.options());
  TORCH_CHECK(dB.sizes() == Bm.sizes() && dC.sizes() == Cm.sizes() && dB.stride(3) == 1 && dC.stride(3) == 1 &&
              dB.scalar_type() == u.scalar_type() && dC.scalar_type() == u.scalar_type(), "dB/dC layout");
  a.dB_ = dB.data_ptr(); a.sdBb = dB.stride(0); a.sdBg = dB.stride(1); a.sdBn = dB.stride(2);
  a.dC_ = dC.data_ptr(); a.sdCb = dC.stride(0); a.sdCg = dC.stride(1); a.sdCn = dC.stride(2);
  auto fo = u.options().dtype(at::kFloat);
  a.Kc = mamba_amd::selscan_bwd_kc(a);
  TORCH_CHECK(!a.dtw_ || (mamba_amd::selscan_bwd_sequential(a) && mamba_amd::selscan_dt_fusable(a)),
              "selscan_bwd_dt: shape / layout not supported by the fused sequential backward");
  const int ndg = (a.D + a.Kc - 1) / a.Kc;
  auto part_bc = at::empty({2, a.B, ndg, a.N, a.L}, fo);
  a.part_dB = part_bc[0].data_ptr<float>(); a.part_dC = part_bc[1].data_ptr<float>();
  // A / D / delta_bias gradient partials: one flat fp32 buffer [dA (B, D, N) | dD (B, D) | dbias (B, D)].
  // part_mode (ops/grad_accum.py::deferred): 0 transient, reduced now; 1 / 2 store / add into the persistent
  // buffer, no reduction (empty dA / dD / dbias); 3 / 4 store / add, then reduce over the batch.
  const PartMode pm = part_mode(part_mode_);
  const int64_t nA = (int64_t)a.B * a.D * a.N, nd = (int64_t)a.B * a.D;
  const bool direct = part_mode_ > 0 && mamba_amd::selscan_bwd_sequential(a);  // kernel writes the buffer itself
  Tensor pb = direct ? part_tensor(part_buf, part_mode_, {nA + 2 * nd}, u.options()) : at::zeros({nA + 2 * nd}, fo);
  a.part_dA = pb.data_ptr<float>(); a.part_dD = a.part_dA + nA; a.part_dbias = a.part_dD + nd;
  a.pacc = direct && pm.pacc;
  HIPCHK(mamba_amd::launch_selscan_bwd(a, cur_stream()));
  if (part_mode_ > 0 && !direct) {  // time-parallel kernels accumulate into zeroed partials: fold them in here
    Tensor dst = part_tensor(part_buf, part_mode_, {nA + 2 * nd}, u.options());
    if (pm.pacc) dst.add_(pb); else dst.copy_(pb);
    pb = dst;
  }
  Tensor dA, dD, dbias;
  if (pm.reduce) {
    dA = pb.narrow(0, 0, nA).view({a.B, a.D, a.N}).sum(0).to(A.scalar_type());
    auto s2 = pb.narrow(0, nA, 2 * nd).view({2, a.B, a.D}).sum(1);
    dD = D.has_value() && D->defined() ? s2[0].to(D->scalar_type()) : at::empty({0}, fo);
    dbias = delta_bias.has_value() && delta_bias->defined() ? s2[1].to(delta_bias->scalar_type()) : at::empty({0}, fo);
  } else {
    dA = at::empty({0}, fo); dD = at::empty({0}, fo); dbias = at::empty({0}, fo);
  }
  if (!dz.defined()) dz = at::empty({0}, u.options());
  return {du, ddelta, dA, dB, dC, dD, dz, dbias};
}

std::vector<Tensor> selscan_bwd(Tensor dout, Tensor u, Tensor delta, Tensor A, Tensor Bm, Tensor Cm, optional<Tensor> D,
                                optional<Tensor> z, optional<Tensor> delta_bias, Tensor carries, bool softplus) {
  return selscan_bwd_impl(dout, u, delta, A, Bm, Cm, D, z, delta_bias, carries, softplus, c10::nullopt, c10::nullopt,
                          c10::nullopt);
}

std::vector<Tensor> selscan_bwd_into(Tensor dout, Tensor u, Tensor delta, Tensor A, Tensor Bm, Tensor Cm,
                                     optional<Tensor> D, optional<Tensor> z, optional<Tensor> delta_bias, Tensor carries,
                                     bool softplus, Tensor dz_out, Tensor dB_out, Tensor dC_out,
                                     optional<Tensor> part_buf, int64_t part_mode) {
  return selscan_bwd_impl(dout, u, delta, A, Bm, Cm, D, z, delta_bias, carries, softplus, dz_out, dB_out, dC_out,
                          part_buf, part_mode);
}

std::vector<Tensor> selscan_bwd_dt_into(Tensor dout, Tensor u, Tensor dtw, Tensor dtx, Tensor A, Tensor Bm, Tensor Cm,
                                        optional<Tensor> D, optional<Tensor> z, optional<Tensor> delta_bias,
                                        Tensor carries, bool softplus, Tensor dz_out, Tensor dB_out, Tensor dC_out,
                                        optional<Tensor> part_buf, int64_t part_mode) {
  return selscan_bwd_impl(dout, u, u, A, Bm, Cm, D, z, delta_bias, carries, softplus, dz_out, dB_out, dC_out, part_buf,
                          part_mode, dtw, dtx);
}

// decode-time recurrent update; Mamba-1: state (b,d,n), x/dt/z (b,d), A (d,n), B/C (b,n), D (d)
//                               Mamba-2: state (b,h,p,n), x/z (b,h,p), dt (b,h), A (h), B/C (b,g,n), D (h)
Tensor ssm_state_update(Tensor state, Tensor x, Tensor dt, Tensor A, Tensor Bm, Tensor Cm, optional<Tensor> D,
                        optional<Tensor> z, optional<Tensor> dt_bias, bool softplus) {
  check_cuda(x, "x");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(state.scalar_type() == at::kFloat && state.is_contiguous(), "state must be contiguous fp32");
  mamba_amd::SSMUpdateArgs a{};
  a.dtype = dcode(x.scalar_type());
  a.softplus = softplus;
  a.B = x.size(0);
  Tensor Af = f32c(A), Df = f32c_opt(D), bf = f32c_opt(dt_bias);
  Tensor xx = x, zz = z.has_value() && z->defined() ? *z : Tensor(), dtt = dt, Bb = Bm, Cc = Cm;
  if (state.dim() == 3) {  // Mamba-1 as H = d, P = 1
    a.H = state.size(1); a.P = 1; a.N = state.size(2); a.G = 1;
    a.A_per_n = true; a.D_per_p = false; a.dt_bias_per_p = false;
    xx = x.unsqueeze(-1);
    if (zz.defined()) zz = zz.unsqueeze(-1);
    dtt = dt.unsqueeze(-1);
    Bb = Bm.unsqueeze(1);
    Cc = Cm.unsqueeze(1);
  } else {
    a.H = state.size(1); a.P = state.size(2); a.N = state.size(3); a.G = Bm.size(1);
    a.A_per_n = false; a.D_per_p = false; a.dt_bias_per_p = false;
    dtt = dt.unsqueeze(-1).expand({a.B, a.H, a.P});
  }
  TORCH_CHECK(xx.stride(2) == 1 && Bb.stride(2) == 1 && Cc.stride(2) == 1, "unit inner strides required");
  TORCH_CHECK(Bb.scalar_type() == x.scalar_type() && Cc.scalar_type() == x.scalar_type() &&
              dtt.scalar_type() == x.scalar_type(), "dtype mismatch");
  a.state = state.data_ptr<float>();
  a.x_ = xx.data_ptr(); a.sxb = xx.stride(0); a.sxh = xx.stride(1);
  a.dt_ = dtt.data_ptr(); a.sdtb = dtt.stride(0); a.sdth = dtt.stride(1); a.sdtp = dtt.stride(2);
  a.A = Af.data_ptr<float>(); a.D = fptr(Df); a.dt_bias = fptr(bf);
  a.Bm_ = Bb.data_ptr(); a.sBb = Bb.stride(0); a.sBg = Bb.stride(1);
  a.Cm_ = Cc.data_ptr(); a.sCb = Cc.stride(0); a.sCg = Cc.stride(1);
  if (zz.defined()) { a.z_ = zz.data_ptr(); a.szb = zz.stride(0); a.szh = zz.stride(1); }
  auto out = at::empty(x.sizes(), x.options());
  a.out_ = out.data_ptr();
  HIPCHK(mamba_amd::launch_ssm_update(a, cur_stream()));
  return out;
}

// C = A . B^T for bf16 K-contiguous operands (the projection forward); out optional (may be a
// row-strided view, e.g. a column slice of a wider buffer)
Tensor gemm_tn(Tensor A, Tensor B, optional<Tensor> out) {
  check_cuda(A, "A");
  at::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "gemm_tn: A (M,K), B (N,K)");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "gemm_tn: bf16 operands");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "gemm_tn: K-contiguous operands");
  const int64_t M = A.size(0), N = B.size(0), K = A.size(1);
  Tensor C = out.has_value() && out->defined() ? *out : at::empty({M, N}, A.options());
  TORCH_CHECK(C.dim() == 2 && C.size(0) == M && C.size(1) == N && C.stride(1) == 1 && C.scalar_type() == at::kBFloat16,
              "gemm_tn: out (M,N) bf16 with unit column stride");
  TORCH_CHECK((uintptr_t)A.data_ptr() % 16 == 0 && (uintptr_t)B.data_ptr() % 16 == 0 && (uintptr_t)C.data_ptr() % 16 == 0,
              "gemm_tn: 16-B aligned operands");
  TORCH_CHECK(mamba_amd::gemm_tn_supported((int)M, (int)N, (int)K, A.stride(0), B.stride(0), C.stride(0)),
              "gemm_tn: needs K % 64 == 0, N % 8 == 0, row strides % 8 == 0");
  HIPCHK(mamba_amd::launch_gemm_tn_bf16(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0),
                                        (int)M, (int)N, (int)K, cur_stream()));
  return C;
}

// Y (C, R) = X (R, C)^T for a bf16 matrix with unit column stride (kernels/gemm.hip transpose_bf16_k)
Tensor transpose_bf16(Tensor X) {
  check_cuda(X, "X");
  at::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  TORCH_CHECK(X.dim() == 2 && X.scalar_type() == at::kBFloat16 && X.stride(1) == 1 && (uintptr_t)X.data_ptr() % 16 == 0,
              "transpose_bf16: 2-D bf16, unit column stride, 16-B aligned");
  const int64_t R = X.size(0), C = X.size(1);
  TORCH_CHECK(R % 8 == 0 && C % 8 == 0 && X.stride(0) % 8 == 0, "transpose_bf16: sizes and row stride % 8 == 0");
  Tensor Y = at::empty({C, R}, X.options());
  HIPCHK(mamba_amd::launch_transpose_bf16(X.data_ptr(), X.stride(0), Y.data_ptr(), R, (int)R, (int)C, cur_stream()));
  return Y;
}

// C (N, M) (+)= A (N, K) . B (K, M) for the channel-major Mamba-1 projections (x_proj / dt_proj and their
// input gradients); B / out rows are contiguous along M and may be row-strided views (x_dbl[:R])
Tensor gemm_skinny(Tensor A, Tensor B, optional<Tensor> out, bool accumulate) {
  check_cuda(A, "A");
  at::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(0), "gemm_skinny: A (N,K), B (K,M)");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "gemm_skinny: bf16 operands");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "gemm_skinny: unit inner strides");
  const int64_t N = A.size(0), K = A.size(1), M = B.size(1);
  Tensor C = out.has_value() && out->defined() ? *out : at::empty({N, M}, B.options());
  TORCH_CHECK(C.dim() == 2 && C.size(0) == N && C.size(1) == M && C.stride(1) == 1 && C.scalar_type() == at::kBFloat16,
              "gemm_skinny: out (N,M) bf16 with unit column stride");
  TORCH_CHECK(!accumulate || (out.has_value() && out->defined()), "gemm_skinny: accumulate needs out");
  TORCH_CHECK((uintptr_t)A.data_ptr() % 16 == 0 && (uintptr_t)B.data_ptr() % 16 == 0 && (uintptr_t)C.data_ptr() % 16 == 0,
              "gemm_skinny: 16-B aligned operands");
  TORCH_CHECK(mamba_amd::gemm_skinny_supported((int)N, (int)K, (int)M, A.stride(0), B.stride(0), C.stride(0)),
              "gemm_skinny: needs K % 8 == 0, M % 8 == 0, row strides % 8 == 0");
  HIPCHK(mamba_amd::launch_gemm_skinny(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0),
                                       (int)N, (int)K, (int)M, accumulate, cur_stream()));
  return C;
}

// dW (fp32, (P, Q)) = dY^T X for token-major bf16 dY (M, P), X (M, Q); out optional (accumulate=True
// adds into it, e.g. an existing fp32 .grad)
// C (+)= dY^T X on the staged-ring split-K engine (kernels/gemm_pipe.hip gemm_wg_k via launch_gemm_pipe): transient
// fp32 slabs, then the fixed-order slab sum into C.  la / lb: 1 = the operand is token-major ((M, P) / (M, Q)),
// 0 = channel-major ((P, M) / (Q, M)).  False when the engine does not take the layout (the caller falls back).
static bool staged_wgrad(const Tensor& dY, int la, const Tensor& X, int lb, int64_t M, int64_t P, int64_t Q,
                         Tensor& C, bool accumulate) {
  if (mamba_amd::gemm_wg_nb() == 0) return false;
  const int64_t lda = dY.size(0) == 1 ? dY.size(1) : dY.stride(0), ldb = X.size(0) == 1 ? X.size(1) : X.stride(0);
  // narrow outputs: the output dimension the engine tiles by rows (128-row tile form) should be the narrow one --
  // the Mamba-1 x_proj (80 x 1536) as is, the dt_proj (1536 x 48) as its transpose (48 x 1536), reduced into a
  // (Q, P) buffer and added transposed (256-column tiles would compute 81% zeros there)
  const bool swap = P > 128 && Q <= 128;
  const int64_t R = swap ? Q : P, Cc = swap ? P : Q;
  if (!(swap ? mamba_amd::gemm_pipe_supported(lb, la, (int)R, (int)Cc, (int)M, ldb, lda, Cc)
             : mamba_amd::gemm_pipe_supported(la, lb, (int)R, (int)Cc, (int)M, lda, ldb, Cc)))
    return false;
  const int S = mamba_amd::gemm_pipe_splits((int)R, (int)Cc, (int)M);
  const int bm = R <= 128 ? 128 : 256;
  auto part = at::empty({S, R, Cc}, dY.options().dtype(at::kFloat));
  const hipError_t e = swap ? mamba_amd::launch_gemm_pipe(lb, la, X.data_ptr(), ldb, dY.data_ptr(), lda, part.data_ptr(),
                                                          Cc, (int)R, (int)Cc, (int)M, S, R * Cc, 1, bm, cur_stream())
                            : mamba_amd::launch_gemm_pipe(la, lb, dY.data_ptr(), lda, X.data_ptr(), ldb, part.data_ptr(),
                                                          Cc, (int)R, (int)Cc, (int)M, S, R * Cc, 1, bm, cur_stream());
  if (e == hipErrorInvalidValue) return false;
  HIPCHK(e);
  if (!swap) {
    HIPCHK(mamba_amd::launch_gp_reduce(part.data_ptr<float>(), S, P * Q, P * Q, C.data_ptr<float>(), accumulate,
                                       cur_stream()));
    return true;
  }
  auto ct = at::empty({Q, P}, dY.options().dtype(at::kFloat));
  HIPCHK(mamba_amd::launch_gp_reduce(part.data_ptr<float>(), S, P * Q, P * Q, ct.data_ptr<float>(), false, cur_stream()));
  if (accumulate) C.add_(ct.t());
  else C.copy_(ct.t());
  return true;
}

Tensor gemm_wgrad(Tensor dY, Tensor X, optional<Tensor> out, bool accumulate) {
  check_cuda(dY, "dY");
  at::hip::HIPGuardMasqueradingAsCUDA guard(dY.device());
  TORCH_CHECK(dY.dim() == 2 && X.dim() == 2 && dY.size(0) == X.size(0), "gemm_wgrad: dY (M,P), X (M,Q)");
  TORCH_CHECK(dY.scalar_type() == at::kBFloat16 && X.scalar_type() == at::kBFloat16, "gemm_wgrad: bf16 operands");
  TORCH_CHECK(dY.stride(1) == 1 && X.stride(1) == 1, "gemm_wgrad: unit column stride");
  TORCH_CHECK((uintptr_t)dY.data_ptr() % 16 == 0 && (uintptr_t)X.data_ptr() % 16 == 0, "gemm_wgrad: 16-B aligned");
  const int64_t M = dY.size(0), P = dY.size(1), Q = X.size(1);
  Tensor C = out.has_value() && out->defined() ? *out : at::empty({P, Q}, dY.options().dtype(at::kFloat));
  TORCH_CHECK(C.scalar_type() == at::kFloat && C.is_contiguous() && C.size(0) == P && C.size(1) == Q,
              "gemm_wgrad: out must be contiguous fp32 (P,Q)");
  TORCH_CHECK(!accumulate || (out.has_value() && out->defined()), "gemm_wgrad: accumulate needs out");
  if (staged_wgrad(dY, 1, X, 1, M, P, Q, C, accumulate)) return C;
  const int S = mamba_amd::gemm_wgrad_splits((int)M, (int)P, (int)Q);
  auto part = at::empty({S, P, Q}, dY.options().dtype(at::kFloat));
  HIPCHK(mamba_amd::launch_gemm_wgrad(dY.data_ptr(), dY.stride(0), X.data_ptr(), X.stride(0), part.data_ptr<float>(),
                                      C.data_ptr<float>(), (int)M, (int)P, (int)Q, accumulate, cur_stream()));
  return C;
}

// dW (fp32, (P, Q)) (+)= dY^T X over M tokens where either operand may be CHANNEL-major:
//   dy_cm: dY given as (P, M) (else (M, P));  x_cm: X given as (Q, M) (else (M, Q)).  At least one is.
Tensor gemm_wgrad_cm(Tensor dY, Tensor X, optional<Tensor> out, bool accumulate, bool dy_cm, bool x_cm,
                     optional<Tensor> part_buf, int64_t part_mode_) {
  check_cuda(dY, "dY");
  at::hip::HIPGuardMasqueradingAsCUDA guard(dY.device());
  TORCH_CHECK(dy_cm || x_cm, "gemm_wgrad_cm: use gemm_wgrad for two token-major operands");
  TORCH_CHECK(dY.dim() == 2 && X.dim() == 2, "gemm_wgrad_cm: 2-D operands");
  TORCH_CHECK(dY.scalar_type() == at::kBFloat16 && X.scalar_type() == at::kBFloat16, "gemm_wgrad_cm: bf16 operands");
  TORCH_CHECK(dY.stride(1) == 1 && X.stride(1) == 1, "gemm_wgrad_cm: unit inner strides");
  TORCH_CHECK((uintptr_t)dY.data_ptr() % 16 == 0 && (uintptr_t)X.data_ptr() % 16 == 0, "gemm_wgrad_cm: 16-B aligned");
  const int64_t P = dy_cm ? dY.size(0) : dY.size(1), M = dy_cm ? dY.size(1) : dY.size(0);
  const int64_t Q = x_cm ? X.size(0) : X.size(1), MX = x_cm ? X.size(1) : X.size(0);
  TORCH_CHECK(M == MX, "gemm_wgrad_cm: token counts differ");
  TORCH_CHECK(mamba_amd::gemm_wgrad_cm_supported((int)M, (int)P, (int)Q, dY.stride(0), X.stride(0)),
              "gemm_wgrad_cm: needs M % 64 == 0, P, Q, strides % 8 == 0");
  Tensor C = out.has_value() && out->defined() ? *out : at::empty({P, Q}, dY.options().dtype(at::kFloat));
  TORCH_CHECK(C.scalar_type() == at::kFloat && C.is_contiguous() && C.size(0) == P && C.size(1) == Q,
              "gemm_wgrad_cm: out must be contiguous fp32 (P,Q)");
  TORCH_CHECK(!accumulate || (out.has_value() && out->defined()), "gemm_wgrad_cm: accumulate needs out");
  if (part_mode_ == 0 && staged_wgrad(dY, dy_cm ? 0 : 1, X, x_cm ? 0 : 1, M, P, Q, C, accumulate)) return C;
  const int S = mamba_amd::gemm_wgrad_splits((int)M, (int)P, (int)Q);
  // part_mode (ops/grad_accum.py::deferred): 0 transient slabs reduced now; 1 / 2 store / add into the
  // persistent slabs, no reduction (returns an empty tensor); 3 / 4 store / add, then reduce into C
  const PartMode pm = part_mode(part_mode_);
  Tensor part = part_tensor(part_buf, part_mode_, {S, P, Q}, dY.options());
  if (!pm.reduce) C = at::empty({0}, dY.options().dtype(at::kFloat));
  HIPCHK(mamba_amd::launch_gemm_wgrad_cm(dY.data_ptr(), dY.stride(0), X.data_ptr(), X.stride(0), part.data_ptr<float>(),
                                         pm.reduce ? C.data_ptr<float>() : nullptr, (int)M, (int)P, (int)Q, accumulate,
                                         dy_cm, x_cm, cur_stream(), pm.pacc, pm.reduce));
  return C;
}

// Pipelined MFMA GEMM (kernels/gemm_pipe.hip): C = A . B^T with each operand as stored:
//   la = 0: A is (M, K) K-contiguous; la = 1: A is (K, M) M-contiguous.  lb likewise for B ((N, K) / (K, N)).
// mode 0: bf16 C (M, N) (out may be a row-strided view); 1: fp32 C; 2: fp32 C += (out required).
// splits > 1 (fp32 modes): out is (splits, M, N) -- one fp32 slab per K split (reduce with gp_reduce).
Tensor gp_mm(Tensor A, Tensor B, optional<Tensor> out, int64_t la, int64_t lb, int64_t mode, int64_t splits,
             int64_t bm) {
  check_cuda(A, "A");
  at::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "gp_mm: 2-D operands");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "gp_mm: bf16 operands");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "gp_mm: unit inner strides");
  TORCH_CHECK((la == 0 || la == 1) && (lb == 0 || lb == 1) && mode >= 0 && mode <= 2 && splits >= 1, "gp_mm: args");
  const int64_t M = la == 0 ? A.size(0) : A.size(1), K = la == 0 ? A.size(1) : A.size(0);
  const int64_t N = lb == 0 ? B.size(0) : B.size(1), KB = lb == 0 ? B.size(1) : B.size(0);
  TORCH_CHECK(K == KB, "gp_mm: contraction sizes differ (", K, " vs ", KB, ")");
  TORCH_CHECK(mode != 0 || splits == 1, "gp_mm: bf16 output needs splits == 1");
  TORCH_CHECK(M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31), "gp_mm: sizes");
  TORCH_CHECK((uintptr_t)A.data_ptr() % 16 == 0 && (uintptr_t)B.data_ptr() % 16 == 0, "gp_mm: 16-B aligned operands");
  Tensor C;
  const auto dt = mode == 0 ? at::kBFloat16 : at::kFloat;
  if (out.has_value() && out->defined()) {
    C = *out;
  } else {
    TORCH_CHECK(mode != 2, "gp_mm: mode 2 accumulates into out");
    // fp32 output is always (splits, M, N) (a 1-slab result reduces with gp_reduce like any other)
    C = mode != 0 ? at::empty({splits, M, N}, A.options().dtype(dt)) : at::empty({M, N}, A.options().dtype(dt));
  }
  TORCH_CHECK(C.scalar_type() == dt && C.stride(-1) == 1 && C.size(-1) == N && C.size(-2) == M, "gp_mm: out shape/dtype");
  TORCH_CHECK(splits == 1 || (C.dim() == 3 && C.size(0) == splits && C.is_contiguous()), "gp_mm: split out (S, M, N)");
  TORCH_CHECK(C.dim() == 2 || (C.dim() == 3 && C.size(0) == splits && C.is_contiguous()), "gp_mm: out rank");
  TORCH_CHECK((uintptr_t)C.data_ptr() % 16 == 0, "gp_mm: 16-B aligned out");
  const int64_t ldc = C.stride(-2);
  // a size-1 leading dim has an arbitrary stride in torch (e.g. (1, n) views): use the dense one
  const int64_t lda = A.size(0) == 1 ? A.size(1) : A.stride(0), ldb = B.size(0) == 1 ? B.size(1) : B.stride(0);
  TORCH_CHECK(mamba_amd::gemm_pipe_supported((int)la, (int)lb, (int)M, (int)N, (int)K, lda, ldb, ldc),
              "gp_mm: unsupported shape/strides (M=", M, " N=", N, " K=", K, " lda=", lda, " ldb=", ldb, " ldc=", ldc,
              "; needs row strides % 8, KC operands K % 8, XC operand rows % 8, N % 4)");
  HIPCHK(mamba_amd::launch_gemm_pipe((int)la, (int)lb, A.data_ptr(), lda, B.data_ptr(), ldb,
                                     C.data_ptr(), ldc, (int)M, (int)N, (int)K, (int)splits, M * ldc, (int)mode,
                                     (int)bm, cur_stream()));
  return C;
}

// Persistent MFMA GEMM (kernels/gemm_pipe.hip, gemm_pk_k): C = A . B^T, layouts as gp_mm, no K split.
// mode 0: bf16 C (optionally row-scaled by the fp32 `rowscale`), 1: fp32 C, 2: fp32 C +=.
Tensor gp_pk(Tensor A, Tensor B, optional<Tensor> out, int64_t la, int64_t lb, int64_t mode,
             optional<Tensor> rowscale) {
  check_cuda(A, "A");
  at::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "gp_pk: 2-D operands");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "gp_pk: bf16 operands");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "gp_pk: unit inner strides");
  TORCH_CHECK((la == 0 || la == 1) && (lb == 0 || lb == 1) && !(la == 1 && lb == 0) && mode >= 0 && mode <= 2,
              "gp_pk: args");
  const int64_t M = la == 0 ? A.size(0) : A.size(1), K = la == 0 ? A.size(1) : A.size(0);
  const int64_t N = lb == 0 ? B.size(0) : B.size(1), KB = lb == 0 ? B.size(1) : B.size(0);
  TORCH_CHECK(K == KB, "gp_pk: contraction sizes differ (", K, " vs ", KB, ")");
  TORCH_CHECK(M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31), "gp_pk: sizes");
  TORCH_CHECK((uintptr_t)A.data_ptr() % 16 == 0 && (uintptr_t)B.data_ptr() % 16 == 0, "gp_pk: 16-B aligned operands");
  const auto dt = mode == 0 ? at::kBFloat16 : at::kFloat;
  Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
  } else {
    TORCH_CHECK(mode != 2, "gp_pk: mode 2 accumulates into out");
    C = at::empty({M, N}, A.options().dtype(dt));
  }
  TORCH_CHECK(C.dim() == 2 && C.scalar_type() == dt && C.stride(1) == 1 && C.size(0) == M && C.size(1) == N,
              "gp_pk: out shape/dtype");
  TORCH_CHECK((uintptr_t)C.data_ptr() % 16 == 0, "gp_pk: 16-B aligned out");
  const float* rs = nullptr;
  if (rowscale.has_value() && rowscale->defined()) {
    TORCH_CHECK(mode == 0 && rowscale->scalar_type() == at::kFloat && rowscale->is_contiguous() &&
                rowscale->numel() == M, "gp_pk: rowscale is a contiguous fp32 (M,) vector, bf16 output only");
    rs = rowscale->data_ptr<float>();
  }
  const int64_t lda = A.size(0) == 1 ? A.size(1) : A.stride(0), ldb = B.size(0) == 1 ? B.size(1) : B.stride(0);
  const int64_t ldc = C.size(0) == 1 ? C.size(1) : C.stride(0);
  TORCH_CHECK(mamba_amd::gemm_pk_supported((int)la, (int)lb, (int)mode, (int)M, (int)N, (int)K, lda, ldb, ldc),
              "gp_pk: unsupported shape/strides (M=", M, " N=", N, " K=", K, " lda=", lda, " ldb=", ldb, " ldc=", ldc,
              "; needs strides and N % 8, KC K % 8, XC A M % 8, operands < 4 GB)");
  const hipError_t e = mamba_amd::launch_gemm_pk((int)la, (int)lb, A.data_ptr(), lda, B.data_ptr(), ldb, C.data_ptr(),
                                                 ldc, (int)M, (int)N, (int)K, (int)mode, rs, cur_stream());
  TORCH_CHECK(e != hipErrorNotReady,
              "gp_pk: no tile-claim counter pair: either the first gp_pk launch of this device is inside a HIP graph "
              "capture (run one eager launch first), or this process has captured more than ",
              mamba_amd::gemm_pk_graph_counter_capacity(), " gp_pk launches into graphs (captured pairs are never "
              "recycled: re-capture less often, e.g. reuse a GraphedDecoder instead of rebuilding it)");
  HIPCHK(e);
  return C;
}

// diagnostic SSD phase timing: a contiguous uint64 (int64) buffer, or None to switch it off (kernels/ssd.hip)
void ssd_stamps(optional<Tensor> buf) {
  if (buf.has_value() && buf->defined()) {
    TORCH_CHECK(buf->is_cuda() && buf->scalar_type() == at::kLong && buf->is_contiguous(), "ssd_stamps: int64 buffer");
    mamba_amd::set_ssd_stamps(buf->data_ptr(), buf->numel());
  } else {
    mamba_amd::set_ssd_stamps(nullptr, 0);
  }
}

// segment-parallel SSD walks: n >= 0 sets the process override (0 = automatic, kernels/ssd.hip), n < 0 leaves it;
// returns the segment count a (B, H, nc) walk gets
int64_t ssd_segments(int64_t n, int64_t B, int64_t H, int64_t nc) {
  if (n >= 0) mamba_amd::set_ssd_segments((int)n);
  const int s = mamba_amd::ssd_pick_segments((int)B, (int)H, (int)nc);
  const int cps = ((int)nc + s - 1) / s;
  return ((int)nc + cps - 1) / cps;
}

// split-K GEMM engine workgroup shape (8 or 4 waves); w <= 0 only reads it
int64_t gp_waves(int64_t w) {
  if (w > 0) mamba_amd::set_gemm_pipe_waves((int)w);
  return mamba_amd::gemm_pipe_waves();
}

// split-K XC . XC weight-gradient engine: LDS slots of gemm_wg_k (4 / 5) or 0 (gemm_pipe_k); nb < 0 only reads it
int64_t gp_wg_nb(int64_t nb) {
  if (nb >= 0) mamba_amd::set_gemm_wg_nb((int)nb);
  return mamba_amd::gemm_wg_nb();
}

// staged-ring KC operand images: 0 = 32-deep, 1 = paired 64-deep for wide long-K KC operands, 2 = paired for every KC
// operand; v < 0 only reads it
int64_t conv_cf_order_knob(int64_t v) {
  if (v >= 0) mamba_amd::set_conv_cf_order((int)v);
  return mamba_amd::conv_cf_order();
}
int64_t selscan_order_knob(int64_t v) {
  if (v >= 0) mamba_amd::set_selscan_order((int)v);
  return mamba_amd::selscan_order();
}
int64_t gp_wg_kcpair(int64_t v) {
  if (v >= 0) mamba_amd::set_gemm_wg_kcpair((int)v);
  return mamba_amd::gemm_wg_kcpair();
}

int64_t wgrad_splits(int64_t M, int64_t P, int64_t Q) { return mamba_amd::gemm_wgrad_splits((int)M, (int)P, (int)Q); }
int64_t gp_splits(int64_t M, int64_t N, int64_t K) { return mamba_amd::gemm_pipe_splits((int)M, (int)N, (int)K); }


// column sums of a (rows, cols) fp32 partial block, as the backward ops reduce their per-workgroup partial rows
// (clobbers part); exposed for the numerics / determinism tests of launch_colsum
Tensor colsum(Tensor part) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() == 2 && part.is_contiguous(),
              "colsum: contiguous 2-D fp32 CUDA tensor");
  auto out = at::empty({part.size(1)}, part.options());
  HIPCHK(mamba_amd::launch_colsum(part.data_ptr<float>(), (int)part.size(0), (int)part.size(1), out.data_ptr<float>(),
                                  cur_stream()));
  return out;
}

// batched late column sums (ops/grad_accum.py::flush_late): tab = uint8 (n, 80) LateCol rows
void late_colsum(Tensor tab, int64_t n, int64_t nblk, int64_t ntile) {
  TORCH_CHECK(tab.is_cuda() && tab.scalar_type() == at::kByte && tab.is_contiguous() && tab.numel() == n * 80,
              "late_colsum: contiguous uint8 CUDA table of n 80-byte rows");
  at::hip::HIPGuardMasqueradingAsCUDA guard(tab.device());
  HIPCHK(mamba_amd::launch_late_colsum(tab.data_ptr(), (int)n, (int)nblk, (int)ntile, cur_stream()));
}

// ---- native optimizer step (ops/optim.py): tab = uint8 OptSeg table, blk = int64 (nblk, 2) chunk table ----
static void check_opt_tables(const Tensor& tab, const Tensor& blk) {
  TORCH_CHECK(tab.is_cuda() && tab.scalar_type() == at::kByte && tab.is_contiguous() && tab.numel() % 64 == 0,
              "optimizer segment table: contiguous uint8 CUDA tensor of 64-byte rows");
  TORCH_CHECK(blk.is_cuda() && blk.scalar_type() == at::kLong && blk.is_contiguous() && blk.dim() == 2 &&
              blk.size(1) == 2 && blk.size(0) > 0, "optimizer block table: (nblk, 2) int64 CUDA tensor");
}

// [|| g / divisor ||_2, clip coefficient / divisor] as a 2-element fp32 tensor (max_norm <= 0: coefficient 1)
Tensor opt_grad_norm(Tensor tab, Tensor blk, double max_norm, double divisor) {
  check_opt_tables(tab, blk);
  const int nblk = (int)blk.size(0);
  auto partial = at::empty({nblk}, blk.options().dtype(at::kFloat));
  auto out = at::empty({2}, blk.options().dtype(at::kFloat));
  HIPCHK(mamba_amd::launch_grad_norm(tab.data_ptr(), blk.data_ptr<int64_t>(), nblk, partial.data_ptr<float>(),
                                     (float)max_norm, (float)divisor, out.data_ptr<float>(), cur_stream()));
  return out;
}

void opt_adamw(Tensor tab, Tensor blk, c10::optional<Tensor> gscale, double b1, double b2, double eps) {
  check_opt_tables(tab, blk);
  const float* gs = nullptr;
  if (gscale.has_value() && gscale->defined()) {
    TORCH_CHECK(gscale->is_cuda() && gscale->scalar_type() == at::kFloat && gscale->numel() >= 2, "gscale: fp32[2]");
    gs = gscale->data_ptr<float>();
  }
  HIPCHK(mamba_amd::launch_adamw(tab.data_ptr(), blk.data_ptr<int64_t>(), (int)blk.size(0), gs, (float)b1, (float)b2,
                                 (float)eps, cur_stream()));
}

int64_t opt_chunk() { return mamba_amd::opt_chunk(); }

// out (+)= sum over the leading dim of part (S, ...) in fixed order; out fp32 contiguous, numel(out) = numel(part[0])
void gp_reduce(Tensor part, Tensor out, bool accumulate) {
  check_cuda(part, "part");
  at::hip::HIPGuardMasqueradingAsCUDA guard(part.device());
  TORCH_CHECK(part.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat && part.is_contiguous() &&
              out.is_contiguous() && part.dim() >= 2 && part.numel() == part.size(0) * out.numel(), "gp_reduce: shapes");
  HIPCHK(mamba_amd::launch_gp_reduce(part.data_ptr<float>(), (int)part.size(0), out.numel(), out.numel(),
                                     out.data_ptr<float>(), accumulate, cur_stream()));
}

// ---------------------------------------------------------------------------------------------
// fused Mamba-2 decode step (kernels/decode.hip).  Every operand is preallocated by the caller
// (inference.FusedMamba2Decoder) so the three launches per layer can be captured in one HIP graph.
void chk_f32(const Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n, "decode: ", name,
              " must be a contiguous fp32 GPU tensor of ", n, " elements");
}

void decode_inproj(Tensor hn, Tensor W, Tensor zxbcdt, int64_t conv_lo, int64_t conv_hi, Tensor conv_state,
                   Tensor conv_w, optional<Tensor> conv_b) {
  check_cuda(hn, "hn");
  at::hip::HIPGuardMasqueradingAsCUDA guard(hn.device());
  TORCH_CHECK(hn.dim() == 2 && hn.is_contiguous() && hn.scalar_type() == at::kBFloat16, "decode: hn must be (b, d) bf16");
  const int64_t b = hn.size(0), d = hn.size(1);
  TORCH_CHECK(W.scalar_type() == at::kBFloat16 && W.is_contiguous() && W.dim() == 2 && W.size(1) == d, "decode: W_in");
  const int64_t n_out = W.size(0);
  TORCH_CHECK(b <= mamba_amd::decode_max_batch() && d % 8 == 0 && b * d * 2 <= 65536, "decode: b*d too large");
  chk_f32(zxbcdt, b * n_out, "zxbcdt");
  const int64_t C = conv_hi - conv_lo;
  TORCH_CHECK(conv_lo >= 0 && conv_hi <= n_out && C > 0, "decode: conv range");
  TORCH_CHECK(conv_state.scalar_type() == at::kBFloat16 && conv_state.dim() == 3 && conv_state.size(0) == b &&
              conv_state.size(1) == C && conv_state.stride(2) == 1, "decode: conv_state (b, C, state_len) bf16");
  TORCH_CHECK(conv_w.numel() % C == 0, "decode: conv_w (C, W)");
  const int64_t Wd = conv_w.numel() / C;
  TORCH_CHECK(conv_state.size(2) >= Wd - 1 && conv_state.size(2) <= 16, "decode: state_len >= W-1");
  chk_f32(conv_w, C * Wd, "conv_w");
  const float* cb = nullptr;
  if (conv_b.has_value() && conv_b->defined()) {
    chk_f32(*conv_b, C, "conv_b");
    cb = conv_b->data_ptr<float>();
  }
  HIPCHK(mamba_amd::launch_decode_inproj(hn.data_ptr(), W.data_ptr(), (int)n_out, (int)d, (int)b,
                                         zxbcdt.data_ptr<float>(), (int)conv_lo, (int)conv_hi, conv_state.data_ptr(),
                                         conv_state.stride(0), conv_state.stride(1), (int)conv_state.size(2),
                                         conv_w.data_ptr<float>(), cb,
                                         (int)Wd, cur_stream()));
}

void decode_ssm(Tensor zxbcdt, Tensor state, Tensor A, optional<Tensor> D, optional<Tensor> dt_bias, int64_t ngroups,
                Tensor g_out, Tensor part) {
  check_cuda(state, "state");
  at::hip::HIPGuardMasqueradingAsCUDA guard(state.device());
  TORCH_CHECK(state.dim() == 4 && state.is_contiguous() && state.scalar_type() == at::kFloat, "decode: state (b,h,p,n) fp32");
  const int64_t b = state.size(0), H = state.size(1), P = state.size(2), N = state.size(3);
  TORCH_CHECK(P % 16 == 0 && (N == 64 || N == 128 || N == 256) && H % ngroups == 0, "decode: ssm shape");
  const int64_t n_out = 2 * H * P + 2 * ngroups * N + H;
  chk_f32(zxbcdt, b * n_out, "zxbcdt");
  chk_f32(A, H, "A");
  const float* Dp = nullptr;
  const float* bp = nullptr;
  if (D.has_value() && D->defined()) { chk_f32(*D, H, "D"); Dp = D->data_ptr<float>(); }
  if (dt_bias.has_value() && dt_bias->defined()) { chk_f32(*dt_bias, H, "dt_bias"); bp = dt_bias->data_ptr<float>(); }
  TORCH_CHECK(g_out.is_cuda() && g_out.scalar_type() == at::kBFloat16 && g_out.is_contiguous() &&
              g_out.numel() == b * H * P, "decode: g_out (b, di) bf16");
  chk_f32(part, b * H * (P / 16), "part");
  HIPCHK(mamba_amd::launch_decode_ssm(zxbcdt.data_ptr<float>(), (int)n_out, state.data_ptr<float>(), A.data_ptr<float>(),
                                      Dp, bp, (int)H, (int)P, (int)ngroups, (int)N, (int)b, g_out.data_ptr(),
                                      part.data_ptr<float>(), cur_stream()));
}

void decode_outproj(Tensor g, Tensor part, double eps, Tensor W, Tensor out) {
  check_cuda(g, "g");
  at::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  TORCH_CHECK(g.dim() == 2 && g.is_contiguous() && g.scalar_type() == at::kBFloat16, "decode: g (b, di) bf16");
  const int64_t b = g.size(0), di = g.size(1);
  TORCH_CHECK(W.scalar_type() == at::kBFloat16 && W.is_contiguous() && W.dim() == 2 && W.size(1) == di, "decode: W_out");
  const int64_t d_out = W.size(0);
  TORCH_CHECK(b <= mamba_amd::decode_max_batch() && di % 8 == 0 && b * di * 2 <= 65536, "decode: b*di too large");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 2 &&
              part.size(0) == b, "decode: part (b, nparts) fp32");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.numel() == b * d_out, "decode: out");
  HIPCHK(mamba_amd::launch_decode_outproj(g.data_ptr(), part.data_ptr<float>(), (int)part.size(1), (float)eps,
                                          W.data_ptr(), (int)d_out, (int)di, (int)b, out.data_ptr(), cur_stream()));
}

}  // namespace

TORCH_LIBRARY(mamba_amd, m) {
  m.def("add_rmsnorm_fwd(Tensor x, Tensor? residual, Tensor weight, float eps, ScalarType out_dtype, "
        "ScalarType res_dtype) -> (Tensor, Tensor, Tensor)");
  m.def("add_rmsnorm_bwd(Tensor dy, Tensor? dres_out, Tensor res_out, Tensor weight, Tensor rstd, "
        "ScalarType dx_dtype, ScalarType dres_dtype, bool write_dres, Tensor(z!)? part_buf=None, int part_mode=0) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("gated_rmsnorm_fwd(Tensor x, Tensor z, Tensor weight, float eps, int group_size, bool norm_before_gate) "
        "-> (Tensor, Tensor)");
  m.def("gated_rmsnorm_bwd(Tensor dy, Tensor x, Tensor z, Tensor weight, Tensor rstd, int group_size, "
        "bool norm_before_gate, Tensor(a!)? dx_out, Tensor(b!)? dz_out, Tensor(z!)? part_buf=None, int part_mode=0) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("ce_fwd(Tensor logits, Tensor targets, int ignore_index, Tensor scale, Tensor(a!)? grad) -> Tensor");
  m.def("conv1d_cf_fwd(Tensor x, Tensor weight, Tensor? bias, bool silu) -> Tensor");
  m.def("conv1d_cf_bwd(Tensor x, Tensor weight, Tensor? bias, Tensor dout, bool silu, Tensor(a!)? dx_out, "
        "Tensor(z!)? part_buf=None, int part_mode=0) -> (Tensor, Tensor, Tensor)");
  m.def("conv1d_cl_fwd(Tensor x, Tensor weight, Tensor? bias, bool silu) -> Tensor");
  m.def("conv1d_cl_bwd(Tensor x, Tensor weight, Tensor? bias, Tensor dout, bool silu, Tensor(a!)? dx_out, "
        "Tensor(z!)? part_buf=None, int part_mode=0) -> (Tensor, Tensor, Tensor)");
  m.def("conv1d_cl_var_fwd(Tensor x, Tensor weight, Tensor? bias, bool silu, Tensor? seq_idx, "
        "Tensor? initial_states, bool want_final) -> (Tensor, Tensor)");
  m.def("conv1d_cl_var_bwd(Tensor x, Tensor weight, Tensor? bias, Tensor dout, bool silu, Tensor? seq_idx, "
        "Tensor? initial_states, Tensor? dfinal, Tensor(a!)? dx_out, Tensor(z!)? part_buf=None, int part_mode=0) "
        "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def("conv1d_update(Tensor x, Tensor(a!) conv_state, Tensor weight, Tensor? bias, bool silu) -> Tensor");
  m.def("ssd_fwd_f32(Tensor x, Tensor dt, Tensor A, Tensor B, Tensor C, Tensor? D, Tensor? dt_bias, Tensor? init, "
        "bool softplus, float dt_min, float dt_max, bool want_final) -> (Tensor, Tensor)");
  m.def("ssd_fwd(Tensor x, Tensor dt, Tensor A, Tensor B, Tensor C, Tensor? D, Tensor? dt_bias, Tensor? init, "
        "int chunk, bool softplus, float dt_min, float dt_max, bool A_is_log=False, Tensor? seq_idx=None) "
        "-> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("ssd_bwd(Tensor dy, Tensor x, Tensor dt, Tensor A, Tensor B, Tensor C, Tensor? D, Tensor? dt_bias, "
        "Tensor? init, Tensor cum, Tensor dtp, Tensor states, Tensor? dfinal, int chunk, bool softplus, float dt_min, "
        "float dt_max, Tensor(a!)? dx_out, Tensor(b!)? ddt_out, Tensor(c!)? dB_out, Tensor(d!)? dC_out, "
        "bool A_is_log=False, Tensor(z!)? part_buf=None, int part_mode=0, int ddt_zero_pad=0) -> Tensor[]");
  m.def("selscan_fwd(Tensor u, Tensor delta, Tensor A, Tensor B, Tensor C, Tensor? D, Tensor? z, Tensor? delta_bias, "
        "bool softplus) -> (Tensor, Tensor, Tensor)");
  m.def("selscan_bwd(Tensor dout, Tensor u, Tensor delta, Tensor A, Tensor B, Tensor C, Tensor? D, Tensor? z, "
        "Tensor? delta_bias, Tensor carries, bool softplus) -> Tensor[]");
  m.def("selscan_bwd_into(Tensor dout, Tensor u, Tensor delta, Tensor A, Tensor B, Tensor C, Tensor? D, Tensor? z, "
        "Tensor? delta_bias, Tensor carries, bool softplus, Tensor(a!) dz_out, Tensor(b!) dB_out, Tensor(c!) dC_out, "
        "Tensor(z!)? part_buf=None, int part_mode=0) -> Tensor[]");
  m.def("selscan_fwd_dt(Tensor u, Tensor dtw, Tensor dtx, Tensor A, Tensor B, Tensor C, Tensor? D, Tensor? z, "
        "Tensor? delta_bias, bool softplus) -> (Tensor, Tensor, Tensor)");
  m.def("selscan_bwd_dt_into(Tensor dout, Tensor u, Tensor dtw, Tensor dtx, Tensor A, Tensor B, Tensor C, Tensor? D, "
        "Tensor? z, Tensor? delta_bias, Tensor carries, bool softplus, Tensor(a!) dz_out, Tensor(b!) dB_out, "
        "Tensor(c!) dC_out, Tensor(z!)? part_buf=None, int part_mode=0) -> Tensor[]");
  m.def("gemm_tn(Tensor A, Tensor B, Tensor(a!)? out=None) -> Tensor");
  m.def("gemm_wgrad(Tensor dY, Tensor X, Tensor(a!)? out=None, bool accumulate=False) -> Tensor");
  m.def("gemm_wgrad_cm(Tensor dY, Tensor X, Tensor(a!)? out=None, bool accumulate=False, bool dy_cm=True, "
        "bool x_cm=False, Tensor(z!)? part_buf=None, int part_mode=0) -> Tensor");
  m.def("wgrad_splits(int M, int P, int Q) -> int", &wgrad_splits);
  m.def("gp_mm(Tensor A, Tensor B, Tensor(a!)? out=None, int la=0, int lb=0, int mode=0, int splits=1, int bm=256) -> Tensor");
  m.def("gp_pk(Tensor A, Tensor B, Tensor(a!)? out=None, int la=0, int lb=0, int mode=0, Tensor? rowscale=None) -> Tensor");
  m.def("gp_waves(int w=0) -> int", &gp_waves);
  m.def("gp_wg_nb(int nb=-1) -> int", &gp_wg_nb);
  m.def("gp_wg_kcpair(int v=-1) -> int", &gp_wg_kcpair);
  m.def("conv_cf_order(int v=-1) -> int", &conv_cf_order_knob);
  m.def("selscan_order(int v=-1) -> int", &selscan_order_knob);
  m.def("ssd_stamps(Tensor? buf) -> ()", &ssd_stamps);
  m.def("ssd_segments(int n, int B, int H, int nc) -> int", &ssd_segments);
  m.def("gp_splits(int M, int N, int K) -> int", &gp_splits);
  m.def("part_rows(str kind, int a, int b=0) -> int", &part_rows);
  m.def("gp_reduce(Tensor part, Tensor(a!) out, bool accumulate=False) -> ()");
  m.def("transpose_bf16(Tensor X) -> Tensor");
  m.def("colsum(Tensor(a!) part) -> Tensor");
  m.def("late_colsum(Tensor tab, int n, int nblk, int ntile) -> ()");
  m.def("opt_grad_norm(Tensor tab, Tensor blk, float max_norm, float divisor) -> Tensor");
  m.def("opt_adamw(Tensor tab, Tensor blk, Tensor? gscale, float b1, float b2, float eps) -> ()");
  m.def("opt_chunk() -> int", &opt_chunk);
  m.def("gemm_skinny(Tensor A, Tensor B, Tensor(a!)? out=None, bool accumulate=False) -> Tensor");
  m.def("ssm_state_update(Tensor(a!) state, Tensor x, Tensor dt, Tensor A, Tensor B, Tensor C, Tensor? D, Tensor? z, "
        "Tensor? dt_bias, bool softplus) -> Tensor");
  m.def("decode_inproj(Tensor hn, Tensor W, Tensor(a!) zxbcdt, int conv_lo, int conv_hi, Tensor(b!) conv_state, "
        "Tensor conv_w, Tensor? conv_b) -> ()");
  m.def("decode_ssm(Tensor zxbcdt, Tensor(a!) state, Tensor A, Tensor? D, Tensor? dt_bias, int ngroups, "
        "Tensor(b!) g_out, Tensor(c!) part) -> ()");
  m.def("decode_outproj(Tensor g, Tensor part, float eps, Tensor W, Tensor(a!) out) -> ()");
}

TORCH_LIBRARY_IMPL(mamba_amd, CUDA, m) {
  m.impl("add_rmsnorm_fwd", &add_rmsnorm_fwd);
  m.impl("gemm_tn", &gemm_tn);
  m.impl("gemm_wgrad", &gemm_wgrad);
  m.impl("gemm_skinny", &gemm_skinny);
  m.impl("gemm_wgrad_cm", &gemm_wgrad_cm);
  m.impl("gp_mm", &gp_mm);
  m.impl("gp_pk", &gp_pk);
  m.impl("gp_reduce", &gp_reduce);
  m.impl("transpose_bf16", &transpose_bf16);
  m.impl("colsum", &colsum);
  m.impl("late_colsum", &late_colsum);
  m.impl("opt_grad_norm", &opt_grad_norm);
  m.impl("opt_adamw", &opt_adamw);
  m.impl("add_rmsnorm_bwd", &add_rmsnorm_bwd);
  m.impl("gated_rmsnorm_fwd", &gated_rmsnorm_fwd);
  m.impl("gated_rmsnorm_bwd", &gated_rmsnorm_bwd);
  m.impl("ce_fwd", &ce_fwd);
  m.impl("conv1d_cf_fwd", &conv1d_cf_fwd);
  m.impl("conv1d_cf_bwd", &conv1d_cf_bwd);
  m.impl("conv1d_cl_fwd", &conv1d_cl_fwd);
  m.impl("conv1d_cl_bwd", &conv1d_cl_bwd);
  m.impl("conv1d_update", &conv1d_update);
  m.impl("conv1d_cl_var_fwd", &conv1d_cl_var_fwd);
  m.impl("conv1d_cl_var_bwd", &conv1d_cl_var_bwd);
  m.impl("ssd_fwd", &ssd_fwd);
  m.impl("ssd_fwd_f32", &ssd_fwd_f32);
  m.impl("ssd_bwd", &ssd_bwd);
  m.impl("selscan_fwd", &selscan_fwd);
  m.impl("selscan_bwd", &selscan_bwd);
  m.impl("selscan_bwd_into", &selscan_bwd_into);
  m.impl("selscan_fwd_dt", &selscan_fwd_dt);
  m.impl("selscan_bwd_dt_into", &selscan_bwd_dt_into);
  m.impl("ssm_state_update", &ssm_state_update);
  m.impl("decode_inproj", &decode_inproj);
  m.impl("decode_ssm", &decode_ssm);
  m.impl("decode_outproj", &decode_outproj);
}
