"""Fused residual-add + RMSNorm and gated RMSNorm.

GPU path: HIP kernels ``add_rmsnorm_fwd/bwd`` and ``gated_rmsnorm_fwd/bwd``
(csrc/kernels/norm.hip: one row per wavefront, 16-byte vector loads, fp32 statistics, per-block
dw partials reduced deterministically).  CPU path: ``reference.add_rms_norm_ref`` /
``reference.gated_rms_norm_ref`` under plain autograd.

API mirrors upstream ``layer_norm_fn``/``rms_norm_fn`` and ``RMSNormGated`` that the reference
reaches through Block / Mamba2 (reference model.py:8 -> mixer_seq_simple).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from . import _ext, grad_accum
from .reference import add_rms_norm_ref, gated_rms_norm_ref


def _rows(t: torch.Tensor) -> torch.Tensor:
    """View as (M, D) keeping a row stride (last dim must be unit-stride)."""
    if t.stride(-1) != 1:
        t = t.contiguous()
    if t.dim() == 2:
        return t
    try:
        return t.view(-1, t.shape[-1])
    except RuntimeError:
        return t.reshape(-1, t.shape[-1])


class _AddRMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, residual, eps, prenorm, residual_in_fp32, out_dtype):
        shape = x.shape
        x2 = _rows(x)
        r2 = _rows(residual) if residual is not None else None
        res_dtype = torch.float32 if residual_in_fp32 else x.dtype
        out_dtype = out_dtype or x.dtype
        y, res_out, rstd = _ext.ops().add_rmsnorm_fwd(x2, r2, weight, eps, out_dtype, res_dtype)
        ctx.save_for_backward(res_out, weight, rstd)
        ctx.param = weight
        ctx.x_dtype = x.dtype
        ctx.res_dtype = residual.dtype if residual is not None else None
        ctx.has_residual = residual is not None
        ctx.prenorm = prenorm
        y = y.view(shape)
        if prenorm:
            return y, res_out.view(shape)
        return y

    @staticmethod
    def backward(ctx, dy, *rest):
        res_out, weight, rstd = ctx.saved_tensors
        dres_out = rest[0] if ctx.prenorm else None
        shape = dy.shape
        dy2 = _rows(dy)
        dr2 = _rows(dres_out) if dres_out is not None else None
        # the same gradient flows to x and to residual: write it once per needed dtype
        want_res = ctx.has_residual and ctx.needs_input_grad[2]
        res_dtype = ctx.res_dtype if want_res else None
        ops = _ext.ops()
        d = grad_accum.deferred(ctx.param, "rmsnorm", (ops.part_rows("add_rmsnorm", dy2.shape[0]), dy2.shape[1]),
                                dy2.device) if ctx.needs_input_grad[1] else None
        # sync micro-step: the weight-gradient partials go to the batched late column sum (grad_accum.flush_late)
        late = d is not None and d[1] >= 3 and grad_accum.late_ok(ctx.param)
        if late:
            d = (d[0], d[1] - 2)
        dx, dres, dw = ops.add_rmsnorm_bwd(dy2, dr2, res_out, weight, rstd, ctx.x_dtype,
                                           res_dtype if res_dtype is not None else ctx.x_dtype,
                                           want_res and res_dtype != ctx.x_dtype, *(d or (None, 0)))
        if dw.numel() == 0:  # deferred to the sync micro-step / to the late column sum
            dw = None
        if late:
            grad_accum.late_colsum(d[0], 0, 0, [ctx.param])
        dx = dx.view(shape)
        dresidual = None
        if want_res:
            dresidual = (dres if res_dtype != ctx.x_dtype else dx).view(shape)
        return dx, grad_accum.defer(ctx.param, dw), dresidual, None, None, None, None


def rms_norm_fn(x, weight, bias=None, residual=None, prenorm=False, residual_in_fp32=False,
                eps=1e-6, out_dtype=None):
    """Fused (optional residual add) + RMSNorm; returns y or (y, residual_out) when prenorm."""
    assert bias is None, "RMSNorm has no bias"
    if _ext.use_native(x, residual):
        return _AddRMSNormFn.apply(x, weight, residual, eps, prenorm, residual_in_fp32, out_dtype)
    return add_rms_norm_ref(x, weight, residual, eps, prenorm, residual_in_fp32, out_dtype)


layer_norm_fn = rms_norm_fn  # the reference only ever uses is_rms_norm=True


class RMSNorm(nn.Module):
    """RMSNorm with the upstream parameter layout (``weight`` only, no ``bias`` key)."""

    def __init__(self, hidden_size, eps=1e-5, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden_size, device=device, dtype=dtype))
        self.register_parameter("bias", None)

    def forward(self, x, residual=None, prenorm=False, residual_in_fp32=False):
        return rms_norm_fn(x, self.weight, None, residual=residual, prenorm=prenorm,
                           residual_in_fp32=residual_in_fp32, eps=self.eps)


# ----------------------------------------------------------------------------------------
class _GatedRMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, z, weight, eps, group_size, norm_before_gate):
        shape = x.shape
        x2, z2 = _rows(x), _rows(z)
        y, rstd = _ext.ops().gated_rmsnorm_fwd(x2, z2, weight, eps, group_size, norm_before_gate)
        ctx.save_for_backward(x2, z2, weight, rstd)
        ctx.param = weight
        ctx.eps, ctx.group_size, ctx.nbg = eps, group_size, norm_before_gate
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, z2, weight, rstd = ctx.saved_tensors
        ops = _ext.ops()
        d = grad_accum.deferred(ctx.param, "gated_rmsnorm", (ops.part_rows("gated_rmsnorm", x2.shape[0]),
                                                             x2.shape[1]), x2.device)
        late = d is not None and d[1] >= 3 and grad_accum.late_ok(ctx.param)
        if late:
            d = (d[0], d[1] - 2)
        dx, dz, dw = ops.gated_rmsnorm_bwd(_rows(dy), x2, z2, weight, rstd, ctx.group_size, ctx.nbg, None, None,
                                           *(d or (None, 0)))
        if dw.numel() == 0:
            dw = None
        if late:
            grad_accum.late_colsum(d[0], 0, 0, [ctx.param])
        return dx.view(ctx.shape), dz.view(ctx.shape), grad_accum.defer(ctx.param, dw), None, None, None


def rmsnorm_gated_fn(x, z, weight, eps=1e-5, group_size=None, norm_before_gate=False):
    group_size = group_size or x.shape[-1]
    if _ext.use_native(x, z):
        return _GatedRMSNormFn.apply(x, z, weight, eps, group_size, norm_before_gate)
    return gated_rms_norm_ref(x, z, weight, eps, group_size, norm_before_gate)


class RMSNormGated(nn.Module):
    def __init__(self, hidden_size, eps=1e-5, group_size=None, norm_before_gate=False,
                 device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.group_size = group_size
        self.norm_before_gate = norm_before_gate
        self.weight = nn.Parameter(torch.ones(hidden_size, device=device, dtype=dtype))
        self.register_parameter("bias", None)

    def forward(self, x, z=None):
        if z is None:
            return rms_norm_fn(x, self.weight, eps=self.eps)
        return rmsnorm_gated_fn(x, z, self.weight, self.eps, self.group_size, self.norm_before_gate)
