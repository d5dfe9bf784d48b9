"""Bias-free projection (nn.Linear without bias) with a native weight-gradient GEMM.

Forward and input-gradient GEMMs stay on hipBLASLt (the pinned TunableOp solutions reach
~1000 TF/s on these shapes).  The weight gradient dW = dY^T X reduces over all B*T tokens into a
small output (768 x 1536 for out_proj), where the library leaves most CUs idle: the native
``gemm_wgrad`` splits the token dimension across workgroups (256 x 256 MFMA tiles, LDS-DMA staged,
fixed-order fp32 reduction) and returns the gradient directly in fp32 -- the parameter's dtype --
so the bf16 -> fp32 cast kernel disappears as well (csrc/kernels/gemm.hip).
Autocast semantics match ``F.linear`` under ``torch.autocast``: compute in the autocast dtype.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext
from . import grad_accum


def _compute_dtype(x: torch.Tensor) -> torch.dtype:
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return x.dtype


def _native_ok(dy: torch.Tensor, x: torch.Tensor) -> bool:
    return (dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.stride(-1) == 1 and x.stride(-1) == 1
            and dy.shape[-1] % 8 == 0 and x.shape[-1] % 8 == 0 and dy.stride(0) % 8 == 0 and x.stride(0) % 8 == 0
            and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0)


class _ProjFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, cd):
        x2 = x.reshape(-1, x.shape[-1]).to(cd)
        w = grad_accum.cached_cast(weight, cd)
        y = F.linear(x2, w)
        ctx.save_for_backward(x2, w)
        ctx.param = weight
        ctx.wdtype = weight.dtype
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != w.dtype:
            dy2 = dy2.to(w.dtype)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = torch.mm(dy2, w) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            p = ctx.param
            native = _native_ok(dy2, x2)
            if (native and grad_accum.accumulable(p) and p.grad.dtype == torch.float32 and p.grad.is_contiguous()
                    and p.grad.shape == w.shape):
                # no-sync micro-step: the split-K reduction adds straight into p.grad, on a side stream
                # beside the rest of the backward (grad_accum.side_stream; joined before the sync step)
                side = grad_accum.side_stream(dy2.device)
                if side is None:
                    _ext.ops().gemm_wgrad(dy2, x2, p.grad, True)
                else:
                    side.wait_stream(torch.cuda.current_stream(dy2.device))
                    with torch.cuda.stream(side):
                        _ext.ops().gemm_wgrad(dy2, x2, p.grad, True)
                    dy2.record_stream(side)
                    x2.record_stream(side)
            else:
                dw = _ext.ops().gemm_wgrad(dy2, x2, None, False) if native else torch.mm(dy2.t(), x2)
                dw = grad_accum.defer(p, dw.to(ctx.wdtype))
        return (dx.view(ctx.xshape) if dx is not None else None), dw, None


def linear(x: torch.Tensor, layer: torch.nn.Linear) -> torch.Tensor:
    """``layer(x)`` for a bias-free nn.Linear, native weight gradient on the GPU."""
    if layer.bias is None and _ext.use_native(x):
        return _ProjFn.apply(x, layer.weight, _compute_dtype(x))
    return layer(x)
