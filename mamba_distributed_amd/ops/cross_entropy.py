"""Cross-entropy for the LM head.

The reference computes ``F.cross_entropy(logits.view(-1, V), targets.view(-1))`` on the
(B*T, 50304) bf16 logits under autocast, which upcasts to a 6.6 GB fp32 copy and writes a second
fp32 gradient (model.py:44-46).  Here the HIP kernel ``ce_fwd`` (csrc/kernels/cross_entropy.hip)
reads each bf16 logit row exactly once (the row lives in registers of one 512-thread workgroup),
computes the log-sum-exp and the loss, and — when a gradient is needed — writes
d(loss)/d(logits) = (softmax - onehot) / n_valid as bf16 in the same pass.

Two entry points:
  * ``cross_entropy(logits, targets)``            — drop-in loss, logits preserved, bf16 grad buffer.
  * ``fused_linear_cross_entropy(h, W, targets)`` — lm_head GEMM + CE in one autograd node; the
    gradient overwrites the logits buffer in place, so the (B*T, V) tensor exists once.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext, grad_accum
from .linear import _pk_wins, mm_nt


def _inv_count(targets, ignore_index):
    return 1.0 / (targets != ignore_index).sum().clamp(min=1).to(torch.float32)


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, ignore_index):
        shape = logits.shape
        l2 = logits.reshape(-1, shape[-1])
        t = targets.reshape(-1)
        inv = _inv_count(t, ignore_index)
        need_grad = ctx.needs_input_grad[0]
        grad = torch.empty_like(l2) if need_grad else None
        losses = _ext.ops().ce_fwd(l2, t, ignore_index, inv, grad)
        loss = losses.sum() * inv
        ctx.save_for_backward(grad if need_grad else None)
        ctx.shape = shape
        return loss

    @staticmethod
    def backward(ctx, gloss):
        (grad,) = ctx.saved_tensors
        return (grad * gloss.to(grad.dtype)).view(ctx.shape), None, None


def cross_entropy(logits, targets, ignore_index=-100):
    if _ext.use_native(logits) and logits.dtype in (torch.bfloat16, torch.float16, torch.float32):
        return _CrossEntropyFn.apply(logits, targets, ignore_index)
    return F.cross_entropy(logits.float().view(-1, logits.size(-1)), targets.view(-1),
                           ignore_index=ignore_index)


class _FusedLinearCEFn(torch.autograd.Function):
    """loss = CE(h @ W^T, targets); the CE kernel turns the logits buffer into dlogits in place."""

    @staticmethod
    def forward(ctx, h, weight, targets, ignore_index, compute_dtype):
        h2 = h.reshape(-1, h.shape[-1]).to(compute_dtype)
        w = grad_accum.cached_cast(weight, compute_dtype)        # once per optimizer step
        t = targets.reshape(-1)
        logits = mm_nt(h2, w)                                    # persistent native GEMM or hipBLASLt
        inv = _inv_count(t, ignore_index)
        need_grad = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        losses = _ext.ops().ce_fwd(logits, t, ignore_index, inv, logits if need_grad else None)
        loss = losses.sum() * inv
        if need_grad:
            ctx.save_for_backward(h2, w, logits)               # logits now hold dlogits
        ctx.hshape, ctx.hdtype, ctx.wdtype = h.shape, h.dtype, weight.dtype
        ctx.param = weight
        return loss

    @staticmethod
    def backward(ctx, gloss):
        h2, w, dlogits = ctx.saved_tensors
        g = gloss.to(torch.float32)
        dh = dw = None
        if ctx.needs_input_grad[0]:
            # dh = dlogits W: a K-contiguous product against W^T (cached once per optimizer step)
            wt = (grad_accum.cached_transpose(ctx.param, w.dtype)
                  if _pk_wins(dlogits.shape[0], w.shape[1], w.shape[0]) else None)
            dh = (mm_nt(dlogits, wt) if wt is not None else torch.mm(dlogits, w)).mul_(g).view(ctx.hshape).to(ctx.hdtype)
        if ctx.needs_input_grad[1]:
            dw = torch.mm(dlogits.t(), h2).to(ctx.wdtype).mul_(g)
        return dh, dw, None, None, None


def fused_linear_cross_entropy(h, weight, targets, ignore_index=-100, compute_dtype=torch.bfloat16):
    if _ext.use_native(h):
        return _FusedLinearCEFn.apply(h, weight, targets, ignore_index, compute_dtype)
    logits = F.linear(h, weight.to(h.dtype))
    return F.cross_entropy(logits.float().view(-1, logits.size(-1)), targets.view(-1),
                           ignore_index=ignore_index)
