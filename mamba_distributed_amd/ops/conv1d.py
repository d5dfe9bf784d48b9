"""Causal depthwise conv1d (+SiLU), both memory layouts.

Same call surface as causal-conv1d's ``causal_conv1d_fn(x, weight, bias, activation, initial_states,
return_final_states, seq_idx)`` with x given as (batch, dim, seqlen) — SURVEY.md D15, K3-K6.  The
layout is taken from the strides:

  * channel-first  (x.stride(2) == 1): Mamba-1 path (x is a slice of the (b, 2di, l) in_proj output)
      -> HIP ``conv1d_cf_fwd/bwd``: one wavefront per (b, channel-block) walks time with a 3-tap
         register window; 16-byte loads along l.
  * channel-last   (x.stride(1) == 1): Mamba-2 path (xBC is a column slice of the (b, l, d_in_proj)
      in_proj output) -> HIP ``conv1d_cl_fwd/bwd``: lanes over channels (8 bf16 per lane, 16 B),
      a block owns a time tile, the w-1 halo rows are re-read (cheap, L2 hits).
  * seq_idx / initial_states / return_final_states (either layout) -> HIP ``conv1d_cl_var_fwd/bwd``.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _ext, grad_accum
from .reference import causal_conv1d_ref, causal_conv1d_update_ref


def _is_channel_last(x: torch.Tensor) -> bool:
    return x.stride(1) == 1 and x.stride(2) != 1


class _CausalConv1dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, silu):
        ops = _ext.ops()
        w2 = weight.reshape(weight.shape[0], -1)
        if _is_channel_last(x):
            xt = x.transpose(1, 2)  # (b, l, d) with unit channel stride
            out = ops.conv1d_cl_fwd(xt, w2, bias, silu).transpose(1, 2)
            ctx.cl = True
        else:
            if x.stride(2) != 1:
                x = x.contiguous()
            out = ops.conv1d_cf_fwd(x, w2, bias, silu)
            ctx.cl = False
        ctx.save_for_backward(x, w2, bias)
        ctx.silu = silu
        ctx.wshape = weight.shape
        ctx.params = (weight, bias)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w2, bias = ctx.saved_tensors
        ops = _ext.ops()
        if ctx.cl:
            dx, dw, db = ops.conv1d_cl_bwd(x.transpose(1, 2), w2, bias, dout.transpose(1, 2), ctx.silu, None)
            dx = dx.transpose(1, 2)
        else:
            dx, dw, db = ops.conv1d_cf_bwd(x, w2, bias, dout, ctx.silu, None)
        pw, pb = ctx.params
        return (dx, grad_accum.defer(pw, dw.reshape(ctx.wshape).to(w2.dtype)),
                (grad_accum.defer(pb, db.to(bias.dtype)) if bias is not None else None), None)


class _CausalConv1dVarFn(torch.autograd.Function):
    """Packed variable-length sequences (seq_idx) and/or state hand-off (initial / final states):
    HIP ``conv1d_cl_var_fwd/bwd`` (channel-last; a tap never reads across a sequence boundary, the
    initial states precede the row's first sequence, the final states are the last w-1 inputs)."""

    @staticmethod
    def forward(ctx, x, weight, bias, silu, seq_idx, initial_states, return_final):
        ops = _ext.ops()
        w2 = weight.reshape(weight.shape[0], -1)
        xt = x.transpose(1, 2)
        if xt.stride(2) != 1:
            xt = xt.contiguous()
        init = initial_states
        if init is not None and init.dtype != x.dtype:
            init = init.to(x.dtype)
        out, fin = ops.conv1d_cl_var_fwd(xt, w2, bias, silu, seq_idx, init, return_final)
        ctx.save_for_backward(xt, w2, bias, seq_idx, init)
        ctx.silu, ctx.wshape, ctx.params = silu, weight.shape, (weight, bias)
        ctx.has_init, ctx.init_dtype = initial_states is not None, getattr(initial_states, "dtype", None)
        ctx.ret_final = return_final
        ctx.set_materialize_grads(False)
        if not return_final:
            ctx.mark_non_differentiable(fin)
        return out.transpose(1, 2), fin

    @staticmethod
    def backward(ctx, dout, dfin):
        xt, w2, bias, seq_idx, init = ctx.saved_tensors
        if dout is None:
            dout = torch.zeros_like(xt).transpose(1, 2)
        dx, dw, db, dinit = _ext.ops().conv1d_cl_var_bwd(xt, w2, bias, dout.transpose(1, 2), ctx.silu, seq_idx,
                                                         init, dfin if ctx.ret_final else None, None)
        pw, pb = ctx.params
        return (dx.transpose(1, 2), grad_accum.defer(pw, dw.reshape(ctx.wshape).to(w2.dtype)),
                (grad_accum.defer(pb, db.to(bias.dtype)) if bias is not None else None), None, None,
                dinit.to(ctx.init_dtype) if ctx.has_init else None, None)


def causal_conv1d_fn(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
                     activation: Optional[str] = None, initial_states=None, return_final_states=False,
                     seq_idx: Optional[torch.Tensor] = None):
    """x: (b, d, l) in either memory layout; weight (d, w) or (d, 1, w).

    ``seq_idx`` (b, l) int: packed variable-length rows (taps never cross a change of seq_idx);
    ``initial_states`` (b, d, w-1): inputs preceding x (CP halo / chunked prefill), gradients flow;
    ``return_final_states``: also return the last w-1 inputs (b, d, w-1) (the decode conv_state)."""
    silu = activation in ("silu", "swish")
    assert activation in (None, "silu", "swish")
    if _ext.use_native(x):
        if initial_states is None and not return_final_states and seq_idx is None:
            return _CausalConv1dFn.apply(x, weight, bias, silu)
        out, fin = _CausalConv1dVarFn.apply(x, weight, bias, silu, seq_idx, initial_states, return_final_states)
        return (out, fin) if return_final_states else out
    w2 = weight.reshape(weight.shape[0], -1)
    return causal_conv1d_ref(x, w2, bias, activation, initial_states, return_final_states, seq_idx=seq_idx)


def causal_conv1d_update(x, conv_state, weight, bias=None, activation=None):
    """Single-token decode step (K6).  conv_state (b, d, w-1) is updated in place."""
    w2 = weight.reshape(weight.shape[0], -1)
    if _ext.use_native(x):
        return _ext.ops().conv1d_update(x, conv_state, w2, bias, activation in ("silu", "swish"))
    return causal_conv1d_update_ref(x, conv_state, w2, bias, activation)
