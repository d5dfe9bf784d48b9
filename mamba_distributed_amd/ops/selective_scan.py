"""Mamba-1 selective scan (S6) and the Mamba-1 inner path.

Call surface mirrors upstream ``selective_scan_fn`` / ``mamba_inner_fn`` (SURVEY.md D9, D10,
K1/K2) that the reference reaches through ``Mamba.forward`` (reference model.py:8).

GPU (csrc/kernels/selective_scan.hip):
  * forward: one wavefront per (batch, channel) row, lanes over time (16 steps per lane), all N
    states per wave; per state each lane composes its steps into one affine map, a DPP prefix
    scan (row_shr / row_bcast) combines the 64 lane maps, and the state at each backward-tile
    boundary is saved ("carries") for the backward.
  * backward: a workgroup owns 64 channels of one batch row and walks 256-step tiles from the
    end; its 4 waves split the states, replay the forward from the saved carries and run the
    adjoint as a DPP suffix scan.  B/C tiles are staged once in LDS for all channels, the next
    channel's rows are prefetched, and dB/dC are summed over the channels in registers (fixed-order,
    no float atomics).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _ext, grad_accum
from .conv1d import causal_conv1d_fn
from .reference import selective_scan_ref


class _SelectiveScanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, delta, A, B, C, D, z, delta_bias, delta_softplus, return_last_state):
        ops = _ext.ops()
        out, carries, last = ops.selscan_fwd(u, delta, A, B, C, D, z, delta_bias, delta_softplus)
        ctx.save_for_backward(u, delta, A, B, C, D, z, delta_bias, carries)
        ctx.softplus = delta_softplus
        ctx.params = (A, D, delta_bias)
        if return_last_state:
            return out, last
        return out

    @staticmethod
    def backward(ctx, dout, *rest):
        u, delta, A, B, C, D, z, delta_bias, carries = ctx.saved_tensors
        ops = _ext.ops()
        du, ddelta, dA, dB, dC, dD, dz, ddelta_bias = ops.selscan_bwd(
            dout, u, delta, A, B, C, D, z, delta_bias, carries, ctx.softplus)
        pA, pD, pdb = ctx.params
        d = grad_accum.defer
        return (du, ddelta, d(pA, dA), dB.to(B.dtype), dC.to(C.dtype),
                d(pD, dD) if D is not None else None,
                dz if z is not None else None,
                d(pdb, ddelta_bias) if delta_bias is not None else None, None, None)


def selective_scan_fn(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                      return_last_state=False):
    """u/delta/z (b,d,l); A (d,n) real; B/C (b,g,n,l) input-dependent (the Mamba-1 layout)."""
    if B.dim() == 3:
        B = B.unsqueeze(1)
    if C.dim() == 3:
        C = C.unsqueeze(1)
    if _ext.use_native(u) and not A.is_complex():
        return _SelectiveScanFn.apply(u, delta, A, B, C, D, z, delta_bias, delta_softplus,
                                      return_last_state)
    return selective_scan_ref(u, delta, A, B, C, D, z, delta_bias, delta_softplus, return_last_state)


def mamba_inner_fn(xz, conv1d_weight, conv1d_bias, x_proj_weight, delta_proj_weight,
                   out_proj_weight, out_proj_bias, A, B=None, C=None, D=None, delta_bias=None,
                   B_proj_bias=None, C_proj_bias=None, delta_softplus=True):
    """Mamba-1 training path on the channel-major (b, 2*d_inner, l) in_proj output.

    conv1d+SiLU (HIP, channel-first) -> x_proj / dt_proj as batched GEMMs that keep the
    channel-major layout (no transposes materialised) -> selective scan (HIP) -> out_proj.
    """
    assert B is None and C is None and B_proj_bias is None and C_proj_bias is None
    d_inner = xz.shape[1] // 2
    x, z = xz[:, :d_inner], xz[:, d_inner:]
    R = delta_proj_weight.shape[1]
    N = A.shape[-1]
    conv_out = causal_conv1d_fn(x, conv1d_weight, conv1d_bias, "silu")       # (b, di, l)
    x_dbl = torch.matmul(x_proj_weight, conv_out)                              # (b, R+2N, l)
    delta = torch.matmul(delta_proj_weight, x_dbl[:, :R])                      # (b, di, l)
    Bm = x_dbl[:, R:R + N].unsqueeze(1)                                        # (b, 1, N, l)
    Cm = x_dbl[:, R + N:].unsqueeze(1)
    y = selective_scan_fn(conv_out, delta, A, Bm, Cm, D, z=z, delta_bias=delta_bias,
                          delta_softplus=delta_softplus)                       # (b, di, l)
    return F.linear(y.transpose(1, 2), out_proj_weight, out_proj_bias)        # (b, l, d)


def selective_state_update(state, x, dt, A, B, C, D=None, z=None, dt_bias=None, dt_softplus=False):
    """One-token recurrent update for cached decode (T10); ``state`` is updated in place."""
    from .reference import selective_state_update_ref
    if _ext.use_native(x):
        return _ext.ops().ssm_state_update(state, x, dt, A, B, C, D, z, dt_bias, dt_softplus)
    return selective_state_update_ref(state, x, dt, A, B, C, D, z, dt_bias, dt_softplus)
