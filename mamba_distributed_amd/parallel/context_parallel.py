"""Context (sequence) parallelism for Mamba-2: the sequence dimension is sharded over CP ranks.

The reference has no sequence parallelism (T=1024 fixed, no attention).  For the
long-context configs (Mamba-2 2.8B at T=8192 and beyond) the SSD's linear recurrence gives an exact
and cheap split: rank r holds tokens [r*L/cp, (r+1)*L/cp) of every sequence.

  conv1d   causal, width W: rank r needs the last W-1 *pre-conv* rows of rank r-1 (a halo of
           (b, W-1, conv_dim) -- a few hundred KB), fed to the conv as its initial states; rank 0
           uses zeros.
  SSD      linear in the entering state S_in:  y = y_0 + e^{cum_t} C_t . S_in,
           S_out = e^{cum_L} S_in + S_0  (y_0 / S_0 = the local scan from a zero state).
           Each rank runs the native SSD once from zero, all-gathers (S_0, cum_L) -- (b,h,p,n) fp32
           + (b,h) per rank -- and folds the exclusive prefix over ranks into S_in locally, then
           adds the off-diagonal term with one batched GEMM.  No second scan, no serial
           rank-to-rank pipeline: one all-gather per layer, latency O(1) in cp.
  norm / out_proj / add-norm / CE   token-local: no communication.

Backward is autograd through the same ops (the all-gathers' backward sums every rank's gradient
contribution for the states it owns).  Parameters are replicated over CP, so DDP over the DP x CP
group averages their gradients with the step's usual bucketed all-reduce (parallel/groups.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..ops.conv1d import causal_conv1d_fn
from ..ops.reference import ssd_dt_transform
from ..ops.ssd import mamba_chunk_scan_combined
from .comm import all_gather_small, group_rank, group_size

_INF = float("inf")


def cp_causal_conv1d(xBC: torch.Tensor, weight: torch.Tensor, bias, cp_group, activation="silu"):
    """Causal depthwise conv over a sequence shard.  xBC: (b, l_local, c) (channel-last)."""
    b, l, c = xBC.shape
    w = weight.shape[-1]
    if group_size(cp_group) > 1 and w > 1:
        assert l >= w - 1, f"context-parallel shard length {l} < conv halo {w - 1}"
        tails = all_gather_small(xBC[:, l - (w - 1):, :], cp_group, dim=0)      # (cp*b, w-1, c)
        r = group_rank(cp_group)
        # rank 0 pads with zeros, but through the graph (0 * tails) so its backward runs the same
        # all-reduce as every other rank's
        halo = tails[(r - 1) * b: r * b] if r > 0 else tails[:b] * 0.0
        # the halo enters as the conv's initial states (native conv1d_cl_var; no padded copy of xBC)
        return causal_conv1d_fn(xBC.transpose(1, 2), weight, bias, activation,
                                initial_states=halo.transpose(1, 2)).transpose(1, 2)
    return causal_conv1d_fn(xBC.transpose(1, 2), weight, bias, activation).transpose(1, 2)


def cp_ssd(x, dt, A, B, C, D, dt_bias, dt_limit, cp_group, chunk_size=64):
    """SSD over a sequence shard with the cross-rank state hand-off.

    x (b,l,h,p), dt (b,l,h) raw, A (h) (negative), B/C (b,l,g,n) -> y (b,l,h,p) in x.dtype."""
    if group_size(cp_group) == 1:
        return mamba_chunk_scan_combined(x, dt, A, B, C, chunk_size, D=D, dt_bias=dt_bias,
                                         dt_softplus=True, dt_limit=dt_limit)
    y0, s0 = mamba_chunk_scan_combined(x, dt, A, B, C, chunk_size, D=D, dt_bias=dt_bias,
                                       dt_softplus=True, dt_limit=dt_limit, return_final_states=True)
    cum = torch.cumsum(ssd_dt_transform(dt, dt_bias, True, dt_limit) * A.float(), dim=1)   # (b,l,h)
    b, l, h, p = x.shape
    n = B.shape[3]
    ws, r = group_size(cp_group), group_rank(cp_group)
    # ONE collective per layer for (S_0, cum_L): two independent gathers could run their backward
    # all-reduces in different orders on different ranks (no data dependency orders them)
    packed = torch.cat([s0.float().reshape(b, h, p * n), cum[:, -1].unsqueeze(-1)], dim=-1)
    gathered = all_gather_small(packed.unsqueeze(0), cp_group, dim=0)              # (cp,b,h,p*n+1)
    finals = gathered[..., :p * n].reshape(ws, b, h, p, n)
    totals = gathered[..., p * n]                                                  # (cp,b,h)
    if r == 0:
        # rank 0 enters from the zero state; keep the gathered tensor in the graph so every rank
        # runs the same backward collective
        return (y0.float() + 0.0 * gathered.sum()).to(x.dtype)
    S = finals[0]
    for k in range(1, r):
        S = torch.exp(totals[k])[..., None, None] * S + finals[k]
    return ssd_state_correction(y0, cum, C, S).to(x.dtype)


def ssd_state_correction(y0, cum, C, S_in):
    """y = y0 + e^{cum_t} C_t . S_in  -- the contribution of an entering state S_in (b,h,p,n) to a
    segment scanned from zero (y0 (b,l,h,p), in-segment cumsum of dt*A cum (b,l,h), C (b,l,g,n))."""
    b, l, h, p = y0.shape
    g, n = C.shape[2], C.shape[3]
    Sg = S_in.float().view(b, g, h // g, p, n)
    corr = torch.einsum("blgn,bgkpn->blgkp", C.float(), Sg).reshape(b, l, h, p)
    return y0.float() + torch.exp(cum)[..., None] * corr


def gated_rmsnorm_dist(y, z, weight, eps, norm_group=None, group_size_local=None):
    """y * silu(z), RMS-normalised over the full (possibly TP-sharded) channel group, times weight.

    ``norm_group``: the TP group when one norm group spans several ranks (Mamba-2 ngroups=1 under
    tensor parallelism); the sum of squares is all-reduced (symmetric backward)."""
    from ..ops.norm import rmsnorm_gated_fn
    from .comm import all_reduce_sym
    if group_size(norm_group) == 1:
        return rmsnorm_gated_fn(y, z, weight, eps, group_size_local or y.shape[-1], False)
    d_local = y.shape[-1]
    g = y.float() * F.silu(z.float())
    ss = all_reduce_sym(g.pow(2).sum(-1, keepdim=True), norm_group)
    rstd = torch.rsqrt(ss / (d_local * group_size(norm_group)) + eps)
    return (g * rstd * weight.float()).to(y.dtype)


def mamba2_inner_parallel(zxbcdt, conv_w, conv_b, dt_bias, A_log, D, norm_w, eps, headdim, ngroups, d_state,
                          dt_limit=(0.0, _INF), cp_group=None, norm_group=None, chunk_size=64):
    """Unfused Mamba-2 inner path (conv1d+SiLU -> SSD -> gated RMSNorm) with context parallelism
    over ``cp_group`` and/or a TP-spanning norm over ``norm_group``.  Each piece runs its native
    HIP kernel on the GPU (conv1d_cl, ssd_fwd/bwd, gated_rmsnorm) and its reference on the CPU."""
    b, l, _ = zxbcdt.shape
    H = dt_bias.shape[0]
    di = H * headdim
    gn = ngroups * d_state
    z, xBC, dt = torch.split(zxbcdt, [di, di + 2 * gn, H], dim=-1)
    xBC = cp_causal_conv1d(xBC, conv_w, conv_b, cp_group)
    x, Bm, Cm = torch.split(xBC, [di, gn, gn], dim=-1)
    A = -torch.exp(A_log.float())
    y = cp_ssd(x.unflatten(-1, (H, headdim)), dt, A, Bm.unflatten(-1, (ngroups, d_state)),
               Cm.unflatten(-1, (ngroups, d_state)), D, dt_bias, dt_limit, cp_group, chunk_size)
    y = y.flatten(-2)
    if y.dtype != zxbcdt.dtype:
        y = y.to(zxbcdt.dtype)
    return gated_rmsnorm_dist(y, z, norm_w, eps, norm_group, di // ngroups)


def shard_sequence(t: torch.Tensor, cp_group, dim: int = 1) -> torch.Tensor:
    """This CP rank's contiguous slice of the sequence dimension (inputs and targets)."""
    ws = group_size(cp_group)
    if ws == 1:
        return t
    L = t.shape[dim]
    assert L % ws == 0, f"sequence length {L} not divisible by cp={ws}"
    n = L // ws
    return t.narrow(dim, group_rank(cp_group) * n, n)
