"""Pure-PyTorch reference implementations of every op the framework has a HIP kernel for.

These are (a) the CPU execution path (tests, gloo plumbing runs) and (b) the numerics
oracles the HIP kernels are checked against (tests/test_ops_*.py).  They are written for
clarity and exact semantics, not speed.

Semantics follow what the reference reaches through its dependencies:
  * fused residual-add + RMSNorm     — upstream ops/triton/layer_norm.py (D13, T6/T7)
  * gated RMSNorm                    — upstream ops/triton/layernorm_gated.py (D14, T8/T9)
  * causal depthwise conv1d          — causal-conv1d (D15, K3-K6)
  * selective scan (Mamba-1)         — csrc/selective_scan (D10, K1/K2)
  * SSD chunked scan (Mamba-2)       — ops/triton/ssd_*.py (D12, T1-T5)
  * single-token state updates       — selective_state_update / causal_conv1d_update (D16, K6, T10)
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def _f(t: torch.Tensor) -> torch.Tensor:
    """Promote to the fp32 compute type (fp64 stays fp64 for the oracle tests)."""
    return t if t.dtype == torch.float64 else t.float()


# --------------------------------------------------------------------------------------
# Normalisation
# --------------------------------------------------------------------------------------
def add_rms_norm_ref(
    x: torch.Tensor,
    weight: torch.Tensor,
    residual: Optional[torch.Tensor] = None,
    eps: float = 1e-5,
    prenorm: bool = False,
    residual_in_fp32: bool = False,
    out_dtype: Optional[torch.dtype] = None,
):
    """residual_out = x + residual ; y = residual_out * rsqrt(mean(residual_out^2) + eps) * w.

    Returns ``y`` or ``(y, residual_out)`` when ``prenorm``.  ``residual_out`` is fp32 when
    ``residual_in_fp32`` (the Block contract of SURVEY.md D6), else x's dtype.
    """
    out_dtype = out_dtype or x.dtype
    res_dtype = torch.float32 if residual_in_fp32 else x.dtype
    r = _f(x) if residual is None else _f(x) + _f(residual)
    rstd = torch.rsqrt(r.pow(2).mean(-1, keepdim=True) + eps)
    y = (r * rstd * _f(weight)).to(out_dtype)
    if prenorm:
        return y, r.to(res_dtype)
    return y


def gated_rms_norm_ref(
    x: torch.Tensor,
    z: Optional[torch.Tensor],
    weight: torch.Tensor,
    eps: float = 1e-5,
    group_size: Optional[int] = None,
    norm_before_gate: bool = False,
):
    """Mamba-2 output norm: y = RMSNorm_group(x * silu(z)) * w  (norm_before_gate=False)."""
    dtype = x.dtype
    xf = _f(x)
    d = xf.shape[-1]
    group_size = group_size or d
    if z is not None and not norm_before_gate:
        xf = xf * F.silu(_f(z))
    xg = xf.reshape(*xf.shape[:-1], d // group_size, group_size)
    rstd = torch.rsqrt(xg.pow(2).mean(-1, keepdim=True) + eps)
    out = (xg * rstd).reshape_as(xf) * _f(weight)
    if z is not None and norm_before_gate:
        out = out * F.silu(_f(z))
    return out.to(dtype)


# --------------------------------------------------------------------------------------
# Causal depthwise conv1d
# --------------------------------------------------------------------------------------
def causal_conv1d_ref(
    x: torch.Tensor,
    weight: torch.Tensor,
    bias: Optional[torch.Tensor] = None,
    activation: Optional[str] = None,
    initial_states: Optional[torch.Tensor] = None,
    return_final_states: bool = False,
    seq_idx: Optional[torch.Tensor] = None,
):
    """x: (b, d, l) channel-first (any strides); weight: (d, w); initial_states: (b, d, w-1).

    out[b,c,t] = act(bias_c + sum_k w[c,k] * x[b,c,t-(w-1)+k]), zero (or initial_states) left pad.
    seq_idx (b, l): a tap contributes only if its input belongs to the output's sequence (the initial
    states belong to the row's first sequence).
    """
    dtype = x.dtype
    b, d, l = x.shape
    w = weight.shape[-1]
    xf = _f(x)
    if initial_states is None:
        xp = F.pad(xf, (w - 1, 0))
    else:
        xp = torch.cat([_f(initial_states), xf], dim=-1)
    if seq_idx is None:
        out = F.conv1d(xp, _f(weight).unsqueeze(1), _f(bias) if bias is not None else None, groups=d)
        out = out[..., :l]
    else:
        sq = seq_idx.long()
        sqp = torch.cat([sq[:, :1].expand(b, w - 1), sq], dim=1)        # pad slots: first sequence
        wf = _f(weight)
        out = xf.new_zeros(b, d, l) + (_f(bias)[None, :, None] if bias is not None else 0.0)
        for k in range(w):
            same = (sqp[:, k:k + l] == sq).to(xf.dtype)[:, None, :]     # input t-(w-1)+k vs output t
            out = out + wf[None, :, k:k + 1] * xp[..., k:k + l] * same
    if activation in ("silu", "swish"):
        out = F.silu(out)
    out = out.to(dtype)
    if return_final_states:
        final = xp[..., -(w - 1):].to(dtype)
        return out, final
    return out


def causal_conv1d_update_ref(x, conv_state, weight, bias=None, activation=None):
    """One decode step.  x: (b, d); conv_state: (b, d, state_len >= w-1) updated IN PLACE (causal-conv1d
    >= 1.4 semantics: the output uses the last w-1 entries and x; the state keeps the last state_len
    inputs).  Upstream Mamba / Mamba2 caches use state_len = d_conv."""
    dtype = x.dtype
    w = weight.shape[-1]
    full = torch.cat([_f(conv_state), _f(x).unsqueeze(-1)], dim=-1)  # (b, d, state_len + 1)
    window = full[..., -w:]
    out = (window * _f(weight)).sum(-1)
    if bias is not None:
        out = out + _f(bias)
    if activation in ("silu", "swish"):
        out = F.silu(out)
    conv_state.copy_(full[..., 1:].to(conv_state.dtype))
    return out.to(dtype)


# --------------------------------------------------------------------------------------
# Selective scan (Mamba-1)
# --------------------------------------------------------------------------------------
def _scan_inputs(u, delta, A, B, C, D, z, delta_bias, delta_softplus):
    delta = _f(delta)
    if delta_bias is not None:
        delta = delta + _f(delta_bias)[..., None]
    if delta_softplus:
        delta = F.softplus(delta)
    return delta


def selective_scan_ref(
    u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
    return_last_state=False, chunk: int = 32,
):
    """u, delta, z: (b, d, l); A: (d, n); B, C: (b, g, n, l) [variable, g groups] or (d, n).

    h_t = exp(delta_t A) h_{t-1} + delta_t B_t u_t ;  y_t = C_t . h_t + D u_t ;  y *= silu(z).

    Evaluated chunk-parallel: inside a chunk the decays are closed-form products
    exp(A * (cumdelta_t - cumdelta_s)), across chunks a short sequential loop.
    """
    dtype_in = u.dtype
    delta = _scan_inputs(u, delta, A, B, C, D, z, delta_bias, delta_softplus)
    uf = _f(u)
    A = _f(A)
    b, d, l = uf.shape
    n = A.shape[1]

    def expand_bc(M):
        if M.dim() == 2:  # (d, n) constant
            return _f(M)[None, :, :, None].expand(b, d, n, l)
        g = M.shape[1]
        return _f(M).repeat_interleave(d // g, dim=1)  # (b, d, n, l)

    Bf = expand_bc(B)
    Cf = expand_bc(C)
    h = uf.new_zeros(b, d, n)
    ys = []
    for c0 in range(0, l, chunk):
        c1 = min(l, c0 + chunk)
        dl = delta[..., c0:c1]                       # (b,d,q)
        cum = torch.cumsum(dl, dim=-1)               # (b,d,q)
        # decay from s to t: exp(A * (cum_t - cum_s)), t >= s
        seg = cum[..., :, None] - cum[..., None, :]  # (b,d,q(t),q(s))
        q = c1 - c0
        mask = torch.ones(q, q, dtype=torch.bool, device=u.device).tril()
        seg = seg.masked_fill(~mask, 0.0)
        Ldec = torch.exp(A[None, :, :, None, None] * seg[:, :, None]) * mask  # (b,d,n,t,s)
        xin = dl * uf[..., c0:c1]                    # (b,d,s)
        Bc = Bf[..., c0:c1]                          # (b,d,n,s)
        Cc = Cf[..., c0:c1]
        # states at each t inside chunk: H[t] = exp(A cum_t) h0 + sum_s L[t,s] B_s x_s
        Hin = torch.einsum("bdnts,bdns,bds->bdnt", Ldec, Bc, xin)
        Hin = Hin + torch.exp(A[None, :, :, None] * cum[:, :, None, :]) * h[..., None]
        y = torch.einsum("bdnt,bdnt->bdt", Hin, Cc)
        ys.append(y)
        h = Hin[..., -1]
    y = torch.cat(ys, dim=-1)
    if D is not None:
        y = y + uf * _f(D)[:, None]
    if z is not None:
        y = y * F.silu(_f(z))
    y = y.to(dtype_in)
    return (y, h) if return_last_state else y


def selective_scan_sequential_ref(u, delta, A, B, C, D=None, z=None, delta_bias=None,
                                  delta_softplus=False, return_last_state=False):
    """Token-by-token recurrence (the definition; slow — for tests only)."""
    dtype_in = u.dtype
    delta = _scan_inputs(u, delta, A, B, C, D, z, delta_bias, delta_softplus)
    uf = _f(u)
    A = _f(A)
    b, d, l = uf.shape
    n = A.shape[1]
    if B.dim() == 2:
        Bf = _f(B)[None, :, :, None].expand(b, d, n, l)
    else:
        Bf = _f(B).repeat_interleave(d // B.shape[1], dim=1)
    if C.dim() == 2:
        Cf = _f(C)[None, :, :, None].expand(b, d, n, l)
    else:
        Cf = _f(C).repeat_interleave(d // C.shape[1], dim=1)
    h = uf.new_zeros(b, d, n)
    ys = []
    for t in range(l):
        dA = torch.exp(delta[..., t, None] * A)
        h = dA * h + (delta[..., t] * uf[..., t])[..., None] * Bf[..., t]
        ys.append((h * Cf[..., t]).sum(-1))
    y = torch.stack(ys, dim=-1)
    if D is not None:
        y = y + uf * _f(D)[:, None]
    if z is not None:
        y = y * F.silu(_f(z))
    y = y.to(dtype_in)
    return (y, h) if return_last_state else y


def selective_state_update_ref(state, x, dt, A, B, C, D=None, z=None, dt_bias=None, dt_softplus=False):
    """One-token SSM update, in place on ``state``.

    Mamba-1 form: state (b, d, n); x, dt, z (b, d); A (d, n); B, C (b, n); D (d,)
    Mamba-2 form: state (b, h, p, n); x, z (b, h, p); dt (b, h); A (h,); B, C (b, g, n); D (h,)
    """
    if state.dim() == 3:
        dtf = _f(dt)
        if dt_bias is not None:
            dtf = dtf + _f(dt_bias)
        if dt_softplus:
            dtf = F.softplus(dtf)
        dA = torch.exp(dtf[..., None] * _f(A))
        dBx = (dtf * _f(x))[..., None] * _f(B)[:, None, :]
        new = _f(state) * dA + dBx
        state.copy_(new.to(state.dtype))
        out = (new * _f(C)[:, None, :]).sum(-1)
        if D is not None:
            out = out + _f(x) * _f(D)
        if z is not None:
            out = out * F.silu(_f(z))
        return out.to(x.dtype)
    b, h, p, n = state.shape
    g = B.shape[1]
    dtf = _f(dt)
    if dt_bias is not None:
        dtf = dtf + _f(dt_bias)
    if dt_softplus:
        dtf = F.softplus(dtf)
    dA = torch.exp(dtf * _f(A))  # (b, h)
    Bh = _f(B).repeat_interleave(h // g, dim=1)  # (b,h,n)
    Ch = _f(C).repeat_interleave(h // g, dim=1)
    new = _f(state) * dA[..., None, None] + (dtf[..., None] * _f(x))[..., None] * Bh[:, :, None, :]
    state.copy_(new.to(state.dtype))
    out = torch.einsum("bhpn,bhn->bhp", new, Ch)
    if D is not None:
        out = out + _f(x) * _f(D)[:, None]
    if z is not None:
        out = out * F.silu(_f(z))
    return out.to(x.dtype)


# --------------------------------------------------------------------------------------
# SSD (Mamba-2 structured state-space duality), chunked
# --------------------------------------------------------------------------------------
def ssd_dt_transform(dt, dt_bias=None, dt_softplus=True, dt_limit=(0.0, float("inf"))):
    dt = _f(dt)
    if dt_bias is not None:
        dt = dt + _f(dt_bias)
    if dt_softplus:
        dt = F.softplus(dt)
    if dt_limit != (0.0, float("inf")):
        dt = dt.clamp(min=dt_limit[0], max=dt_limit[1])
    return dt


def ssd_chunked_ref(
    x: torch.Tensor,              # (b, l, h, p)
    dt: torch.Tensor,             # (b, l, h)   raw (pre-bias / pre-softplus)
    A: torch.Tensor,              # (h,)
    B: torch.Tensor,              # (b, l, g, n)
    C: torch.Tensor,              # (b, l, g, n)
    chunk_size: int = 64,
    D: Optional[torch.Tensor] = None,   # (h,) or (h, p)
    z: Optional[torch.Tensor] = None,   # (b, l, h, p)
    dt_bias: Optional[torch.Tensor] = None,
    dt_softplus: bool = True,
    dt_limit=(0.0, float("inf")),
    initial_states: Optional[torch.Tensor] = None,  # (b, h, p, n)
    return_final_states: bool = False,
    seq_idx: Optional[torch.Tensor] = None,         # (b, l) int, non-decreasing per row
):
    """Chunked SSD.  Exact semantics of upstream ``mamba_chunk_scan_combined``:

    dt' = softplus(dt + dt_bias) ; a_t = dt'_t A_h ; within chunk cum = cumsum(a)
    y_t = sum_{s<=t in chunk} (C_t.B_s) e^{cum_t-cum_s} dt'_s x_s + e^{cum_t} C_t . S_prev + D x_t
    S_next = e^{cum_last} S_prev + sum_s e^{cum_last-cum_s} dt'_s x_s B_s^T
    seq_idx (packed rows): explicit masks -- every term that links two tokens (or a token and the
    carried state) of different sequences is dropped; the initial state belongs to the row's first
    sequence; the final state is the last sequence's.
    """
    dtype = x.dtype
    b, l, h, p = x.shape
    g, n = B.shape[2], B.shape[3]
    q = chunk_size
    dtp = ssd_dt_transform(dt, dt_bias, dt_softplus, dt_limit)  # (b,l,h) fp32
    pad = (-l) % q
    xf, Bf, Cf = _f(x), _f(B), _f(C)
    if pad:
        xf = F.pad(xf, (0, 0, 0, 0, 0, pad))
        Bf = F.pad(Bf, (0, 0, 0, 0, 0, pad))
        Cf = F.pad(Cf, (0, 0, 0, 0, 0, pad))
        dtp = F.pad(dtp, (0, 0, 0, pad))
    nc = (l + pad) // q
    if seq_idx is not None:
        sq = seq_idx.long()
        if pad:
            sq = torch.cat([sq, sq[:, -1:].expand(b, pad)], dim=1)
        sq = sq.reshape(b, nc, q)
        sq_last = sq[:, :, -1]                                         # (b,c)
        sq_prev = torch.cat([sq[:, :1, 0], sq_last[:, :-1]], dim=1)   # state owner entering chunk c
    xf = xf.reshape(b, nc, q, h, p)
    Bf = Bf.reshape(b, nc, q, g, n).repeat_interleave(h // g, dim=3)
    Cf = Cf.reshape(b, nc, q, g, n).repeat_interleave(h // g, dim=3)
    dtc = dtp.reshape(b, nc, q, h)
    a = dtc * _f(A)
    cum = torch.cumsum(a, dim=2)                                   # (b,c,q,h)
    seg = cum[:, :, :, None, :] - cum[:, :, None, :, :]            # (b,c,t,s,h)
    mask = torch.ones(q, q, dtype=torch.bool, device=x.device).tril()[None, None, :, :, None]
    if seq_idx is not None:
        mask = mask & (sq[:, :, :, None] == sq[:, :, None, :])[..., None]
    Ldec = torch.exp(seg.masked_fill(~mask, float("-inf")))
    CB = torch.einsum("bcthn,bcshn->bctsh", Cf, Bf)
    xdt = xf * dtc[..., None]
    y = torch.einsum("bctsh,bcshp->bcthp", CB * Ldec, xdt)
    decay_states = torch.exp(cum[:, :, -1:, :] - cum)              # (b,c,q,h)
    if seq_idx is not None:
        decay_states = decay_states * (sq == sq_last[..., None]).to(cum.dtype)[..., None]
    states = torch.einsum("bcshn,bcsh,bcshp->bchpn", Bf, decay_states, xdt)
    S = xf.new_zeros(b, h, p, n) if initial_states is None else _f(initial_states)
    chunk_decay = torch.exp(cum[:, :, -1, :])                       # (b,c,h)
    if seq_idx is not None:
        chunk_decay = chunk_decay * (sq_last == sq_prev).to(cum.dtype)[..., None]
    s_in = []
    for c in range(nc):
        s_in.append(S)
        S = chunk_decay[:, c, :, None, None] * S + states[:, c]
    S_in = torch.stack(s_in, dim=1)                                  # (b,c,h,p,n)
    state_w = torch.exp(cum)
    if seq_idx is not None:
        state_w = state_w * (sq == sq_prev[..., None]).to(cum.dtype)[..., None]
    y = y + torch.einsum("bcthn,bchpn->bcthp", Cf, S_in) * state_w[..., None]
    y = y.reshape(b, nc * q, h, p)[:, :l]
    if D is not None:
        Df = _f(D)
        y = y + _f(x) * (Df[:, None] if Df.dim() == 1 else Df)
    if z is not None:
        y = y * F.silu(_f(z))
    y = y.to(dtype)
    return (y, S) if return_final_states else y


def ssd_sequential_ref(x, dt, A, B, C, D=None, z=None, dt_bias=None, dt_softplus=True,
                       dt_limit=(0.0, float("inf")), initial_states=None, return_final_states=False,
                       seq_idx=None):
    """Token-by-token Mamba-2 recurrence (definition; tests only).  seq_idx: the state restarts
    from zero wherever seq_idx changes."""
    dtype = x.dtype
    b, l, h, p = x.shape
    g, n = B.shape[2], B.shape[3]
    dtp = ssd_dt_transform(dt, dt_bias, dt_softplus, dt_limit)
    Bh = _f(B).repeat_interleave(h // g, dim=2)
    Ch = _f(C).repeat_interleave(h // g, dim=2)
    S = _f(x).new_zeros(b, h, p, n) if initial_states is None else _f(initial_states)
    ys = []
    for t in range(l):
        dA = torch.exp(dtp[:, t] * _f(A))  # (b,h)
        if seq_idx is not None and t > 0:
            dA = dA * (seq_idx[:, t] == seq_idx[:, t - 1]).to(dA.dtype)[:, None]
        S = S * dA[..., None, None] + (dtp[:, t, :, None] * _f(x[:, t]))[..., None] * Bh[:, t, :, None, :]
        ys.append(torch.einsum("bhpn,bhn->bhp", S, Ch[:, t]))
    y = torch.stack(ys, dim=1)
    if D is not None:
        Df = _f(D)
        y = y + _f(x) * (Df[:, None] if Df.dim() == 1 else Df)
    if z is not None:
        y = y * F.silu(_f(z))
    y = y.to(dtype)
    return (y, S) if return_final_states else y


# --------------------------------------------------------------------------------------
# Loss
# --------------------------------------------------------------------------------------
def cross_entropy_ref(logits, targets, ignore_index=-100, reduction="mean"):
    return F.cross_entropy(_f(logits).view(-1, logits.size(-1)), targets.view(-1),
                           ignore_index=ignore_index, reduction=reduction)


def softplus_inverse(x: torch.Tensor) -> torch.Tensor:
    """inv_softplus(x) = x + log(-expm1(-x)) (upstream dt-bias init)."""
    return x + torch.log(-torch.expm1(-x))


__all__ = [n for n in dir() if n.endswith("_ref")] + ["ssd_dt_transform", "softplus_inverse"]