"""Tensor parallelism (TP) with optional sequence parallelism (SP) for Mamba-2.

Capability parity with upstream mamba-ssm's ``distributed/tensor_parallel.py``
(``ColumnParallelLinear``, ``RowParallelLinear``, ``VocabParallelEmbedding``) and
``Mamba2(process_group=..., sequence_parallel=True)``.  The reference never
uses them (DDP only); on MI355X with 288 GB per GPU even the 2.8B model fits replicated, so TP is
for model sizes beyond the BASELINE configs and for latency-bound serving.

Head-sharded Mamba-2 (one TP rank owns nheads/tp heads):

  in_proj   column-parallel, per-rank rows  [z_r | x_r | B_g | C_g | dt_r]
  conv1d    channel-sharded                 [x_r | B_g | C_g]
  SSD       local heads, native kernel, no communication
  norm      gated RMSNorm: local when the norm groups are sharded (ngroups % tp == 0, the fused
            native conv->SSD->norm kernel chain runs unchanged on the local heads); for ngroups == 1
            the B/C projections are *replicated* on every TP rank (upstream requires
            ngroups % tp == 0, so the published ngroups=1 checkpoints could not use TP at all) and
            the norm's sum of squares is all-reduced over TP (one (tokens,) fp32 vector per layer)
  out_proj  row-parallel: all-reduce (TP) or reduce-scatter over tokens (SP)

Two collectives per layer, both on the xGMI full mesh: all-gather / identity before in_proj and
reduce-scatter / all-reduce after out_proj.  Gradients of replicated rows (the ngroups == 1 B/C
projections) and, under SP, of the token-sharded replicated parameters (block norms, embedding)
are summed over TP by ``sync_tp_grads`` (parallel/api.py) before the optimizer step.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.linear import linear
from ..ops.ssd import mamba2_inner_fn
from .comm import (all_gather_raw, copy_to_group, gather_along, group_rank, group_size, reduce_from_group,
                   reduce_scatter_along)
from .context_parallel import mamba2_inner_parallel

_INF = float("inf")


def _proj(x, layer: nn.Linear):
    return linear(x, layer) if layer.bias is None else layer(x)


class ColumnParallelLinear(nn.Linear):
    """y_r = x W_r^T: output features sharded.  Input replicated (TP) or token-sharded (SP: all-gathered
    along dim 0 -- the flattened batch*seq dim -- forward, reduce-scattered backward)."""

    def __init__(self, in_features, out_features, process_group, bias=True, sequence_parallel=True,
                 multiple_of=1, device=None, dtype=None):
        ws = group_size(process_group)
        if out_features % multiple_of:
            raise ValueError(f"out_features ({out_features}) must be a multiple of {multiple_of}")
        units = out_features // multiple_of
        r = group_rank(process_group)
        local = (units // ws + int(r < units % ws)) * multiple_of
        super().__init__(in_features, local, bias=bias, device=device, dtype=dtype)
        self.process_group = process_group
        self.sequence_parallel = sequence_parallel
        for p in self.parameters():
            p._tp_sharded = True

    def forward(self, x):
        pg = self.process_group
        x = gather_along(x, pg, 0) if self.sequence_parallel else copy_to_group(x, pg)
        return _proj(x, self)


class RowParallelLinear(nn.Linear):
    """y = sum_r x_r W_r^T: input features sharded; partial outputs all-reduced (TP) or
    reduce-scattered along the token dim (SP).  The bias is added once, after the reduction."""

    def __init__(self, in_features, out_features, process_group, bias=True, sequence_parallel=True,
                 multiple_of=1, device=None, dtype=None):
        ws = group_size(process_group)
        units = in_features // multiple_of
        r = group_rank(process_group)
        local = (units // ws + int(r < units % ws)) * multiple_of
        super().__init__(local, out_features, bias=False, device=device, dtype=dtype)
        self.weight._tp_sharded = True
        self.process_group = process_group
        self.sequence_parallel = sequence_parallel
        if bias:
            self.bias = nn.Parameter(torch.zeros(out_features, device=device, dtype=dtype))

    def forward(self, x):
        y = linear(x, self) if self.bias is None else F.linear(x, self.weight)
        y = (reduce_scatter_along(y, self.process_group, 0) if self.sequence_parallel
             else reduce_from_group(y, self.process_group))
        return y if self.bias is None else y + self.bias


class VocabParallelEmbedding(nn.Embedding):
    """Rows of the (vocab, d) table sharded over TP; each rank looks up the ids it owns, zeros the
    rest, and the partial embeddings are summed (all-reduce, or reduce-scatter over tokens under SP)."""

    def __init__(self, num_embeddings, embedding_dim, process_group=None, padding_idx=None,
                 sequence_parallel=False, device=None, dtype=None):
        ws = group_size(process_group)
        assert num_embeddings % ws == 0, f"vocab {num_embeddings} not divisible by tp={ws}"
        self.process_group = process_group
        self.sequence_parallel = sequence_parallel
        self.vocab_start = group_rank(process_group) * (num_embeddings // ws)
        super().__init__(num_embeddings // ws, embedding_dim, padding_idx=padding_idx, device=device, dtype=dtype)
        self.weight._tp_sharded = True

    def forward(self, ids):
        if group_size(self.process_group) == 1:
            return super().forward(ids)
        local = ids - self.vocab_start
        mask = (local < 0) | (local >= self.num_embeddings)
        emb = super().forward(local.masked_fill(mask, 0)).masked_fill(mask[..., None], 0.0)
        if self.sequence_parallel:
            return reduce_scatter_along(emb.flatten(0, -2), self.process_group, 0)
        return reduce_from_group(emb, self.process_group)


class Mamba2TP(nn.Module):
    """Head-sharded Mamba-2 mixer (see module docstring).  Build it from a full ``Mamba2`` with
    ``Mamba2TP.from_full(mixer, process_group, sequence_parallel)`` -- every rank must hold the same
    full weights (same seed, or a loaded checkpoint) -- and recover the full parameters with
    ``full_state_dict()`` (collective)."""

    def __init__(self, full, process_group, sequence_parallel=False):
        super().__init__()
        ws, r = group_size(process_group), group_rank(process_group)
        self.process_group = process_group
        self.sequence_parallel = sequence_parallel
        self.cp_group = None
        self.tp, self.tp_rank = ws, r
        self.d_model, self.d_state, self.d_conv = full.d_model, full.d_state, full.d_conv
        self.headdim, self.layer_idx = full.headdim, full.layer_idx
        self.dt_limit, self.chunk_size = full.dt_limit, full.chunk_size
        self.norm_before_gate = full.norm_before_gate
        assert not self.norm_before_gate, "norm_before_gate=True is not supported under TP"
        H, G, N, di = full.nheads, full.ngroups, full.d_state, full.d_inner
        assert H % ws == 0, f"nheads {H} not divisible by tp={ws}"
        if G % ws == 0:
            self.groups_replicated = False
            self.ngroups = G // ws
        else:
            assert G == 1, "ngroups must be divisible by tp, or 1 (replicated B/C)"
            self.groups_replicated = True
            self.ngroups = 1
        self.nheads = H // ws
        self.d_inner = di // ws
        self.full_dims = (H, G, N, di)
        Hl, Gl, dil = self.nheads, self.ngroups, self.d_inner
        g0 = 0 if self.groups_replicated else r * Gl
        W = full.in_proj.weight.detach()
        zr = W[r * dil:(r + 1) * dil]
        xr = W[di + r * dil: di + (r + 1) * dil]
        Br = W[2 * di + g0 * N: 2 * di + (g0 + Gl) * N]
        Cr = W[2 * di + G * N + g0 * N: 2 * di + G * N + (g0 + Gl) * N]
        dtr = W[2 * di + 2 * G * N + r * Hl: 2 * di + 2 * G * N + (r + 1) * Hl]
        dev, dt_ = W.device, W.dtype
        self.in_proj = nn.Linear(self.d_model, 2 * dil + 2 * Gl * N + Hl, bias=False, device=dev, dtype=dt_)
        assert full.in_proj.bias is None and full.out_proj.bias is None, "bias=True is not supported under TP"
        with torch.no_grad():
            self.in_proj.weight.copy_(torch.cat([zr, xr, Br, Cr, dtr], 0))
        conv_full = full.conv1d.weight.detach()
        cdim = dil + 2 * Gl * N
        self.conv1d = nn.Conv1d(cdim, cdim, kernel_size=full.d_conv, groups=cdim, padding=full.d_conv - 1,
                                bias=full.conv1d.bias is not None, device=dev, dtype=conv_full.dtype)

        def conv_rows(t):
            return torch.cat([t[r * dil:(r + 1) * dil], t[di + g0 * N: di + (g0 + Gl) * N],
                              t[di + G * N + g0 * N: di + G * N + (g0 + Gl) * N]], 0)

        with torch.no_grad():
            self.conv1d.weight.copy_(conv_rows(conv_full))
            if full.conv1d.bias is not None:
                self.conv1d.bias.copy_(conv_rows(full.conv1d.bias.detach()))
        hs = slice(r * Hl, (r + 1) * Hl)
        self.dt_bias = nn.Parameter(full.dt_bias.detach()[hs].clone())
        self.A_log = nn.Parameter(full.A_log.detach()[hs].clone())
        self.D = nn.Parameter(full.D.detach()[hs].clone())
        for p in (self.dt_bias, self.A_log, self.D):
            p._no_weight_decay = True
        from ..ops.norm import RMSNormGated
        self.norm = RMSNormGated(dil, eps=full.norm.eps, norm_before_gate=False,
                                 group_size=dil // Gl, device=dev, dtype=full.norm.weight.dtype)
        with torch.no_grad():
            self.norm.weight.copy_(full.norm.weight.detach()[r * dil:(r + 1) * dil])
        self.out_proj = nn.Linear(dil, self.d_model, bias=False, device=dev, dtype=full.out_proj.weight.dtype)
        with torch.no_grad():
            self.out_proj.weight.copy_(full.out_proj.weight.detach()[:, r * dil:(r + 1) * dil])
        for p in self.parameters():
            p._tp_sharded = True
        if self.groups_replicated and ws > 1:
            # rows of in_proj / conv1d that every TP rank holds in full: their gradients are partial
            # (each rank back-propagates through its own heads only) and are summed by sync_tp_grads
            self.in_proj.weight._tp_rep_rows = (2 * dil, 2 * dil + 2 * N)
            self.conv1d.weight._tp_rep_rows = (dil, dil + 2 * N)
            if self.conv1d.bias is not None:
                self.conv1d.bias._tp_rep_rows = (dil, dil + 2 * N)

    @classmethod
    def from_full(cls, full, process_group, sequence_parallel=False):
        assert not getattr(full, "_general", False), \
            "TP shards the default Mamba2 configuration (rmsnorm, per-head D, d_ssm == d_inner)"
        return cls(full, process_group, sequence_parallel)

    # ------------------------------------------------------------------------------------------
    def forward(self, u, seqlen=None, inference_params=None, **kw):
        assert inference_params is None, "cached decode is not supported on the TP mixer"
        pg = self.process_group
        if self.sequence_parallel:
            assert seqlen is not None, "sequence-parallel input is (tokens/tp, d): pass seqlen"
            u_full = gather_along(u.reshape(-1, u.shape[-1]), pg, 0)
            u3 = u_full.view(-1, seqlen, self.d_model)
        else:
            u3 = copy_to_group(u, pg)
        zxbcdt = _proj(u3, self.in_proj)
        norm_group = pg if self.groups_replicated else None
        if norm_group is None and self.cp_group is None:
            y = mamba2_inner_fn(zxbcdt, self.conv1d.weight, self.conv1d.bias, self.dt_bias, self.A_log, self.D,
                                self.norm.weight, self.norm.eps, self.headdim, self.ngroups, self.d_state,
                                self.dt_limit, False, ref_chunk_size=min(64, self.chunk_size), A_is_log=True)
        else:
            y = mamba2_inner_parallel(zxbcdt, self.conv1d.weight, self.conv1d.bias, self.dt_bias, self.A_log,
                                      self.D, self.norm.weight, self.norm.eps, self.headdim, self.ngroups,
                                      self.d_state, self.dt_limit, self.cp_group, norm_group,
                                      min(64, self.chunk_size))
        out = _proj(y, self.out_proj)
        if self.sequence_parallel:
            return reduce_scatter_along(out.reshape(-1, self.d_model), pg, 0)
        return reduce_from_group(out, pg)

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def full_state_dict(self, prefix=""):
        """Reassemble the full (upstream-layout) Mamba2 parameters on every rank (collective)."""
        pg = self.process_group
        H, G, N, di = self.full_dims
        dil, Gl, Hl = self.d_inner, self.ngroups, self.nheads

        def gather0(t):
            return all_gather_raw(t.contiguous(), pg, 0)

        W = self.in_proj.weight
        z = gather0(W[:dil])
        x = gather0(W[dil:2 * dil])
        Bw, Cw = W[2 * dil:2 * dil + Gl * N], W[2 * dil + Gl * N:2 * dil + 2 * Gl * N]
        if not self.groups_replicated:
            Bw, Cw = gather0(Bw), gather0(Cw)
        dtw = gather0(W[2 * dil + 2 * Gl * N:])
        sd = {"in_proj.weight": torch.cat([z, x, Bw, Cw, dtw], 0)}

        def conv_full(t):
            xs = gather0(t[:dil])
            b_, c_ = t[dil:dil + Gl * N], t[dil + Gl * N:]
            if not self.groups_replicated:
                b_, c_ = gather0(b_), gather0(c_)
            return torch.cat([xs, b_, c_], 0)

        sd["conv1d.weight"] = conv_full(self.conv1d.weight)
        if self.conv1d.bias is not None:
            sd["conv1d.bias"] = conv_full(self.conv1d.bias)
        sd["dt_bias"] = gather0(self.dt_bias)
        sd["A_log"] = gather0(self.A_log)
        sd["D"] = gather0(self.D)
        sd["norm.weight"] = gather0(self.norm.weight)
        sd["out_proj.weight"] = gather0(self.out_proj.weight.t()).t().contiguous()
        return {prefix + k: v for k, v in sd.items()}

