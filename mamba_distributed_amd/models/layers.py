"""Auxiliary layers for hybrid configs: gated MLP (d_intermediate > 0) and causal MHA
(attn_layer_idx).  The reference never enables them (attn_layer_idx=[],
d_intermediate=0) but MambaConfig exposes them, so the model API accepts such configs.

Attention uses ``F.scaled_dot_product_attention`` (PyTorch-ROCm's own flash path); a KV cache
supports cached decoding next to the SSM caches.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class GatedMLP(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, activation=F.silu,
                 bias=False, multiple_of=128, device=None, dtype=None):
        factory = {"device": device, "dtype": dtype}
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or int(8 * in_features / 3)
        hidden_features = (hidden_features + multiple_of - 1) // multiple_of * multiple_of
        self.fc1 = nn.Linear(in_features, 2 * hidden_features, bias=bias, **factory)
        self.activation = activation
        self.fc2 = nn.Linear(hidden_features, out_features, bias=bias, **factory)

    def forward(self, x):
        y = self.fc1(x)
        y, gate = y.chunk(2, dim=-1)
        return self.fc2(y * self.activation(gate))


def _rotary(x, pos, dim, base=10000.0):
    """Apply rotary embedding (non-interleaved halves) to the first ``dim`` features of x (b,l,h,d)."""
    if dim == 0:
        return x
    half = dim // 2
    inv = 1.0 / (base ** (torch.arange(0, half, device=x.device, dtype=torch.float32) / half))
    ang = pos.float()[:, None] * inv[None, :]                 # (l, half)
    cos, sin = ang.cos()[None, :, None, :], ang.sin()[None, :, None, :]
    xr, xp = x[..., :dim].float(), x[..., dim:]
    x1, x2 = xr[..., :half], xr[..., half:]
    out = torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)
    return torch.cat([out, xp], dim=-1)


class MHA(nn.Module):
    """Causal multi-head (grouped-query) attention with optional rotary embedding, and upstream's two
    extras (mamba_ssm/modules/mha.py): a causal depthwise conv over q/k/v (``d_conv``, native conv
    kernels, with its own decode state) and a gated-MLP branch that shares in_proj / out_proj with the
    attention (``mlp_dim``, rounded up to a multiple of 256)."""

    def __init__(self, embed_dim, num_heads, num_heads_kv=None, head_dim=None, qkv_proj_bias=True,
                 out_proj_bias=True, softmax_scale=None, causal=True, layer_idx=None, d_conv=0,
                 rotary_emb_dim=0, rotary_emb_base=10000.0, mlp_dim=0, device=None, dtype=None, **kw):
        factory = {"device": device, "dtype": dtype}
        super().__init__()
        self.embed_dim = embed_dim
        self.d_conv = d_conv
        self.mlp_dim = math.ceil(mlp_dim / 256) * 256
        self.layer_idx = layer_idx
        self.num_heads = num_heads
        self.num_heads_kv = num_heads_kv or num_heads
        assert self.num_heads % self.num_heads_kv == 0
        self.head_dim = head_dim or embed_dim // num_heads
        self.rotary_emb_dim = rotary_emb_dim
        self.rotary_emb_base = rotary_emb_base
        self.softmax_scale = softmax_scale
        self.causal = causal
        qkv_dim = self.head_dim * (self.num_heads + 2 * self.num_heads_kv)
        if d_conv > 0:
            self.conv1d = nn.Conv1d(qkv_dim, qkv_dim, kernel_size=d_conv, padding=d_conv - 1, groups=qkv_dim,
                                    **factory)
        self.in_proj = nn.Linear(embed_dim, qkv_dim + self.mlp_dim, bias=qkv_proj_bias, **factory)
        self.out_proj = nn.Linear(self.head_dim * num_heads + self.mlp_dim // 2, embed_dim, bias=out_proj_bias,
                                  **factory)

    def allocate_inference_cache(self, batch_size, max_seqlen, dtype=None, **kw):
        dtype = dtype or self.out_proj.weight.dtype
        device = self.out_proj.weight.device
        kv = torch.empty(batch_size, max_seqlen, 2, self.num_heads_kv, self.head_dim, dtype=dtype, device=device)
        if self.d_conv == 0:
            return kv
        conv_state = torch.zeros(batch_size, self.conv1d.weight.shape[0], self.d_conv, dtype=dtype, device=device)
        return kv, conv_state

    def _conv(self, qkv, inference_params):
        """Causal depthwise conv over q/k/v (no activation, as upstream); the decode state holds the last
        d_conv INPUTS (pre-conv), so prefill + token steps equal the full-sequence conv."""
        from ..ops.conv1d import causal_conv1d_fn, causal_conv1d_update
        w = self.conv1d.weight
        offset = 0 if inference_params is None else inference_params.seqlen_offset
        conv_state = None
        if inference_params is not None:
            d = inference_params.key_value_memory_dict
            if self.layer_idx not in d:
                d[self.layer_idx] = self.allocate_inference_cache(qkv.shape[0], inference_params.max_seqlen,
                                                                  dtype=qkv.dtype)
            conv_state = d[self.layer_idx][1]
        if conv_state is not None and offset > 0:
            assert qkv.shape[1] == 1, "cached decode takes one token at a time"
            return causal_conv1d_update(qkv.squeeze(1).contiguous(), conv_state, w, self.conv1d.bias).unsqueeze(1)
        xt = qkv.transpose(1, 2)
        if conv_state is not None:
            conv_state.copy_(F.pad(xt, (max(0, self.d_conv - xt.shape[-1]), 0))[..., -self.d_conv:])
        return causal_conv1d_fn(xt, w, self.conv1d.bias).transpose(1, 2)

    def forward(self, x, inference_params=None, **kw):
        b, l, _ = x.shape
        qkv = self.in_proj(x)
        x_mlp = None
        if self.mlp_dim > 0:
            qkv, x_mlp = qkv.split([qkv.shape[-1] - self.mlp_dim, self.mlp_dim], dim=-1)
            up, gate = x_mlp.chunk(2, dim=-1)
            x_mlp = up * F.silu(gate)
        if self.d_conv > 0:
            qkv = self._conv(qkv, inference_params)
        hq, hk, hd = self.num_heads, self.num_heads_kv, self.head_dim
        q, k, v = torch.split(qkv, [hq * hd, hk * hd, hk * hd], dim=-1)
        q, k, v = q.view(b, l, hq, hd), k.view(b, l, hk, hd), v.view(b, l, hk, hd)
        offset = 0 if inference_params is None else inference_params.seqlen_offset
        pos = torch.arange(offset, offset + l, device=x.device)
        q = _rotary(q, pos, self.rotary_emb_dim, self.rotary_emb_base)
        k = _rotary(k, pos, self.rotary_emb_dim, self.rotary_emb_base)
        if inference_params is not None:
            d = inference_params.key_value_memory_dict
            if self.layer_idx not in d:
                d[self.layer_idx] = self.allocate_inference_cache(b, inference_params.max_seqlen, dtype=k.dtype)
            cache = d[self.layer_idx]
            if isinstance(cache, tuple):
                cache = cache[0]
            cache[:b, offset:offset + l, 0] = k
            cache[:b, offset:offset + l, 1] = v
            k, v = cache[:b, :offset + l, 0], cache[:b, :offset + l, 1]
        rep = hq // hk
        qt = q.transpose(1, 2)
        kt = k.transpose(1, 2).repeat_interleave(rep, dim=1)
        vt = v.transpose(1, 2).repeat_interleave(rep, dim=1)
        causal = self.causal and (inference_params is None or offset == 0)
        if self.causal and inference_params is not None and offset > 0 and l > 1:
            mask = torch.ones(l, offset + l, dtype=torch.bool, device=x.device).tril(offset)
            o = F.scaled_dot_product_attention(qt, kt, vt, attn_mask=mask, scale=self.softmax_scale)
        else:
            o = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal and l > 1, scale=self.softmax_scale)
        o = o.transpose(1, 2).reshape(b, l, hq * hd)
        if x_mlp is not None:
            o = torch.cat([o, x_mlp], dim=-1)
        return self.out_proj(o)

