"""Mamba-2 (SSD) mixer.

Parameter names, shapes and init follow upstream ``mamba_ssm/modules/mamba2.py::Mamba2``
 so checkpoints interchange.  Training forward:

    zxbcdt = in_proj(u)                      native persistent GEMM fwd into 64-aligned padded rows,
                                             native persistent dgrad (K = padded width), native split-K wgrad
    y      = mamba2_inner_fn(zxbcdt, ...)    HIP: conv1d(xBC)+SiLU -> SSD -> gated RMSNorm
    out    = out_proj(y)                     native persistent fwd and dgrad, native split-K wgrad
(projection routing: ops/linear.py; the native engines for every model, hipBLASLt only under the
MAMBA_AMD_PROJ_GEMM A/B switches)

The conv, SSD and norm kernels read their operands straight out of the strided zxbcdt buffer
and the backward writes d(zxbcdt) as one buffer in the same padded layout (ops/ssd.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.conv1d import causal_conv1d_update
from ..ops.linear import linear
from ..ops.norm import RMSNormGated
from ..ops.reference import softplus_inverse
from ..ops.selective_scan import selective_state_update
from ..ops.ssd import mamba2_inner_fn


class Mamba2(nn.Module):
    def __init__(self, d_model, d_state=128, d_conv=4, conv_init=None, expand=2, headdim=64,
                 d_ssm=None, ngroups=1, A_init_range=(1, 16), D_has_hdim=False, rmsnorm=True,
                 norm_before_gate=False, dt_min=0.001, dt_max=0.1, dt_init_floor=1e-4,
                 dt_limit=(0.0, float("inf")), bias=False, conv_bias=True, chunk_size=256,
                 use_mem_eff_path=True, layer_idx=None, process_group=None, sequence_parallel=True,
                 device=None, dtype=None):
        factory = {"device": device, "dtype": dtype}
        super().__init__()
        assert process_group is None, "head-sharded TP: parallel.tensor_parallel.Mamba2TP.from_full / parallel.parallelize"
        self.d_model = d_model
        self.d_state = d_state
        self.d_conv = d_conv
        self.conv_init = conv_init
        self.expand = expand
        self.d_inner = int(expand * d_model)
        self.headdim = headdim
        self.d_ssm = self.d_inner if d_ssm is None else d_ssm
        assert self.d_ssm <= self.d_inner
        self.ngroups = ngroups
        assert self.d_ssm % headdim == 0
        self.nheads = self.d_ssm // headdim
        self.D_has_hdim = D_has_hdim
        self.rmsnorm = rmsnorm
        self.norm_before_gate = norm_before_gate
        self.dt_limit = dt_limit
        self.activation = "silu"
        self.chunk_size = chunk_size
        self.use_mem_eff_path = use_mem_eff_path
        self.layer_idx = layer_idx
        self.cp_group = None  # context parallelism (parallel/api.py::parallelize sets it)

        d_in_proj = 2 * self.d_inner + 2 * ngroups * d_state + self.nheads
        self.in_proj = nn.Linear(d_model, d_in_proj, bias=bias, **factory)
        conv_dim = self.d_ssm + 2 * ngroups * d_state
        self.conv1d = nn.Conv1d(conv_dim, conv_dim, bias=conv_bias, kernel_size=d_conv, groups=conv_dim,
                                padding=d_conv - 1, **factory)
        if conv_init is not None:
            nn.init.uniform_(self.conv1d.weight, -conv_init, conv_init)
        self.act = nn.SiLU()

        dt = torch.exp(torch.rand(self.nheads, **factory) * (math.log(dt_max) - math.log(dt_min))
                       + math.log(dt_min)).clamp(min=dt_init_floor)
        self.dt_bias = nn.Parameter(softplus_inverse(dt))
        self.dt_bias._no_weight_decay = True

        assert A_init_range[0] > 0 and A_init_range[1] >= A_init_range[0]
        A = torch.empty(self.nheads, dtype=torch.float32, device=device).uniform_(*A_init_range)
        self.A_log = nn.Parameter(torch.log(A).to(dtype=dtype or torch.float32))
        self.A_log._no_weight_decay = True
        self.D = nn.Parameter(torch.ones(self.d_ssm if D_has_hdim else self.nheads, device=device))
        self.D._no_weight_decay = True
        if rmsnorm:
            self.norm = RMSNormGated(self.d_ssm, eps=1e-5, norm_before_gate=norm_before_gate,
                                     group_size=self.d_ssm // ngroups, **factory)
        self.out_proj = nn.Linear(self.d_inner, d_model, bias=bias, **factory)
        # upstream's other Mamba2 variants (mamba_ssm/modules/mamba2.py): the gate-only output without the
        # norm (rmsnorm=False), a per-channel skip D (D_has_hdim) and a gated-MLP branch beside a narrower
        # SSM (d_ssm < d_inner).  They run the same native ops unfused (_forward_general); the default
        # configuration keeps the fused chain.
        self.d_mlp = (d_in_proj - 2 * self.d_ssm - 2 * ngroups * d_state - self.nheads) // 2
        self._general = D_has_hdim or not rmsnorm or self.d_mlp > 0

    # ------------------------------------------------------------------
    def forward(self, u, seqlen=None, seq_idx=None, cu_seqlens=None, inference_params=None):
        b, l, _ = u.shape
        conv_state = ssm_state = None
        if inference_params is not None:
            conv_state, ssm_state = self._get_states_from_cache(inference_params, b)
            if inference_params.seqlen_offset > 0:
                out, _, _ = self.step(u, conv_state, ssm_state)
                return out
        fused = not self._general and self.cp_group is None and conv_state is None
        # the fused chain writes d(zxbcdt) into the padded layout itself (ops/linear.py: padded output rows)
        zxbcdt = linear(u, self.in_proj, pad=fused)
        if seq_idx is None and cu_seqlens is not None:
            seq_idx = seq_idx_from_cu_seqlens(cu_seqlens, l, u.device).expand(b, l)
        if self._general:
            assert self.cp_group is None, "context parallelism runs the default Mamba2 configuration only"
            y = self._forward_general(zxbcdt, seq_idx, conv_state, ssm_state)
        elif self.cp_group is not None and conv_state is None:
            assert seq_idx is None, "packed sequences (seq_idx) are not supported with context parallelism"
            from ..parallel.context_parallel import mamba2_inner_parallel
            y = mamba2_inner_parallel(zxbcdt, self.conv1d.weight, self.conv1d.bias, self.dt_bias, self.A_log,
                                      self.D, self.norm.weight, self.norm.eps, self.headdim, self.ngroups,
                                      self.d_state, self.dt_limit, self.cp_group, None, min(64, self.chunk_size))
        elif conv_state is None:
            y = mamba2_inner_fn(zxbcdt, self.conv1d.weight, self.conv1d.bias, self.dt_bias, self.A_log, self.D,
                                self.norm.weight, self.norm.eps, self.headdim, self.ngroups, self.d_state,
                                self.dt_limit, self.norm_before_gate, ref_chunk_size=min(64, self.chunk_size),
                                A_is_log=True, seq_idx=seq_idx)
        else:
            y = self._prefill(zxbcdt, conv_state, ssm_state)
        return linear(y, self.out_proj)

    def _forward_general(self, zxbcdt, seq_idx=None, conv_state=None, ssm_state=None):
        """Unfused forward for rmsnorm=False / D_has_hdim / d_mlp > 0 (upstream Mamba2.forward's
        non-fused branch): conv1d+SiLU -> SSD -> skip / gate / norm -> [silu(z0) x0, y].  With
        ``conv_state`` / ``ssm_state`` (prefill) the decode cache is filled too."""
        from ..ops.conv1d import causal_conv1d_fn
        from ..ops.ssd import mamba_chunk_scan_combined
        b, l, _ = zxbcdt.shape
        di, gn, H, P = self.d_ssm, self.ngroups * self.d_state, self.nheads, self.headdim
        z0, x0, z, xBC, dt = torch.split(zxbcdt, [self.d_mlp, self.d_mlp, di, di + 2 * gn, H], dim=-1)
        if zxbcdt.stride(-2) % 8:  # e.g. an odd in_proj width (d_mlp > 0): the native ops want aligned rows
            z, xBC, dt = z.contiguous(), xBC.contiguous(), dt.contiguous()
        xt = xBC.transpose(1, 2)
        if conv_state is not None:
            sl = conv_state.shape[-1]  # upstream layout: the last d_conv inputs
            conv_state.copy_(F.pad(xt, (max(0, sl - xt.shape[-1]), 0))[..., -sl:])
        xBC = causal_conv1d_fn(xt, self.conv1d.weight, self.conv1d.bias, "silu", seq_idx=seq_idx).transpose(1, 2)
        x, B, C = torch.split(xBC, [di, gn, gn], dim=-1)
        xh = x.unflatten(-1, (H, P))
        res = mamba_chunk_scan_combined(
            xh, dt, -torch.exp(self.A_log.float()), B.unflatten(-1, (self.ngroups, self.d_state)),
            C.unflatten(-1, (self.ngroups, self.d_state)), min(64, self.chunk_size),
            D=None if self.D_has_hdim else self.D, dt_bias=self.dt_bias, dt_softplus=True,
            dt_limit=self.dt_limit, seq_idx=seq_idx, return_final_states=ssm_state is not None)
        y, last = res if ssm_state is not None else (res, None)
        if last is not None:
            ssm_state.copy_(last)
        y = self._skip_gate_norm(y, xh, z)
        if self.d_mlp > 0:
            y = torch.cat([F.silu(z0) * x0, y], dim=-1)
        return y

    def _skip_gate_norm(self, y, xh, z):
        """y (.., H, P) from the scan -> (.., d_ssm): + x D (per channel), then the gate: silu(z) without
        the norm (rmsnorm=False, upstream's z inside the scan) or the gated RMSNorm."""
        if self.D_has_hdim:
            y = y + xh * self.D.view(self.nheads, self.headdim).to(y.dtype)
        y = y.flatten(-2)
        if not self.rmsnorm:
            return y * F.silu(z)
        return self.norm(y, z)

    def _prefill(self, zxbcdt, conv_state, ssm_state):
        """Prompt pass that also fills the decode cache (conv window + final SSM state): the same fused
        native chain as training (conv1d -> SSD -> gated norm) with ``return_final_states``."""
        di, gn = self.d_ssm, self.ngroups * self.d_state
        xt = zxbcdt[..., di:2 * di + 2 * gn].transpose(1, 2)
        sl = conv_state.shape[-1]  # upstream layout: the last d_conv inputs
        conv_state.copy_(F.pad(xt, (max(0, sl - xt.shape[-1]), 0))[..., -sl:])
        y, last = mamba2_inner_fn(zxbcdt, self.conv1d.weight, self.conv1d.bias, self.dt_bias, self.A_log, self.D,
                                  self.norm.weight, self.norm.eps, self.headdim, self.ngroups, self.d_state,
                                  self.dt_limit, self.norm_before_gate, ref_chunk_size=min(64, self.chunk_size),
                                  A_is_log=True, return_final_states=True)
        ssm_state.copy_(last)
        return y

    @torch.no_grad()
    def step(self, hidden_states, conv_state, ssm_state):
        dtype = hidden_states.dtype
        zxbcdt = self.in_proj(hidden_states.squeeze(1))
        di, gn, H = self.d_ssm, self.ngroups * self.d_state, self.nheads
        z0, x0, z, xBC, dt = torch.split(zxbcdt, [self.d_mlp, self.d_mlp, di, di + 2 * gn, H], dim=-1)
        if zxbcdt.stride(-2) % 8:
            z, xBC, dt = z.contiguous(), xBC.contiguous(), dt.contiguous()
        xBC = causal_conv1d_update(xBC, conv_state, self.conv1d.weight, self.conv1d.bias, "silu")
        x, B, C = torch.split(xBC, [di, gn, gn], dim=-1)
        A = -torch.exp(self.A_log.float())
        xh = x.unflatten(-1, (H, self.headdim))
        y = selective_state_update(ssm_state, xh, dt, A,
                                   B.unflatten(-1, (self.ngroups, self.d_state)),
                                   C.unflatten(-1, (self.ngroups, self.d_state)),
                                   None if self.D_has_hdim else self.D,
                                   z=None, dt_bias=self.dt_bias, dt_softplus=True)
        y = self._skip_gate_norm(y, xh, z)
        if self.d_mlp > 0:
            y = torch.cat([F.silu(z0) * x0, y], dim=-1)
        out = self.out_proj(y)
        return out.unsqueeze(1).to(dtype), conv_state, ssm_state

    def allocate_inference_cache(self, batch_size, max_seqlen, dtype=None, **kwargs):
        device = self.out_proj.weight.device
        conv_dtype = self.conv1d.weight.dtype if dtype is None else dtype
        conv_state = torch.zeros(batch_size, self.conv1d.weight.shape[0], self.d_conv, device=device,
                                 dtype=conv_dtype)
        ssm_state = torch.zeros(batch_size, self.nheads, self.headdim, self.d_state, device=device,
                                dtype=torch.float32)
        return conv_state, ssm_state

    def _get_states_from_cache(self, inference_params, batch_size):
        assert self.layer_idx is not None
        if self.layer_idx not in inference_params.key_value_memory_dict:
            inference_params.key_value_memory_dict[self.layer_idx] = self.allocate_inference_cache(
                batch_size, inference_params.max_seqlen)
        return inference_params.key_value_memory_dict[self.layer_idx]


def seq_idx_from_cu_seqlens(cu_seqlens: torch.Tensor, seqlen: int, device=None) -> torch.Tensor:
    """(1, seqlen) int32 sequence index of every packed token from cumulative lengths [0, l1, l1+l2, ...]."""
    cu = cu_seqlens.to(device=device, dtype=torch.long)
    lens = (cu[1:] - cu[:-1]).clamp(min=0)
    idx = torch.repeat_interleave(torch.arange(lens.numel(), device=cu.device, dtype=torch.int32), lens)
    assert idx.numel() == seqlen, f"cu_seqlens covers {idx.numel()} tokens, sequence has {seqlen}"
    return idx.unsqueeze(0)
