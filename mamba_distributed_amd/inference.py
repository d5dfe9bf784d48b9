"""Cached decoding with the per-token step captured in a HIP graph.

Upstream's ``GenerationMixin`` keeps a CUDA-graph decode cache (utils/generation.py);
the reference never uses it (its ``generate`` re-runs the full prefix per token, model.py:49-75).
On MI355X one decode token of a 64-layer stack is ~400 tiny kernels (a few GEMVs, the conv/SSM
state updates and norms per layer), so host launch overhead, not the GPU, sets the latency.
``GraphedDecoder`` allocates the conv/SSM state caches once, runs the prompt through the normal
(chunked) path, then records ONE decode step for the whole stack into a ``torch.cuda.CUDAGraph``
(a HIP graph on ROCm) and replays it per token: one launch per token instead of hundreds.

Only pure Mamba stacks are graphed: attention layers index their KV cache by a Python-side offset
that changes every token.

For pure Mamba-2 stacks in bf16 the step is additionally FUSED (``fused=None`` -> automatic): each
layer runs four native kernels (residual-add+RMSNorm, then csrc/kernels/decode.hip: in_proj GEMV+conv
window, SSM state update+gate, gated-norm+out_proj GEMV) on fp32 parameter copies prepared once,
instead of ~7 library / elementwise kernels plus per-call parameter casts.
"""
from __future__ import annotations

from typing import Optional

import torch

from .models.mixer_seq import InferenceParams, MambaLMHeadModel


class _FusedMamba2Step:
    """Buffers + fp32 parameter copies for the fused per-layer decode kernels (decode.hip)."""

    def __init__(self, model: MambaLMHeadModel, params: InferenceParams, batch_size: int):
        dev = next(model.parameters()).device
        bb = model.backbone
        self.model, self.params, self.b = model, params, batch_size
        f32 = lambda t: None if t is None else t.detach().float().contiguous()  # noqa: E731
        bf = lambda t: t.detach().to(torch.bfloat16).contiguous()  # noqa: E731
        self.layers = []
        for i, blk in enumerate(bb.layers):
            m = blk.mixer
            H, P, G, N = m.nheads, m.headdim, m.ngroups, m.d_state
            di = m.d_inner
            conv_state, ssm_state = params.key_value_memory_dict[i]
            self.layers.append(dict(
                norm_w=f32(blk.norm.weight), eps=float(blk.norm.eps), W_in=bf(m.in_proj.weight),
                conv_lo=di, conv_hi=2 * di + 2 * G * N, conv_w=f32(m.conv1d.weight.reshape(m.conv1d.weight.shape[0], -1)),
                conv_b=f32(m.conv1d.bias), A=(-torch.exp(m.A_log.detach().float())).contiguous(), D=f32(m.D),
                dt_bias=f32(m.dt_bias), G=G, geps=float(m.norm.eps),
                # gate-norm weight folded into out_proj (decode.hip K3 applies rstd in its epilogue)
                W_out=bf(m.out_proj.weight.float() * m.norm.weight.float()[None, :]),
                conv_state=conv_state, ssm_state=ssm_state, n_out=m.in_proj.weight.shape[0], di=di, nparts=H * (P // 16)))
        d = bb.embedding.weight.shape[1]
        n_out = max(l["n_out"] for l in self.layers)
        di = max(l["di"] for l in self.layers)
        nparts = max(l["nparts"] for l in self.layers)
        b = batch_size
        self.h = [torch.empty(b, d, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        self.zx = torch.empty(b * n_out, device=dev, dtype=torch.float32)
        self.g = torch.empty(b * di, device=dev, dtype=torch.bfloat16)
        self.part = torch.empty(b * nparts, device=dev, dtype=torch.float32)
        self.norm_f = bb.norm_f
        self.norm_f_w = f32(bb.norm_f.weight)

    @torch.no_grad()
    def refresh(self):
        """Re-derive the parameter copies IN PLACE from the model's current weights (after training steps), so
        a captured graph that points at them stays valid."""
        bb = self.model.backbone
        for blk, L in zip(bb.layers, self.layers):
            m = blk.mixer
            L["norm_w"].copy_(blk.norm.weight)
            L["W_in"].copy_(m.in_proj.weight)
            L["conv_w"].copy_(m.conv1d.weight.reshape(m.conv1d.weight.shape[0], -1))
            if L["conv_b"] is not None:
                L["conv_b"].copy_(m.conv1d.bias)
            L["A"].copy_(-torch.exp(m.A_log.float()))
            L["D"].copy_(m.D)
            L["dt_bias"].copy_(m.dt_bias)
            L["W_out"].copy_(m.out_proj.weight.float() * m.norm.weight.float()[None, :])
        self.norm_f_w.copy_(bb.norm_f.weight)

    @staticmethod
    def supported(model: MambaLMHeadModel, batch_size: int) -> bool:
        from .models.mamba2 import Mamba2
        from .ops import _ext
        bb = model.backbone
        dev = next(model.parameters()).device
        if dev.type != "cuda" or not _ext.use_native(next(model.parameters())) or batch_size > 16:
            return False
        from .ops.norm import RMSNorm
        if not (bb.fused_add_norm and bb.residual_in_fp32) or bb.embedding.weight.dtype != torch.bfloat16 \
                or not isinstance(bb.norm_f, RMSNorm):
            return False
        d = bb.embedding.weight.shape[1]
        if d % 8 or batch_size * d * 2 > 65536:
            return False
        for blk in bb.layers:
            m = blk.mixer
            if type(m) is not Mamba2 or m._general or blk.mlp is not None or m.norm_before_gate or m.in_proj.bias is not None \
                    or m.out_proj.bias is not None or getattr(m, "cp_group", None) is not None:
                return False
            if m.conv1d.weight.dtype != torch.bfloat16 or m.headdim % 16 or m.d_state not in (64, 128, 256):
                return False
            if m.d_inner % 8 or batch_size * m.d_inner * 2 > 65536 or m.d_ssm != m.d_inner:
                return False
        return True

    def __call__(self, tok: torch.Tensor) -> torch.Tensor:
        ops = torch.ops.mamba_amd
        b = self.b
        h = self.model.backbone.embedding(tok.reshape(b)).to(torch.bfloat16)
        res = None
        for i, L in enumerate(self.layers):
            zx = self.zx[: b * L["n_out"]]
            g = self.g[: b * L["di"]].view(b, L["di"])
            part = self.part[: b * L["nparts"]].view(b, L["nparts"])
            hn, res, _ = ops.add_rmsnorm_fwd(h, res, L["norm_w"], L["eps"], torch.bfloat16, torch.float32)
            ops.decode_inproj(hn, L["W_in"], zx, L["conv_lo"], L["conv_hi"], L["conv_state"], L["conv_w"], L["conv_b"])
            ops.decode_ssm(zx, L["ssm_state"], L["A"], L["D"], L["dt_bias"], L["G"], g, part)
            h = self.h[i % 2]
            ops.decode_outproj(g, part, L["geps"], L["W_out"], h)
        hn, _, _ = ops.add_rmsnorm_fwd(h, res, self.norm_f_w, self.norm_f.eps, torch.bfloat16, torch.float32)
        return torch.nn.functional.linear(hn, self.model.lm_head.weight)


class GraphedDecoder:
    def __init__(self, model: MambaLMHeadModel, batch_size: int = 1, max_seqlen: int = 2048,
                 use_graph: Optional[bool] = None, fused: Optional[bool] = None):
        self.model = model
        self.device = next(model.parameters()).device
        attn = getattr(model.config, "attn_layer_idx", None)
        if use_graph is None:
            use_graph = self.device.type == "cuda" and not attn
        if use_graph and attn:
            raise ValueError("HIP-graph decode supports pure Mamba stacks only (attention KV offsets vary per token)")
        self.use_graph = use_graph
        self.batch_size = batch_size
        self.params = InferenceParams(max_seqlen=max_seqlen, max_batch_size=batch_size)
        self.params.key_value_memory_dict = model.allocate_inference_cache(batch_size, max_seqlen)
        self.tok = torch.zeros(batch_size, 1, dtype=torch.long, device=self.device)
        self.graph = None
        self.out = None
        if fused is None:
            fused = _FusedMamba2Step.supported(model, batch_size)
        self.fused = _FusedMamba2Step(model, self.params, batch_size) if fused else None

    def _states(self):
        return [t for v in self.params.key_value_memory_dict.values() for t in v]

    def reset(self):
        for t in self._states():
            t.zero_()
        self.params.seqlen_offset = 0

    def refresh(self):
        """Pick up weight updates made since construction (the fused step's derived copies)."""
        if self.fused is not None:
            self.fused.refresh()

    @torch.no_grad()
    def prefill(self, input_ids: torch.Tensor) -> torch.Tensor:
        """Run the prompt (b, l), fill the caches, return the last position's logits (b, V)."""
        assert input_ids.shape[0] == self.batch_size
        self.reset()
        logits = MambaLMHeadModel.forward(self.model, input_ids, inference_params=self.params,
                                          num_last_tokens=1).logits
        self.params.seqlen_offset = input_ids.shape[1]
        return logits[:, -1]

    def _eager_step(self) -> torch.Tensor:
        if self.fused is not None:
            return self.fused(self.tok)
        return MambaLMHeadModel.forward(self.model, self.tok, inference_params=self.params).logits[:, -1]

    def _capture(self):
        # warm up on a side stream (lazy library handles, extension load) without disturbing the caches
        saved = [t.clone() for t in self._states()]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                self._eager_step()
        torch.cuda.current_stream().wait_stream(side)
        for t, s in zip(self._states(), saved):
            t.copy_(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = self._eager_step()  # recorded, not executed

    @torch.no_grad()
    def step(self, token_ids: torch.Tensor) -> torch.Tensor:
        """Feed one token per sequence (b,) or (b, 1); returns next-token logits (b, V)."""
        assert self.params.seqlen_offset > 0, "call prefill() first"
        self.tok.copy_(token_ids.reshape(self.batch_size, 1))
        if not self.use_graph:
            out = self._eager_step()
        else:
            if self.graph is None:
                self._capture()
            self.graph.replay()
            out = self.out
        self.params.seqlen_offset += 1
        return out
