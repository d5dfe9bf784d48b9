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
"""
from __future__ import annotations

from typing import Optional

import torch

from .models.mixer_seq import InferenceParams, MambaLMHeadModel


class GraphedDecoder:
    def __init__(self, model: MambaLMHeadModel, batch_size: int = 1, max_seqlen: int = 2048,
                 use_graph: Optional[bool] = None):
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

    def _states(self):
        return [t for v in self.params.key_value_memory_dict.values() for t in v]

    def reset(self):
        for t in self._states():
            t.zero_()
        self.params.seqlen_offset = 0

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
