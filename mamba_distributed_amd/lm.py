"""``LMHeadModel`` — the reference's model API façade (reference model.py:15-149).

Same constructor and methods:
  LMHeadModel(config, device, enc=None)
  .forward(input_ids, targets=None, position_ids=None, inference_params=None, num_last_tokens=0)
        -> (logits, loss)
  .generate(text, top_k=50, max_length=32, seed=42) -> str
  .top_k_sampling(logits, k=50, seed=42) -> int
  LMHeadModel.load_from_hf(model_name, device)
  .configure_optimizers(weight_decay, learning_rate, device_type, master_process) -> AdamW

Deliberate differences:
  * A7: no stray ``self.type = type``;  A8: ``seed`` is honoured, no debug prints.
  * ``forward(..., return_logits=False)`` with targets runs the fused lm_head+cross-entropy HIP
    path (the (B*T, V) logits tensor is never materialised twice; logits come back as None).
  * ``generate`` uses the O(L) cached-state decode (A12) instead of full-prefix recompute;
    ``generate(..., use_cache=False)`` keeps the reference's recompute behaviour.
  * A9: weight decay is applied to every >=2-D tensor (incl. A_log, conv1d.weight) exactly like the
    reference; ``honor_no_weight_decay=True`` opts into upstream's ``_no_weight_decay`` flags.
"""
from __future__ import annotations

import inspect
from typing import Optional

import torch

from .config import MambaConfig
from .models.mixer_seq import InferenceParams, MambaLMHeadModel
from .ops.cross_entropy import cross_entropy, fused_linear_cross_entropy
from .utils.tokenizer import get_encoding


class LMHeadModel(MambaLMHeadModel):
    def __init__(self, config: MambaConfig, device=None, enc=None, dtype=None):
        self.device = device
        super().__init__(config, device=device, dtype=dtype)
        self.enc = enc if enc is not None else get_encoding("gpt2")

    # nn.Module defines `.to`; keep self.device in sync for generate()
    def to(self, *args, **kwargs):
        out = super().to(*args, **kwargs)
        dev = next(self.parameters()).device
        self.device = str(dev) if dev.type != "cpu" else "cpu"
        return out

    def forward(self, input_ids, targets=None, position_ids=None, inference_params=None,
                num_last_tokens=0, return_logits=True, **mixer_kwargs):
        par = getattr(self, "parallel", None)
        if par is not None and targets is not None:
            from .parallel.api import shard_batch
            targets = shard_batch(self, targets)
        if targets is not None and not return_logits:
            h = self.backbone(input_ids, inference_params=inference_params, **mixer_kwargs)
            cd = torch.get_autocast_dtype("cuda") if (h.is_cuda and torch.is_autocast_enabled("cuda")) else h.dtype
            loss = fused_linear_cross_entropy(h, self.lm_head.weight, targets, compute_dtype=cd)
            return None, self._parallel_loss(loss)
        logits = super().forward(input_ids, position_ids=position_ids, inference_params=inference_params,
                                 num_last_tokens=num_last_tokens, **mixer_kwargs).logits
        loss = None
        if targets is not None:
            loss = self._parallel_loss(cross_entropy(logits.reshape(-1, logits.size(-1)), targets.reshape(-1)))
        return logits, loss

    def _parallel_loss(self, loss):
        """Sequence parallelism: every TP rank holds 1/tp of the tokens; return the TP-group mean
        (forward all-reduce, identity backward -> each rank back-propagates its own mean / tp).
        Context parallelism keeps the rank-local mean (DDP over DP x CP averages the gradients)."""
        par = getattr(self, "parallel", None)
        if par is None or not par.sequence_parallel:
            return loss
        from .parallel.comm import reduce_from_group
        return reduce_from_group(loss, par.tp_group) / par.tp

    # ------------------------------------------------------------------------------------
    def top_k_sampling(self, logits: torch.Tensor, k: int = 50, seed: Optional[int] = 42,
                       generator: Optional[torch.Generator] = None) -> int:
        top_k_logits, top_k_indices = torch.topk(logits.float(), k)
        probabilities = torch.softmax(top_k_logits, dim=-1)
        if generator is None:
            generator = torch.Generator(device=logits.device)
            if seed is not None:
                generator.manual_seed(seed)
        sampled = torch.multinomial(probabilities, num_samples=1, generator=generator)
        return int(top_k_indices[sampled].item())

    @torch.no_grad()
    def generate(self, text: str, top_k: int = 50, max_length: int = 32, seed: int = 42,
                 use_cache: bool = True, use_graph: Optional[bool] = None) -> str:
        """Top-k sampling (reference model.py:49-75).  ``use_cache`` (default): O(1) state-cached
        decode; on a GPU with a pure Mamba stack the per-token step replays a HIP graph
        (``inference.GraphedDecoder``).  ``use_cache=False``: the reference's full recompute."""
        dev = next(self.parameters()).device
        ids = self.enc.encode(text)
        eot = self.enc.eot_token if hasattr(self.enc, "eot_token") else getattr(self.enc, "eos_token_id", None)
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed)
        xgen = torch.tensor([ids], device=dev, dtype=torch.long)
        if not use_cache:
            for _ in range(max_length):
                logits, _ = self(xgen)
                nxt = self.top_k_sampling(logits[0, -1], k=top_k, generator=gen)
                xgen = torch.cat([xgen, torch.tensor([[nxt]], device=dev)], dim=1)
                if nxt == eot:
                    break
            return self.enc.decode(xgen[0].tolist())
        from .inference import GraphedDecoder
        dec = GraphedDecoder(self, batch_size=1, max_seqlen=xgen.shape[1] + max_length, use_graph=use_graph)
        logits = dec.prefill(xgen)
        out = list(ids)
        for i in range(max_length):
            nxt = self.top_k_sampling(logits[0], k=top_k, generator=gen)
            out.append(nxt)
            if nxt == eot or i == max_length - 1:
                break
            logits = dec.step(torch.tensor([nxt], device=dev))
        return self.enc.decode(out)

    # ------------------------------------------------------------------------------------
    @classmethod
    def load_from_hf(cls, model_name: str, device: str, enc=None) -> "LMHeadModel":
        from .utils.hf import load_config_hf, load_state_dict_hf
        config = MambaConfig.from_dict(load_config_hf(model_name))
        if enc is None:
            try:
                from transformers import AutoTokenizer
                enc = AutoTokenizer.from_pretrained("state-spaces/mamba-370m-hf", local_files_only=True)
            except Exception:
                enc = None
        model = cls(config, device=device, enc=enc)
        model.load_state_dict(load_state_dict_hf(model_name))
        return model

    def configure_optimizers(self, weight_decay, learning_rate, device_type, master_process,
                             honor_no_weight_decay: bool = False, betas=(0.9, 0.95), eps=1e-8):
        param_dict = {pn: p for pn, p in self.named_parameters() if p.requires_grad}

        def decays(p):
            if honor_no_weight_decay and getattr(p, "_no_weight_decay", False):
                return False
            return p.dim() >= 2

        decay_params = [p for _, p in param_dict.items() if decays(p)]
        nodecay_params = [p for _, p in param_dict.items() if not decays(p)]
        optim_groups = [
            {"params": decay_params, "weight_decay": weight_decay},
            {"params": nodecay_params, "weight_decay": 0.0},
        ]
        if master_process:
            print(f"num decayed parameter tensors: {len(decay_params)}, with "
                  f"{sum(p.numel() for p in decay_params):,} parameters")
            print(f"num non-decayed parameter tensors: {len(nodecay_params)}, with "
                  f"{sum(p.numel() for p in nodecay_params):,} parameters")
        fused_available = "fused" in inspect.signature(torch.optim.AdamW).parameters
        use_fused = fused_available and device_type == "cuda"
        if master_process:
            print(f"using fused AdamW: {use_fused}")
        # on the GPU the native multi-tensor AdamW (ops/optim.py: same update, clip and bf16 weight images folded
        # in); MAMBA_AMD_NATIVE_ADAMW=0 keeps torch's fused AdamW
        import os
        from .ops.optim import NativeAdamW, native_available
        if (use_fused and os.environ.get("MAMBA_AMD_NATIVE_ADAMW", "1") != "0"
                and native_available(decay_params + nodecay_params)):
            return NativeAdamW(optim_groups, lr=learning_rate, betas=betas, eps=eps)
        return torch.optim.AdamW(optim_groups, lr=learning_rate, betas=betas, eps=eps, fused=use_fused)

