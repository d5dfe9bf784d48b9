"""Backbone and LM head: Block, create_block, MixerModel, MambaLMHeadModel.

Behaviour contract = upstream ``mamba_ssm/models/mixer_seq_simple.py`` + ``modules/block.py``
as reached by the reference (reference model.py:8, train.py:75):
  * pre-norm residual blocks, fp32 residual stream, fused add+RMSNorm (HIP kernel on GPU),
  * ``ssm_cfg["layer"]`` selects Mamba1 (default) or Mamba2,
  * vocab padded to ``pad_vocab_size_multiple``, tied embeddings,
  * ``_init_weights``: N(0, 0.02) embeddings, zero linear biases (except ``_no_reinit``),
    out_proj re-scaled by 1/sqrt(n_residuals_per_layer * n_layer),
  * state-dict keys identical to SURVEY.md §2.8 (``backbone.embedding.weight``, ...).
"""
from __future__ import annotations

import copy
import json
import math
import os
from collections import namedtuple
from dataclasses import dataclass, field
from functools import partial
from typing import Optional

import torch
import torch.utils.checkpoint
import torch.nn as nn
import torch.nn.functional as F

from ..config import MambaConfig
from ..ops.norm import RMSNorm, rms_norm_fn
from .layers import MHA, GatedMLP
from .mamba1 import Mamba
from .mamba2 import Mamba2
from ..utils.generation import GenerationMixin


@dataclass
class InferenceParams:
    """Decode cache bookkeeping (upstream utils/generation.py InferenceParams)."""
    max_seqlen: int
    max_batch_size: int
    seqlen_offset: int = 0
    batch_size_offset: int = 0
    key_value_memory_dict: dict = field(default_factory=dict)
    lengths_per_sample: Optional[torch.Tensor] = None

    def reset(self, max_seqlen, max_batch_size):
        self.max_seqlen = max_seqlen
        self.max_batch_size = max_batch_size
        self.seqlen_offset = 0
        if self.lengths_per_sample is not None:
            self.lengths_per_sample.zero_()


class Block(nn.Module):
    def __init__(self, dim, mixer_cls, mlp_cls, norm_cls=nn.LayerNorm, fused_add_norm=False,
                 residual_in_fp32=False):
        super().__init__()
        self.residual_in_fp32 = residual_in_fp32
        self.fused_add_norm = fused_add_norm
        self.norm = norm_cls(dim)
        self.mixer = mixer_cls(dim)
        if mlp_cls is not nn.Identity:
            self.norm2 = norm_cls(dim)
            self.mlp = mlp_cls(dim)
        else:
            self.mlp = None
        # the fused add+norm kernel is RMSNorm's; with LayerNorm (rms_norm=False) the same prenorm math runs
        # unfused (upstream's layer_norm_fn with is_rms_norm=False)
        self._fused_rms = fused_add_norm and isinstance(self.norm, RMSNorm)

    def _add_norm(self, norm, hidden_states, residual):
        if self._fused_rms:
            return rms_norm_fn(hidden_states, norm.weight, None, residual=residual, prenorm=True,
                               residual_in_fp32=self.residual_in_fp32, eps=norm.eps)
        residual = (hidden_states + residual) if residual is not None else hidden_states
        hidden_states = norm(residual.to(dtype=norm.weight.dtype))
        if self.residual_in_fp32:
            residual = residual.to(torch.float32)
        return hidden_states, residual

    def forward(self, hidden_states, residual=None, inference_params=None, **mixer_kwargs):
        hidden_states, residual = self._add_norm(self.norm, hidden_states, residual)
        hidden_states = self.mixer(hidden_states, inference_params=inference_params, **mixer_kwargs)
        if self.mlp is not None:
            hidden_states, residual = self._add_norm(self.norm2, hidden_states, residual)
            hidden_states = self.mlp(hidden_states)
        return hidden_states, residual

    def allocate_inference_cache(self, batch_size, max_seqlen, dtype=None, **kw):
        return self.mixer.allocate_inference_cache(batch_size, max_seqlen, dtype=dtype, **kw)


def create_block(d_model, d_intermediate, ssm_cfg=None, attn_layer_idx=None, attn_cfg=None,
                 norm_epsilon=1e-5, rms_norm=False, residual_in_fp32=False, fused_add_norm=False,
                 layer_idx=None, device=None, dtype=None):
    factory = {"device": device, "dtype": dtype}
    ssm_cfg = copy.deepcopy(ssm_cfg) if ssm_cfg is not None else {}
    attn_layer_idx = attn_layer_idx or []
    attn_cfg = attn_cfg or {}
    if layer_idx not in attn_layer_idx:
        ssm_layer = ssm_cfg.pop("layer", "Mamba1")
        if ssm_layer not in ("Mamba1", "Mamba2"):
            raise ValueError(f"Invalid ssm_layer: {ssm_layer}, only support Mamba1 and Mamba2")
        cls = Mamba2 if ssm_layer == "Mamba2" else Mamba
        mixer_cls = partial(cls, layer_idx=layer_idx, **ssm_cfg, **factory)
    else:
        mixer_cls = partial(MHA, layer_idx=layer_idx, **attn_cfg, **factory)
    norm_cls = partial(RMSNorm if rms_norm else nn.LayerNorm, eps=norm_epsilon, **factory)
    if d_intermediate == 0:
        mlp_cls = nn.Identity
    else:
        mlp_cls = partial(GatedMLP, hidden_features=d_intermediate, out_features=d_model, **factory)
    block = Block(d_model, mixer_cls, mlp_cls, norm_cls=norm_cls, fused_add_norm=fused_add_norm,
                  residual_in_fp32=residual_in_fp32)
    block.layer_idx = layer_idx
    return block


def _init_weights(module, n_layer, initializer_range=0.02, rescale_prenorm_residual=True,
                  n_residuals_per_layer=1):
    if isinstance(module, nn.Linear):
        if module.bias is not None and not getattr(module.bias, "_no_reinit", False):
            nn.init.zeros_(module.bias)
    elif isinstance(module, nn.Embedding):
        nn.init.normal_(module.weight, std=initializer_range)
    if rescale_prenorm_residual:
        for name, p in module.named_parameters():
            if name in ("out_proj.weight", "fc2.weight"):
                nn.init.kaiming_uniform_(p, a=math.sqrt(5))
                with torch.no_grad():
                    p /= math.sqrt(n_residuals_per_layer * n_layer)


class MixerModel(nn.Module):
    def __init__(self, d_model, n_layer, d_intermediate, vocab_size, ssm_cfg=None, attn_layer_idx=None,
                 attn_cfg=None, norm_epsilon=1e-5, rms_norm=False, initializer_cfg=None,
                 fused_add_norm=False, residual_in_fp32=False, device=None, dtype=None):
        factory = {"device": device, "dtype": dtype}
        super().__init__()
        self.residual_in_fp32 = residual_in_fp32
        self.fused_add_norm = fused_add_norm
        self.embedding = nn.Embedding(vocab_size, d_model, **factory)
        self.layers = nn.ModuleList([
            create_block(d_model, d_intermediate=d_intermediate, ssm_cfg=ssm_cfg,
                         attn_layer_idx=attn_layer_idx, attn_cfg=attn_cfg, norm_epsilon=norm_epsilon,
                         rms_norm=rms_norm, residual_in_fp32=residual_in_fp32,
                         fused_add_norm=fused_add_norm, layer_idx=i, **factory)
            for i in range(n_layer)])
        self.norm_f = (RMSNorm if rms_norm else nn.LayerNorm)(d_model, eps=norm_epsilon, **factory)
        self.apply(partial(_init_weights, n_layer=n_layer, **(initializer_cfg or {}),
                           n_residuals_per_layer=1 if d_intermediate == 0 else 2))

    def allocate_inference_cache(self, batch_size, max_seqlen, dtype=None, **kw):
        return {i: layer.allocate_inference_cache(batch_size, max_seqlen, dtype=dtype, **kw)
                for i, layer in enumerate(self.layers)}

    def forward(self, input_ids, inference_params=None, **mixer_kwargs):
        ctx = getattr(self, "parallel", None)
        if ctx is not None and inference_params is None:
            # context / sequence parallelism (parallel/api.py): compute on this rank's token shard
            from ..parallel.api import shard_batch
            mixer_kwargs = dict(mixer_kwargs, seqlen=input_ids.shape[1] // max(1, ctx.cp))
            input_ids = shard_batch(self, input_ids)
        hidden_states = self.embedding(input_ids)
        residual = None
        every = getattr(self, "checkpoint_every", 0)
        recompute = every > 0 and inference_params is None and self.training and torch.is_grad_enabled()
        for i, layer in enumerate(self.layers):
            if recompute and i % every == 0:
                # activation checkpointing: keep only the block inputs, recompute the block in backward
                hidden_states, residual = torch.utils.checkpoint.checkpoint(
                    layer, hidden_states, residual, use_reentrant=False, **mixer_kwargs)
            else:
                hidden_states, residual = layer(hidden_states, residual, inference_params=inference_params,
                                                **mixer_kwargs)
        if self.fused_add_norm and isinstance(self.norm_f, RMSNorm):
            return rms_norm_fn(hidden_states, self.norm_f.weight, None, residual=residual, prenorm=False,
                               residual_in_fp32=self.residual_in_fp32, eps=self.norm_f.eps)
        residual = (hidden_states + residual) if residual is not None else hidden_states
        return self.norm_f(residual.to(dtype=self.norm_f.weight.dtype))


CausalLMOutput = namedtuple("CausalLMOutput", ["logits"])


class MambaLMHeadModel(nn.Module, GenerationMixin):
    def __init__(self, config: MambaConfig, initializer_cfg=None, device=None, dtype=None):
        super().__init__()
        self.config = config
        factory = {"device": device, "dtype": dtype}
        vocab_size = config.padded_vocab_size
        self.backbone = MixerModel(
            d_model=config.d_model, n_layer=config.n_layer, d_intermediate=config.d_intermediate,
            vocab_size=vocab_size, ssm_cfg=config.ssm_cfg, attn_layer_idx=config.attn_layer_idx,
            attn_cfg=config.attn_cfg, rms_norm=config.rms_norm, initializer_cfg=initializer_cfg,
            fused_add_norm=config.fused_add_norm, residual_in_fp32=config.residual_in_fp32, **factory)
        self.lm_head = nn.Linear(config.d_model, vocab_size, bias=False, **factory)
        self.apply(partial(_init_weights, n_layer=config.n_layer, **(initializer_cfg or {})))
        self.tie_weights()

    def tie_weights(self):
        if self.config.tie_embeddings:
            self.lm_head.weight = self.backbone.embedding.weight

    def allocate_inference_cache(self, batch_size, max_seqlen, dtype=None, **kw):
        return self.backbone.allocate_inference_cache(batch_size, max_seqlen, dtype=dtype, **kw)

    def set_activation_checkpointing(self, every: int = 1) -> None:
        """Recompute every ``every``-th block in the backward instead of keeping its activations
        (0 = off).  The memory/compute trade upstream exposes as the fused ops' ``checkpoint_lvl``,
        applied per block: at T = 8192+ or large micro-batches it bounds activation memory to the
        block inputs plus one block's working set.  Gradients are unchanged: the native kernels
        are deterministic, so the recomputed forward is bitwise the original."""
        self.backbone.checkpoint_every = int(every)

    def forward_hidden(self, input_ids, inference_params=None, **mixer_kwargs):
        return self.backbone(input_ids, inference_params=inference_params, **mixer_kwargs)

    def forward(self, input_ids, position_ids=None, inference_params=None, num_last_tokens=0,
                **mixer_kwargs):
        hidden_states = self.backbone(input_ids, inference_params=inference_params, **mixer_kwargs)
        if num_last_tokens > 0:
            hidden_states = hidden_states[:, -num_last_tokens:]
        return CausalLMOutput(logits=self.lm_head(hidden_states))

    # ---- upstream-style (de)serialisation: config.json + pytorch_model.bin -----------------
    @classmethod
    def from_pretrained(cls, pretrained_model_name, device=None, dtype=None, **kw):
        from ..utils.hf import load_config_hf, load_state_dict_hf
        config = MambaConfig.from_dict(load_config_hf(pretrained_model_name))
        model = cls(config, device=device, dtype=dtype, **kw)
        model.load_state_dict(load_state_dict_hf(pretrained_model_name, device=device, dtype=dtype))
        return model

    def save_pretrained(self, save_directory):
        os.makedirs(save_directory, exist_ok=True)
        torch.save(self.state_dict(), os.path.join(save_directory, "pytorch_model.bin"))
        with open(os.path.join(save_directory, "config.json"), "w") as f:
            json.dump(self.config.to_dict(), f, indent=4)
