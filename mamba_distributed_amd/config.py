"""Model configuration.

`MambaConfig` keeps the exact field names and defaults of the dataclass the reference
builds its model from (reference train.py:75 ``MambaConfig(d_model=768, vocab_size=50304)``,
eval.py:34; upstream ``mamba_ssm/models/config_mamba.py`` — SURVEY.md §2.2 D1), so
``MambaConfig(d_model=768, vocab_size=50304)`` builds the same 64-layer, 280,019,712-param
Mamba-1 model the reference trains.

Differences that are deliberate:
  * ``to_dict`` / ``from_dict`` so checkpoints store the config as a plain dict, which
    loads under ``torch.load``'s ``weights_only=True`` default (torch >= 2.6).
"""
from __future__ import annotations

import copy
import dataclasses
from dataclasses import dataclass, field
from typing import Any, Dict, List


@dataclass
class MambaConfig:
    d_model: int = 2560
    d_intermediate: int = 0
    n_layer: int = 64
    vocab_size: int = 50277
    ssm_cfg: Dict[str, Any] = field(default_factory=dict)
    attn_layer_idx: List[int] = field(default_factory=list)
    attn_cfg: Dict[str, Any] = field(default_factory=dict)
    rms_norm: bool = True
    residual_in_fp32: bool = True
    fused_add_norm: bool = True
    pad_vocab_size_multiple: int = 8
    tie_embeddings: bool = True

    # ---- helpers (not part of the upstream field set) ----
    def to_dict(self) -> Dict[str, Any]:
        return copy.deepcopy(dataclasses.asdict(self))

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "MambaConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: copy.deepcopy(v) for k, v in d.items() if k in names})

    @property
    def layer_type(self) -> str:
        return self.ssm_cfg.get("layer", "Mamba1")

    @property
    def padded_vocab_size(self) -> int:
        m = self.pad_vocab_size_multiple
        v = self.vocab_size
        return v if v % m == 0 else v + (m - v % m)


# Named configs used by bench.py / train.py (BASELINE.json "configs").
PRESETS: Dict[str, Dict[str, Any]] = {
    # reference default: Mamba-1 mixers, "280M" (train.py:75)
    "mamba1-280m": dict(d_model=768, n_layer=64, vocab_size=50304, ssm_cfg={"layer": "Mamba1"}),
    # BASELINE headline: the same width/depth with Mamba-2 (SSD) mixers, 279.6M params
    "mamba2-280m": dict(d_model=768, n_layer=64, vocab_size=50304, ssm_cfg={"layer": "Mamba2"}),
    "mamba1-370m": dict(d_model=1024, n_layer=48, vocab_size=50304, ssm_cfg={"layer": "Mamba1"}),
    "mamba2-1.4b": dict(d_model=2048, n_layer=48, vocab_size=50304, ssm_cfg={"layer": "Mamba2"}),
    "mamba2-2.8b": dict(d_model=2560, n_layer=64, vocab_size=50304, ssm_cfg={"layer": "Mamba2"}),
    # tiny plumbing config (BASELINE "Tiny Mamba-2 (2 layers, d_model=256)")
    "mamba2-tiny": dict(d_model=256, n_layer=2, vocab_size=50304, ssm_cfg={"layer": "Mamba2"}),
    "mamba1-tiny": dict(d_model=256, n_layer=2, vocab_size=50304, ssm_cfg={"layer": "Mamba1"}),
}


def preset(name: str, **overrides) -> MambaConfig:
    d = copy.deepcopy(PRESETS[name])
    d.update(overrides)
    return MambaConfig(**d)
