"""Checkpoints (reference train.py:152-163 writer, eval.py:29-43 reader).

Layout kept: ``log/model_{step:05d}.pt`` holding ``{"model", "config", "step", "val_loss"}`` with
the §2.8 state-dict keys.  Changes:
  * ``config`` is a plain dict -> a bare ``torch.load(path)`` works under torch>=2.6's
    ``weights_only=True`` default (the reference's pickled dataclass does not load there),
  * optional ``optimizer`` / ``rng`` / ``loader`` / ``lr_step`` entries make real resume possible,
  * atomic write (tmp file + rename) so a crash mid-save never leaves a truncated checkpoint.
"""
from __future__ import annotations

import glob
import os
import random
import re
from typing import Optional

import numpy as np
import torch

from ..config import MambaConfig


def rng_state():
    st = {"torch": torch.get_rng_state(), "numpy": np.random.get_state()[1].tolist(),
          "python": list(random.getstate()[1])}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st):
    torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])


def save_checkpoint(path: str, model, step: int, val_loss: Optional[float] = None, optimizer=None,
                    loader_state=None, extra=None, include_rng: bool = False, model_state=None):
    """``model_state``: an explicit state dict (e.g. the reassembled full layout of a tensor-parallel
    model, parallel/api.py::full_state_dict); default ``model.state_dict()``."""
    cfg = model.config.to_dict() if hasattr(model.config, "to_dict") else dict(model.config)
    sd = model_state if model_state is not None else model.state_dict()
    ckpt = {"model": sd, "config": cfg, "step": step, "val_loss": val_loss}
    if optimizer is not None:
        ckpt["optimizer"] = optimizer.state_dict()
    if loader_state is not None:
        ckpt["loader"] = loader_state
    if include_rng:
        ckpt["rng"] = rng_state()
    if extra:
        ckpt.update(extra)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(ckpt, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str, map_location="cpu"):
    """Safe load (weights_only=True: nothing in the file is executed)."""
    return torch.load(path, map_location=map_location, weights_only=True)


def config_from_checkpoint(ckpt) -> MambaConfig:
    cfg = ckpt.get("config")
    if isinstance(cfg, MambaConfig):
        return cfg
    if isinstance(cfg, dict):
        return MambaConfig.from_dict(cfg)
    # reference-era checkpoint without a readable config: the hard-coded eval.py:34 config
    return MambaConfig(d_model=768, vocab_size=50304)


def latest_checkpoint(log_dir: str) -> Optional[str]:
    paths = glob.glob(os.path.join(log_dir, "model_*.pt"))
    best, best_step = None, -1
    for p in paths:
        m = re.search(r"model_(\d+)\.pt$", p)
        if m and int(m.group(1)) > best_step:
            best, best_step = p, int(m.group(1))
    return best
