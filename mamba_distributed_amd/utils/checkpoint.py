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
    """Every RNG this process draws from, as plain tensors / lists (weights_only-loadable)."""
    name, keys, pos, has_gauss, cached = np.random.get_state()
    ver, pstate, gauss_next = random.getstate()
    st = {"torch": torch.get_rng_state(),
          "numpy": {"name": name, "keys": keys.tolist(), "pos": int(pos), "has_gauss": int(has_gauss),
                    "cached": float(cached)},
          "python": {"version": int(ver), "state": list(pstate), "gauss_next": gauss_next}}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st):
    """Inverse of ``rng_state`` (torch, CUDA, numpy and python).  Older checkpoints stored only the
    numpy / python key arrays: those are restored with default positions."""
    torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])
    npst = st.get("numpy")
    if isinstance(npst, dict):
        np.random.set_state((npst["name"], np.asarray(npst["keys"], dtype=np.uint32), npst["pos"],
                             npst["has_gauss"], npst["cached"]))
    elif npst is not None:
        np.random.set_state(("MT19937", np.asarray(npst, dtype=np.uint32), 624, 0, 0.0))
    pyst = st.get("python")
    if isinstance(pyst, dict):
        random.setstate((pyst["version"], tuple(pyst["state"]), pyst["gauss_next"]))
    elif pyst is not None:
        random.setstate((3, tuple(pyst), None))


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


class _RefMambaConfig:
    """Stand-in for ``mamba_ssm.models.config_mamba.MambaConfig``, the dataclass the reference pickles
    into its checkpoints (train.py:152-163).  Registered as a weights_only safe global under that
    module path: the unpickler builds this inert object (attribute dict only, no code from the file
    runs) and ``config_from_checkpoint`` turns it into our MambaConfig."""

    def __setstate__(self, state):
        self.__dict__.update(state if isinstance(state, dict) else {})

    def to_dict(self):
        return dict(self.__dict__)


_RefMambaConfig.__module__ = "mamba_ssm.models.config_mamba"
_RefMambaConfig.__qualname__ = "MambaConfig"
_RefMambaConfig.__name__ = "MambaConfig"


def load_checkpoint(path: str, map_location="cpu"):
    """Safe load (weights_only=True: nothing in the file is executed).  Reference-format checkpoints
    (a pickled mamba_ssm MambaConfig under "config") load through the inert ``_RefMambaConfig``."""
    with torch.serialization.safe_globals([_RefMambaConfig]):
        return torch.load(path, map_location=map_location, weights_only=True)


def config_from_checkpoint(ckpt) -> MambaConfig:
    cfg = ckpt.get("config")
    if isinstance(cfg, MambaConfig):
        return cfg
    if isinstance(cfg, dict):
        return MambaConfig.from_dict(cfg)
    if isinstance(cfg, _RefMambaConfig):
        return MambaConfig.from_dict(cfg.to_dict())
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
