"""Hugging Face hub helpers (upstream utils/hf.py; reference model.py:97-116 re-implements this).

There is no network on the boxes this framework targets, so these resolve either a local
directory containing ``config.json`` / ``pytorch_model.bin`` (or ``model.safetensors``) or a
hub id already present in the local HF cache (``transformers.utils.hub.cached_file``).
Weights are always loaded with ``weights_only=True`` (nothing in the file is executed).
"""
from __future__ import annotations

import json
import os

import torch

CONFIG_NAME = "config.json"
WEIGHTS_NAME = "pytorch_model.bin"
SAFE_WEIGHTS_NAME = "model.safetensors"


def _resolve(model_name: str, filename: str):
    if os.path.isdir(model_name):
        p = os.path.join(model_name, filename)
        return p if os.path.exists(p) else None
    try:
        from transformers.utils.hub import cached_file
        return cached_file(model_name, filename, _raise_exceptions_for_missing_entries=False,
                           local_files_only=True)
    except Exception:
        return None


def load_config_hf(model_name: str) -> dict:
    path = _resolve(model_name, CONFIG_NAME)
    if path is None:
        raise FileNotFoundError(f"{CONFIG_NAME} for {model_name!r} not found locally (offline)")
    with open(path) as f:
        return json.load(f)


def load_state_dict_hf(model_name: str, device=None, dtype=None) -> dict:
    path = _resolve(model_name, SAFE_WEIGHTS_NAME)
    if path is not None:
        from safetensors.torch import load_file
        sd = load_file(path, device="cpu")
    else:
        path = _resolve(model_name, WEIGHTS_NAME)
        if path is None:
            raise FileNotFoundError(f"weights for {model_name!r} not found locally (offline)")
        sd = torch.load(path, weights_only=True, map_location="cpu", mmap=True)
    if dtype is not None:
        sd = {k: v.to(dtype=dtype) for k, v in sd.items()}
    if device is not None:
        sd = {k: v.to(device=device) for k, v in sd.items()}
    return sd
