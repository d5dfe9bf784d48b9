"""Loader for the in-tree native extension ``mamba_distributed_amd/_C.so``.

The .so is built by ``mamba_distributed_amd/csrc/build.py`` (hipcc, ``--offload-arch=gfx950``)
and registers its operators under ``torch.ops.mamba_amd``.

Dispatch policy (one place, used by every op module):
  * CPU tensors            -> the pure-PyTorch reference path (``ops/reference.py``)
  * GPU tensors            -> the HIP kernels.  If the extension is missing on a GPU box we
                              raise instead of silently falling back: a silent eager fallback would
                              make a GPU test pass without the native code ever running.
  * ``MAMBA_AMD_FORCE_REFERENCE=1`` is the one explicit opt-in to run the reference ops on the
    GPU (used for A/B baselines in bench.py --reference-ops).
"""
from __future__ import annotations

import os
import threading

import torch

_LOCK = threading.Lock()
_LOADED = None  # None = not tried, False = failed, str = path
_ERR = None

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MAMBA_AMD_SO: load another build of the extension (kernel A/B runs against a saved baseline .so)
SO_PATH = os.environ.get("MAMBA_AMD_SO") or os.path.join(_PKG_DIR, "_C.so")


def load() -> bool:
    global _LOADED, _ERR
    if _LOADED is not None:
        return bool(_LOADED)
    with _LOCK:
        if _LOADED is not None:
            return bool(_LOADED)
        if not os.path.exists(SO_PATH):
            _LOADED, _ERR = False, f"{SO_PATH} not built (run python -m mamba_distributed_amd.csrc.build)"
            return False
        try:
            torch.ops.load_library(SO_PATH)
            _LOADED = SO_PATH
        except Exception as e:  # pragma: no cover - depends on the box
            _LOADED, _ERR = False, f"failed to load {SO_PATH}: {e}"
    return bool(_LOADED)


def available() -> bool:
    return load()


def error() -> str:
    load()
    return _ERR or ""


def force_reference() -> bool:
    return os.environ.get("MAMBA_AMD_FORCE_REFERENCE", "0") == "1"


def use_native(*tensors) -> bool:
    """True when the op should run on the HIP kernels.

    Raises if any tensor is on the GPU, the reference path was not explicitly requested and the
    extension cannot be loaded (fail loudly — see module docstring).
    """
    on_gpu = any(t is not None and isinstance(t, torch.Tensor) and t.is_cuda for t in tensors)
    if not on_gpu or force_reference():
        return False
    if not load():
        raise RuntimeError(
            "mamba_distributed_amd native HIP extension is required for GPU tensors but is not "
            f"available: {_ERR}.  Build it with `python -m mamba_distributed_amd.csrc.build` or set "
            "MAMBA_AMD_FORCE_REFERENCE=1 to run the (slow) PyTorch reference ops explicitly."
        )
    return True


def ops():
    load()
    return torch.ops.mamba_amd
