"""Reference-compatible model module (reference model.py): `from model import LMHeadModel`."""
from mamba_distributed_amd.config import MambaConfig  # noqa: F401
from mamba_distributed_amd.lm import LMHeadModel  # noqa: F401

__all__ = ["LMHeadModel", "MambaConfig"]
