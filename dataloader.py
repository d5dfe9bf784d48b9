"""Reference-compatible data module (reference dataloader.py): `from dataloader import DataLoaderLite`."""
from mamba_distributed_amd.data.loader import DataLoaderLite, load_tokens  # noqa: F401

__all__ = ["DataLoaderLite", "load_tokens"]
