"""Op layer: autograd Functions that dispatch to the gfx950 HIP kernels (GPU) or to the
pure-PyTorch references (CPU).  See ``_ext.py`` for the dispatch policy."""
from . import _ext, reference
from .conv1d import causal_conv1d_fn, causal_conv1d_update
from .cross_entropy import cross_entropy, fused_linear_cross_entropy
from .norm import RMSNorm, RMSNormGated, layer_norm_fn, rms_norm_fn, rmsnorm_gated_fn
from .selective_scan import mamba_inner_fn, selective_scan_fn, selective_state_update
from .ssd import mamba2_inner_fn, mamba_chunk_scan_combined, mamba_split_conv1d_scan_combined

native_available = _ext.available

__all__ = [
    "causal_conv1d_fn", "causal_conv1d_update", "cross_entropy", "fused_linear_cross_entropy",
    "RMSNorm", "RMSNormGated", "layer_norm_fn", "rms_norm_fn", "rmsnorm_gated_fn",
    "mamba_inner_fn", "selective_scan_fn", "selective_state_update", "mamba2_inner_fn",
    "mamba_chunk_scan_combined", "mamba_split_conv1d_scan_combined", "native_available", "reference",
]
