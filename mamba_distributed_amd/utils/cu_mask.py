"""CU-partitioned HIP streams (hipExtStreamCreateWithCUMask) for the concurrent training streams.

The step runs compute-bound GEMMs (weight gradients on the side stream, ops/grad_accum.py; the next
micro-batch's forward, parallel/microbatch.py) beside memory-bound norm / conv / scan kernels.  A GEMM
workgroup fills a CU (128 KB of LDS, 256+ registers per lane), so with unrestricted streams the two
kinds time-share CUs; a CU mask reserves a fixed share of every XCD for each stream instead, so the
bandwidth-bound kernels keep enough CUs to saturate HBM while the GEMMs run on the rest.

Masks are given in eighths: ``eighths=k`` enables CUs whose logical index i has ((i >> 2) & 7) < k, i.e.
4k of every 32 -- the same share of each shader engine under either mapping the runtime uses (bit i ->
SE i % 4, or 32 bits per XCD).  Off unless the environment asks for it:

  MAMBA_AMD_SIDE_CUS=k    weight-gradient side stream on k/8 of the CUs
  MAMBA_AMD_OTHER_CUS=k   the second micro-batch stream on k/8 of the CUs

Measured on one MI355X (profiles/r2_v7_cumask_ab.txt): every side-stream mask from 3/8 to 6/8 is 15-31 %
slower on the Mamba-2 280M step than the unrestricted stream, so both knobs stay off by default.
(The reference has no counterpart: it runs one CUDA stream under DDP, train.py:203-231.)
"""
import os
from typing import Dict, Optional, Tuple

import torch

_CACHE: Dict[Tuple[int, int], "torch.cuda.ExternalStream"] = {}


def mask_words(n_cus: int, eighths: int):
    """The CU mask (list of 32-bit words covering ``n_cus`` CUs) with ``eighths``/8 of them enabled."""
    if not 1 <= eighths <= 8:
        raise ValueError(f"eighths must be in 1..8, got {eighths}")
    words = []
    for w in range((n_cus + 31) // 32):
        v = 0
        for b in range(32):
            i = 32 * w + b
            if i < n_cus and ((i >> 2) & 7) < eighths:
                v |= 1 << b
        words.append(v)
    return words


def env_eighths(name: str) -> Optional[int]:
    v = os.environ.get(name, "").strip()
    if not v:
        return None
    k = int(v)
    return None if k >= 8 else k


def masked_stream(device: int, eighths: int) -> "torch.cuda.ExternalStream":
    """A cached stream on ``device`` restricted to ``eighths``/8 of the CUs (native, needs the extension)."""
    key = (device, eighths)
    s = _CACHE.get(key)
    if s is None:
        from ..ops import _ext
        n = torch.cuda.get_device_properties(device).multi_processor_count
        ptr = _ext.ops().cu_masked_stream(device, mask_words(n, eighths))
        s = torch.cuda.ExternalStream(ptr, device=torch.device("cuda", device))
        _CACHE[key] = s
    return s
