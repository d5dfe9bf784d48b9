"""Decode out_proj GEMV (ops.decode_outproj) time vs batch rows, Mamba-2 280M layer shapes (d_out 768, di 1536)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mamba_distributed_amd.ops import _ext  # noqa: E402

ops = _ext.ops()
dev = "cuda"
W = torch.randn(768, 1536, device=dev).to(torch.bfloat16)
for b in (1, 2, 4, 8, 16):
    g = torch.randn(b, 1536, device=dev).to(torch.bfloat16)
    part = torch.rand(b, 96, device=dev)
    out = torch.empty(b, 768, device=dev, dtype=torch.bfloat16)
    for _ in range(20):
        ops.decode_outproj(g, part, 1e-5, W, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        ops.decode_outproj(g, part, 1e-5, W, out)
    e1.record()
    torch.cuda.synchronize()
    print(f"decode_outproj b={b:2d}  {e0.elapsed_time(e1) / 200 * 1000:7.2f} us", flush=True)
