"""launch_colsum timing at the backward's partial shapes (norm weights, gated norm, conv taps, SSD sums), HIP events,
us per column sum (profiles/r5/colsum_single_launch_rejected.txt compared a single-launch form against it)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.error()
ops = _ext.ops()
res = {}
for rows, cols in [(2048, 768), (2048, 1536), (512, 8960), (1024, 72)]:
    parts = [torch.randn(rows, cols, device="cuda") for _ in range(8)]
    for p in parts:
        ops.colsum(p)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(25):
        for p in parts:
            ops.colsum(p)
    e.record()
    torch.cuda.synchronize()
    res[f"{rows}x{cols}_us"] = round(s.elapsed_time(e) * 1e3 / 200, 2)
print(json.dumps(res))
