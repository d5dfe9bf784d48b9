"""Mamba-1 selective-scan forward walk (selscan_fwd_sg_k) at the 280M / 370M layer shapes, channel-major buffers
as in models/mamba1.py: microseconds per call (HIP events).
  python scripts/selscan_fwd_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402


def main():
    assert _ext.load(), _ext.error()
    ops = torch.ops.mamba_amd
    b, L, n = 64, 1024, 16
    for name, d in (("m1_280m", 1536), ("m1_370m", 2048)):
        cm = lambda t2: t2.view(t2.shape[0], b, L).permute(1, 0, 2)  # noqa: E731
        g = torch.Generator(device="cuda").manual_seed(0)
        u = cm(torch.randn(d, b * L, device="cuda", generator=g).to(torch.bfloat16))
        z = cm(torch.randn(d, b * L, device="cuda", generator=g).to(torch.bfloat16))
        delta = cm((torch.randn(d, b * L, device="cuda", generator=g) * 0.5 - 1).to(torch.bfloat16))
        xd = torch.randn(2 * n, b * L, device="cuda", generator=g).to(torch.bfloat16)
        Bm, Cm = cm(xd[:n]).unsqueeze(1), cm(xd[n:]).unsqueeze(1)
        A = -torch.rand(d, n, device="cuda") * 4 - 0.1
        D = torch.randn(d, device="cuda")
        db = torch.randn(d, device="cuda") * 0.3
        f = lambda: ops.selscan_fwd(u, delta, A, Bm, Cm, D, z, db, True)  # noqa: E731
        f()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                f()
            e.record()
            torch.cuda.synchronize()
            best = min(best, s.elapsed_time(e) * 100)
        print(json.dumps({"shape": name, "fwd_us": round(best, 1)}), flush=True)


if __name__ == "__main__":
    main()
