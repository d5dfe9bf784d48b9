"""Wide short-K streaming GEMMs of the Mamba-1 280M layer (kernels/gemm.hip gemm_skinny_k): the delta product
(W_dt 1536 x 48 . x_dbl[:48], write-only 201 MB) and dconv += W_x^T dx_dbl (1536 x 80, read + write 201 MB each).
  python scripts/skinny_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402


def timeit(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    assert _ext.load(), _ext.error()
    ops = _ext.ops()
    M = 65536
    g = torch.Generator(device="cuda").manual_seed(0)
    wdt = (torch.randn(1536, 48, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    xd = torch.randn(80, M, device="cuda", generator=g).to(torch.bfloat16)
    wxt = (torch.randn(80, 1536, device="cuda", generator=g) * 0.1).to(torch.bfloat16).t().contiguous()
    out = torch.empty(1536, M, device="cuda", dtype=torch.bfloat16)
    y = ops.gemm_skinny(wdt, xd[:48], None, False)
    ref = wdt.float() @ xd[:48].float()
    rel = ((y.float() - ref).norm() / ref.norm()).item()
    t1 = timeit(lambda: ops.gemm_skinny(wdt, xd[:48], out, False))
    t2 = timeit(lambda: ops.gemm_skinny(wxt, xd, out, True))
    nb = 1536 * M * 2
    print(json.dumps({"delta_us": round(t1, 1),
                      "delta_TBs": round(nb / t1 / 1e6, 2), "dconv_acc_us": round(t2, 1),
                      "dconv_TBs": round(2 * nb / t2 / 1e6, 2), "rel": round(rel, 5)}), flush=True)


if __name__ == "__main__":
    main()
