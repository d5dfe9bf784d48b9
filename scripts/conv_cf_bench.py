"""Channel-first causal conv (Mamba-1 conv1d, kernels/conv1d.hip conv_cf_*) at the Mamba-1 280M / 370M layer shapes:
forward and backward microseconds (HIP events) and effective HBM bandwidth, plus a check against the fp32 reference.

  python scripts/conv_cf_bench.py [--reps 20] [--orders 0,1]   (conv_cf_order knob values, interleaved)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402
from mamba_distributed_amd.ops.reference import causal_conv1d_ref  # noqa: E402


def timeit(fn, reps):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--orders", default="")
    a = ap.parse_args()
    assert _ext.load(), _ext.error()
    ops = _ext.ops()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (b, d, L) in {"m1_280m": (64, 1536, 1024), "m1_370m": (64, 2048, 1024)}.items():
        xm = torch.randn(d, b, L, device="cuda", generator=g).to(torch.bfloat16)
        x = xm.permute(1, 0, 2)  # logical (b, d, l), channel-major memory as in models/mamba1.py
        w = torch.randn(d, 4, device="cuda", generator=g) * 0.5
        bias = torch.randn(d, device="cuda", generator=g) * 0.1
        go = torch.randn(d, b, L, device="cuda", generator=g).to(torch.bfloat16).permute(1, 0, 2)
        dxm = torch.empty(d, b, L, device="cuda", dtype=torch.bfloat16)
        dx = dxm.permute(1, 0, 2)
        y = ops.conv1d_cf_fwd(x, w, bias, True)
        ref = causal_conv1d_ref(x.float(), w, bias, "silu")
        rel = ((y.float() - ref).norm() / ref.norm()).item()
        knobs = [int(v) for v in a.orders.split(",")] if a.orders else [ops.conv_cf_order(-1)]
        for rep in range(2 if a.orders else 1):
            for kv in knobs:
                ops.conv_cf_order(kv)
                t_f = timeit(lambda: ops.conv1d_cf_fwd(x, w, bias, True), a.reps)
                t_b = timeit(lambda: ops.conv1d_cf_bwd(x, w, bias, go, True, dx), a.reps)
                nb = x.numel() * 2
                print(json.dumps({"shape": name, "order": kv, "fwd_us": round(t_f, 1),
                                  "fwd_TBs": round(2 * nb / t_f / 1e6, 2), "bwd_us": round(t_b, 1),
                                  "bwd_TBs": round(3 * nb / t_b / 1e6, 2), "fwd_rel": round(rel, 5)}), flush=True)


if __name__ == "__main__":
    main()
