"""Segment-parallel SSD walks: time the native ssd_fwd / ssd_bwd ops per segment count (kernels/ssd.hip).

Usage: python scripts/ssd_seg_bench.py [--shapes 2p8b,280m,prefill] [--segs 1,2,4,8,16] [--reps 10]
Prints one line per (shape, segments) with the forward and backward op times (cumsum + walks + combine for the
forward; segment pass + reverse walk + chunk backward for the backward) and the automatic choice.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402

SHAPES = {"2p8b": (4, 8192, 80), "1p4b": (32, 1024, 48), "280m": (64, 1024, 24), "prefill": (1, 32768, 24)}


def inputs(b, L, H, N=128, G=1):
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g, device="cuda")  # noqa: E731
    x = r(b, L, H, 64).to(torch.bfloat16)
    Bm = (r(b, L, G, N) * 0.5).to(torch.bfloat16)
    Cm = (r(b, L, G, N) * 0.5).to(torch.bfloat16)
    dt = (r(b, L, H) * 0.5 - 1.0).to(torch.bfloat16)
    A = -torch.rand(H, generator=g, device="cuda") * 8 - 0.5
    D = r(H)
    bias = r(H) * 0.3
    dy = r(b, L, H, 64).to(torch.bfloat16)
    return x, dt, A, Bm, Cm, D, bias, dy


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="2p8b,280m,prefill")
    ap.add_argument("--segs", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    assert _ext.load(), _ext.error()
    ops = _ext.ops()
    for name in args.shapes.split(","):
        b, L, H = SHAPES[name]
        nc = (L + 63) // 64
        x, dt, A, Bm, Cm, D, bias, dy = inputs(b, L, H)
        ops.ssd_segments(0, 1, 1, 1)
        auto = int(ops.ssd_segments(-1, b, H, nc))
        ref = None
        for s in [int(v) for v in args.segs.split(",")]:
            got = int(ops.ssd_segments(s, b, H, nc))
            fwd = lambda: ops.ssd_fwd(x, dt, A, Bm, Cm, D, bias, None, 64, True, 0.0, float("inf"))  # noqa: E731
            y, cum, dtp, states, fin = fwd()
            bwd = lambda: ops.ssd_bwd(dy, x, dt, A, Bm, Cm, D, bias, None, cum, dtp, states, None, 64, True, 0.0,  # noqa: E731
                                      float("inf"), None, None, None, None)
            tf = timed(fwd, args.reps)
            tb = timed(bwd, args.reps)
            g = bwd()
            if ref is None:
                ref = (y.float(), fin, [t.float() for t in g[:5]])
                err = 0.0
            else:
                rel = lambda a, c: ((a - c).norm() / (c.norm() + 1e-12)).item()  # noqa: E731
                err = max([rel(y.float(), ref[0]), rel(fin, ref[1])] + [rel(a.float(), c) for a, c in zip(g[:5], ref[2])])
            print(f"{name} b={b} L={L} H={H} segs={got}{' (auto)' if got == auto else ''}: fwd {tf:8.1f} us  "
                  f"bwd {tb:8.1f} us  max rel diff vs first {err:.2e}", flush=True)
        ops.ssd_segments(0, 1, 1, 1)


if __name__ == "__main__":
    main()
