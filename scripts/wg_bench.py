"""Weight-gradient GEMM engines A/B: dW = dY^T X as XC . XC fp32 split-K slabs (ops.gp_mm, both operands token-major)
on gemm_pipe_k (nb 0) and on gemm_wg_k with a 4- or 5-slot ring of 32-deep stages (nb 4 / 5), at the projection
shapes of the Mamba-2 models (csrc/kernels/gemm_pipe.hip).  Interleaved rounds in one process, HIP events, random
operands; one JSON line per shape with us, TF/s and the split count.

  python scripts/wg_bench.py [--reps 10] [--rounds 3] [--only in280,out280] [--nb 0,4,5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402

# name: (P = dY width, Q = X width, tokens)
SHAPES = {
    "in280": (3392, 768, 65536), "out280": (768, 1536, 65536),
    "lmdw": (50304, 768, 16384),
    "in1.4b": (8512, 2048, 32768), "out1.4b": (2048, 4096, 32768),
    "in2.8b": (10576, 2560, 32768), "out2.8b": (2560, 5120, 32768),
}


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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--nb", default="0,4,5")
    a = ap.parse_args()
    assert _ext.load(), _ext.error()
    ops = _ext.ops()
    nbs = [int(v) for v in a.nb.split(",")]
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (P, Q, T) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        dY = (torch.randn(T, P, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
        X = (torch.randn(T, Q, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
        S = ops.gp_splits(P, Q, T)
        part = torch.empty(S, P, Q, device="cuda")
        res = {nb: [] for nb in nbs}
        outs = {}
        for _ in range(a.rounds):
            for nb in nbs:
                ops.gp_wg_nb(nb)
                res[nb].append(timeit(lambda: ops.gp_mm(dY, X, part, 1, 1, 1, S, 256), a.reps))
                outs[nb] = part.clone()
        ops.gp_wg_nb(0)
        fl = 2.0 * P * Q * T
        out = {"shape": name, "P": P, "Q": Q, "T": T, "splits": S}
        for nb in nbs:
            t = min(res[nb])
            out[f"nb{nb}_us"] = round(t, 1)
            out[f"nb{nb}_tflops"] = round(fl / t / 1e6, 1)
            out[f"nb{nb}_equal_nb{nbs[0]}"] = bool(torch.equal(outs[nb], outs[nbs[0]]))
        print(json.dumps(out), flush=True)
        del dY, X, part, outs


if __name__ == "__main__":
    main()
