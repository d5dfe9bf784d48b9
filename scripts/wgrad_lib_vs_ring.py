"""Weight-gradient products of the wide Mamba-2 models: the native staged ring (fp32 split-K slabs + fixed-order
reduce, the training path) vs hipBLASLt (torch.mm of the transposed token-major operands, bf16 output -- a lower
bound for the library, which would still need an fp32 result).  HIP events, tuned table on.

  python scripts/wgrad_lib_vs_ring.py [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402
from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms  # noqa: E402

SHAPES = {"in1.4b": (8512, 2048, 32768), "out1.4b": (2048, 4096, 32768),
          "in2.8b": (10576, 2560, 32768), "out2.8b": (2560, 5120, 32768), "in280": (3392, 768, 65536)}


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
    a = ap.parse_args()
    assert _ext.load(), _ext.error()
    print(json.dumps({"tuned_table": enable_tuned_gemms()}), flush=True)
    ops = _ext.ops()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (P, Q, T) in SHAPES.items():
        dy = (torch.randn(T, P, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
        x = (torch.randn(T, Q, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
        S = ops.gp_splits(P, Q, T)
        out = torch.empty(P, Q, device="cuda", dtype=torch.float32)

        def ring():
            part = ops.gp_mm(dy, x, None, 1, 1, 1, S, 256)
            ops.gp_reduce(part, out, False)

        t_ring = min(timeit(ring, a.reps) for _ in range(2))
        t_lib = min(timeit(lambda: torch.mm(dy.t(), x), a.reps) for _ in range(2))
        fl = 2.0 * P * Q * T
        print(json.dumps({"shape": name, "splits": S, "ring_us": round(t_ring, 1), "ring_tflops": round(fl / t_ring / 1e6),
                          "lib_bf16_us": round(t_lib, 1), "lib_tflops": round(fl / t_lib / 1e6)}), flush=True)
        del dy, x, out


if __name__ == "__main__":
    main()
