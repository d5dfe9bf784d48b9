"""In/out-projection GEMMs of the Mamba-2 280M layer (32768 tokens): hipBLASLt (torch, TunableOp table
as shipped) vs the native pipelined MFMA GEMM (gp_mm), forward and dgrad, HIP events.

  python scripts/proj_gemm_bench.py [--reps 30]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402


def timeit(f, reps):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--M", type=int, default=32768)
    a = ap.parse_args()
    assert _ext.load(), _ext.error()
    from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
    print("tuned table:", enable_tuned_gemms())
    ops = torch.ops.mamba_amd
    dev = "cuda"
    M = a.M
    for name, K, N in (("in_proj", 768, 3352), ("out_proj", 1536, 768)):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        ref = torch.nn.functional.linear(x, w)
        for bm in (256, 192, 128):
            try:
                y = ops.gp_mm(x, w, None, 0, 0, 0, 1, bm)
            except RuntimeError as e:
                print(f"{name} fwd gp_mm bm={bm}: {e}")
                continue
            err = ((y.float() - ref.float()).norm() / ref.float().norm()).item()
            t = timeit(lambda: ops.gp_mm(x, w, None, 0, 0, 0, 1, bm), a.reps)
            print(f"{name:8s} fwd   gp_mm bm={bm:4d} {t:8.1f} us {fl / t / 1e6:7.1f} TF/s  rel_err {err:.1e}")
        t = timeit(lambda: torch.nn.functional.linear(x, w), a.reps)
        print(f"{name:8s} fwd   hipBLASLt      {t:8.1f} us {fl / t / 1e6:7.1f} TF/s")
        refd = dy @ w
        wT = w.t().contiguous()  # (in, out): dgrad as a KC.KC product (a per-step cached transpose)
        for bm in (192, 256):
            d = ops.gp_mm(dy, wT, None, 0, 0, 0, 1, bm)
            err = ((d.float() - refd.float()).norm() / refd.float().norm()).item()
            t = timeit(lambda: ops.gp_mm(dy, wT, None, 0, 0, 0, 1, bm), a.reps)
            print(f"{name:8s} dgrad gp_mm(W^T KC) bm={bm:4d} {t:8.1f} us {fl / t / 1e6:7.1f} TF/s  rel_err {err:.1e}")
        for bm in (256, 128):
            try:
                d = ops.gp_mm(dy, w, None, 0, 1, 0, 1, bm)
            except RuntimeError as e:
                print(f"{name} dgrad gp_mm bm={bm}: {e}")
                continue
            err = ((d.float() - refd.float()).norm() / refd.float().norm()).item()
            t = timeit(lambda: ops.gp_mm(dy, w, None, 0, 1, 0, 1, bm), a.reps)
            print(f"{name:8s} dgrad gp_mm bm={bm:4d} {t:8.1f} us {fl / t / 1e6:7.1f} TF/s  rel_err {err:.1e}")
        t = timeit(lambda: dy @ w, a.reps)
        print(f"{name:8s} dgrad hipBLASLt      {t:8.1f} us {fl / t / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    main()
