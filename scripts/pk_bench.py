"""Persistent MFMA GEMM (gp_pk, kernels/gemm_pipe.hip::gemm_pk_k) against hipBLASLt (torch, shipped TunableOp
table) and the non-persistent engine (gp_mm) on the projection / lm_head forward and input-gradient shapes of
the 280M models (32768 tokens), HIP events, interleaved rounds.  Input gradients are KC . KC products against a
transposed weight copy (cached once per optimizer step in training).

  python scripts/pk_bench.py [--reps 20] [--rounds 3] [--only in_fwd,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402


def timeit(f, reps):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--only", default="")
    ap.add_argument("--no-wgrad", action="store_true")
    a = ap.parse_args()
    assert _ext.load(), _ext.error()
    from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
    print("tuned table:", enable_tuned_gemms(), flush=True)
    ops = torch.ops.mamba_amd
    dev = "cuda"
    M = a.M
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(torch.bfloat16)

    # (name, A (M,K), B (N,K)) : C = A B^T
    cases = []
    for name, K, N in (("in_fwd", 768, 3352), ("out_fwd", 1536, 768), ("in_dgrad", 3352, 768),
                       ("out_dgrad", 768, 1536), ("lm_fwd", 768, 50304), ("lm_dgrad", 50304, 768),
                       ("in_fwd_pad", 768, 3392), ("in_dgrad_pad", 3392, 768), ("odd", 200, 200), ("odd2", 328, 1000)):
        if a.only and name not in a.only.split(","):
            continue
        m = 1000 if name.startswith("odd") else M
        cases.append((name, rnd(m, K), rnd(N, K, scale=0.05)))
    for name, A, B in cases:
        m, K = A.shape
        N = B.shape[0]
        fl = 2.0 * m * N * K
        ref = torch.nn.functional.linear(A, B)
        if name == "lm_dgrad" and m * K * 2 >= (1 << 32):  # operand past the engine's 4 GB offset range
            print(json.dumps({"case": name, "M": m, "skipped": "operand >= 4 GB"}), flush=True)
            continue
        rs = torch.rand(m, device=dev, generator=g) + 0.5
        res = {"case": name, "M": m, "N": N, "K": K}
        err = rel(ops.gp_pk(A, B), ref)
        # row scale (the gated-norm rstd folded out of the out_proj operand)
        err_rs = rel(ops.gp_pk(A, B, None, 0, 0, 0, rs), ref.float() * rs[:, None])
        res["rel_err"], res["rel_err_rowscale"] = float(f"{err:.2e}"), float(f"{err_rs:.2e}")
        if not name.startswith("odd") and not (name == "lm_dgrad" and m * K * 2 >= (1 << 32)):
            t = {"pk": [], "lib": [], "gp_mm": []}
            for _ in range(a.rounds):
                t["pk"].append(timeit(lambda: ops.gp_pk(A, B), a.reps))
                t["lib"].append(timeit(lambda: torch.nn.functional.linear(A, B), a.reps))
                # the non-persistent engines: the staged ring (gemm_wg_k, default) and gemm_pipe_k (nb 0)
                t["gp_mm"].append(timeit(lambda: ops.gp_mm(A, B, None, 0, 0, 0, 1, 256), a.reps))
                ops.gp_wg_nb(0)
                t.setdefault("gp_pipe", []).append(timeit(lambda: ops.gp_mm(A, B, None, 0, 0, 0, 1, 256), a.reps))
                ops.gp_wg_nb(4)
            for k, v in t.items():
                if v:
                    res[k + "_us"] = round(min(v), 1)
                    res[k + "_tflops"] = round(fl / min(v) / 1e6, 1)
        if name in ("in_fwd", "in_fwd_pad", "out_fwd") and not a.no_wgrad:
            # weight gradient of the same projection: dW (N, K) = dY^T X, both token-major (XC . XC split-K slabs)
            dY = rnd(m, N)
            S = ops.gp_splits(N, K, m)
            ref_w = dY.float().t() @ A.float()
            tw, tw4 = [], []
            for w in (8, 4):  # the split-K engine as 8 waves (shipped) and 4 waves (one per SIMD)
                ops.gp_waves(w)
                part = ops.gp_mm(dY, A, None, 1, 1, 1, S, 256)
                res[f"wgrad_err_w{w}"] = float(f"{rel(part.sum(0), ref_w):.2e}")
            for _ in range(a.rounds):
                ops.gp_waves(8)
                tw.append(timeit(lambda: ops.gp_mm(dY, A, None, 1, 1, 1, S, 256), a.reps))
                ops.gp_waves(4)
                tw4.append(timeit(lambda: ops.gp_mm(dY, A, None, 1, 1, 1, S, 256), a.reps))
            ops.gp_waves(8)
            res["wgrad_us"] = round(min(tw), 1)
            res["wgrad_tflops"] = round(fl / min(tw) / 1e6, 1)
            res["wgrad4_us"] = round(min(tw4), 1)
            res["wgrad_splits"] = S
        print(json.dumps(res), flush=True)
        assert err < 1e-2 and err_rs < 1e-2, res


if __name__ == "__main__":
    main()
