"""Forward / input-gradient projection products on the two native engines: the persistent engine (gp_pk,
gemm_pk_k) as KC . KC against a (N, K) weight image, and the staged ring (gp_mm, gemm_wg_k) as KC . XC against the
(K, N) image -- the same product, C = A B^T with B^T given k-major, so the weight-side operand is DMA'd in whole
128-B lines (only the token-major activation keeps 64-B stage rows).  Shapes: the Mamba-2 280M and 1.4B projections
at 64k / 32k tokens (padded in_proj width).  HIP events, interleaved rounds, one JSON line per shape.

  python scripts/fwd_engine_ab.py [--reps 10] [--rounds 3] [--only in_fwd280,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402

# name: (tokens, K, N)  C (tokens, N) = A (tokens, K) . W (N, K)^T
SHAPES = {
    "in_fwd280": (65536, 768, 3392), "out_fwd280": (65536, 1536, 768),
    "in_dgrad280": (65536, 3392, 768), "out_dgrad280": (65536, 768, 1536),
    "in_fwd1.4b": (32768, 2048, 8512), "out_fwd1.4b": (32768, 4096, 2048),
    "in_dgrad1.4b": (32768, 8512, 2048), "out_dgrad1.4b": (32768, 2048, 4096),
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
    a = ap.parse_args()
    assert _ext.load(), _ext.error()
    ops = _ext.ops()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (T, K, N) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        A = (torch.randn(T, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
        W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
        Wt = W.t().contiguous()
        c_pk = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        c_wg = torch.empty_like(c_pk)
        res = {"pk": [], "wg": []}
        for _ in range(a.rounds):
            res["pk"].append(timeit(lambda: ops.gp_pk(A, W, c_pk), a.reps))
            res["wg"].append(timeit(lambda: ops.gp_mm(A, Wt, c_wg, 0, 1, 0, 1, 256), a.reps))
        fl = 2.0 * T * K * N
        ref = A.float() @ W.float().t()
        out = {"shape": name, "T": T, "K": K, "N": N}
        for k, c in (("pk", c_pk), ("wg", c_wg)):
            t = min(res[k])
            out[f"{k}_us"] = round(t, 1)
            out[f"{k}_tflops"] = round(fl / t / 1e6, 1)
            out[f"{k}_rel"] = round(((c.float() - ref).norm() / ref.norm()).item(), 5)
        print(json.dumps(out), flush=True)
        del A, W, Wt, c_pk, c_wg, ref


if __name__ == "__main__":
    main()
