"""lm_head GEMMs at the 280M training shape (32768 x 768 hidden, vocab 50304) with the tuned table, and
the fused lm_head + CE node end to end.   python scripts/lmhead_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kbench import timeit  # noqa: E402  (scripts/ on sys.path when run from scripts/)


def main():
    from mamba_distributed_amd.ops import _ext
    from mamba_distributed_amd.ops.cross_entropy import fused_linear_cross_entropy
    from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
    assert _ext.load(), _ext.error()
    print("tuned:", enable_tuned_gemms())
    dev = "cuda"
    T, d, V = 32768, 768, 50304
    h = torch.randn(T, d, device=dev).to(torch.bfloat16)
    W = (torch.randn(V, d, device=dev) * 0.02).to(torch.bfloat16)
    g = torch.randn(T, V, device=dev).to(torch.bfloat16)
    fl = 2 * T * d * V
    for name, fn in [("fwd  h.W^T", lambda: torch.nn.functional.linear(h, W)),
                     ("fwd  mm(h, W.t())", lambda: torch.mm(h, W.t())),
                     ("dgrad g.W", lambda: torch.mm(g, W)),
                     ("wgrad g^T.h", lambda: torch.mm(g.t(), h))]:
        t = timeit(fn, 10)
        print(f"{name:20s} {t * 1e3:9.1f} us  {fl / t / 1e9:7.0f} TF/s", flush=True)
    Wp = (torch.randn(V, d, device=dev) * 0.02).requires_grad_(True)
    hh = h.clone().requires_grad_(True)
    tg = torch.randint(0, V, (T,), device=dev)

    def node():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = fused_linear_cross_entropy(hh, Wp, tg)
        loss.backward()
    t = timeit(node, 5)
    print(f"fused lm_head+CE fwd+bwd {t * 1e3:9.1f} us")


if __name__ == "__main__":
    main()
