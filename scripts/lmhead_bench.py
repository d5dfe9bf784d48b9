"""lm_head GEMMs at the 280M training shape (32768 x 768 hidden, vocab 50304) with the tuned table, and
the fused lm_head + CE node end to end (native row-chunked engines vs hipBLASLt).   python scripts/lmhead_bench.py"""
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
    T, d, V = int(os.environ.get("LM_T", 65536)), 768, 50304
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
    # the row-chunked node's three products at one 16384-row chunk: native engines vs hipBLASLt
    R = 16384
    ops = torch.ops.mamba_amd
    hc, gc = h[:R], g[:R]
    Wt = W.t().contiguous()
    dwb = torch.zeros(1, V, d, device=dev)
    fc = 2 * R * d * V
    for name, fn in [("chunk fwd  pk", lambda: ops.gp_pk(hc, W)), ("chunk fwd  lib", lambda: torch.mm(hc, W.t())),
                     ("chunk dh   pk", lambda: ops.gp_pk(gc, Wt)), ("chunk dh   lib", lambda: torch.mm(gc, W)),
                     ("chunk dW   gp_mm+=", lambda: ops.gp_mm(gc, hc, dwb, 1, 1, 2, 1, 256)),
                     ("chunk dW   lib", lambda: torch.mm(gc.t(), hc))]:
        t = timeit(fn, 10)
        print(f"{name:20s} {t * 1e3:9.1f} us  {fc / t / 1e9:7.0f} TF/s", flush=True)
    Wp = (torch.randn(V, d, device=dev) * 0.02).requires_grad_(True)
    hh = h.clone().requires_grad_(True)
    tg = torch.randint(0, V, (T,), device=dev)

    def node():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = fused_linear_cross_entropy(hh, Wp, tg)
        loss.backward()
    import importlib
    ce = importlib.import_module("mamba_distributed_amd.ops.cross_entropy")
    for eng, cap, f32 in (("lib", 16384, True), ("lib", 32768, True), ("lib", 16384, False), ("native", 16384, True)):
        os.environ["MAMBA_AMD_LMHEAD"] = eng
        ce._ROW_CAP = cap
        ce._F32_OUT[0] = None if f32 else False
        node()
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        t = timeit(node, 5)
        peak = (torch.cuda.max_memory_allocated() - base) / 2**30
        print(f"fused lm_head+CE fwd+bwd [{eng} rows<={cap} dW-f32-out={ce._F32_OUT[0]}] {t * 1e3:9.1f} us"
              f"  ({3 * fl / t / 1e9:6.0f} TF/s over the 3 GEMMs)  transient peak {peak:.2f} GB", flush=True)

if __name__ == "__main__":
    main()
