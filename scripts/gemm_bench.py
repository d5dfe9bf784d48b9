"""A/B of the projection GEMMs at the Mamba-2 280M micro-batch shape (32 x 1024 tokens): the pipelined
native engine (ops.gp_mm, csrc/kernels/gemm_pipe.hip) vs hipBLASLt with the pinned TunableOp table (what
the training step used before) and the previous native weight-gradient kernel.  Interleaved rounds in one
process (cdna_hip_programming.md §5.4 rule 24), random operands; prints one JSON line per product.

  python scripts/gemm_bench.py [--reps 30] [--rounds 3] [--T 32768]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps):
    fn(); fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record(); fn(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=30)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--T", type=int, default=32768)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--dp", type=int, default=3352)
    p.add_argument("--di", type=int, default=1536)
    p.add_argument("--only", default="")
    p.add_argument("--sweep", action="store_true", help="K sweep at M=32768, N=4096 (8 full tile rounds)")
    p.add_argument("--ablate", action="store_true", help="diagnostic ablations of the native kernel (garbage out)")
    a = p.parse_args()
    from mamba_distributed_amd.ops import _ext
    from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
    assert _ext.load(), _ext.error()
    enable_tuned_gemms()
    ops = _ext.ops()
    dev = "cuda"
    T, d, dp, di = a.T, a.d, a.dp, a.di
    g = torch.Generator(device=dev).manual_seed(0)
    if a.ablate:
        for K in (768, 3072):
            A = (torch.randn(T, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            B = (torch.randn(4096, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            out = {"K": K}
            for bits, name in ((0, "full"), (1, "no_vmwait"), (2, "no_dma"), (4, "no_barrier"), (8, "no_epi"),
                               (5, "no_wait_no_bar"), (6, "no_dma_no_bar"), (14, "mfma_lds_only")):
                ops.gp_set_ablate(bits)
                out[name + "_us"] = round(timeit(lambda: ops.gp_mm(A, B, None, 0, 0, 0, 1, 256), a.reps)[0], 1)
            ops.gp_set_ablate(0)
            print(json.dumps(out), flush=True)
        return
    if a.sweep:
        for K in (128, 256, 512, 768, 1536, 3072):
            A = (torch.randn(T, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            B = (torch.randn(4096, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            r = {}
            for _ in range(a.rounds):
                for k, fn in {"lib": lambda: torch.nn.functional.linear(A, B),
                              "gp": lambda: ops.gp_mm(A, B, None, 0, 0, 0, 1, 256)}.items():
                    r.setdefault(k, []).append(timeit(fn, a.reps)[0])
            out = {"K": K, "flop": 2 * T * 4096 * K}
            for k, v in r.items():
                out[k + "_us"] = round(sorted(v)[len(v) // 2], 1)
                out[k + "_tflops"] = round(out["flop"] / out[k + "_us"] / 1e6, 1)
            print(json.dumps(out), flush=True)
        return
    rnd = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.5).to(torch.bfloat16)  # noqa: E731
    x, zx, W_in, y, dout, W_out = rnd(T, d), rnd(T, dp), rnd(dp, d), rnd(T, di), rnd(T, d), rnd(d, di)
    cases = {
        # name: (flop, {arm: fn})
        "in_fwd": (2 * T * d * dp, {"lib": lambda: torch.nn.functional.linear(x, W_in),
                                    "gp": lambda: ops.gp_mm(x, W_in, None, 0, 0, 0, 1, 256),
                                    "gp4w": lambda: ops.gp_mm(x, W_in, None, 0, 0, 0, 1, 1256)}),
        "in_dgrad": (2 * T * d * dp, {"lib": lambda: torch.mm(zx, W_in),
                                      "gp": lambda: ops.gp_mm(zx, W_in, None, 0, 1, 0, 1, 256),
                                      "gp128": lambda: ops.gp_mm(zx, W_in, None, 0, 1, 0, 1, 128)}),
        "out_fwd": (2 * T * d * di, {"lib": lambda: torch.nn.functional.linear(y, W_out),
                                     "gp": lambda: ops.gp_mm(y, W_out, None, 0, 0, 0, 1, 256),
                                     "gp128": lambda: ops.gp_mm(y, W_out, None, 0, 0, 0, 1, 128),
                                     "gp4w": lambda: ops.gp_mm(y, W_out, None, 0, 0, 0, 1, 1256)}),
        "out_dgrad": (2 * T * d * di, {"lib": lambda: torch.mm(dout, W_out),
                                       "gp": lambda: ops.gp_mm(dout, W_out, None, 0, 1, 0, 1, 256)}),
    }
    gin = torch.zeros(dp, d, device=dev)
    gout = torch.zeros(d, di, device=dev)
    S_in, S_out = ops.gp_splits(dp, d, T), ops.gp_splits(d, di, T)
    part_in = torch.empty(S_in, dp, d, device=dev)
    part_out = torch.empty(S_out, d, di, device=dev)

    def gp_w(A, B, part, out):
        ops.gp_mm(A, B, part, 1, 1, 1, part.shape[0], 256)
        ops.gp_reduce(part, out, True)

    cases["in_wgrad"] = (2 * T * d * dp, {"old_native": lambda: ops.gemm_wgrad(zx, x, gin, True),
                                          "lib": lambda: torch.mm(zx.t(), x),
                                          "gp_slab_only": lambda: ops.gp_mm(zx, x, part_in, 1, 1, 1, S_in, 256),
                                          "gp+reduce": lambda: gp_w(zx, x, part_in, gin)})
    cases["out_wgrad"] = (2 * T * d * di, {"old_native": lambda: ops.gemm_wgrad(dout, y, gout, True),
                                           "lib": lambda: torch.mm(dout.t(), y),
                                           "gp_slab_only": lambda: ops.gp_mm(dout, y, part_out, 1, 1, 1, S_out, 256),
                                           "gp+reduce": lambda: gp_w(dout, y, part_out, gout)})
    only = set(a.only.split(",")) if a.only else None
    for name, (flop, arms) in cases.items():
        if only and name not in only:
            continue
        res = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                res[k].append(timeit(fn, a.reps)[0])
        out = {"case": name, "flop": flop}
        for k, v in res.items():
            med = sorted(v)[len(v) // 2]
            out[k + "_us"] = round(med, 1)
            out[k + "_tflops"] = round(flop / med / 1e6, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
