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


def m1_cases(T=65536, d=768, di=1536, R=48, N=16):
    """The gp_mm products of one Mamba-1 280M layer (models/mamba1.py, ops/linear.py), as (name, A, B, la, lb, mode,
    splits, bm, flop).  Channel-major activations are (features, tokens)."""
    g = torch.Generator(device="cuda").manual_seed(1)
    rnd = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(torch.bfloat16)  # noqa: E731
    dxz, w_in, h2 = rnd(2 * di, T), rnd(2 * di, d), rnd(T, d)
    wx, co2, wdt, dd2 = rnd(R + 2 * N, di), rnd(di, T), rnd(di, R), rnd(di, T)
    y2, w_out, dout = rnd(di, T), rnd(d, di), rnd(T, d)
    dxdbl = rnd(R + 2 * N, T)
    return [
        ("m1_in_dgrad XC.XC bf16", dxz, w_in, 1, 1, 0, 1, 256, 2.0 * T * d * 2 * di),
        ("m1_x_proj KC.XC 128-row", wx, co2, 0, 1, 0, 1, 128, 2.0 * T * di * (R + 2 * N)),
        ("m1_dxdbl XC.XC 128-row", wdt, dd2, 1, 1, 0, 1, 128, 2.0 * T * di * R),
        ("m1_out_fwd XC.KC bf16", y2, w_out, 1, 0, 0, 1, 256, 2.0 * T * di * d),
        ("m1_out_wgrad XC.KC slabs", dout, y2, 1, 0, 1, 0, 256, 2.0 * T * di * d),
        ("m1_in_wgrad KC.XC slabs", dxz, h2, 0, 1, 1, 0, 256, 2.0 * T * d * 2 * di),
        ("m1_in_wgrad^T XC.KC slabs (768 x 3072)", h2, dxz, 1, 0, 1, 0, 256, 2.0 * T * d * 2 * di),
        ("m1_in_wgrad XC.XC slabs (dxz token-major copy)", dxz.t().contiguous(), h2, 1, 1, 1, 0, 256,
         2.0 * T * d * 2 * di),
        ("m1_out_wgrad XC.XC slabs (y2 token-major copy)", dout, y2.t().contiguous(), 1, 1, 1, 0, 256,
         2.0 * T * di * d),
        ("m1_out_fwd KC.KC bf16 (y2 token-major copy)", y2.t().contiguous(), w_out, 0, 0, 0, 1, 256, 2.0 * T * di * d),
        ("m1_x_wgrad KC.KC slabs", dxdbl, co2, 0, 0, 1, 0, 256, 2.0 * T * di * (R + 2 * N)),
        ("m1_x_wgrad KC.KC slabs 128-row", dxdbl, co2, 0, 0, 1, 0, 128, 2.0 * T * di * (R + 2 * N)),
        ("m1_dt_wgrad KC.KC slabs (1536 x 48)", dd2, dxdbl[:R], 0, 0, 1, 0, 256, 2.0 * T * di * R),
        ("m1_dt_wgrad^T KC.KC slabs 128-row (48 x 1536)", dxdbl[:R], dd2, 0, 0, 1, 0, 128, 2.0 * T * di * R),
    ]


def run_m1_kp(a, ops, kps):
    """The Mamba-1 cases on the staged-ring engine with the KC operand images paired (kp 1, gemm_wg_kp_k) or not."""
    for name, A, B, la, lb, mode, S, bm, fl in m1_cases():
        if la == 1 and lb == 1 or (la == 0 and lb == 0 and mode == 0):
            continue
        M = A.shape[0] if la == 0 else A.shape[1]
        N = B.shape[0] if lb == 0 else B.shape[1]
        K = A.shape[1] if la == 0 else A.shape[0]
        if S == 0:
            S = ops.gp_splits(M, N, K)
        out = torch.empty(S, M, N, device="cuda") if mode else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        res = {kp: [] for kp in kps}
        outs = {}
        for _ in range(a.rounds):
            for kp in kps:
                ops.gp_wg_kcpair(kp)  # 0 off, 1 default rule, 2 every KC operand
                res[kp].append(timeit(lambda: ops.gp_mm(A, B, out, la, lb, mode, S, bm), a.reps))
                outs[kp] = out.clone()
        ops.gp_wg_kcpair(1)
        r = {"case": name, "M": M, "N": N, "K": K, "splits": S}
        for kp in kps:
            t = min(res[kp])
            r[f"kp{kp}_us"] = round(t, 1)
            r[f"kp{kp}_tflops"] = round(fl / t / 1e6, 1)
            r[f"kp{kp}_equal_kp{kps[0]}"] = bool(torch.equal(outs[kp], outs[kps[0]]))
        print(json.dumps(r), flush=True)


def run_m1(a, ops, nbs):
    for name, A, B, la, lb, mode, S, bm, fl in m1_cases():
        M = A.shape[0] if la == 0 else A.shape[1]
        N = B.shape[0] if lb == 0 else B.shape[1]
        K = A.shape[1] if la == 0 else A.shape[0]
        if S == 0:
            S = ops.gp_splits(M, N, K)
        out = torch.empty(S, M, N, device="cuda") if mode else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        res = {nb: [] for nb in nbs}
        outs = {}
        for _ in range(a.rounds):
            for nb in nbs:
                ops.gp_wg_nb(nb)
                res[nb].append(timeit(lambda: ops.gp_mm(A, B, out, la, lb, mode, S, bm), a.reps))
                outs[nb] = out.clone()
        ops.gp_wg_nb(4)
        r = {"case": name, "M": M, "N": N, "K": K, "splits": S}
        for nb in nbs:
            t = min(res[nb])
            r[f"nb{nb}_us"] = round(t, 1)
            r[f"nb{nb}_tflops"] = round(fl / t / 1e6, 1)
            r[f"nb{nb}_equal_nb{nbs[0]}"] = bool(torch.equal(outs[nb], outs[nbs[0]]))
        print(json.dumps(r), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--nb", default="0,4")
    ap.add_argument("--m1", action="store_true", help="the Mamba-1 layer's gp_mm products instead")
    ap.add_argument("--kp", default="", help="with --m1: compare KC image modes (0 off, 1 default rule, 2 all), e.g. 0,2")
    a = ap.parse_args()
    assert _ext.load(), _ext.error()
    ops = _ext.ops()
    nbs = [int(v) for v in a.nb.split(",")]
    if a.m1 and a.kp:
        run_m1_kp(a, ops, [int(v) for v in a.kp.split(",")])
        return
    if a.m1:
        run_m1(a, ops, nbs)
        return
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
        ops.gp_wg_nb(4)
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
