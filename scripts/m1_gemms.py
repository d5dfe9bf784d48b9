"""Time every GEMM of one Mamba-1 280M layer (B=32, T=1024) in the exact call forms of
models/mamba1.py, with the shipped TunableOp table (isolated, HIP events, median of 20)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms  # noqa: E402


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    enable_tuned_gemms()
    dev, bf = "cuda", torch.bfloat16
    M, d, di, R, N = 32 * 1024, 768, 1536, 48, 16
    h2 = torch.randn(M, d, device=dev, dtype=bf)
    Win = torch.randn(2 * di, d, device=dev, dtype=bf)
    co2 = torch.randn(di, M, device=dev, dtype=bf)
    Wx = torch.randn(R + 2 * N, di, device=dev, dtype=bf)
    Wdt = torch.randn(di, R, device=dev, dtype=bf)
    xdbl = torch.randn(R + 2 * N, M, device=dev, dtype=bf)
    dd2 = torch.randn(di, M, device=dev, dtype=bf)
    dxdbl = torch.randn(R + 2 * N, M, device=dev, dtype=bf)
    y2 = torch.randn(di, M, device=dev, dtype=bf)
    Wout = torch.randn(d, di, device=dev, dtype=bf)
    dout = torch.randn(M, d, device=dev, dtype=bf)
    dxz = torch.randn(2 * di, M, device=dev, dtype=bf)
    rows = [
        ("in_proj fwd   xz = Win @ h2^T", lambda: torch.mm(Win, h2.t())),
        ("x_proj fwd    Wx @ co2", lambda: torch.mm(Wx, co2)),
        ("dt_proj fwd   Wdt @ xdbl[:R]", lambda: torch.mm(Wdt, xdbl[:R])),
        ("out_proj fwd  y2^T @ Wout^T", lambda: torch.nn.functional.linear(y2.t(), Wout)),
        ("out_proj dX   dout @ Wout", lambda: torch.mm(dout, Wout)),
        ("out_proj dW   dout^T @ y2^T", lambda: torch.mm(dout.t(), y2.t())),
        ("dWdt          dd2 @ xdbl[:R]^T", lambda: torch.mm(dd2, xdbl[:R].t())),
        ("dxdbl[:R]     Wdt^T @ dd2", lambda: torch.mm(Wdt.t(), dd2)),
        ("dWx           dxdbl @ co2^T", lambda: torch.mm(dxdbl, co2.t())),
        ("dco2 +=       Wx^T @ dxdbl", lambda: co2.clone().addmm_(Wx.t(), dxdbl)),
        ("in_proj dX    dxz^T @ Win", lambda: torch.mm(dxz.t(), Win)),
        ("in_proj dW    dxz @ h2", lambda: torch.mm(dxz, h2)),
    ]
    from mamba_distributed_amd.ops import _ext
    sk = _ext.ops().gemm_skinny
    WdtT, WxT = Wdt.t().contiguous(), Wx.t().contiguous()
    dco = co2.clone()
    rows += [
        ("native x_proj fwd", lambda: sk(Wx, co2, None, False)),
        ("native dt_proj fwd", lambda: sk(Wdt, xdbl[:R], None, False)),
        ("native dxdbl[:R]", lambda: sk(WdtT, dd2, None, False)),
        ("native dco2 +=", lambda: sk(WxT, dxdbl, dco, True)),
    ]
    tot = 0.0
    for name, fn in rows:
        us = t(fn)
        tot += us
        print(f"{name:34s} {us:8.1f} us", flush=True)
    print(f"{'total':34s} {tot:8.1f} us")


if __name__ == "__main__":
    main()
