"""Per-phase cycle breakdown of the SSD forward walk and chunk backward (kernels/ssd.hip, STAMPS builds): wave 0 of
every workgroup sums s_memtime deltas per phase of its loop.  Prints mean cycles per chunk (forward) / per head
(chunk backward) for each phase, plus the un-stamped kernel times for reference.

  python scripts/ssd_stamps.py [--B 64]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402

FWD = ["top barrier", "LDS stage (+load wait)", "barrier 2", "y/S stores + prefetch", "Y_off MFMA",
       "CB mask + Y_diag", "D x + Y staging", "state update"]
BWD = ["top barrier", "LDS stage (+load wait)", "barrier 2 + prefetch", "(1)(2) dM/M", "(4)(6) BdS/Yoff",
       "barrier 3 + (3) dXdt", "(5)(7) dX/dB/dC", "(9) + dX store + flush"]


def ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--L", type=int, default=1024)
    ap.add_argument("--H", type=int, default=24, help="heads (24: Mamba-2 280M, 80: 2.8B)")
    a = ap.parse_args()
    assert _ext.load(), _ext.error()
    ops = torch.ops.mamba_amd
    dev = "cuda"
    B, L, H, P, N, G = a.B, a.L, a.H, 64, 128, 1
    di = H * P
    conv_dim = di + 2 * G * N
    torch.manual_seed(0)
    xc = torch.randn(B, L, conv_dim, device=dev).to(torch.bfloat16)
    x = xc[..., :di].unflatten(-1, (H, P))
    Bm = xc[..., di:di + N].unflatten(-1, (G, N))
    Cm = xc[..., di + N:].unflatten(-1, (G, N))
    dt = torch.randn(B, L, H, device=dev).to(torch.bfloat16)
    A = -torch.rand(H, device=dev) * 8 - 0.5
    D = torch.randn(H, device=dev)
    dtb = torch.randn(H, device=dev) * 0.3
    fwd = lambda: ops.ssd_fwd(x, dt, A, Bm, Cm, D, dtb, None, 64, True, 0.0, float("inf"))  # noqa: E731
    y, cum, dtp, states, fin = fwd()
    dy = torch.randn_like(y)
    bwd = lambda: ops.ssd_bwd(dy, x, dt, A, Bm, Cm, D, dtb, None, cum, dtp, states, None, 64, True, 0.0,  # noqa: E731
                              float("inf"), None, None, None, None)
    print(f"unstamped: ssd_fwd {ms(fwd):.3f} ms, ssd_bwd {ms(bwd):.3f} ms", flush=True)
    nc = (L + 63) // 64
    n_f = H * B
    # the chunk backward writes nc * nhg * B rows; nhg (head groups, pick_hg / MAMBA_AMD_SSD_HG) is at most H, so
    # size for that and read back the rows actually written (the kernels skip stamping when the buffer is short)
    n_b = nc * H * B
    buf = torch.full(((n_f + n_b) * 8,), -1, dtype=torch.int64, device=dev)
    ops.ssd_stamps(buf)
    t_f = ms(fwd, 1)
    t_b = ms(bwd, 1)
    ops.ssd_stamps(None)
    st = buf.view(-1, 8).double().cpu()
    f, b = st[:n_f], st[n_f:n_f + n_b]
    b = b[b[:, 0] >= 0]  # the rows of the nc * nhg * B workgroups that ran
    print(f"stamped: ssd_fwd {t_f:.3f} ms, ssd_bwd {t_b:.3f} ms (s_memtime ticks)")
    ftot = f.sum(1).mean().item()
    print(f"forward walk: {ftot / nc:.0f} ticks per chunk per workgroup ({nc} chunks)")
    for k, name in enumerate(FWD):
        v = f[:, k].mean().item() / nc
        print(f"  F{k} {name:28s} {v:8.0f}  {100 * v * nc / ftot:5.1f}%")
    hpw = H // max(1, b.shape[0] // (nc * B))  # heads per workgroup
    btot = b.sum(1).mean().item()
    print(f"chunk backward: {btot / hpw:.0f} ticks per head per workgroup ({hpw} heads)")
    for k, name in enumerate(BWD):
        v = b[:, k].mean().item() / hpw
        print(f"  B{k} {name:28s} {v:8.0f}  {100 * v * hpw / btot:5.1f}%")


if __name__ == "__main__":
    main()
