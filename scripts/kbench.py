"""Microbenchmarks of the hot native ops at the headline shape (Mamba-2 280M micro-batch:
B=32, L=1024, d_model=768 -> H=24, P=64, N=128, conv_dim=1792).  Times fwd and bwd of each op with
HIP events (median of N reps after warmup) and prints achieved bytes/s where meaningful.

  python scripts/kbench.py [--only ssd,conv,norm,gnorm,ce,selscan] [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--only", default="ssd,conv,norm,gnorm,ce,selscan,gemm")
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--B", type=int, default=32)
    p.add_argument("--L", type=int, default=1024)
    a = p.parse_args()
    only = set(a.only.split(","))
    from mamba_distributed_amd.ops import _ext
    from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
    assert _ext.load(), _ext.error()
    enable_tuned_gemms()  # library GEMMs with the same pinned solutions as training
    ops = torch.ops.mamba_amd
    dev = "cuda"
    B, L, H, P, N, G = a.B, a.L, 24, 64, 128, 1
    di = H * P
    dproj = 2 * di + 2 * G * N + H
    conv_dim = di + 2 * G * N
    torch.manual_seed(0)
    zx = torch.randn(B, L, dproj, device=dev).to(torch.bfloat16)
    res = {}
    if "conv" in only:
        xBC = zx[..., di:di + conv_dim]
        w = torch.randn(conv_dim, 4, device=dev) * 0.3
        bias = torch.randn(conv_dim, device=dev)
        out = ops.conv1d_cl_fwd(xBC, w, bias, True)
        g = torch.randn_like(out)
        t = timeit(lambda: ops.conv1d_cl_fwd(xBC, w, bias, True), a.reps)
        res["conv_cl_fwd"] = (t, 2 * out.numel() * 2)
        t = timeit(lambda: ops.conv1d_cl_bwd(xBC, w, bias, g, True, None), a.reps)
        res["conv_cl_bwd"] = (t, 3 * out.numel() * 2)
    if "gemm" in only:
        import torch.nn.functional as F
        for (M, Nn, K, tag) in [(B * L, dproj, 768, "in_proj"), (B * L, 768, di, "out_proj")]:
            A = torch.randn(M, K, device=dev).to(torch.bfloat16)
            W = torch.randn(Nn, K, device=dev).to(torch.bfloat16)
            t = timeit(lambda: F.linear(A, W), a.reps)
            res[f"gemm_{tag}_hipblaslt"] = (t, 0)
            print(f"{tag}: hipBLASLt {2 * M * Nn * K / t / 1e9:.0f} TF/s", flush=True)
            t = timeit(lambda: ops.gemm_tn(A, W, None), a.reps)
            res[f"gemm_{tag}_native"] = (t, 0)
            print(f"{tag}: native    {2 * M * Nn * K / t / 1e9:.0f} TF/s", flush=True)
            # weight gradient dW (N, K) = dY^T (N, M) . X (M, K)
            dY = torch.randn(M, Nn, device=dev).to(torch.bfloat16)
            t = timeit(lambda: torch.mm(dY.t(), A).float(), a.reps)
            res[f"wgrad_{tag}_hipblaslt"] = (t, 0)
            print(f"{tag} wgrad: hipBLASLt(+fp32 cast) {2 * M * Nn * K / t / 1e9:.0f} TF/s", flush=True)
            t = timeit(lambda: ops.gemm_wgrad(dY, A, None, False), a.reps)
            res[f"wgrad_{tag}_native"] = (t, 0)
            print(f"{tag} wgrad: native fp32          {2 * M * Nn * K / t / 1e9:.0f} TF/s", flush=True)
    if "ssd" in only:
        xc = torch.randn(B, L, conv_dim, device=dev).to(torch.bfloat16)
        x = xc[..., :di].unflatten(-1, (H, P))
        Bm = xc[..., di:di + N].unflatten(-1, (G, N))
        Cm = xc[..., di + N:].unflatten(-1, (G, N))
        dt = zx[..., -H:]
        A = -torch.rand(H, device=dev) * 8 - 0.5
        D = torch.randn(H, device=dev)
        dtb = torch.randn(H, device=dev) * 0.3
        y, cum, dtp, states, fin = ops.ssd_fwd(x, dt, A, Bm, Cm, D, dtb, None, 64, True, 0.0, float("inf"))
        dy = torch.randn_like(y)
        t = timeit(lambda: ops.ssd_fwd(x, dt, A, Bm, Cm, D, dtb, None, 64, True, 0.0, float("inf")), a.reps)
        res["ssd_fwd"] = (t, 0)
        t = timeit(lambda: ops.ssd_bwd(dy, x, dt, A, Bm, Cm, D, dtb, None, cum, dtp, states, None, 64, True, 0.0,
                                       float("inf"), None, None, None, None), a.reps)
        res["ssd_bwd"] = (t, 0)
    if "gnorm" in only:
        y = torch.randn(B * L, di, device=dev).to(torch.bfloat16)
        z = zx[..., :di].flatten(0, 1)
        w = torch.rand(di, device=dev)
        yn, rstd = ops.gated_rmsnorm_fwd(y, z, w, 1e-5, di, False)
        t = timeit(lambda: ops.gated_rmsnorm_fwd(y, z, w, 1e-5, di, False), a.reps)
        res["gated_fwd"] = (t, 3 * y.numel() * 2)
        t = timeit(lambda: ops.gated_rmsnorm_bwd(yn, y, z, w, rstd, di, False, None, None), a.reps)
        res["gated_bwd"] = (t, 5 * y.numel() * 2)
    if "norm" in only:
        x = torch.randn(B * L, 768, device=dev).to(torch.bfloat16)
        r = torch.randn(B * L, 768, device=dev)
        w = torch.rand(768, device=dev)
        y, ro, rstd = ops.add_rmsnorm_fwd(x, r, w, 1e-5, torch.bfloat16, torch.float32)
        t = timeit(lambda: ops.add_rmsnorm_fwd(x, r, w, 1e-5, torch.bfloat16, torch.float32), a.reps)
        res["add_norm_fwd"] = (t, x.numel() * (2 + 4 + 4 + 2))
        t = timeit(lambda: ops.add_rmsnorm_bwd(y, ro, ro, w, rstd, torch.bfloat16, torch.float32, True), a.reps)
        res["add_norm_bwd"] = (t, x.numel() * (2 + 4 + 4 + 2 + 4))
    if "ce" in only:
        logits = torch.randn(B * L, 50304, device=dev).to(torch.bfloat16)
        tg = torch.randint(0, 50304, (B * L,), device=dev)
        sc = torch.tensor(1.0 / (B * L), device=dev)
        t = timeit(lambda: ops.ce_fwd(logits, tg, -100, sc, logits), a.reps)
        res["ce_fwd_inplace_grad"] = (t, 2 * logits.numel() * 2)
    if "selscan" in only:
        d, n = 1536, 16
        # the Mamba-1 layer's layouts: u / delta / z channel-major per batch row (b, d, l), B / C (b, 1, n, l)
        # (the previous (d, b, l)-permuted views put consecutive channels 64 KB apart, an HBM stride
        # the model never produces)
        xz = torch.randn(B, 2 * d, L, device=dev).to(torch.bfloat16)
        u, z = xz[:, :d], xz[:, d:]
        delta = (torch.randn(B, d, L, device=dev) * 0.5 - 1).to(torch.bfloat16)
        A = -torch.rand(d, n, device=dev) * 4
        Bm = torch.randn(B, 1, n, L, device=dev).to(torch.bfloat16)
        Cm = torch.randn(B, 1, n, L, device=dev).to(torch.bfloat16)
        D = torch.randn(d, device=dev)
        db = torch.randn(d, device=dev)
        out, carries, last = ops.selscan_fwd(u, delta, A, Bm, Cm, D, z, db, True)
        t = timeit(lambda: ops.selscan_fwd(u, delta, A, Bm, Cm, D, z, db, True), a.reps)
        res["selscan_fwd"] = (t, 4 * u.numel() * 2)
        t = timeit(lambda: ops.selscan_bwd(out, u, delta, A, Bm, Cm, D, z, db, carries, True), a.reps)
        res["selscan_bwd"] = (t, 7 * u.numel() * 2)
    for k, (t, by) in res.items():
        bw = f"  {by / t / 1e9:.2f} TB/s" if by else ""
        print(f"{k:22s} {t * 1000:9.1f} us{bw}")


if __name__ == "__main__":
    main()
