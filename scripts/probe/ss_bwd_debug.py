"""Debug: sequential selscan backward vs time-parallel, per-gradient error and dB error pattern."""
import os
import torch
import mamba_distributed_amd  # noqa: F401
from mamba_distributed_amd.ops import _ext
_ext.load()
ops = torch.ops.mamba_amd
torch.manual_seed(8)
b, d, L, G, n = 32, 1536, 64, 1, 16
dev = "cuda"
u = torch.randn(b, d, L, device=dev).to(torch.bfloat16)
delta = (torch.randn(b, d, L, device=dev) * 0.5 - 1).to(torch.bfloat16)
A = -torch.rand(d, n, device=dev) * 4 - 0.1
Bm = torch.randn(b, G, n, L, device=dev).to(torch.bfloat16)
Cm = torch.randn(b, G, n, L, device=dev).to(torch.bfloat16)
D = torch.randn(d, device=dev)
z = torch.randn(b, d, L, device=dev).to(torch.bfloat16)
db = torch.randn(d, device=dev) * 0.3
dout = torch.randn(b, d, L, device=dev).to(torch.bfloat16)
res = {}
for sg in ("1", "0"):
    os.environ["MAMBA_AMD_SELSCAN_BWD_SG"] = sg
    out, carries, last = ops.selscan_fwd(u, delta, A, Bm, Cm, D, z, db, True)
    res[sg] = ops.selscan_bwd(dout, u, delta, A, Bm, Cm, D, z, db, carries, True)
    print(sg, "carries", tuple(carries.shape))
names = ["du", "ddelta", "dA", "dB", "dC", "dD", "dz", "dbias"]
for nm, x, y in zip(names, res["1"], res["0"]):
    x, y = x.float(), y.float()
    print(f"{nm:7s} rel {((x - y).norm() / (y.norm() + 1e-12)).item():.3e}")
x, y = res["1"][3].float()[0, 0], res["0"][3].float()[0, 0]  # (n, L)
err = (x - y).abs()
print("dB err by n:", [f"{v:.2f}" for v in (err.mean(1) / y.abs().mean(1)).tolist()])
print("dB err by t (first 32):", [f"{v:.2f}" for v in (err.mean(0) / y.abs().mean(0)).tolist()[:32]])
print("x[0,:8]", x[0, :8].tolist())
print("y[0,:8]", y[0, :8].tolist())
# is x a permutation / scaled version of y?
for nn in range(4):
    for tt in range(4):
        cands = [(i, j) for i in range(n) for j in range(L) if abs(y[i, j] - x[nn, tt]) < 1e-2 * abs(x[nn, tt]) + 1e-3]
        print("x", nn, tt, x[nn, tt].item(), "matches y at", cands[:4])
