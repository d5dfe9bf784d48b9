"""Channel-last conv (Mamba-2 conv1d, kernels/conv1d.hip) bandwidth on the in_proj output's strided xBC slice vs a
contiguous copy, next to torch's own copy kernels (the practical 1:1 read/write ceiling on the box).

  python scripts/conv_stride_probe.py      (one MI355X; results: profiles/r6/conv_bandwidth_probe.txt)
"""
import torch, sys, os
sys.path.insert(0, os.getcwd())
from mamba_distributed_amd.ops import _ext
assert _ext.load()
ops = torch.ops.mamba_amd
def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps): fn()
        e.record(); torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / reps)
    return best
B, L, di, cd, dproj = 64, 1024, 1536, 1792, 3392
zx = torch.randn(B, L, dproj, device="cuda").to(torch.bfloat16)
xs = zx[..., di:di + cd]
xc = xs.contiguous()
w = torch.randn(cd, 4, device="cuda") * 0.3; b = torch.randn(cd, device="cuda")
for name, x in (("strided slice", xs), ("contiguous", xc)):
    t = timeit(lambda: ops.conv1d_cl_fwd(x, w, b, True))
    print(f"conv_cl_fwd {name:14s} {t:7.1f} us  {2 * B * L * cd * 2 / t / 1e6:.2f} TB/s")
g = torch.randn(B, L, cd, device="cuda").to(torch.bfloat16)
for name, x in (("strided slice", xs), ("contiguous", xc)):
    t = timeit(lambda: ops.conv1d_cl_bwd(x, w, b, g, True, None))
    print(f"conv_cl_bwd {name:14s} {t:7.1f} us  {3 * B * L * cd * 2 / t / 1e6:.2f} TB/s")
t = timeit(lambda: xs.contiguous()); print(f"torch copy strided->contig {t:7.1f} us  {2*B*L*cd*2/t/1e6:.2f} TB/s")
t = timeit(lambda: xc.clone()); print(f"torch copy contig->contig  {t:7.1f} us  {2*B*L*cd*2/t/1e6:.2f} TB/s")
