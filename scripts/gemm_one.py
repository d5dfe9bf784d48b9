"""Run one projection GEMM engine on one shape (for rocprofv3 counter passes):
python scripts/gemm_one.py {pk,lib} M N K [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load()
eng = sys.argv[1]
M, N, K = (int(x) for x in sys.argv[2:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
if eng == "lib":
    from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
    enable_tuned_gemms()
A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
B = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
ops = torch.ops.mamba_amd
f = {"pp": lambda: ops.gp_pp(A, B, C), "pk": lambda: ops.gp_pk(A, B, C),
     "lib": lambda: torch.nn.functional.linear(A, B)}[eng]
for _ in range(reps):
    f()
torch.cuda.synchronize()
print("done", eng, M, N, K)
