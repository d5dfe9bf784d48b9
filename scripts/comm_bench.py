"""Collective bandwidth microbenchmark (rccl-tests style) for the gradient all-reduce and the TP/CP
collectives (SURVEY.md §4 'Perf' row, §5.1, §5.8).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 scripts/comm_bench.py [--ops all_reduce,...]
             [--min-mb 1 --max-mb 1024] [--dtype fp32|bf16] [--iters 20]

For each op and message size: mean time, algorithm bandwidth (bytes / t) and bus bandwidth with the
rccl-tests correction factors (all-reduce 2(n-1)/n, all-gather / reduce-scatter (n-1)/n), as one
JSON line per point on rank 0.  On one 8x MI355X node every GPU has 7 xGMI links (~153 GB/s each),
so a ring that uses one link per direction tops out near 153 GB/s bus bandwidth; RCCL's multi-ring /
direct algorithms should approach the 7-link aggregate for large messages.  The DDP bucket size
(parallel/ddp.py, 100 MB default) should sit where this curve has flattened.
Runs on gloo / CPU too (functional check; the numbers are meaningless there).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mamba_distributed_amd.parallel.dist import destroy, init_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="all_reduce,all_gather,reduce_scatter")
    ap.add_argument("--min-mb", type=float, default=1.0)
    ap.add_argument("--max-mb", type=float, default=1024.0)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    info = init_distributed("auto")
    assert info.ddp, "run under torchrun"
    n = info.world_size
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    esz = torch.tensor([], dtype=dt).element_size()
    gpu = info.device.startswith("cuda")
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    gloo = dist.get_backend() != "nccl"
    mb = a.min_mb
    while mb <= a.max_mb + 1e-9:
        count = max(n, int(mb * 2**20 / esz) // n * n)
        nbytes = count * esz
        buf = torch.ones(count, dtype=dt, device=info.device)
        shard = torch.ones(count // n, dtype=dt, device=info.device)
        for op in a.ops.split(","):
            if op == "all_reduce":
                def fn():
                    dist.all_reduce(buf)
                factor = 2 * (n - 1) / n
            elif op == "all_gather":
                def fn():
                    if gloo:
                        dist.all_gather(list(buf.chunk(n)), shard)
                    else:
                        dist.all_gather_into_tensor(buf, shard)
                factor = (n - 1) / n
            elif op == "reduce_scatter":
                if gloo:
                    continue  # gloo has no reduce-scatter
                def fn():
                    dist.reduce_scatter_tensor(shard, buf)
                factor = (n - 1) / n
            else:
                raise ValueError(op)
            for _ in range(a.warmup):
                fn()
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                fn()
            sync()
            t = (time.perf_counter() - t0) / a.iters
            tt = torch.tensor([t], dtype=torch.float64, device=info.device)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
            if info.master:
                alg = nbytes / t / 1e9
                print(json.dumps({"op": op, "bytes": nbytes, "dtype": a.dtype, "n_ranks": n,
                                  "time_us": round(t * 1e6, 1), "algbw_GBs": round(alg, 2),
                                  "busbw_GBs": round(alg * factor, 2), "backend": dist.get_backend()}),
                      flush=True)
        mb *= 2
    destroy()


if __name__ == "__main__":
    main()
