"""Headline benchmark: Mamba-2 280M DDP training throughput (tokens/s, whole job).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
         --master-port P bench.py --gpus N --steps K --warmup W

Config = BASELINE.json's headline: Mamba-2 280M (d_model 768, 64 layers, vocab 50304), seq 1024,
global batch 524,288 tokens (= 512 sequences; micro-batch auto: 64 sequences per micro-step for the 280M models,
grad-accum 8/N), bf16 autocast,
fused AdamW, grad clip 1.0, data parallel over RCCL (native bucketed reducer; --dp-impl ddp = torch DDP).  Synthetic tokens, random init (no dataset/weights
on the box).  A "step" is one full optimizer step (all micro-batches + all-reduce + clip + AdamW).
W untimed warmup steps, then exactly K steps between barrier+synchronize pairs; the MAX elapsed
over ranks is reported; rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

BASELINE_TOK_S = 238000.0  # BASELINE.md derived 8xA100 node throughput (no published tok/s)
BASELINE_GPUS = 8
BASELINE_PER_GPU = BASELINE_TOK_S / BASELINE_GPUS  # 29.75k tok/s per A100
METRIC = "tokens/sec (whole node) Mamba-2 280M DDP at 1/2/4/8 MI355X; HellaSwag acc"


def _relaunch_under_torchrun(argv, n):
    """``python bench.py --gpus N`` outside torchrun: start N ranks with torch.distributed.run as a
    CHILD process (before this process touches the GPU: no exec from a GPU-initialised process)
    and exit with its return code, so a multi-GPU request can never silently measure one GPU."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _allreduce_probe(dev: str, world: int, bucket_mb: float, iters: int = 10) -> dict:
    """Mean time and bus bandwidth of an fp32 all-reduce of one gradient bucket (and of 4x that), every rank."""
    import torch.distributed as dist
    out = {}
    on_gpu = dev.startswith("cuda")
    for mb in (bucket_mb, 4 * bucket_mb):
        n = max(world, int(mb * 2**20) // 4 // world * world)
        buf = torch.ones(n, dtype=torch.float32, device=dev)
        for _ in range(3):
            dist.all_reduce(buf)
        if on_gpu:
            torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(buf)
        if on_gpu:
            torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / iters
        tt = torch.tensor(t, device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
        key = f"allreduce_{int(round(mb))}MB"
        out[key + "_ms"] = round(1e3 * t, 3)
        out[key + "_busbw_GBps"] = round(2 * (world - 1) / world * n * 4 / t / 1e9, 1)
        del buf
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--model", default="mamba2-280m")
    p.add_argument("--B", default="auto",
                   help="micro-batch (sequences); auto: parallel/microbatch.py::auto_micro_batch (64 for the 280M "
                        "models when a rank has >= 64 sequences per step, else 32) -- the global batch and the "
                        "gradient are the same for any micro-batch")
    p.add_argument("--T", type=int, default=1024)
    p.add_argument("--global-batch-tokens", type=int, default=524288)
    p.add_argument("--bucket-cap-mb", type=float, default=100.0)
    p.add_argument("--grad-comm-dtype", default="fp32")
    p.add_argument("--reference-ops", action="store_true", help="A/B: run the PyTorch reference ops")
    p.add_argument("--no-fused-ce", action="store_true")
    p.add_argument("--no-tuned-gemms", action="store_true", help="library-default GEMM solutions")
    p.add_argument("--profile-steps", type=int, default=0, help="torch.profiler trace of N extra steps")
    p.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                   help="next micro-batch's forward on a second stream beside the backward "
                        "(auto: d_model <= 1024, parallel/microbatch.py::auto_overlap)")
    p.add_argument("--no-overlap", action="store_true", help="same as --overlap off")
    p.add_argument("--trace-loss", action="store_true",
                   help="diagnostics: print every step's loss and grad norm (syncs each step; not for timing)")
    p.add_argument("--activation-checkpointing", type=int, default=0,
                   help="recompute every N-th block in the backward (memory for long sequences; 0 = off)")
    p.add_argument("--dp-impl", default="native", choices=["native", "ddp"],
                   help="gradient all-reduce: native bucketed reducer (parallel/reducer.py) or torch DDP")
    a = p.parse_args()
    if a.gpus > 1 and "RANK" not in os.environ:
        sys.exit(_relaunch_under_torchrun(sys.argv[1:], a.gpus))
    if a.reference_ops:
        os.environ["MAMBA_AMD_FORCE_REFERENCE"] = "1"

    from mamba_distributed_amd import LMHeadModel, preset
    from mamba_distributed_amd.data.loader import SyntheticTokens
    from mamba_distributed_amd.ops import grad_accum
    from mamba_distributed_amd.parallel import ddp as ddp_mod
    from mamba_distributed_amd.parallel.microbatch import auto_defer_reduce, resolve_overlap, run_micro_batches
    from mamba_distributed_amd.parallel.dist import all_reduce_avg, all_reduce_max, barrier, destroy, init_distributed

    info = init_distributed("auto")
    world = info.world_size
    dev = info.device
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the job has {world} rank(s); refusing to report", file=sys.stderr)
        destroy()
        sys.exit(2)
    cfg = preset(a.model)
    assert a.global_batch_tokens % (a.T * world) == 0
    if str(a.B) == "auto":
        from mamba_distributed_amd.parallel.microbatch import auto_micro_batch
        a.B = auto_micro_batch(cfg, a.global_batch_tokens // (a.T * world), a.T)
    a.B = int(a.B)
    assert a.global_batch_tokens % (a.B * a.T * world) == 0
    accum = a.global_batch_tokens // (a.B * a.T * world)
    from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
    # the TunableOp table only matters when a library GEMM can run: the hipBLASLt A/B switches, or the reference ops
    from mamba_distributed_amd.ops.linear import library_gemms_possible
    lib_gemms = library_gemms_possible(cfg) or os.environ.get("MAMBA_AMD_LMHEAD") == "lib" or a.reference_ops
    tuned = False if (a.no_tuned_gemms or not lib_gemms) else enable_tuned_gemms()
    torch.manual_seed(1337)
    model = LMHeadModel(cfg, device=dev)
    if a.activation_checkpointing:
        model.set_activation_checkpointing(a.activation_checkpointing)
    dmodel = ddp_mod.wrap_data_parallel(model, info, a.dp_impl, a.bucket_cap_mb, a.grad_comm_dtype)
    opt = model.configure_optimizers(0.1, 6e-4, "cuda" if dev.startswith("cuda") else "cpu", False)
    # the reducer leaves the gradients summed for the native AdamW, which divides (parallel/ddp.py)
    ddp_mod.configure_grad_average(dmodel, opt)
    loader = SyntheticTokens(a.B, a.T, cfg.vocab_size, info.rank, world, device=dev)
    fused = not a.no_fused_ce
    overlap = resolve_overlap("off" if a.no_overlap else a.overlap, cfg, a.B * a.T)

    on_gpu = dev.startswith("cuda")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    def compute_loss(x, y):
        # bf16 autocast on the GPU; the CPU path (gloo rehearsal of the multi-rank flow) stays fp32
        with torch.autocast(device_type="cuda" if on_gpu else "cpu", dtype=torch.bfloat16, enabled=on_gpu):
            _, loss = dmodel(x, y, return_logits=not fused)
        return loss / accum

    def step():
        ddp_mod.zero_grad(dmodel, opt)
        with grad_accum.accumulation_scope(defer_reduce=auto_defer_reduce(cfg)):
            # micro-batch k+1's forward runs on a second stream beside micro-batch k's backward
            loss_acc = run_micro_batches(dmodel, loader.next_batch, accum, compute_loss,
                                         overlap=overlap)
        all_reduce_avg(loss_acc)
        norm = ddp_mod.clip_and_step(dmodel, opt, 1.0)
        if a.trace_loss and info.master:
            print(f"step loss {loss_acc.item():.5f} grad_norm {norm.item():.4f}", flush=True)
        return loss_acc

    red = ddp_mod._reducer(dmodel)
    for _ in range(a.warmup):
        step()
    if red is not None:
        red.timing = True
        red.exposed_ms()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        last = step()
    barrier()
    sync()
    elapsed = torch.tensor(time.perf_counter() - t0, device=dev, dtype=torch.float64)
    all_reduce_max(elapsed)
    elapsed = float(elapsed.item())
    comm_probe = {}
    if world > 1:
        # after the timed region: the gradient all-reduce's bus bandwidth at the bucket size over this job's RCCL
        # rings (xGMI on one node), rccl-tests convention busbw = 2 (n - 1) / n x bytes / t
        comm_probe = _allreduce_probe(dev, world, a.bucket_cap_mb)
    comm = {"backend": info.backend, "world_size": world}
    if world > 1:
        comm.update(comm_probe)
    if red is not None:
        exp = red.exposed_ms()
        red.timing = False
        ex = torch.tensor([sorted(exp)[len(exp) // 2] if exp else 0.0], device=dev, dtype=torch.float64)
        all_reduce_max(ex)
        bb = red.bucket_bytes()
        comm.update({"exposed_allreduce_ms_per_step": round(float(ex.item()), 3), "n_buckets": len(bb),
                     "bucket_mb": [round(b / 2**20, 1) for b in bb],
                     "grad_bytes": int(sum(bb)), "grad_comm_dtype": a.grad_comm_dtype})
    peak_gb = torch.cuda.max_memory_allocated() / 2**30 if dev.startswith("cuda") else 0.0
    reserved_gb = torch.cuda.max_memory_reserved() / 2**30 if dev.startswith("cuda") else 0.0
    # caching-allocator retries (a failed cudaMalloc -> free cached blocks -> device sync -> retry): nonzero means
    # the run is memory-bound on the allocator, not on the kernels
    alloc_retries = int(torch.cuda.memory_stats().get("num_alloc_retries", 0)) if dev.startswith("cuda") else 0
    loss_v = float(last.item())
    if a.profile_steps and info.master:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(a.profile_steps):
                step()
            torch.cuda.synchronize()
        os.makedirs("gpurun_out", exist_ok=True)
        with open("gpurun_out/torch_profile.txt", "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
    tokens = a.global_batch_tokens * a.steps
    value = tokens / elapsed
    if info.master:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 2),
            "higher_is_better": True,
            "scaling": "strong",
            # the derived A100 figure at the SAME GPU count (per-GPU rate x N): at N = 8 this is the node
            # ratio against BASELINE.md's 238k; at N < 8 it never divides a partial node by a whole one
            "vs_baseline": round(value / (BASELINE_PER_GPU * world), 3),
            "vs_a100_per_gpu": round(value / world / BASELINE_PER_GPU, 3),
            "vs_a100_node": round(value / BASELINE_TOK_S, 3) if world == BASELINE_GPUS else None,
            "dtype": "bf16" if on_gpu else "fp32",
            "data": "synthetic (uniform random tokens, random-init weights)",
            "config": {
                "model": f"{a.model} (d_model={cfg.d_model}, n_layer={cfg.n_layer}, vocab={cfg.vocab_size}, "
                         f"layer={cfg.layer_type})",
                "global_batch": a.global_batch_tokens // a.T,
                "global_batch_tokens": a.global_batch_tokens,
                "micro_batch": a.B,
                "grad_accum": accum,
                "seq_len": a.T,
                "parallelism": f"dp{world}",
                "ops": "pytorch-reference" if (a.reference_ops or not on_gpu) else "native-hip",
                "gemm_table": ("tunableop-gfx950" if tuned else "library-default") if lib_gemms
                              else "unused (every GEMM on the native engines)",
                "microbatch_overlap": overlap,
                "dp_impl": a.dp_impl if world > 1 else "none",
                "activation_checkpointing": a.activation_checkpointing,
                "final_loss": round(loss_v, 4),
                "peak_mem_gb": round(peak_gb, 1),
                "peak_reserved_gb": round(reserved_gb, 1),
                "alloc_retries": alloc_retries,
                "comm": comm,
                "per_gpu_tok_s": round(value / world, 1),
            },
        }
        print(json.dumps(out), flush=True)
    from mamba_distributed_amd.ops import grad_accum
    grad_accum.release_buffers()
    destroy()


if __name__ == "__main__":
    main()
