"""Host-side timeline of one headline training step (where does the GPU wait for the host?).

Runs the bench.py step (Mamba-2 280M, 16 micro-batches, overlap) and records host timestamps at phase
boundaries together with CUDA events on the main stream, then prints, per phase, when the host finished
enqueueing it and when the GPU finished executing it.   python scripts/diag_step.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mamba_distributed_amd import LMHeadModel, preset
    from mamba_distributed_amd.data.loader import SyntheticTokens
    from mamba_distributed_amd.ops import grad_accum
    from mamba_distributed_amd.parallel import ddp as ddp_mod
    from mamba_distributed_amd.parallel.dist import init_distributed
    from mamba_distributed_amd.parallel.microbatch import auto_defer_reduce, resolve_overlap, run_micro_batches
    from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
    info = init_distributed()
    dev = info.device
    enable_tuned_gemms()
    torch.manual_seed(1337)
    model_name = sys.argv[1] if len(sys.argv) > 1 else "mamba2-280m"
    cfg = preset(model_name)
    model = LMHeadModel(cfg, device=dev)
    dmodel = ddp_mod.wrap_data_parallel(model, info, "native", 100.0, "fp32")
    opt = model.configure_optimizers(0.1, 6e-4, "cuda", False)
    loader = SyntheticTokens(32, 1024, cfg.vocab_size, 0, 1, device=dev)
    overlap = resolve_overlap("auto", cfg)
    print("overlap", overlap, flush=True)
    accum = 16

    def compute_loss(x, y):
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            _, loss = dmodel(x, y, return_logits=False)
        return loss / accum

    marks = []

    def mark(name):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((name, time.perf_counter(), ev))

    def step():
        mark("start")
        ddp_mod.zero_grad(dmodel, opt)
        mark("zero_grad")
        with grad_accum.accumulation_scope(defer_reduce=auto_defer_reduce(cfg)):
            loss_acc = run_micro_batches(dmodel, loader.next_batch, 1, compute_loss, overlap=False)
            mark("micro-batch 0")
            loss_acc = run_micro_batches(dmodel, loader.next_batch, accum - 1, compute_loss, overlap=overlap)
            mark("micro-batches enqueued")
        mark("scope exited")
        norm = ddp_mod.clip_grad_norm_(dmodel, 1.0)
        mark("clip enqueued")
        opt.step()
        mark("opt.step enqueued")
        return loss_acc

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    marks.clear()
    step()
    torch.cuda.synchronize()
    t0, e0 = marks[0][1], marks[0][2]
    for name, t, ev in marks:
        print(f"{name:28s} host {1e3 * (t - t0):9.1f} ms   gpu {e0.elapsed_time(ev):9.1f} ms", flush=True)


if __name__ == "__main__":
    main()
