"""Long-prompt prefill latency (batch 1 by default) with the segment-parallel SSD walks on (automatic) and off.

  python scripts/bench_prefill.py [--model mamba2-280m] [--prompt 8192 32768] [--batch 1] [--reps 3]
One JSON line per (prompt, segments): ms per prefill (eager, bf16, random-init weights, random tokens) and the
last-position logits' max difference between the two settings.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="mamba2-280m")
    p.add_argument("--prompt", type=int, nargs="+", default=[8192, 32768])
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    from mamba_distributed_amd import LMHeadModel, preset
    from mamba_distributed_amd.inference import GraphedDecoder
    from mamba_distributed_amd.ops import _ext
    assert _ext.load(), _ext.error()
    ops = _ext.ops()
    torch.manual_seed(0)
    cfg = preset(a.model)
    m = LMHeadModel(cfg, device="cuda").to(torch.bfloat16).eval()
    for L in a.prompt:
        ids = torch.randint(0, cfg.vocab_size, (a.batch, L), device="cuda")
        dec = GraphedDecoder(m, batch_size=a.batch, max_seqlen=L + 8, use_graph=False)
        ref = None
        for forced in (1, 0):  # 1: one walk per (h, b); 0: automatic segments
            ops.ssd_segments(forced, 1, 1, 1)
            nseg = int(ops.ssd_segments(-1, a.batch, cfg.d_model * 2 // 64, (L + 63) // 64))
            logits = dec.prefill(ids)
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                logits = dec.prefill(ids)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            diff = 0.0 if ref is None else (logits.float() - ref).abs().max().item()
            ref = logits.float() if ref is None else ref
            print(json.dumps({"model": a.model, "batch": a.batch, "prompt": L, "ssd_segments": nseg,
                              "prefill_ms": round(min(ts), 2), "tok_per_s": round(a.batch * L / min(ts) * 1e3),
                              "max_logit_diff_vs_one_walk": round(diff, 4)}), flush=True)
        ops.ssd_segments(0, 1, 1, 1)
        del dec


if __name__ == "__main__":
    main()
