"""Decode benchmark: per-token latency / throughput of cached generation, eager vs HIP-graph replay.

  python scripts/bench_decode.py [--model mamba2-280m] [--batch 1 16] [--prompt 512] [--tokens 128]
Prints one JSON line per (batch, mode).  Random-init weights, bf16 model, random prompt tokens.
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
    p.add_argument("--batch", type=int, nargs="+", default=[1, 16])
    p.add_argument("--prompt", type=int, default=512)
    p.add_argument("--tokens", type=int, default=128)
    a = p.parse_args()
    from mamba_distributed_amd import LMHeadModel, preset
    from mamba_distributed_amd.inference import GraphedDecoder
    from mamba_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
    enable_tuned_gemms()
    torch.manual_seed(0)
    cfg = preset(a.model)
    m = LMHeadModel(cfg, device="cuda").to(torch.bfloat16).eval()
    for bs in a.batch:
        ids = torch.randint(0, cfg.vocab_size, (bs, a.prompt), device="cuda")
        for mode in ("eager", "graph_unfused", "graph"):
            # eager / graph: fused Mamba-2 decode kernels (decode.hip) when supported; graph_unfused: the
            # per-op cached step (library GEMVs + separate conv / SSM / norm kernels) in one HIP graph
            dec = GraphedDecoder(m, batch_size=bs, max_seqlen=a.prompt + a.tokens + 8, use_graph=mode != "eager",
                                 fused=False if mode == "graph_unfused" else None)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            logits = dec.prefill(ids)
            torch.cuda.synchronize()
            t_prefill = time.perf_counter() - t0
            tok = logits.argmax(-1)
            for _ in range(3):  # warm-up (and graph capture)
                tok = dec.step(tok).argmax(-1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.tokens):
                tok = dec.step(tok).argmax(-1)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"model": a.model, "batch": bs, "mode": mode, "fused": dec.fused is not None,
                              "prompt": a.prompt,
                              "prefill_ms": round(t_prefill * 1e3, 2),
                              "ms_per_token": round(dt * 1e3 / a.tokens, 3),
                              "tokens_per_s": round(bs * a.tokens / dt, 1)}), flush=True)


if __name__ == "__main__":
    main()
