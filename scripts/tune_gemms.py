"""Search hipBLASLt/rocBLAS solutions for every GEMM of a training step and write the table
that ``utils.gemm_tuning.enable_tuned_gemms`` replays (run on an MI355X):

    python scripts/tune_gemms.py --models mamba2-280m mamba1-280m --B 32 --T 1024
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mamba_distributed_amd import LMHeadModel, preset  # noqa: E402
from mamba_distributed_amd.utils import gemm_tuning  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--models", nargs="+", default=["mamba2-280m"])
    p.add_argument("--B", type=int, default=32)
    p.add_argument("--T", type=int, default=1024)
    p.add_argument("--out", default=gemm_tuning.DEFAULT_TABLE)
    p.add_argument("--max-ms", type=int, default=40)
    p.add_argument("--decode-batch", type=int, nargs="*", default=[],
                   help="also tune the decode GEMVs (M = batch) of a bf16 model")
    a = p.parse_args()
    if os.path.exists(a.out):
        torch.cuda.tunable.read_file(a.out)  # keep earlier shapes
    gemm_tuning.enable_tuned_gemms(a.out, tune=True, max_tuning_ms=a.max_ms)
    for name in a.models:
        cfg = preset(name)
        model = LMHeadModel(cfg, device="cuda")
        for fused in (True, False):
            x = torch.randint(0, cfg.vocab_size, (a.B, a.T), device="cuda")
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
                _, loss = model(x, x, return_logits=not fused)
            loss.backward()
            torch.cuda.synchronize()
            print(f"{name} fused_ce={fused}: {len(torch.cuda.tunable.get_results())} tuned GEMMs", flush=True)
        if a.decode_batch:
            from mamba_distributed_amd.inference import GraphedDecoder
            mb = model.to(torch.bfloat16).eval()
            for bs in a.decode_batch:
                dec = GraphedDecoder(mb, batch_size=bs, max_seqlen=64, use_graph=False)
                logits = dec.prefill(torch.randint(0, cfg.vocab_size, (bs, 16), device="cuda"))
                for _ in range(2):
                    logits = dec.step(logits.argmax(-1))
                torch.cuda.synchronize()
                print(f"{name} decode batch {bs}: {len(torch.cuda.tunable.get_results())} tuned GEMMs", flush=True)
        del model
        torch.cuda.empty_cache()
    n = gemm_tuning.flush(a.out)
    for r in torch.cuda.tunable.get_results():
        print(r)
    print(f"wrote {n} rows -> {a.out}")


if __name__ == "__main__":
    main()
