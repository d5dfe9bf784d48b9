"""HellaSwag evaluation (reference eval.py:15-200).

Same protocol: GPT-2 BPE, context + " " + ending for the 4 endings, zero-padded (4, maxlen),
completion mask, per-token CE on shifted logits, masked sum and masked mean, ``pred_norm =
argmin(mean)``, first 2000 validation examples, ``log/hellaswag_eval.txt`` gets
``"2000 {correct}/2000 {acc:.4f}"`` (no trailing newline).

Fixed reference bugs: A1 ``(str, Enum)``; A2 the HF branch loads the model
(``LMHeadModel.load_from_hf``); A3 the device is passed through; A4 ``--checkpoint`` flag (default
keeps ``log/model_mamba_03000.pt``); A5 the checkpoint's config is read (plain dict) instead of the
hard-coded Mamba-1 config, so Mamba-2 checkpoints evaluate too.
Offline: ``download`` only works when the jsonl is already in ``--data-dir``; otherwise it raises.
If fewer than ``num_examples`` exist, the result line is written at the end with the real count.
"""
from __future__ import annotations

import json
import os
from enum import Enum
from typing import Iterator, Optional

import torch
import torch.nn.functional as F

from ..lm import LMHeadModel
from ..utils.checkpoint import config_from_checkpoint, load_checkpoint
from ..utils.tokenizer import get_encoding

CHECKPOINT_PATH = "log/model_mamba_03000.pt"
HELLASWAG_DATA = {
    "train": "https://raw.githubusercontent.com/rowanz/hellaswag/master/data/hellaswag_train.jsonl",
    "val": "https://raw.githubusercontent.com/rowanz/hellaswag/master/data/hellaswag_val.jsonl",
    "test": "https://raw.githubusercontent.com/rowanz/hellaswag/master/data/hellaswag_test.jsonl",
}


class ModelType(str, Enum):
    CUSTOM = "custom"
    HF = "hugging_face"


def load_model_from_checkpoint(checkpoint_path: str = CHECKPOINT_PATH, device: str = "cuda", enc=None) -> LMHeadModel:
    ckpt = load_checkpoint(checkpoint_path, map_location="cpu")
    config = config_from_checkpoint(ckpt)
    model = LMHeadModel(config=config, device=device, enc=enc)
    model.load_state_dict(ckpt["model"])
    return model


def download_file(url: str, fname: str, chunk_size: int = 1024):
    import requests
    from tqdm import tqdm
    resp = requests.get(url, stream=True, timeout=30)
    total = int(resp.headers.get("content-length", 0))
    with open(fname, "wb") as file, tqdm(desc=fname, total=total, unit="iB", unit_scale=True,
                                         unit_divisor=1024) as bar:
        for data in resp.iter_content(chunk_size=chunk_size):
            bar.update(file.write(data))


def download(split: str, data_dir: str):
    os.makedirs(data_dir, exist_ok=True)
    fname = os.path.join(data_dir, f"hellaswag_{split}.jsonl")
    if not os.path.exists(fname):
        print(f"Downloading {HELLASWAG_DATA[split]} to {fname}...")
        download_file(HELLASWAG_DATA[split], fname)


def render_example(example, enc):
    ctx, label, endings = example["ctx"], example["label"], example["endings"]
    data = {"label": label, "ctx_tokens": None, "ending_tokens": []}
    ctx_tokens = enc.encode(ctx)
    data["ctx_tokens"] = ctx_tokens
    tok_rows, mask_rows = [], []
    for end in endings:
        end_tokens = enc.encode(" " + end)  # GPT-2 BPE: the leading space belongs to the word
        tok_rows.append(ctx_tokens + end_tokens)
        mask_rows.append([0] * len(ctx_tokens) + [1] * len(end_tokens))
        data["ending_tokens"].append(end_tokens)
    max_len = max(len(r) for r in tok_rows)
    tokens = torch.zeros((4, max_len), dtype=torch.long)
    mask = torch.zeros((4, max_len), dtype=torch.long)
    for i, (tr, mr) in enumerate(zip(tok_rows, mask_rows)):
        tokens[i, : len(tr)] = torch.tensor(tr)
        mask[i, : len(mr)] = torch.tensor(mr)
    return data, tokens, mask, label


def iterate_examples(split: str, data_dir: str) -> Iterator[dict]:
    download(split, data_dir)
    with open(os.path.join(data_dir, f"hellaswag_{split}.jsonl")) as f:
        for line in f:
            if line.strip():
                yield json.loads(line)


@torch.no_grad()
def score_example(model, tokens, mask, autocast_dtype: Optional[torch.dtype] = None):
    if autocast_dtype is not None and tokens.is_cuda:
        with torch.autocast("cuda", dtype=autocast_dtype):
            logits, _ = model(tokens)
    else:
        logits, _ = model(tokens)
    shift_logits = logits[..., :-1, :].contiguous().float()
    shift_tokens = tokens[..., 1:].contiguous()
    losses = F.cross_entropy(shift_logits.view(-1, shift_logits.size(-1)), shift_tokens.view(-1), reduction="none")
    losses = losses.view(tokens.size(0), -1)
    shift_mask = mask[..., 1:].contiguous()
    masked = losses * shift_mask
    sum_loss = masked.sum(dim=1)
    avg_loss = sum_loss / shift_mask.sum(dim=1)
    return sum_loss, avg_loss


@torch.no_grad()
def evaluate(model_type, hf_model_name: str, device: str = "cuda", checkpoint_path: str = CHECKPOINT_PATH,
             data_dir: str = "hellaswag", num_examples: int = 2000, out_file: str = "log/hellaswag_eval.txt",
             dtype: str = "fp32", model: Optional[LMHeadModel] = None, verbose: bool = True,
             allow_byte_tokenizer: bool = False, enc=None) -> float:
    # the reference's "high" (TF32 on A100, eval.py:125) has no gfx950 counterpart, and under "high" a
    # replayed TunableOp table can select garbage GEMMs (utils/gemm_tuning.py): keep exact fp32
    torch.set_float32_matmul_precision("highest")
    enc = enc if enc is not None else get_encoding("gpt2")
    tok_name = getattr(enc, "name", type(enc).__name__)
    if tok_name == "bytes" and not allow_byte_tokenizer:
        # a GPT-2-BPE-trained model scored on byte ids prints a plausible-looking, meaningless accuracy
        raise RuntimeError("HellaSwag needs the GPT-2 BPE (tiktoken or MAMBA_AMD_TOKENIZER_DIR); only the byte "
                           "fallback tokenizer is available.  Pass --allow-byte-tokenizer to score anyway.")
    if model is None:
        if ModelType(model_type) == ModelType.CUSTOM:
            model = load_model_from_checkpoint(checkpoint_path, device, enc=enc)
        else:
            model = LMHeadModel.load_from_hf(hf_model_name, device)
    model.to(device)
    model.eval()
    ac = {"fp32": None, "bf16": torch.bfloat16}[dtype]
    num_correct_norm = num_correct = num_total = 0
    for example in iterate_examples("val", data_dir):
        _, tokens, mask, label = render_example(example, enc)
        tokens, mask = tokens.to(device), mask.to(device)
        sum_loss, avg_loss = score_example(model, tokens, mask, ac)
        pred = sum_loss.argmin().item()
        pred_norm = avg_loss.argmin().item()
        num_total += 1
        num_correct += int(pred == label)
        num_correct_norm += int(pred_norm == label)
        if verbose:
            print(f"{num_total} acc_norm: {num_correct_norm}/{num_total}={num_correct_norm / num_total:.4f}")
            if num_total < 10:
                print("---")
                print(f"Context:\n {example['ctx']}")
                print("Endings:")
                for i, end in enumerate(example["endings"]):
                    print(f"{i} (loss: {avg_loss[i].item():.4f}) {end}")
                print(f"predicted: {pred_norm}, actual: {label}")
        if num_total == num_examples:
            break
    acc = num_correct_norm / max(1, num_total)
    if out_file:
        os.makedirs(os.path.dirname(out_file) or ".", exist_ok=True)
        with open(out_file, "a") as f:
            f.write(f"{num_total} {num_correct_norm}/{num_total} {acc:.4f}" +
                    ("" if tok_name != "bytes" else f" tokenizer={tok_name}"))
    if verbose:
        print(f"hellaswag acc_norm {acc:.4f} over {num_total} examples (tokenizer={tok_name})")
    return acc


def main(argv=None):
    import argparse
    p = argparse.ArgumentParser()
    p.add_argument("-m", "--model_type", type=str, default="custom", help="use custom or hugging_face")
    p.add_argument("-v", "--hf_model_name", type=str, default="state-spaces/mamba2-370m",
                   help="the hugging face model name (local directory or cached hub id)")
    p.add_argument("-d", "--device", type=str, default="cuda", help="the device to use")
    p.add_argument("--checkpoint", type=str, default=CHECKPOINT_PATH)
    p.add_argument("--data-dir", type=str, default=os.path.join(os.getcwd(), "hellaswag"))
    p.add_argument("--num-examples", type=int, default=2000)
    p.add_argument("--out-file", type=str, default="log/hellaswag_eval.txt")
    p.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    p.add_argument("--allow-byte-tokenizer", action="store_true",
                   help="score with the byte fallback tokenizer when no GPT-2 BPE is available (result tagged)")
    a = p.parse_args(argv)
    return evaluate(a.model_type, a.hf_model_name, a.device, a.checkpoint, a.data_dir, a.num_examples, a.out_file,
                    a.dtype, allow_byte_tokenizer=a.allow_byte_tokenizer)
