"""Tokenizer resolution (the reference uses tiktoken GPT-2 BPE: train.py:41, model.py:20).

This environment is offline and tiktoken is not installed, so ``get_encoding`` resolves, in order:
  1. ``tiktoken.get_encoding(name)`` when tiktoken is importable,
  2. GPT-2 BPE files (``vocab.json`` + ``merges.txt``) in ``$MAMBA_AMD_TOKENIZER_DIR`` loaded with the
     ``tokenizers`` library (same byte-level BPE as tiktoken's gpt2 encoding),
  3. ``ByteTokenizer``: UTF-8 bytes as ids 0..255, EOT = 50256.  Keeps sampling / eval plumbing
     runnable end to end; token ids differ from GPT-2's so quality numbers need 1 or 2.
"""
from __future__ import annotations

import os
import warnings
from typing import List


class ByteTokenizer:
    name = "bytes"
    eot_token = 50256
    n_vocab = 50257

    def encode(self, text: str, **kw) -> List[int]:
        return list(text.encode("utf-8"))

    def encode_ordinary(self, text: str) -> List[int]:
        return self.encode(text)

    def decode(self, ids) -> str:
        return bytes(int(i) for i in ids if 0 <= int(i) < 256).decode("utf-8", errors="replace")


class _HFBPE:
    def __init__(self, tok):
        self._tok = tok
        self.eot_token = tok.token_to_id("<|endoftext|>") or 50256
        self.name = "gpt2-bpe"

    def encode(self, text: str, **kw) -> List[int]:
        return self._tok.encode(text).ids

    encode_ordinary = encode

    def decode(self, ids) -> str:
        return self._tok.decode([int(i) for i in ids])


def get_encoding(name: str = "gpt2"):
    try:
        import tiktoken  # type: ignore
        return tiktoken.get_encoding(name)
    except Exception:
        pass
    d = os.environ.get("MAMBA_AMD_TOKENIZER_DIR")
    if d and os.path.exists(os.path.join(d, "vocab.json")) and os.path.exists(os.path.join(d, "merges.txt")):
        from tokenizers import ByteLevelBPETokenizer
        tok = ByteLevelBPETokenizer(os.path.join(d, "vocab.json"), os.path.join(d, "merges.txt"))
        return _HFBPE(tok)
    warnings.warn("GPT-2 BPE unavailable (no tiktoken, no MAMBA_AMD_TOKENIZER_DIR): using the byte "
                  "tokenizer fallback", stacklevel=2)
    return ByteTokenizer()
