"""Token-shard data loading (reference dataloader.py:7-52).

``DataLoaderLite`` keeps the reference's semantics exactly — sorted shards whose names contain
the split, rank r starts at B*T*r and strides B*T*world, x = buf[:-1], y = buf[1:], rollover to
the next shard (mod #shards) when the next global window would overflow, ``reset()`` rewinds.

Differences: shards are memory-mapped instead of materialised as int64 in host
RAM.  With the native extension loaded (``backend="auto"``), batches come from the C++
``TokenLoader`` (csrc/runtime/token_loader.cpp): a producer thread assembles them ``prefetch``
batches ahead, straight into pinned memory when a GPU is present, so the training loop only issues
a non_blocking H2D copy.  ``backend="python"`` is the numpy path with identical semantics.
``SyntheticTokens`` is the no-dataset source used by bench.py / tests (BASELINE: synthetic data).
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np
import torch


def load_tokens(filename: str) -> torch.Tensor:
    npt = np.load(filename, mmap_mode="r")
    return torch.from_numpy(np.ascontiguousarray(npt).astype(np.int64, copy=False))


def _load_tokens_np(filename: str) -> np.ndarray:
    return np.load(filename, mmap_mode="r")


class DataLoaderLite:
    def __init__(self, B, T, process_rank, num_processes, split, master_process=True,
                 data_root: str = "edu_fineweb10B", verbose: bool = True, backend: str = "auto",
                 prefetch: int = 4, pin_memory: Optional[bool] = None):
        self.B = B
        self.T = T
        self.process_rank = process_rank
        self.num_processes = num_processes
        assert split in {"train", "val"}
        shards = sorted(s for s in os.listdir(data_root) if split in s)
        self.shards: List[str] = [os.path.join(data_root, s) for s in shards]
        assert len(self.shards) > 0, f"no shards found for split {split}"
        if master_process and verbose:
            print(f"found {len(self.shards)} shards for split {split}")
        assert backend in {"auto", "native", "python"}
        self._native = None
        if backend != "python":
            from ..ops import _ext
            if _ext.load():
                if pin_memory is None:
                    pin_memory = torch.cuda.is_available()
                self._native = torch.classes.mamba_amd.TokenLoader(
                    self.shards, B, T, process_rank, num_processes, prefetch, bool(pin_memory))
            elif backend == "native":
                raise RuntimeError(f"native TokenLoader unavailable: {_ext.error()}")
        self.backend = "native" if self._native is not None else "python"
        self.reset()

    def reset(self):
        if self._native is not None:
            self._native.reset()
            return
        self.current_shard = 0
        self.tokens = _load_tokens_np(self.shards[self.current_shard])
        self.current_position = self.B * self.T * self.process_rank

    # the reference attribute names stay readable on both backends
    def __getattr__(self, name):
        if name in ("current_shard", "current_position") and self.__dict__.get("_native") is not None:
            return self._native.state()[0 if name == "current_shard" else 1]
        raise AttributeError(name)

    def state_dict(self):
        return {"current_shard": self.current_shard, "current_position": self.current_position}

    def load_state_dict(self, s):
        if self._native is not None:
            self._native.set_state(int(s["current_shard"]), int(s["current_position"]))
            return
        self.current_shard = s["current_shard"]
        self.tokens = _load_tokens_np(self.shards[self.current_shard])
        self.current_position = s["current_position"]

    def next_batch(self):
        if self._native is not None:
            return self._native.next()
        B, T = self.B, self.T
        buf = torch.from_numpy(np.asarray(
            self.tokens[self.current_position: self.current_position + B * T + 1]).astype(np.int64))
        x = buf[:-1].view(B, T)
        y = buf[1:].view(B, T)
        self.current_position += B * T * self.num_processes
        if self.current_position + (B * T * self.num_processes + 1) > len(self.tokens):
            self.current_shard = (self.current_shard + 1) % len(self.shards)
            self.tokens = _load_tokens_np(self.shards[self.current_shard])
            self.current_position = B * T * self.process_rank
        return x, y


class SyntheticTokens:
    """Deterministic random tokens with the DataLoaderLite interface (no dataset on the box).

    Batches are generated on ``device`` directly (no H2D copy) from a per-rank seeded generator.
    """

    def __init__(self, B, T, vocab_size, process_rank=0, num_processes=1, device="cpu", seed=1234):
        self.B, self.T, self.V = B, T, vocab_size
        self.process_rank, self.num_processes = process_rank, num_processes
        self.device = torch.device(device)
        self.seed = seed
        self.reset()

    def reset(self):
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(self.seed + 7919 * self.process_rank)

    def next_batch(self):
        buf = torch.randint(0, self.V, (self.B * self.T + 1,), generator=self.gen, device=self.device)
        return buf[:-1].view(self.B, self.T), buf[1:].view(self.B, self.T)

    def state_dict(self):
        return {"generator": self.gen.get_state().cpu()}

    def load_state_dict(self, s):
        self.gen.set_state(s["generator"])


def markov_tokens(n: int, vocab_size: int, rng, p_follow: float = 0.75, zipf_a: float = 1.1,
                  succ: Optional[np.ndarray] = None, zipf_map: Optional[np.ndarray] = None) -> np.ndarray:
    """A LEARNABLE synthetic token stream: with probability ``p_follow`` the next token is a fixed
    successor of the previous one (a random permutation ``succ``), otherwise it is drawn from a Zipf
    unigram.  A model that learns the unigram and the successor map reaches a loss far below ln(V)
    (uniform random tokens cannot go below it), so training curves on it show real learning.
    Generated run-wise (runs of successors have geometric length), vectorised over runs."""
    if succ is None:
        succ = rng.permutation(vocab_size)
    ranks = np.arange(1, vocab_size + 1, dtype=np.float64)
    pz = ranks ** -zipf_a
    pz /= pz.sum()
    if zipf_map is None:
        zipf_map = rng.permutation(vocab_size)  # which token gets which Zipf rank
    # run lengths: 1 Zipf draw followed by Geometric(1 - p_follow) - 1 successors
    lens = rng.geometric(1.0 - p_follow, size=n // max(1, int(1 / (1 - p_follow))) + 16)
    while lens.sum() < n:
        lens = np.concatenate([lens, rng.geometric(1.0 - p_follow, size=len(lens))])
    lens = lens[: np.searchsorted(np.cumsum(lens), n) + 1]
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    out = np.empty(int(lens.sum()), dtype=np.int64)
    cur = zipf_map[rng.choice(vocab_size, size=len(lens), p=pz)]
    idx = starts.copy()
    alive = np.arange(len(lens))
    k = 0
    while len(alive):
        out[idx[alive]] = cur[alive]
        k += 1
        alive = alive[lens[alive] > k]
        cur[alive] = succ[cur[alive]]
        idx[alive] += 1
    return out[:n]


def write_synthetic_shards(root: str, n_train: int = 2, n_val: int = 1, tokens_per_shard: int = 1 << 16,
                           vocab_size: int = 50304, seed: int = 0, dtype=np.uint16,
                           kind: str = "uniform") -> List[str]:
    """Write edu_fineweb-style ``*_train_XXXXXX.npy`` / ``*_val_XXXXXX.npy`` shards.
    kind = "uniform": i.i.d. uniform tokens (throughput runs); "markov": ``markov_tokens`` (learning runs;
    every train and val shard shares the successor map and the unigram, i.e. one stationary source)."""
    os.makedirs(root, exist_ok=True)
    rng = np.random.default_rng(seed)
    succ = rng.permutation(vocab_size)
    zipf_map = rng.permutation(vocab_size)
    paths = []
    for split, n in (("val", n_val), ("train", n_train)):
        for i in range(n):
            p = os.path.join(root, f"edufineweb_{split}_{i:06d}.npy")
            if kind == "markov":
                toks = markov_tokens(tokens_per_shard, vocab_size, rng, succ=succ, zipf_map=zipf_map)
            else:
                toks = rng.integers(0, vocab_size, size=tokens_per_shard, dtype=np.int64)
            np.save(p, toks.astype(dtype))
            paths.append(p)
    return paths

