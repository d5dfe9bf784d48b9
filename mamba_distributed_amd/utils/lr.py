"""LR schedule of the reference (train.py:89-110): linear warmup, cosine decay, floor."""
import math


def get_lr(it: int, max_lr: float = 6e-4, min_lr: float = 6e-5, warmup_steps: int = 715,
           max_steps: int = 19073) -> float:
    if it < warmup_steps:
        return max_lr * (it + 1) / warmup_steps
    if it > max_steps:
        return min_lr
    decay_ratio = (it - warmup_steps) / (max_steps - warmup_steps)
    assert 0 <= decay_ratio <= 1
    coeff = 0.5 * (1.0 + math.cos(math.pi * decay_ratio))
    return min_lr + coeff * (max_lr - min_lr)
