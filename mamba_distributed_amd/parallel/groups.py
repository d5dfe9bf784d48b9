"""Process groups for the parallel dimensions: data (DP), context (CP) and tensor (TP).

The reference is DDP-only (train.py:86).  Upstream mamba-ssm's Mamba2 accepts a
``process_group`` for head-sharded tensor parallelism (D18) and the SSD state hand-off is the
natural context-parallel hook (§5.7); this module lays the ranks out for both.

Layout (TP innermost, then CP, then DP)::

    global_rank = (dp_idx * cp + cp_idx) * tp + tp_idx

On one 8x MI355X node every GPU has a direct xGMI link to every other, so any group is a full
mesh; TP innermost keeps the per-layer activation collectives on consecutive GPU ids (and on one
node once jobs span several).  Gradients of parameters replicated over DP *and* CP (everything
under CP, the non-sharded params under TP) are averaged by DDP over ``dp_cp`` -- one bucketed
all-reduce per step, no extra collective for CP.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch.distributed as dist


@dataclass
class ParallelGroups:
    world: int
    rank: int
    tp: int
    cp: int
    dp: int
    tp_group: Optional[object] = None
    cp_group: Optional[object] = None
    dp_group: Optional[object] = None
    dp_cp_group: Optional[object] = None

    @property
    def tp_rank(self) -> int:
        return self.rank % self.tp

    @property
    def cp_rank(self) -> int:
        return (self.rank // self.tp) % self.cp

    @property
    def dp_rank(self) -> int:
        return self.rank // (self.tp * self.cp)


_GROUPS: Optional[ParallelGroups] = None


def init_parallel_groups(tp: int = 1, cp: int = 1) -> ParallelGroups:
    """Create the TP / CP / DP / DP x CP groups (collective: every rank must call it)."""
    global _GROUPS
    if not (dist.is_available() and dist.is_initialized()):
        assert tp == 1 and cp == 1, "tensor/context parallelism needs an initialised process group"
        _GROUPS = ParallelGroups(1, 0, 1, 1, 1)
        return _GROUPS
    world, rank = dist.get_world_size(), dist.get_rank()
    assert world % (tp * cp) == 0, f"world {world} not divisible by tp*cp = {tp * cp}"
    dp = world // (tp * cp)
    g = ParallelGroups(world, rank, tp, cp, dp)

    def rank_of(d, c, t):
        return (d * cp + c) * tp + t

    # new_group is collective over the WORLD: create every group on every rank, in one order
    for d in range(dp):
        for c in range(cp):
            ranks = [rank_of(d, c, t) for t in range(tp)]
            pg = dist.new_group(ranks)
            if rank in ranks:
                g.tp_group = pg
    for d in range(dp):
        for t in range(tp):
            ranks = [rank_of(d, c, t) for c in range(cp)]
            pg = dist.new_group(ranks)
            if rank in ranks:
                g.cp_group = pg
    for c in range(cp):
        for t in range(tp):
            ranks = [rank_of(d, c, t) for d in range(dp)]
            pg = dist.new_group(ranks)
            if rank in ranks:
                g.dp_group = pg
    for t in range(tp):
        ranks = [rank_of(d, c, t) for d in range(dp) for c in range(cp)]
        pg = dist.new_group(ranks)
        if rank in ranks:
            g.dp_cp_group = pg
    _GROUPS = g
    return g


def get_parallel_groups() -> ParallelGroups:
    global _GROUPS
    if _GROUPS is None:
        if dist.is_available() and dist.is_initialized():
            w = dist.get_world_size()
            _GROUPS = ParallelGroups(w, dist.get_rank(), 1, 1, w, dp_group=dist.group.WORLD,
                                     dp_cp_group=dist.group.WORLD)
        else:
            _GROUPS = ParallelGroups(1, 0, 1, 1, 1)
    return _GROUPS


def reset_parallel_groups() -> None:
    global _GROUPS
    _GROUPS = None
