"""Autograd-aware collectives for tensor / sequence / context parallelism.

Upstream mamba-ssm reaches these through ``mamba_ssm/distributed/distributed_utils.py``
(``all_gather_raw``, ``reduce_scatter_raw``, ``all_reduce_raw`` and the ``AllGatherFunc`` /
``ReduceScatterFunc`` / ``AllReduceFunc`` autograd wrappers).  The reference itself
never calls them (it is DDP-only), so they are a capability of the framework, not a parity item.

MI355X-first choices:
  * one communicator per parallel dimension (``parallel/groups.py``); on the 8-GPU xGMI mesh a TP or
    CP group of <= 8 ranks is a full mesh, so RCCL's all-gather / reduce-scatter run over direct
    links -- the large activation collectives use the ``*_into_tensor`` / ``*_tensor`` single-buffer
    forms (no list of per-rank tensors, no extra copy);
  * every op also runs on gloo (CPU tests, the BASELINE "tiny gloo world=2" config): gloo lacks
    reduce-scatter, so it is all-reduce + slice there.

All ops treat a ``None`` group or a group of size 1 as the identity.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


def group_size(group) -> int:
    if group is None or not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def group_rank(group) -> int:
    if group is None or not (dist.is_available() and dist.is_initialized()):
        return 0
    return dist.get_rank(group)


def _is_nccl(group) -> bool:
    return dist.get_backend(group) == "nccl"


# ---------------------------------------------------------------------------------------------
# raw (non-autograd) primitives
# ---------------------------------------------------------------------------------------------
def all_reduce_raw(x: torch.Tensor, group, op=dist.ReduceOp.SUM) -> torch.Tensor:
    x = x.contiguous()
    dist.all_reduce(x, op=op, group=group)
    return x


def all_gather_raw(x: torch.Tensor, group, dim: int = 0) -> torch.Tensor:
    """Concatenate every rank's ``x`` along ``dim`` (rank order)."""
    ws = group_size(group)
    if ws == 1:
        return x
    x = x.contiguous()
    if _is_nccl(group) and dim == 0:
        out = torch.empty((ws * x.shape[0], *x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x, group=group)
        return out
    parts = [torch.empty_like(x) for _ in range(ws)]
    dist.all_gather(parts, x, group=group)
    return torch.cat(parts, dim=dim)


def reduce_scatter_raw(x: torch.Tensor, group, dim: int = 0) -> torch.Tensor:
    """Sum over ranks, then keep this rank's 1/ws slice along ``dim``."""
    ws = group_size(group)
    if ws == 1:
        return x
    assert x.shape[dim] % ws == 0, (x.shape, dim, ws)
    n = x.shape[dim] // ws
    r = group_rank(group)
    if _is_nccl(group) and dim == 0:
        x = x.contiguous()
        out = torch.empty((n, *x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.reduce_scatter_tensor(out, x, group=group)
        return out
    x = all_reduce_raw(x.clone(), group)
    return x.narrow(dim, r * n, n).contiguous()


# ---------------------------------------------------------------------------------------------
# autograd wrappers (Megatron-style f / g operators)
# ---------------------------------------------------------------------------------------------
class _CopyToGroup(torch.autograd.Function):
    """fwd identity, bwd all-reduce(sum): input replicated on every rank, consumed by sharded work."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        return all_reduce_raw(g.clone(), ctx.group), None


class _ReduceFromGroup(torch.autograd.Function):
    """fwd all-reduce(sum), bwd identity: partial sums -> replicated total."""

    @staticmethod
    def forward(ctx, x, group):
        return all_reduce_raw(x.clone(), group)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _AllReduceSym(torch.autograd.Function):
    """fwd all-reduce(sum), bwd all-reduce(sum): a sum whose result every rank uses in its own
    (rank-local) loss term, e.g. the sum-of-squares of a norm whose group spans TP ranks."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return all_reduce_raw(x.clone(), group)

    @staticmethod
    def backward(ctx, g):
        return all_reduce_raw(g.clone(), ctx.group), None


class _GatherAlong(torch.autograd.Function):
    """fwd all-gather along dim, bwd reduce-scatter along dim (sequence-parallel entry)."""

    @staticmethod
    def forward(ctx, x, group, dim):
        ctx.group, ctx.dim = group, dim
        return all_gather_raw(x, group, dim)

    @staticmethod
    def backward(ctx, g):
        return reduce_scatter_raw(g, ctx.group, ctx.dim), None, None


class _ReduceScatterAlong(torch.autograd.Function):
    """fwd reduce-scatter along dim, bwd all-gather along dim (sequence-parallel exit)."""

    @staticmethod
    def forward(ctx, x, group, dim):
        ctx.group, ctx.dim = group, dim
        return reduce_scatter_raw(x, group, dim)

    @staticmethod
    def backward(ctx, g):
        return all_gather_raw(g, ctx.group, ctx.dim), None, None


class _GatherAlongSumGrad(torch.autograd.Function):
    """fwd all-gather along dim, bwd: each rank's slice of the gradient summed over ranks.  Used for
    small per-rank values (context-parallel boundary states / conv halos) that every rank reads."""

    @staticmethod
    def forward(ctx, x, group, dim):
        ctx.group, ctx.dim, ctx.n = group, dim, x.shape[dim]
        return all_gather_raw(x, group, dim)

    @staticmethod
    def backward(ctx, g):
        g = all_reduce_raw(g.clone(), ctx.group)
        return g.narrow(ctx.dim, group_rank(ctx.group) * ctx.n, ctx.n).contiguous(), None, None


def copy_to_group(x, group):
    return x if group_size(group) == 1 else _CopyToGroup.apply(x, group)


def reduce_from_group(x, group):
    return x if group_size(group) == 1 else _ReduceFromGroup.apply(x, group)


def all_reduce_sym(x, group):
    return x if group_size(group) == 1 else _AllReduceSym.apply(x, group)


def gather_along(x, group, dim: int = 0):
    return x if group_size(group) == 1 else _GatherAlong.apply(x, group, dim)


def reduce_scatter_along(x, group, dim: int = 0):
    return x if group_size(group) == 1 else _ReduceScatterAlong.apply(x, group, dim)


def all_gather_small(x, group, dim: int = 0):
    return x if group_size(group) == 1 else _GatherAlongSumGrad.apply(x, group, dim)


def split_along(x: torch.Tensor, group, dim: int = 0) -> torch.Tensor:
    """This rank's contiguous 1/ws slice along ``dim`` (no communication; gradient stays local)."""
    ws = group_size(group)
    if ws == 1:
        return x
    assert x.shape[dim] % ws == 0, (x.shape, dim, ws)
    n = x.shape[dim] // ws
    return x.narrow(dim, group_rank(group) * n, n)


def broadcast_tensors(tensors, src_group_rank: int, group: Optional[object]):
    """In-place broadcast from group rank ``src_group_rank`` (used to make replicated params equal)."""
    if group_size(group) == 1:
        return
    src = dist.get_global_rank(group, src_group_rank)
    for t in tensors:
        dist.broadcast(t.data, src=src, group=group)
