"""Turn a (full, identically initialised) Mamba-2 LM into its TP / SP / CP form, and the optimizer-side
helpers those layouts need.

    groups = init_parallel_groups(tp=2, cp=2)            # after init_distributed()
    model  = LMHeadModel(cfg, device)                    # same seed on every rank
    parallelize(model, groups, sequence_parallel=True)   # in place
    ddp    = wrap_ddp(model, info, process_group=groups.dp_cp_group)
    ...
    loss.backward()
    sync_tp_grads(model, groups)                         # replicated-row / SP-replicated grads
    clip_grad_norm_(model, 1.0, groups)                  # TP-aware global norm
    full_sd = full_state_dict(model)                     # upstream layout, loads into a 1-GPU model

Data layout seen by ``LMHeadModel.forward``: every rank of a TP/CP group passes the *same* full
(b, T) batch; the model takes its own token shard (CP: the rank's contiguous T/cp slice; SP: the
rank's slice of the flattened b*T tokens).  The returned loss is the mean over this rank's tokens
(CP; DDP over DP x CP averages) or the TP-group mean (SP; identical on every TP rank).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from .comm import all_reduce_raw, group_size
from .groups import ParallelGroups


@dataclass
class ParallelContext:
    tp_group: Optional[object] = None
    cp_group: Optional[object] = None
    sequence_parallel: bool = False

    @property
    def tp(self) -> int:
        return group_size(self.tp_group)

    @property
    def cp(self) -> int:
        return group_size(self.cp_group)


def parallelize(model, groups: ParallelGroups, sequence_parallel: bool = False):
    """Shard every Mamba-2 mixer over ``groups.tp_group`` (heads) and/or mark it for context parallelism
    over ``groups.cp_group`` (sequence).  Call on every rank with identical full weights."""
    from ..models.mamba2 import Mamba2
    from .tensor_parallel import Mamba2TP
    tp_group = groups.tp_group if groups.tp > 1 else None
    cp_group = groups.cp_group if groups.cp > 1 else None
    if tp_group is None:
        sequence_parallel = False
    if tp_group is None and cp_group is None:
        return model
    for block in model.backbone.layers:
        mixer = block.mixer
        if tp_group is None and cp_group is None:
            continue
        if not isinstance(mixer, Mamba2):
            raise NotImplementedError("tensor / context parallelism is implemented for Mamba-2 mixers")
        if block.mlp is not None:
            raise NotImplementedError("TP/CP with d_intermediate > 0 (GatedMLP) is not supported")
        if tp_group is not None:
            mixer = Mamba2TP.from_full(mixer, tp_group, sequence_parallel)
            block.mixer = mixer
        mixer.cp_group = cp_group
    model.parallel = ParallelContext(tp_group, cp_group, sequence_parallel)
    model.backbone.parallel = model.parallel
    return model


def _ctx(model) -> Optional[ParallelContext]:
    m = getattr(model, "module", model)
    return getattr(m, "parallel", None)


@torch.no_grad()
def sync_tp_grads(model, groups: Optional[ParallelGroups] = None) -> None:
    """Sum over TP the gradients that are partial on each TP rank:
      * rows of TP-sharded params that every rank holds in full (``_tp_rep_rows``: the ngroups=1 B/C
        projections), and
      * under sequence parallelism, every non-sharded parameter (block norms, norm_f, embedding /
        tied lm_head) -- each rank saw only its token shard.
    One flattened all-reduce per call (a single RCCL launch)."""
    ctx = _ctx(model)
    if ctx is None or ctx.tp == 1:
        return
    m = getattr(model, "module", model)
    views = []
    for p in m.parameters():
        if p.grad is None:
            continue
        rows = getattr(p, "_tp_rep_rows", None)
        if rows is not None:
            views.append(p.grad[rows[0]:rows[1]])
        elif ctx.sequence_parallel and not getattr(p, "_tp_sharded", False):
            views.append(p.grad)
    if not views:
        return
    flat = torch.cat([v.reshape(-1).float() for v in views])
    all_reduce_raw(flat, ctx.tp_group)
    off = 0
    for v in views:
        n = v.numel()
        v.copy_(flat[off:off + n].view_as(v))
        off += n


@torch.no_grad()
def grad_norm(model) -> torch.Tensor:
    """Global L2 norm of the gradients of a (possibly TP-sharded) model: sharded params are summed
    over TP, replicated rows / params counted once (of the data-parallel AVERAGE: a deferred 1/world is applied)."""
    from .ddp import averaged_grads
    averaged_grads(model)
    m = getattr(model, "module", model)
    ctx = _ctx(model)
    tp = ctx.tp if ctx is not None else 1
    dev = next(m.parameters()).device
    shard_sq = torch.zeros((), device=dev, dtype=torch.float32)
    rep_sq = torch.zeros((), device=dev, dtype=torch.float32)
    for p in m.parameters():
        if p.grad is None:
            continue
        g = p.grad.float()
        if tp > 1 and getattr(p, "_tp_sharded", False):
            sq = g.pow(2).sum()
            rows = getattr(p, "_tp_rep_rows", None)
            if rows is not None:  # replicated rows appear on every TP rank: count them once
                sq = sq - g[rows[0]:rows[1]].pow(2).sum() * (1.0 - 1.0 / tp)
            shard_sq += sq
        else:
            rep_sq += g.pow(2).sum()
    if tp > 1:
        all_reduce_raw(shard_sq, ctx.tp_group)
        shard_sq = shard_sq.reshape(())
    return torch.sqrt(shard_sq + rep_sq)


@torch.no_grad()
def clip_grad_norm_(model, max_norm: float, groups: Optional[ParallelGroups] = None) -> torch.Tensor:
    """TP-aware ``torch.nn.utils.clip_grad_norm_`` (identical to it when tp == 1)."""
    from .ddp import averaged_grads
    averaged_grads(model)  # a deferred data-parallel 1/world average (parallel/reducer.py) is applied first
    ctx = _ctx(model)
    if ctx is None or ctx.tp == 1:
        m = getattr(model, "module", model)
        return torch.nn.utils.clip_grad_norm_(m.parameters(), max_norm)
    total = grad_norm(model)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    m = getattr(model, "module", model)
    grads = [p.grad for p in m.parameters() if p.grad is not None]
    torch._foreach_mul_(grads, coef.to(grads[0].device))
    return total


@torch.no_grad()
def full_state_dict(model) -> dict:
    """Upstream-layout state dict of a parallelized model, on every rank (collective
    over TP).  Loads into an unsharded ``LMHeadModel`` of the same config."""
    from .tensor_parallel import Mamba2TP
    m = getattr(model, "module", model)
    sd = {k: v for k, v in m.state_dict().items()}
    for name, mod in m.named_modules():
        if isinstance(mod, Mamba2TP):
            pre = name + "."
            for k in [k for k in sd if k.startswith(pre)]:
                del sd[k]
            sd.update(mod.full_state_dict(pre))
    return sd


def shard_batch(model, x: torch.Tensor) -> torch.Tensor:
    """The slice of a full (b, T) batch tensor this rank computes on (what ``forward`` does to its
    inputs and targets internally) -- for callers that evaluate per-token quantities."""
    ctx = _ctx(model)
    if ctx is None:
        return x
    from .comm import split_along
    from .context_parallel import shard_sequence
    x = shard_sequence(x, ctx.cp_group, dim=1)
    if ctx.sequence_parallel:
        x = split_along(x.reshape(-1), ctx.tp_group, 0)
    return x.contiguous()

