"""Data parallelism over RCCL / xGMI (reference train.py:86, 209-221).

The reference wraps the model in torch DDP with defaults (25 MB buckets).  On one 8x MI355X node
the GPUs form a fully connected xGMI mesh (7 links x ~153 GB/s per GPU).  RCCL's ring
all-reduce is per-link bound, so for the 1.12 GB fp32 gradient of the 280M model the
all-reduce itself costs ~6-13 ms — small next to a 300+ ms step — and what matters is (a) that it
overlaps the LAST micro-step's backward and (b) that the per-collective launch latency is
amortised.  Defaults chosen for that regime:

  * ``bucket_cap_mb=100``  (4x fewer collectives than 25 MB; a 100 MB bucket moves in
    ~0.5-1 ms over xGMI, still much shorter than the backward of the 64 layers it overlaps)
  * ``gradient_as_bucket_view=True``  (grads live in the buckets: no copy in / copy out)
  * ``static_graph`` off: validation / sampling run no-grad forwards through the same wrapper
  * optional bf16 compression hook (``grad_comm_dtype="bf16"``) halves the bytes on the links.

Gradient accumulation uses ``require_backward_grad_sync`` exactly like the reference
(train.py:209-210): only the last micro-step's backward launches the bucketed all-reduce.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as DDP

from .dist import DistInfo


def wrap_ddp(model: torch.nn.Module, info: DistInfo, bucket_cap_mb: float = 100.0,
             grad_comm_dtype: str = "fp32", static_graph: bool = False,
             gradient_as_bucket_view: bool = True, process_group=None):
    """DDP over ``process_group`` (default: WORLD; the DP x CP group under tensor / context
    parallelism, parallel/groups.py)."""
    if not info.ddp:
        return model
    device_ids = [info.local_rank] if info.device.startswith("cuda") else None
    m = DDP(model, device_ids=device_ids, bucket_cap_mb=bucket_cap_mb,
            gradient_as_bucket_view=gradient_as_bucket_view, static_graph=static_graph,
            broadcast_buffers=False, process_group=process_group)
    hook_group = process_group if process_group is not None else dist.group.WORLD
    if grad_comm_dtype == "bf16":
        from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
        m.register_comm_hook(hook_group, default_hooks.bf16_compress_hook)
    elif grad_comm_dtype == "fp16":
        from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
        m.register_comm_hook(hook_group, default_hooks.fp16_compress_hook)
    return m


def wrap_data_parallel(model: torch.nn.Module, info: DistInfo, impl: str = "native", bucket_cap_mb: float = 100.0,
                       grad_comm_dtype: str = "fp32", process_group=None):
    """Data-parallel wrapper: ``impl="native"`` -> parallel/reducer.py (flat gradient buffer,
    explicitly armed buckets; lets every micro-batch forward overlap the previous backward),
    ``impl="ddp"`` -> torch DDP exactly as the reference uses it."""
    if not info.ddp:
        return model
    if impl == "native":
        from .reducer import wrap_reducer
        return wrap_reducer(model, process_group, bucket_cap_mb, grad_comm_dtype)
    assert impl == "ddp", impl
    return wrap_ddp(model, info, bucket_cap_mb, grad_comm_dtype, process_group=process_group)


def _reducer(model):
    from .reducer import ReducedModule
    return model.reducer if isinstance(model, ReducedModule) else None


def unwrap(model):
    from .reducer import ReducedModule
    return model.module if isinstance(model, (DDP, ReducedModule)) else model


def zero_grad(model, optimizer) -> None:
    """Start of an optimizer step: the native reducer keeps .grad as views of its flat buffer and
    zeroes that; otherwise gradients are dropped (set_to_none) like the reference."""
    r = _reducer(model)
    if r is not None:
        r.zero_grad()
    elif optimizer is not None:
        optimizer.zero_grad(set_to_none=True)
    else:
        model.zero_grad(set_to_none=True)


def set_grad_sync(model, enabled: bool):
    """Per micro-step: True only on the last one (reference train.py:209-210).  Also tells the native
    ops whether they may accumulate parameter gradients in place (ops/grad_accum.py).  With the
    native reducer, True arms its bucket hooks for the next backward; call ``finish_grad_sync``
    after that backward."""
    from ..ops import grad_accum
    grad_accum.set_direct(not enabled)
    if isinstance(model, DDP):
        model.require_backward_grad_sync = enabled
    r = _reducer(model)
    if r is not None and enabled:
        r.arm()


def configure_grad_average(model, optimizer) -> bool:
    """Once, before the first optimizer step: with the native reducer, fp32 collectives and the native AdamW as the
    gradient consumer, the reducer leaves the all-reduced gradients SUMMED (``reducer.grad_divisor = world``) and
    ``clip_and_step`` hands that divisor to the optimizer, which folds it into its clip coefficient.  Every step takes
    the same path.  Returns whether the average is deferred.  Any other consumer (a torch optimizer, the TP clip,
    ``averaged_grads``) divides first (``materialize_average``)."""
    from ..ops.optim import NativeAdamW
    r = _reducer(model)
    if r is None:
        return False
    r.defer_average = isinstance(optimizer, NativeAdamW) and r.world > 1 and r.comm_dtype is None
    return r.defer_average


def averaged_grads(model) -> None:
    """Make every ``.grad`` hold the data-parallel AVERAGE (a deferred 1/world is applied now): call before reading
    gradients outside clip_and_step (logging a norm, a custom optimizer, hooks)."""
    r = _reducer(model)
    if r is not None:
        r.materialize_average()


def clip_grad_norm_(model, max_norm: float) -> torch.Tensor:
    """``torch.nn.utils.clip_grad_norm_`` (reference train.py:222).  Under the native reducer every
    gradient is a view into one flat fp32 buffer, so the global 2-norm and the rescale are one
    reduction and one scale kernel over that buffer instead of per-tensor foreach launches (a deferred
    1/world average is applied first)."""
    r = _reducer(model)
    if r is None:
        return torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm)
    r.materialize_average()
    total = torch.linalg.vector_norm(r.flat, 2.0)
    r.flat.mul_(torch.clamp(max_norm / (total + 1e-6), max=1.0))
    return total


def clip_and_step(model, optimizer, max_norm: float) -> torch.Tensor:
    """``clip_grad_norm_(model, max_norm)`` then ``optimizer.step()`` (reference train.py:222, :227).  With the
    native AdamW (ops/optim.py) the two are one norm pass and one update pass with the clip coefficient folded into
    the update's gradient read; a deferred 1/world average (configure_grad_average) rides on the same coefficient,
    passed explicitly from the reducer's ``grad_divisor`` on every step.  The returned norm is always the norm of
    the AVERAGED gradients."""
    from ..ops.optim import NativeAdamW
    if not isinstance(optimizer, NativeAdamW):
        norm = clip_grad_norm_(model, max_norm)  # materialises a deferred average first
        optimizer.step()
        return norm
    r = _reducer(model)
    return optimizer.clip_and_step(max_norm, grad_divisor=r.grad_divisor if r is not None else 1.0)


def finish_grad_sync(model) -> None:
    """Wait for the native reducer's bucket all-reduces (no-op for DDP / single process)."""
    r = _reducer(model)
    if r is not None:
        r.finish()


def params_in_sync(model, atol: float = 0.0) -> bool:
    """Debug / test helper: every rank holds bit-identical parameters (max-abs-diff over ranks)."""
    if not (dist.is_available() and dist.is_initialized()):
        return True
    ok = torch.ones(1, device=next(model.parameters()).device)
    for p in unwrap(model).parameters():
        ref = p.detach().clone()
        dist.broadcast(ref, src=0)
        if (ref - p.detach()).abs().max().item() > atol:
            ok.zero_()
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    return bool(ok.item() == 1)
