"""Gradient-accumulation loop with the next micro-batch's forward overlapped on a second HIP stream.

The reference runs its micro-steps strictly one after the other (train.py:205-219).  Within one
optimizer step the weights are frozen, so micro-batch k+1's forward depends on nothing that micro-batch
k's backward produces.  Here it is enqueued on a second stream right before backward k, so the
GEMM- and MFMA-heavy forward fills the CUs the memory- and latency-bound backward kernels (norms,
conv, scan) leave idle:

    stream A:  fwd0 | bwd0 ......... | fwd2 | (wait bwd1) bwd2 ...
    stream B:       | (wait fwd0) fwd1 | (wait bwd0) bwd1 | fwd3 ...

Ordering rules, each enforced with one stream wait:
  * the other stream waits for the caller's stream on entry (the previous optimizer step);
  * backward k waits for backward k-1 (they accumulate into the same ``p.grad``), captured BEFORE
    forward k+1 is enqueued behind backward k-1, so forward k+1 still runs beside backward k;
  * forward 1 waits for forward 0, which builds the step's bf16 weight casts (ops/grad_accum.py);
  * the last micro-step runs on the caller's stream; under torch DDP its forward (which arms the
    gradient-reduction hooks) is only issued after every earlier backward has been enqueued; the
    native reducer (parallel/reducer.py) is armed right before the last backward instead, so with
    it every forward -- the sync one included -- overlaps the previous backward;
  * the caller's stream waits for the other stream before returning.
Every micro-step's reductions happen in the same order as in the sequential loop, so the gradients
are bitwise identical (tests/test_kernels_gpu.py::test_microbatch_overlap_is_bitwise_identical).
"""
from __future__ import annotations

from typing import Callable, Dict

import torch

from ..ops import grad_accum

_OTHER: Dict[int, "torch.cuda.Stream"] = {}


def _is_ddp(model) -> bool:
    from torch.nn.parallel import DistributedDataParallel as DDP
    return isinstance(model, DDP)


def _set_ddp_sync(model, enabled: bool) -> None:
    if _is_ddp(model):
        model.require_backward_grad_sync = enabled


def _reducer(model):
    from .reducer import ReducedModule
    return model.reducer if isinstance(model, ReducedModule) else None


def auto_micro_batch(cfg, seqs_per_rank: int, seq_len: int) -> int:
    """Micro-batch (sequences) for a rank that processes ``seqs_per_rank`` sequences per optimizer step; the
    global batch and the gradient are the same for any choice (the loss is averaged over all micro-batches).
    Measured on one MI355X at Mamba-2 280M, T = 1024 (profiles/r3/ab5_micro_batch.txt): 64 sequences
    without the overlap match 32 with it at grad-accum 16 (289.6k vs 289.5k tok/s, same 128 GB peak) and
    beat it in the 8-GPU per-rank regime (65,536 tokens per rank: one micro-batch of 64 at 282k vs two of 32
    at 264k, which leaves the second backward with nothing to overlap).  Wider models keep 32 (their
    activations at 64 would not fit next to a second micro-batch, and the 1.4B GEMMs already fill the chip)."""
    best = 64 if getattr(cfg, "d_model", 0) <= 1024 and seq_len <= 1024 else 32
    while best > 1 and (best > seqs_per_rank or seqs_per_rank % best):
        best //= 2
    return max(1, best)


def auto_overlap(cfg, micro_tokens: int = 32768) -> bool:
    """Default for the two-stream micro-batch overlap, by model width.  Measured on one MI355X
    (interleaved runs, native wgrad side stream on): Mamba-2 280M 262k -> 275k tok/s with overlap,
    Mamba-1 280M / 370M +0.4% / +1.3%, but Mamba-2 1.4B (d_model 2048) 91k -> 67k: its GEMMs already
    fill the chip, and a second forward stream beside the backward and its side-stream weight-gradient
    GEMMs only thrashes the caches.  So: on for d_model <= 1024, and only up to 32k-token micro-batches: two
    micro-batches of 64 x 1024 in flight peak at 241 GB and run at 109k tok/s (allocator pressure) against
    290k for one at a time (profiles/r3/ab5_micro_batch.txt)."""
    return getattr(cfg, "d_model", 0) <= 1024 and micro_tokens <= 32768


def auto_defer_reduce(cfg) -> bool:
    """Default for the deferred partial reductions (ops/grad_accum.py::deferred), by model width.  Round 3 measured
    Mamba-2 1.4B at 88k -> 41k and Mamba-1 280M -1% with deferral: both were the allocator pressure of the side
    stream's record_stream lifetimes, gone since the stream-ordered keep-alive (ops/grad_accum.py::side_keep).
    Re-measured on one MI355X, interleaved (profiles/r5/defer_reduce_ab.txt): 1.4B +0.5% (172.8 vs 148.8 GB
    reserved), Mamba-1 280M +0.5%.  So: on up to d_model 2048; off above (2.8B, whose persistent fp32 K-split slabs
    would add ~30 GB to a 230 GB peak)."""
    return getattr(cfg, "d_model", 0) <= 2048


def resolve_overlap(mode, cfg, micro_tokens: int = 32768) -> bool:
    """``mode``: "auto" (auto_overlap), "on"/"off", or a bool."""
    if isinstance(mode, bool):
        return mode
    mode = str(mode).lower()
    if mode == "auto":
        return auto_overlap(cfg, micro_tokens)
    if mode in ("on", "true", "1", "yes"):
        return True
    if mode in ("off", "false", "0", "no"):
        return False
    raise ValueError(f"overlap mode must be auto/on/off, got {mode!r}")


def run_micro_batches(model, next_batch: Callable, accum: int, compute_loss: Callable,
                      overlap: bool = True) -> torch.Tensor:
    """Forward + backward of ``accum`` micro-batches for ONE optimizer step; returns the summed
    (already 1/accum-scaled by ``compute_loss``) loss as an fp32 scalar tensor.

    ``next_batch() -> (x, y)``; ``compute_loss(x, y) -> loss`` runs the forward (with autocast).
    Must be called inside ``grad_accum.accumulation_scope()``.  With the native reducer
    (parallel/reducer.py) the gradients are averaged over the data-parallel group on return."""
    cuda = torch.cuda.is_available() and torch.cuda.is_initialized()
    reducer = _reducer(model)
    if not overlap or not cuda or accum < 2:
        total = None
        for k in range(accum):
            sync = k == accum - 1
            _set_ddp_sync(model, sync)
            grad_accum.set_direct(not sync)
            x, y = next_batch()
            loss = compute_loss(x, y)
            total = loss.detach().float() if total is None else total + loss.detach().float()
            if sync and reducer is not None:
                reducer.arm()
            if sync:
                grad_accum.set_late(not _is_ddp(model))
            loss.backward()
        if reducer is not None:
            reducer.finish()
        grad_accum.flush_late()
        grad_accum.set_late(False)
        return total
    ddp = _is_ddp(model)
    main = torch.cuda.current_stream()
    dev = main.device.index if main.device.index is not None else torch.cuda.current_device()
    other = _OTHER.get(dev)
    if other is None:
        # same priority as the caller's stream (a high-priority compute stream makes both micro-batch
        # streams outrank the weight-gradient side stream, ops/grad_accum.py)
        other = _OTHER[dev] = torch.cuda.Stream(device=dev, priority=main.priority)
    streams = [main if (accum - 1 - k) % 2 == 0 else other for k in range(accum)]
    # everything the caller queued on ``main`` (the previous optimizer step updating the weights and
    # reading the gradients that zero_grad just released) precedes the first forward when that runs
    # on the other stream (even ``accum``): without this wait, blocks freed by zero_grad are handed
    # to forward 0's activations while AdamW may still be reading them as gradients
    other.wait_stream(main)
    # A leaf's AccumulateGrad node lives as long as any in-flight graph holds it, so with two
    # micro-batch graphs alive at once it was usually created on the other stream; autograd then
    # accumulates on that stream behind an event wait on the producer.  That is ordered (see the
    # module docstring's bitwise test) and adds no wait beyond "backward k after backward k-1": silence the
    # per-backward warning torch emits about it.
    _quiet = getattr(torch.autograd.graph, "set_warn_on_accumulate_grad_stream_mismatch", None)
    if _quiet is not None:
        _quiet(False)
    losses = [None] * accum

    def forward(k):
        with torch.cuda.stream(streams[k]):
            _set_ddp_sync(model, k == accum - 1)
            x, y = next_batch()
            losses[k] = compute_loss(x, y)

    forward(0)
    streams[1].wait_stream(streams[0])  # forward 0 built the step's cached weight casts
    for k in range(accum):
        nxt = k + 1
        if k > 0:
            streams[k].wait_stream(streams[k - 1])  # after backward k-1 (forward k+1 is not queued yet)
        early = nxt < accum and (not ddp or nxt < accum - 1)
        if early:
            forward(nxt)  # on streams[k-1] (or the other stream for k = 0): beside backward k
        grad_accum.set_direct(k != accum - 1)
        if k == accum - 1 and reducer is not None:
            reducer.arm()
        if k == accum - 1:
            # the sync backward leaves its small parameter-gradient partials for ONE batched column sum after it
            # (ops/grad_accum.py::flush_late; not under torch DDP, whose hooks would reduce the missing gradients)
            grad_accum.set_late(not ddp)
        with torch.cuda.stream(streams[k]):
            losses[k].backward()
        if nxt < accum and not early:
            # DDP's sync forward arms the reducer hooks: only after every earlier backward is queued
            streams[nxt].wait_stream(streams[k])
            forward(nxt)
    main.wait_stream(other)
    if reducer is not None:
        reducer.finish()
    grad_accum.flush_late()
    grad_accum.set_late(False)
    total = losses[0].detach().float()
    for l in losses[1:]:
        total = total + l.detach().float()
    return total
