"""Native bucketed gradient all-reduce (the framework's replacement for torch DDP's reducer).

Reference: ``DDP(model, device_ids=[local_rank])`` with default 25 MB buckets (train.py:86; SURVEY.md
§2.6-2.7, C2-C3).  Same semantics -- parameters broadcast from rank 0 once, gradients averaged over
the data-parallel group with bucketed all-reduces that overlap the last micro-step's backward -- but
built around how this framework accumulates gradients:

  * every parameter's ``.grad`` is a persistent view into ONE flat fp32 buffer laid out in reverse
    registration order (about the order the backward produces them), so a bucket is a contiguous
    slice of it: the all-reduce runs in place, with no copy into or out of bucket storage;
  * the micro-steps accumulate straight into those views (ops/grad_accum.py's in-place weight
    gradients and batched adds); ``zero_grad`` zeroes the buffer;
  * the bucket hooks are armed explicitly for the sync micro-step only (``arm``).  Unlike DDP's
    forward-armed reducer this lets the next micro-batch's forward -- including the sync one -- run
    on a second stream beside the previous backward (parallel/microbatch.py), at every DP size;
  * buckets launch strictly in index order on every rank (a bucket completes -> every consecutive
    ready bucket from the next unlaunched one is launched), so ranks issue identical collective
    sequences.  ``bucket_cap_mb`` defaults to 100 MB: on the 8-GPU xGMI mesh a 100 MB all-reduce
    is well into the bandwidth-bound regime (scripts/comm_bench.py), and ~11 buckets for the 280M
    model keep the exposed tail (the last bucket after the backward ends) short.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist


def held_param(p: torch.Tensor) -> bool:
    """The parameters whose gradients the sync micro-step may produce AFTER the backward, in the batched late column
    sum (ops/grad_accum.py::flush_late): the small non-matrix ones -- norm weights, conv taps / bias, A_log / D /
    dt_bias.  Their buckets are held until finish(); every other parameter's bucket launches from the backward's
    hooks (small 2-D weights such as Mamba-1's x_proj / dt_proj included, so they keep overlapping the backward)."""
    return p.numel() < GradReducer.SMALL_NUMEL and p.dim() != 2


class GradReducer:
    SMALL_NUMEL = 1 << 17

    def __init__(self, module: torch.nn.Module, process_group=None, bucket_cap_mb: float = 100.0,
                 broadcast_params: bool = True, comm_dtype: str = "fp32"):
        self.group = process_group
        # "bf16" / "fp16": each bucket is pre-divided by the world size and cast before the
        # all-reduce (half the bytes on the links), like DDP's bf16/fp16 compress hooks
        self.comm_dtype = {"fp32": None, "bf16": torch.bfloat16, "fp16": torch.float16}[comm_dtype]
        self.world = dist.get_world_size(process_group)
        params = [p for p in module.parameters() if p.requires_grad]
        assert params, "no trainable parameters"
        dtypes = {p.dtype for p in params}
        assert dtypes == {torch.float32}, f"GradReducer keeps fp32 gradients for fp32 parameters, got {dtypes}"
        # the held parameters (held_param: norm weights, conv taps, A_log / D / dt_bias) go last, in buckets of their
        # own that are HELD until finish(): on the sync micro-step their gradients come from the batched late column
        # sum after the backward (ops/grad_accum.py::flush_late), so their hooks fire before the gradients exist.  A
        # few MB per model, all-reduced once at the end.  grad_accum.late_ok refuses any other parameter.
        order = [p for p in reversed(params) if not held_param(p)]
        small = [p for p in reversed(params) if held_param(p)]
        total = sum(p.numel() for p in params)
        self.flat = torch.zeros(total, dtype=torch.float32, device=params[0].device)
        cap = max(1, int(bucket_cap_mb * 2**20 / 4))
        self.buckets: List[tuple] = []  # (start, end, n_params)
        self._bucket_of: Dict[int, int] = {}
        self._offset: Dict[int, int] = {}
        off, start, count = 0, 0, 0
        self._held_from = None
        for p in order + small:
            if p is (small[0] if small else None) and count:
                self.buckets.append((start, off, count))  # bucket boundary before the held small parameters
                start, count = off, 0
            if p is (small[0] if small else None):
                self._held_from = len(self.buckets)
            self._offset[id(p)] = off
            self._bucket_of[id(p)] = len(self.buckets)
            off += p.numel()
            count += 1
            if off - start >= cap:
                self.buckets.append((start, off, count))
                start, count = off, 0
        if count:
            self.buckets.append((start, off, count))
        if self._held_from is None:
            self._held_from = len(self.buckets)
        self._params = params
        from ..ops import grad_accum
        grad_accum.register_held([p for p in params if held_param(p)])
        for p in params:
            self._attach(p)
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in params]
        self._armed = False
        # The 1/world average.  finish() multiplies the summed gradients by 1/world unless ``defer_average`` is set
        # (parallel/ddp.py::configure_grad_average, once, before the first step, when the consumer is the native
        # AdamW: it folds the factor into its clip coefficient, one full pass over the buffer less per step).
        # ``grad_divisor`` is the explicit state of .grad: the gradients in the flat buffer are the data-parallel
        # average times grad_divisor (1.0, or world after a deferred finish) until the next zero_grad.  Consumers go
        # through parallel/ddp.py (clip_grad_norm_ / clip_and_step / averaged_grads), which divide or materialise.
        self.defer_average = False
        self.grad_divisor = 1.0
        self._main = None  # the stream that called arm() (the caller's / main micro-batch stream)
        # exposed all-reduce time per sync step: stream time from the end of the last backward
        # (finish() entry, in stream order) to the averaged gradients being ready (finish() exit)
        self.timing = False
        self._exposed: List[tuple] = []
        self._left: List[int] = []
        self._next = 0
        self._works = []
        if broadcast_params and self.world > 1:
            src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
            with torch.no_grad():
                for p in module.parameters():
                    dist.broadcast(p.data, src=src, group=process_group)
                for b in module.buffers():
                    dist.broadcast(b.data, src=src, group=process_group)

    def _attach(self, p) -> None:
        off = self._offset[id(p)]
        p.grad = self.flat[off:off + p.numel()].view_as(p)

    # ------------------------------------------------------------------------------------------
    def zero_grad(self) -> None:
        """Zero every gradient, keeping (or restoring) the .grad views into the flat buffer."""
        base = self.flat.data_ptr()
        for p in self._params:
            if p.grad is None or p.grad.data_ptr() != base + 4 * self._offset[id(p)]:
                self._attach(p)
        self.flat.zero_()
        self.grad_divisor = 1.0

    def materialize_average(self) -> None:
        """Make .grad hold the averaged gradients (divide a deferred 1/world now)."""
        if self.grad_divisor != 1.0:
            self.flat.mul_(1.0 / self.grad_divisor)
            self.grad_divisor = 1.0

    def arm(self) -> None:
        """Call right before the sync micro-step's backward: its gradient hooks launch the buckets."""
        self._main = torch.cuda.current_stream(self.flat.device) if self.flat.is_cuda else None
        self._armed = True
        self._left = [n for _, _, n in self.buckets]
        self._next = 0
        self._works = []

    def _hook(self, p) -> None:
        if not self._armed:
            return
        self._left[self._bucket_of[id(p)]] -= 1
        while self._next < self._held_from and self._left[self._next] == 0:
            s, e, _ = self.buckets[self._next]
            self._works.append(self._all_reduce(self.flat[s:e]))
            self._next += 1

    def _join_producers(self) -> None:
        """Order the bucket's collective after EVERY stream that may have produced or accumulated one of its
        gradients.  Autograd runs a parameter's AccumulateGrad (and fires this hook) on whichever stream its
        node was created on -- with two micro-batch graphs alive that is often the other micro-batch stream
        (parallel/microbatch.py) -- so the stream current here need not be the one that wrote every
        gradient of the bucket.  RCCL orders its collective after the current stream only: make that stream
        wait for the default, the second micro-batch and the weight-gradient side stream first."""
        if not self.flat.is_cuda:
            return
        from ..ops import grad_accum
        from .microbatch import _OTHER
        dev = self.flat.device.index if self.flat.device.index is not None else torch.cuda.current_device()
        cur = torch.cuda.current_stream(dev)
        for s in (torch.cuda.default_stream(dev), self._main, _OTHER.get(dev), grad_accum._side.get(dev)):
            if s is not None and s != cur:
                cur.wait_stream(s)

    def _all_reduce(self, t: torch.Tensor):
        if self.world == 1:
            return None
        self._join_producers()
        if self.comm_dtype is None:
            return (dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True), None, None)
        tmp = t.mul(1.0 / self.world).to(self.comm_dtype)
        return (dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=self.group, async_op=True), t, tmp)

    def finish(self) -> None:
        """After the sync backward: launch any bucket not launched yet, wait for all, average."""
        if not self._armed:
            return
        t0 = self._stamp()
        from ..ops import grad_accum
        grad_accum.flush_late()  # the held small-parameter gradients (late column sums), on this stream
        while self._next < len(self.buckets):  # held buckets; parameters that got no gradient this step
            s, e, _ = self.buckets[self._next]
            self._works.append(self._all_reduce(self.flat[s:e]))
            self._next += 1
        for w in self._works:
            if w is not None:
                w[0].wait()
                if w[1] is not None:
                    w[1].copy_(w[2])
        if self.world > 1 and self.comm_dtype is None:
            if self.defer_average:
                self.grad_divisor = float(self.world)
            else:
                self.flat.mul_(1.0 / self.world)
                self.grad_divisor = 1.0
        if t0 is not None:
            self._exposed.append((t0, self._stamp()))
        self._armed = False
        self._works = []

    def _stamp(self):
        if not self.timing:
            return None
        if self.flat.is_cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        import time
        return time.perf_counter()

    def exposed_ms(self, clear: bool = True) -> List[float]:
        """Exposed all-reduce time (ms) of every timed sync step since the last call (syncs)."""
        out = []
        for a, b in self._exposed:
            if isinstance(a, float):
                out.append(1000.0 * (b - a))
            else:
                b.synchronize()
                out.append(a.elapsed_time(b))
        if clear:
            self._exposed = []
        return out

    def bucket_bytes(self) -> List[int]:
        return [4 * (e - s) for s, e, _ in self.buckets]

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


class ReducedModule(torch.nn.Module):
    """Wrapper exposing ``.module`` (like DDP, so callers that unwrap keep working) and ``.reducer``."""

    def __init__(self, module: torch.nn.Module, reducer: GradReducer):
        super().__init__()
        self.module = module
        self.reducer = reducer

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)


def wrap_reducer(module: torch.nn.Module, process_group=None, bucket_cap_mb: float = 100.0,
                 comm_dtype: str = "fp32") -> Optional[ReducedModule]:
    if not (dist.is_available() and dist.is_initialized()):
        return None
    return ReducedModule(module, GradReducer(module, process_group, bucket_cap_mb, comm_dtype=comm_dtype))
