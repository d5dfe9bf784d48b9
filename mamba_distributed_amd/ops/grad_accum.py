"""Micro-batch gradient accumulation without per-parameter add kernels (reference train.py:205-219,
SURVEY.md R14).

With 16 micro-batches per optimizer step (1 GPU) autograd's AccumulateGrad runs ``p.grad += g``
for every parameter on every micro-step: ~450 tiny add kernels per micro-batch for the 280M
Mamba-2 model (~2.3 ms, mostly launch latency), plus the full read-modify-write of the two large
projection gradients.  Inside an ``accumulation_scope`` on the no-sync micro-steps:

  * the projection weight gradients are accumulated by the weight-gradient GEMM itself
    (``gemm_wgrad(..., out=p.grad, accumulate=True)``: the fixed-order split-K reduction adds into
    the existing gradient, still deterministic);
  * every other parameter gradient produced by a native op is queued and applied by ONE
    ``torch._foreach_add_`` when the backward pass finishes.

  * parameter gradients that kernels produce as per-workgroup partial rows (norm weights, conv taps,
    A_log / D / dt_bias) or as K-split fp32 slabs (projection weights) are NOT reduced on the no-sync
    micro-steps at all: the kernels add into persistent per-parameter buffers (``deferred``) and the
    column sum / slab sum runs once, on the sync micro-step, whose autograd return then carries the
    whole step's gradient.  ``accumulation_scope(defer_reduce=...)`` picks this per model
    (parallel/microbatch.py::auto_defer_reduce); MAMBA_AMD_DEFER_REDUCE=0 / 1 forces it off / on.

The last micro-step (the one that triggers the bucketed all-reduce) and anything outside a scope use the normal
autograd path, so torch DDP's gradient hooks fire exactly as usual.  Under the native reducer or in a single process
(``set_late``, parallel/microbatch.py) the sync micro-step additionally (a) adds the projection weight gradients into
the existing flat-buffer .grad instead of returning them (``sync_accumulable``) and (b) leaves the small parameter-
gradient partials for one batched column sum after the backward (``late_colsum`` / ``flush_late``).  The scope also caches
bf16 copies of the projection weights: weights cannot change between the micro-steps of one
optimizer step, and the fused AdamW update does not bump tensor versions, so the cache is tied to
the scope rather than to version counters.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional, Tuple

import torch

_scope_depth = 0
_direct = False
_defer_scope = True   # deferred reductions requested by the outermost accumulation_scope
_side = {}            # device index -> side stream for in-place weight-gradient GEMMs
_side_dirty = set()   # devices whose side stream has work the main stream has not waited for
_pending: List[Tuple[torch.Tensor, torch.Tensor]] = []
_flush_queued = False
_wcache: Dict[Tuple[int, torch.dtype], Tuple[torch.Tensor, torch.Tensor]] = {}
_bufs: Dict[Tuple[int, str], list] = {}  # (id(param), tag) -> [param, fp32 buffer, holds this step's partials]


@contextlib.contextmanager
def accumulation_scope(defer_reduce: bool = True):
    """Wrap the micro-batch loop of ONE optimizer step (no parameter updates inside).
    ``defer_reduce``: keep per-parameter partial buffers across the micro-steps (``deferred``)."""
    global _scope_depth, _direct, _defer_scope
    if _scope_depth == 0:
        _defer_scope = bool(defer_reduce)
    _scope_depth += 1
    ok = False
    try:
        yield
        ok = True
    finally:
        _scope_depth -= 1
        if _scope_depth == 0:
            _direct = False
            _wcache.clear()
            # partials added on a no-sync micro-step and never reduced on the sync one would be lost: the
            # parameter got no gradient on the last micro-step.  Fail loudly on a normal exit.
            stuck = [key[1] for key, ent in _bufs.items() if ent[2]]
            for ent in _bufs.values():  # buffers are kept (reused next step); their contents are dead
                ent[2] = False
            join_side()
            if _late:  # a loop that queued late column sums without flushing them (parallel/microbatch.py flushes)
                if ok:
                    flush_late()
                else:
                    _late.clear()
            set_late(False)
            if ok and stuck:
                raise RuntimeError(
                    f"grad_accum: deferred gradient partials ({sorted(set(stuck))}) were accumulated on no-sync "
                    "micro-steps but never reduced: the last micro-step produced no gradient for those "
                    "parameters. Run with MAMBA_AMD_DEFER_REDUCE=0 for such models.")


def set_direct(enabled: bool) -> None:
    """Called per micro-step (parallel/ddp.py::set_grad_sync): True on the no-sync micro-steps."""
    global _direct
    _direct = bool(enabled) and _scope_depth > 0
    if not _direct:
        join_side()  # the sync micro-step's autograd accumulation must see every in-place wgrad


def side_stream(device: torch.device):
    """Stream for the no-sync micro-steps' in-place weight-gradient GEMMs.  They have no autograd
    consumer (they add straight into p.grad), so they can run beside the rest of the backward: the
    compute-bound wgrad GEMMs overlap the memory- / latency-bound norm, conv and scan kernels of the
    main stream.  Returns None when disabled (MAMBA_AMD_WGRAD_STREAM=0)."""
    import os
    if os.environ.get("MAMBA_AMD_WGRAD_STREAM", "1") == "0" or device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _side.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _side[idx] = s
    _side_dirty.add(idx)
    return s


def join_side() -> None:
    """Make every device's current stream wait for its side stream's queued weight-gradient work."""
    if not _side_dirty:
        return
    for idx in list(_side_dirty):
        torch.cuda.current_stream(idx).wait_stream(_side[idx])
        _kept.pop(idx, None)  # every kept operand's side-stream use is now ordered before the main stream
    _side_dirty.clear()


_kept = {}     # device index -> deque of (side-stream event, operands kept alive for it)
_KEEP_BATCH = 8


def _keep_lag() -> int:
    """Side-stream launches whose operands stay referenced (MAMBA_AMD_SIDE_LAG; < 0: record_stream instead)."""
    import os
    return int(os.environ.get("MAMBA_AMD_SIDE_LAG", "16"))


def side_keep(device: torch.device, *tensors) -> None:
    """Keep the main-stream operands of the side-stream work just queued alive, stream-ordered, instead of
    ``record_stream``.  record_stream defers every reuse of the block to a HOST-side event query, and the host runs
    a whole micro-batch ahead, so each backward's freed activations stayed unusable while the next forward
    allocated fresh ones: 239 GB reserved for 124 GB allocated at the Mamba-2 280M bench shape.  Here the side
    stream records an event after the work; once more than MAMBA_AMD_SIDE_LAG (16) launches are queued, the main stream waits for
    the oldest one's event (a GPU-side wait that is normally long satisfied) and its references are dropped, so any
    later main-stream reuse of that memory is ordered after the side-stream reads."""
    from collections import deque
    idx = device.index if device.index is not None else torch.cuda.current_device()
    side = _side[idx]
    lag = _keep_lag()
    if lag < 0:  # the old form (A/B): the allocator defers each block's reuse to a host-side event query
        for t in tensors:
            t.record_stream(side)
        return
    ev = torch.cuda.Event()
    ev.record(side)
    q = _kept.get(idx)
    if q is None:
        q = _kept[idx] = deque()
    q.append((ev, tensors))
    if len(q) > lag + _KEEP_BATCH:
        # release the oldest _KEEP_BATCH entries behind ONE main-stream wait (on the newest of them: the side stream
        # runs in order, so it covers the older ones): a wait per launch cost ~0.5 % of the step
        last = None
        for _ in range(_KEEP_BATCH):
            last, _t = q.popleft()
        torch.cuda.current_stream(idx).wait_event(last)


def deferred(param, tag: str, shape, device, force: bool = False):
    """Deferred reduction of ``param``'s gradient inside an accumulation scope.

    Returns None outside a scope (the op reduces as usual), else ``(buffer, part_mode)``: a persistent fp32
    buffer of ``shape`` owned by (param, tag) and the mode for the op -- 1 / 2: store / add this
    micro-step's partials, no reduction, the op returns an empty gradient (no-sync micro-step); 3 / 4:
    store / add, then reduce: the op returns the gradient of every micro-step of this optimizer step
    (sync micro-step).  A second call in the same sync micro-step starts over (3) and its gradient is
    added by autograd as usual.  ``force``: defer even when the scope did not ask for deferred reductions
    (small partials whose per-micro-step reduction is pure launch overhead; MAMBA_AMD_DEFER_REDUCE=0 still wins)."""
    import os
    if _scope_depth == 0 or not isinstance(param, torch.Tensor) or not param.requires_grad:
        return None
    env = os.environ.get("MAMBA_AMD_DEFER_REDUCE", "")
    if env == "0" or (env != "1" and not _defer_scope and not force):
        return None
    key = (id(param), tag)
    shape = tuple(int(v) for v in shape)
    ent = _bufs.get(key)
    if ent is not None and ent[0] is param and ent[2] and (tuple(ent[1].shape) != shape or ent[1].device != device):
        # the partial-row / slab layout depends on the micro-batch shape (rows = f(B*L)); a different shape
        # inside one optimizer step (a short last micro-batch, varlen packing) cannot add into the pending
        # partials, and starting a new buffer would drop them: refuse instead
        raise RuntimeError(
            f"grad_accum: micro-batch shape changed inside one optimizer step ({tag}: partials {tuple(ent[1].shape)} "
            f"-> {shape}); deferred reductions need equal micro-batches. Run with MAMBA_AMD_DEFER_REDUCE=0.")
    if ent is None or ent[0] is not param or tuple(ent[1].shape) != shape or ent[1].device != device:
        ent = [param, torch.empty(shape, device=device, dtype=torch.float32), False]
        _bufs[key] = ent
    final = not _direct
    mode = (4 if ent[2] else 3) if final else (2 if ent[2] else 1)
    ent[2] = not final
    return ent[1], mode


def release_buffers() -> None:
    """Free every deferred-reduction buffer and cached weight copy (training end, switching models)."""
    if _scope_depth:
        raise RuntimeError("grad_accum.release_buffers() inside an accumulation_scope")
    _bufs.clear()
    _wcache.clear()
    drop_images()


def in_scope() -> bool:
    return _scope_depth > 0


def direct() -> bool:
    return _direct and _scope_depth > 0


# ---- late column sums: the sync micro-step's deferred partials reduced by one batched launch pair ----------------
# On the sync micro-step each deferred partial block (norm weights, conv taps + bias, A_log / D / dt_bias) used to be
# column-summed by its op -- two small launches per block, ~4 blocks per layer, 3.4 ms of a 209 ms step at one
# micro-batch per optimizer step (profiles/r5/accum1_native_adamw_table.md).  With ``set_late(True)`` (the micro-batch
# loop, parallel/microbatch.py, for the native reducer or a single process; never under torch DDP, whose hooks would
# all-reduce the missing gradients) the ops instead leave the partials in their buffers, queue them here and return
# no gradient; ``flush_late`` reduces every queued block with ONE pair of launches (csrc/kernels/norm.hip
# late_colsum) straight into the parameters' .grad -- before the native reducer launches its held last bucket
# (the small parameters, parallel/reducer.py) or, single process, before the micro-batch loop returns.
_late_on = False
_late: List[tuple] = []       # (part (rows, cols) fp32, mode, G, [destination params])
_late_tab: Dict[int, tuple] = {}  # device index -> (key, device table, n, nblk, ntile)
_LATE_ROWS = 64               # rows per stage-1 split

try:
    import numpy as _np
    _LATE_DTYPE = _np.dtype([("part", "<u8"), ("d0", "<u8"), ("d1", "<u8"), ("d2", "<u8"), ("nrows", "<i4"),
                             ("ncols", "<i4"), ("R", "<i4"), ("RS", "<i4"), ("G", "<i4"), ("mode", "<i4"),
                             ("acc", "<i4"), ("pad0", "<i4"), ("blk0", "<i4"), ("tile0", "<i4"), ("pad1", "<i4"),
                             ("pad2", "<i4")])
    assert _LATE_DTYPE.itemsize == 80
except ImportError:  # pragma: no cover
    _np = None


def set_late(enabled: bool) -> None:
    global _late_on
    _late_on = bool(enabled)


_held: Optional[set] = None  # ids of the native reducer's held parameters (parallel/reducer.py::held_param), if any


def register_held(params) -> None:
    """The native reducer's held parameters: with a reducer alive, only these may take the late path (a late
    gradient of any other parameter would be all-reduced from its hook before flush_late wrote it)."""
    global _held
    _held = {id(p) for p in params}


def late_ok(*params) -> bool:
    """The sync micro-step may queue ``params``' partials for ``flush_late`` (fp32 parameters whose .grad, if any, is
    fp32 contiguous; MAMBA_AMD_LATE_REDUCE=0 turns it off)."""
    import os
    if not (_late_on and _scope_depth > 0 and not _direct and _np is not None):
        return False
    if os.environ.get("MAMBA_AMD_LATE_REDUCE", "1") == "0":
        return False
    from ..parallel.reducer import held_param
    for p in params:
        if p is None:
            continue
        if not (isinstance(p, torch.Tensor) and p.is_leaf and p.requires_grad and p.dtype == torch.float32 and p.is_cuda):
            return False
        if p.grad is not None and (p.grad.dtype != torch.float32 or not p.grad.is_contiguous()):
            return False
        # only parameters the reducer holds until finish() (small non-matrix ones): a late gradient of a parameter
        # whose bucket launches from the backward's hooks would be all-reduced before flush_late writes it
        if not held_param(p) or (_held is not None and id(p) not in _held):
            return False
    return True


def sync_accumulable(param) -> bool:
    """Sync micro-step (native reducer or single process: the same condition as the late column sums) and ``param``
    already holds an fp32 contiguous gradient (the reducer's flat-buffer view, or earlier micro-steps' sum): a weight
    gradient op may add its result into ``param.grad`` itself, on the current stream, and return none -- autograd's
    AccumulateGrad would otherwise write the gradient and add it in a second pass (136 add kernels per step at one
    micro-batch per step).  The parameter's AccumulateGrad still runs (with no gradient) and fires the reducer hook
    after the add was queued.  MAMBA_AMD_SYNC_INPLACE=0 turns it off."""
    import os
    return (_late_on and _scope_depth > 0 and not _direct and isinstance(param, torch.nn.Parameter)
            and param.requires_grad and param.grad is not None and param.grad.dtype == torch.float32
            and param.grad.is_contiguous() and param.grad.is_cuda
            and os.environ.get("MAMBA_AMD_SYNC_INPLACE", "1") != "0")


def late_colsum(part: torch.Tensor, mode: int, G: int, params) -> None:
    """Queue the column sums of ``part`` (rows x cols after flattening the trailing dims) for ``flush_late``.
    mode 0: params = [p], column j -> p.grad[j]; 1: [weight, bias], columns grouped by G = taps + 1 ([taps | bias]
    per channel); 2: [p0, p1, p2], column o G + i -> p_o.grad[i] (None: skipped)."""
    _late.append((part.reshape(part.shape[0], -1), int(mode), int(G), list(params)))


def flush_late() -> None:
    """Reduce every queued partial block into its parameters' .grad with one pair of launches (on the current
    stream, which must be ordered after the backward that wrote the partials)."""
    global _late
    if not _late:
        return
    entries, _late = _late, []
    from . import _ext
    dev = entries[0][0].device
    # destinations: add into an existing fp32 .grad, else store into fresh views of one flat buffer
    need = []
    seen = set()
    for part, mode, G, ps in entries:
        for p in ps:
            if p is None:
                continue
            if id(p) in seen:
                raise RuntimeError("grad_accum.flush_late: a parameter is the destination of two partial blocks")
            seen.add(id(p))
            if p.grad is None:
                need.append(p)
    if need:
        flat = torch.empty(sum(p.numel() for p in need), device=dev, dtype=torch.float32)
        o = 0
        for p in need:
            p.grad = flat[o:o + p.numel()].view_as(p)
            o += p.numel()
    fresh = {id(p) for p in need}
    rows = []
    key = []
    blk = tile = 0
    for part, mode, G, ps in entries:
        nrows, ncols = part.shape
        R = min(_LATE_ROWS, nrows)
        RS = (nrows + R - 1) // R
        tiles = (ncols + 63) // 64
        d = [0, 0, 0]
        acc = 0
        for k, p in enumerate(ps):
            if p is None:
                continue
            d[k] = p.grad.data_ptr()
            if id(p) not in fresh:
                acc |= 1 << k
        rows.append((part.data_ptr(), d[0], d[1], d[2], nrows, ncols, R, RS, G, mode, acc, 0, blk, tile, 0, 0))
        key.append((part.data_ptr(), d[0], d[1], d[2], nrows, ncols, G, mode, acc))
        blk += tiles * RS
        tile += tiles
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = tuple(key)
    ent = _late_tab.get(idx)
    if ent is None or ent[0] != key:
        tab = _np.array(rows, dtype=_LATE_DTYPE)
        t = torch.from_numpy(tab.view(_np.uint8).copy()).pin_memory().to(dev, non_blocking=True)
        ent = _late_tab[idx] = (key, t, len(rows), blk, tile)
    _ext.ops().late_colsum(ent[1], ent[2], ent[3], ent[4])


# ---- bf16 weight images written by the native optimizer step (ops/optim.py) ----------------------------------
# The scope records which images of which parameters its GEMMs asked for (``image_demand``); the native AdamW writes
# exactly those images in its update pass (same bytes the per-step cast / zero-padded copy would produce) and
# ``provide_image`` registers them; the next scope takes them instead of casting again.  An image is valid while the
# parameter's version counter is unchanged (the optimizer's raw-pointer update does not bump it; any other in-place
# write -- load_state_dict, a manual edit -- does, and the image is ignored from then on).
_demand: Dict[Tuple[int, tuple], Tuple[torch.Tensor, tuple]] = {}
_images: Dict[Tuple[int, tuple], Tuple[torch.Tensor, torch.Tensor, int]] = {}


def _want(w: torch.Tensor, kind: tuple):
    """Record the demand for image ``kind`` of parameter ``w``; return the provided image if it is fresh.  Only
    where autograd is off (inside a custom Function's forward, which computes the weight gradient itself): an image
    is a plain tensor, so a differentiable use (F.linear on it in module code) would lose the weight's gradient."""
    if not (isinstance(w, torch.nn.Parameter) and w.requires_grad and w.is_cuda) or torch.is_grad_enabled():
        return None
    key = (id(w), kind)
    _demand[key] = (w, kind)
    ent = _images.get(key)
    if ent is not None and ent[0] is w and ent[2] == w._version:
        return ent[1]
    return None


def image_demand() -> List[Tuple[torch.Tensor, tuple]]:
    """(parameter, kind) pairs the GEMMs asked for since the process started; kind = ("cast", dtype) or
    ("pad_rows", dtype, rows)."""
    return list(_demand.values())


def provide_image(w: torch.Tensor, kind: tuple, img: torch.Tensor) -> None:
    _images[(id(w), kind)] = (w, img, w._version)


def drop_images() -> None:
    _images.clear()
    _demand.clear()


def cached_cast(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """``w.to(dtype)``, reused across the micro-steps of the current scope (or the optimizer's fresh image)."""
    if w.dtype == dtype or _scope_depth == 0:
        return w.to(dtype)
    key = (id(w), dtype)
    ent = _wcache.get(key)
    if ent is not None and ent[0] is w:
        return ent[1]
    t = _want(w, ("cast", dtype))
    if t is None:
        t = w.to(dtype)
    _wcache[key] = (w, t)  # holding w keeps id(w) unique for the scope's lifetime
    return t


def cached_value(w: torch.Tensor, tag, fn):
    """``fn(w)`` (a function of a parameter only, e.g. A = -exp(A_log)), computed once per scope like
    ``cached_cast``; outside a scope it is computed every call.  ("pad_rows", dtype, rows) tags may come from the
    optimizer's images."""
    if _scope_depth == 0:
        return fn(w)
    key = (id(w), tag)
    ent = _wcache.get(key)
    if ent is not None and ent[0] is w:
        return ent[1]
    t = _want(w, tag) if isinstance(tag, tuple) and tag and tag[0] == "pad_rows" else None
    if t is None:
        with torch.no_grad():
            t = fn(w)
    _wcache[key] = (w, t)
    return t


def _transpose(w: torch.Tensor) -> torch.Tensor:
    """``w.t().contiguous()``; bf16 GPU matrices on the native 64 x 64-tile transpose (csrc/kernels/gemm.hip
    transpose_bf16_k: 16-B row loads and stores; torch copies a transposed view element by element)."""
    if (w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and w.stride(1) == 1 and w.shape[0] % 8 == 0
            and w.shape[1] % 8 == 0 and w.stride(0) % 8 == 0 and w.data_ptr() % 16 == 0):
        from . import _ext
        if _ext.use_native(w):
            return _ext.ops().transpose_bf16(w)
    return w.t().contiguous()


def cached_transpose(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """``w.to(dtype).t().contiguous()`` (the input-gradient GEMM's k-contiguous B operand), reused across
    the micro-steps of the current scope like ``cached_cast``."""
    if _scope_depth == 0:
        return _transpose(w.to(dtype))
    key = (id(w), dtype, "t")
    ent = _wcache.get(key)
    if ent is not None and ent[0] is w:
        return ent[1]
    t = _transpose(cached_cast(w, dtype))
    _wcache[key] = (w, t)
    return t


def accumulable(param) -> bool:
    """The parameter already holds a gradient the current micro-step may add into directly."""
    return (direct() and isinstance(param, torch.Tensor) and param.is_leaf and param.requires_grad
            and param.grad is not None)


_pending_stream = None  # stream the queued gradients were produced on (the backward's stream)


def _foreach_accumulate(pairs) -> None:
    """dst += src for every pair with ONE multi-tensor kernel.  torch's fused foreach route needs
    every tensor of both lists dense with identical strides (and one dtype); a single odd gradient
    (a strided view, a broadcast) silently drops the whole call to one add kernel per tensor, so
    non-contiguous sources are made contiguous first and odd destinations are added one by one."""
    by_dtype = {}
    for d, s in pairs:
        if d.is_contiguous():
            by_dtype.setdefault(d.dtype, ([], []))
            by_dtype[d.dtype][0].append(d)
            by_dtype[d.dtype][1].append(s if s.is_contiguous() else s.contiguous())
        else:
            d.add_(s)
    for dst, src in by_dtype.values():
        torch._foreach_add_(dst, src)


def _flush() -> None:
    global _flush_queued, _pending_stream
    _flush_queued = False
    if _pending:
        pairs = list(_pending)
        _pending.clear()
        st, _pending_stream = _pending_stream, None
        if st is not None:
            with torch.cuda.stream(st):  # the callback thread's current stream may be another one
                _foreach_accumulate(pairs)
        else:
            _foreach_accumulate(pairs)


def defer(param, grad):
    """Return value for ``param``'s slot in an autograd backward: ``grad`` itself on the normal
    path, or None after queueing it for the batched accumulation at the end of this backward."""
    global _flush_queued, _pending_stream
    if grad is None or not accumulable(param):
        return grad
    g = param.grad
    if g.shape != grad.shape or g.dtype != grad.dtype or g.device != grad.device:
        return grad
    _pending.append((g, grad))
    if grad.is_cuda and _pending_stream is None:
        _pending_stream = torch.cuda.current_stream(grad.device)
    if not _flush_queued:
        torch.autograd.Variable._execution_engine.queue_callback(_flush)
        _flush_queued = True
    return None
