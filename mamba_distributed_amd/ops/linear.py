"""Bias-free projection (nn.Linear without bias) on the native MFMA GEMM engines.

Forward and input-gradient GEMMs run on the persistent engine (``gp_pk``: one workgroup per CU walks the
output tiles; the next tile's operands stream into LDS while the previous tile's bf16 epilogue drains as
whole-row stores), the input gradient as dY . (W^T)^T against a transposed weight cached per optimizer step,
for every training-size shape of every model (``_pk_wins``; torch.mm only below the engine's minimum token count,
hipBLASLt only under the MAMBA_AMD_PROJ_GEMM A/B switch).  The weight
gradient dW = dY^T X reduces over all B*T tokens into a small output (3352 x 768 for in_proj), where the
library leaves most CUs idle: the native engine (csrc/kernels/gemm_pipe.hip, ``gp_mm`` with both operands
token-major) splits the tokens into S K-slices written as fp32 slabs.  Inside an accumulation scope the
slabs are PERSISTENT per weight: the no-sync micro-steps add into them (on a side stream, beside the rest
of the backward) and the fixed-order slab sum runs once per optimizer step, on the sync micro-step, which
returns the whole step's gradient in fp32 -- the parameter's dtype.
Autocast semantics match ``F.linear`` under ``torch.autocast``: compute in the autocast dtype.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext
from . import grad_accum


def _compute_dtype(x: torch.Tensor) -> torch.dtype:
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return x.dtype


def _native_ok(dy: torch.Tensor, x: torch.Tensor) -> bool:
    return (dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.stride(-1) == 1 and x.stride(-1) == 1
            and dy.shape[-1] % 8 == 0 and x.shape[-1] % 8 == 0 and dy.stride(0) % 8 == 0 and x.stride(0) % 8 == 0
            and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0)


def _wgrad_native(p, dy2: torch.Tensor, x2: torch.Tensor, lb: int = 1):
    """dW = dy2^T x2 (fp32) on the native engine; None when deferred to the sync micro-step.  dy2 is token-major
    (T, P); x2 is token-major (T, Q) (lb = 1) or channel-major (Q, T) (lb = 0: the Mamba-1 out_proj input)."""
    ops = _ext.ops()
    T, P = dy2.shape[0], dy2.shape[1]
    Q = x2.shape[1] if lb == 1 else x2.shape[0]
    S = ops.gp_splits(P, Q, T)
    d = grad_accum.deferred(p, "wgrad", (S, P, Q), dy2.device)
    if grad_accum.sync_accumulable(p):
        # sync micro-step with the gradient already in place (the reducer's flat-buffer view): the fixed-order slab
        # sum adds straight into it instead of autograd writing dW and adding it in a second pass
        if d is None:
            buf = ops.gp_mm(dy2, x2, None, 1, lb, 1, S, 256)
        else:
            buf, mode = d
            ops.gp_mm(dy2, x2, buf, 1, lb, 1 if mode in (1, 3) else 2, S, 256)
        ops.gp_reduce(buf, p.grad, True)
        return None
    if (d is None and lb == 1 and _wgrad_inplace(dy2.device) and grad_accum.accumulable(p) and p.grad.dtype == torch.float32
            and p.grad.is_contiguous()):
        # not deferred (wide models: auto_defer_reduce) on a no-sync micro-step: the split-K wgrad kernel adds
        # its fixed-order slab sum straight into p.grad on the weight-gradient side stream, beside the rest of
        # the backward (the round-1 path; running it on the main stream cost Mamba-2 1.4B 89k -> 84k tok/s,
        # profiles/r3/ab4_mamba2_1.4b_bisect.txt)
        side = grad_accum.side_stream(dy2.device)
        if side is None:
            ops.gemm_wgrad(dy2, x2, p.grad, True)
        else:
            side.wait_stream(torch.cuda.current_stream(dy2.device))
            with torch.cuda.stream(side):
                ops.gemm_wgrad(dy2, x2, p.grad, True)
            grad_accum.side_keep(dy2.device, dy2, x2)
        return None
    if d is None:  # outside an accumulation scope / sync micro-step: transient slabs, reduce now
        part = ops.gp_mm(dy2, x2, None, 1, lb, 1, S, 256)
        dw = torch.empty(P, Q, device=dy2.device, dtype=torch.float32)
        ops.gp_reduce(part, dw, False)
        return dw
    buf, mode = d
    slab_mode = 1 if mode in (1, 3) else 2  # store / add
    if mode <= 2:
        # no-sync micro-step: nothing consumes the slabs before the sync step, so the GEMM runs on the side
        # stream beside the rest of the backward (joined before the sync micro-step)
        side = grad_accum.side_stream(dy2.device)
        if side is None:
            ops.gp_mm(dy2, x2, buf, 1, lb, slab_mode, S, 256)
        else:
            side.wait_stream(torch.cuda.current_stream(dy2.device))
            with torch.cuda.stream(side):
                ops.gp_mm(dy2, x2, buf, 1, lb, slab_mode, S, 256)
            grad_accum.side_keep(dy2.device, dy2, x2)
        return None
    ops.gp_mm(dy2, x2, buf, 1, lb, slab_mode, S, 256)
    dw = torch.empty(P, Q, device=dy2.device, dtype=torch.float32)
    ops.gp_reduce(buf, dw, False)
    return dw


_INPLACE_STATE: dict = {}   # device index -> [calls until the next re-check, decision, device bytes]


def _wgrad_inplace(dev) -> bool:
    """Non-deferred no-sync micro-steps: the split-K wgrad adds into p.grad in place on the side stream, or (False)
    transient fp32 slabs on the persistent engine, reduced on the main stream. MAMBA_AMD_WGRAD_INPLACE=1/0 forces
    either; auto takes the side stream while the allocated peak stays under 70% of the device, the reserved peak
    under 96%, and the caching allocator has never had to retry (re-checked every 64 calls: memory_stats() is not free). The side-stream form
    keeps dy/x alive past the main stream's frees (grad_accum.side_keep: a few launches, stream-ordered; with
    record_stream it was a whole micro-batch, and near capacity that turned into allocator retries, which
    synchronise the device: Mamba-2 2.8B @ 8192 (222 GiB peak) ran 29.6k tok/s with it (17 retries) vs 46.8k
    without, while 1.4B @ 1024 (130 GiB) gains ~8% from it, profiles/r3/ab15_*)."""
    import os
    env = os.environ.get("MAMBA_AMD_WGRAD_INPLACE", "auto")
    if env in ("0", "1"):
        return env == "1"
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _INPLACE_STATE.get(key)
    if st is None:
        st = _INPLACE_STATE[key] = [0, True, torch.cuda.get_device_properties(key).total_memory]
    if st[0] <= 0:
        s = torch.cuda.memory_stats(key)
        # reserved: the side stream's record_stream lifetimes grow the reserved peak well past the allocated one
        # (Mamba-1 370M: 112 GB allocated, 269 GB reserved); at the cap every allocation retries first
        st[1] = (s.get("allocated_bytes.all.peak", 0) < 0.7 * st[2] and s.get("num_alloc_retries", 0) == 0
                 and s.get("reserved_bytes.all.peak", 0) < 0.96 * st[2])
        st[0] = 64
    st[0] -= 1
    return st[1]


def _proj_engine() -> str:
    """Forward / input-gradient projection GEMM engine: "pk" (default: the persistent native engine, gemm_pk_k, for
    every product), "auto" (pk only for the short-K shapes, K <= 1024), "lib" (hipBLASLt), or a comma list of roles on
    pk: fwd / dgrad, each optionally suffixed _short (K <= 1024) or _long (K > 1024), e.g. "fwd_short,dgrad".
    Everything but "pk" is an A/B switch (MAMBA_AMD_PROJ_GEMM).  hipBLASLt measured 2.2% / 1.0% faster whole-step at
    the 1.4B / 2.8B long-K shapes (profiles/r5/proj_engine_routing.txt); the native engine stays the default there
    (profiles/r6/pp_ring_gemm_rejected.txt has the round-6 attempt at closing that gap)."""
    import os
    return os.environ.get("MAMBA_AMD_PROJ_GEMM", "pk")


def library_gemms_possible(cfg) -> bool:
    """Whether a training step can run a library (hipBLASLt) projection GEMM under the current switches (only the
    A/B switches route there); the callers load the tuned solution table only then."""
    return _proj_engine() != "pk"


def _pk_wins(m: int, n_out: int, k: int, role: str = "fwd") -> bool:
    """Engine choice for an (m, n_out, k) product of one role ("fwd" / "dgrad"; the Mamba-1 channel-major products
    pass "fwd_cm" / "dgrad_xc").  The default ("pk") takes the native engine for every training-size product; the
    other settings are the A/B switches described in _proj_engine."""
    e = _proj_engine()
    if e == "lib":
        return False
    if e == "pk":
        return True
    role = {"fwd_cm": "fwd", "dgrad_xc": "dgrad"}.get(role, role)
    if e == "auto":
        return k <= 1024 and m * n_out <= (1 << 28)
    if m * n_out > (1 << 28):  # never the lm_head
        return False
    roles = set(e.split(","))
    return role in roles or f"{role}_{'short' if k <= 1024 else 'long'}" in roles


def _pk_ok(a2: torch.Tensor, n_out: int, k: int, role: str = "fwd") -> bool:
    """The native persistent GEMM for a forward or input-gradient projection: a2 (T, k) token-major bf16 times a
    k-contiguous (n_out, k) weight image (csrc/kernels/gemm_pipe.hip)."""
    return (a2.is_cuda and a2.dtype == torch.bfloat16 and a2.dim() == 2 and a2.stride(-1) == 1
            and a2.stride(0) % 8 == 0 and a2.data_ptr() % 16 == 0 and a2.shape[0] >= 4096 and k > 192
            and k % 8 == 0 and n_out % 8 == 0 and _pk_wins(a2.shape[0], n_out, k, role))


def _pk_mm(a2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return _ext.ops().gp_pk(a2, w)


def mm_nt(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b.T`` for two K-contiguous bf16 operands (a: (M, K), b: (N, K)) on the native persistent GEMM when
    the shape suits it (M * N >= 2^23, K > 192), else torch.mm.  E.g. the Mamba-1 channel-major in_proj
    xz = W_in h^T."""
    ok = (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 2
          and a.stride(-1) == 1 and b.stride(-1) == 1 and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
          and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0 and a.shape[1] > 192 and a.shape[1] % 8 == 0
          and b.shape[0] % 8 == 0 and a.shape[0] * b.shape[0] >= (1 << 23)
          and _pk_wins(a.shape[0], b.shape[0], a.shape[1], "fwd_cm"))
    return _pk_mm(a, b) if ok else torch.mm(a, b.t())


# ---- padded output rows --------------------------------------------------------------------------------------
# An output width that is not a multiple of 64 elements (the Mamba-2 in_proj: 3352 = 2 d_inner + 2 N + H at the
# 280M shape) makes every row of the product start off a 128-B line, and the input gradient then reads a
# K = 3352 operand whose K-tiles straddle two lines each.  The padded layout computes the output into a
# (T, Np) buffer (Np = width rounded up to 64) against a weight copy with zero rows appended (made once per
# optimizer step) and hands the consumer the (T, width) column view.  A consumer that writes the output's
# gradient into the same padded layout with zeroed pad columns registers it (register_zero_padded_grad); the
# backward then runs the input gradient as a K = Np product (zero rows of W^T meet zero columns of dY):
# in_proj dgrad 290 -> 252 us and forward 342 -> 316 us per layer at 64 x 1024 tokens
# (profiles/r3/pk5_inproj_padded_width.log).  Any other gradient layout takes the unpadded product.
_ZERO_PADDED: dict = {}


def pad_width(n: int) -> int:
    return (n + 63) // 64 * 64


def register_zero_padded_grad(full: torch.Tensor) -> None:
    """``full`` (T, Np) [or (b, l, Np)] is a gradient buffer whose columns past the consumer's width are zero;
    the view handed back as the gradient of a padded projection output starts at its first element."""
    for k in [k for k, (ref, _) in _ZERO_PADDED.items() if ref() is None]:
        del _ZERO_PADDED[k]
    import weakref
    _ZERO_PADDED[full.data_ptr()] = (weakref.ref(full), full._version)


def _zero_padded_full(dy2: torch.Tensor, np_: int):
    """The registered (T, Np) buffer behind the gradient view dy2 (T, width), or None."""
    ent = _ZERO_PADDED.get(dy2.data_ptr())
    if ent is None or dy2.stride(0) != np_ or dy2.stride(1) != 1:
        return None
    full = ent[0]()
    if full is None or full._version != ent[1] or full.data_ptr() != dy2.data_ptr() or full.shape[-1] != np_:
        return None
    del _ZERO_PADDED[dy2.data_ptr()]
    return full.reshape(-1, np_)


def _pad_rows(w: torch.Tensor, cd: torch.dtype, np_: int) -> torch.Tensor:
    wp = torch.zeros(np_, w.shape[1], device=w.device, dtype=cd)
    wp[:w.shape[0]].copy_(w)
    return wp


class _ProjFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, cd, pad):
        x2 = x.reshape(-1, x.shape[-1]).to(cd)
        n = weight.shape[0]
        np_ = pad_width(n) if pad else n
        if np_ != n:
            w = grad_accum.cached_value(weight, ("pad_rows", cd, np_), lambda t: _pad_rows(t, cd, np_))
        else:
            w = grad_accum.cached_cast(weight, cd)
        if _pk_ok(x2, w.shape[0], w.shape[1]) and w.is_contiguous():
            y = _pk_mm(x2, w)
        else:
            y = F.linear(x2, w)
        ctx.save_for_backward(x2, w)
        ctx.param = weight
        ctx.wdtype = weight.dtype
        ctx.xshape = x.shape
        ctx.n = n
        return y[:, :n].view(*x.shape[:-1], n) if np_ != n else y.view(*x.shape[:-1], n)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        n = ctx.n
        np_ = w.shape[0]
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != w.dtype:
            dy2 = dy2.to(w.dtype)
        full = _zero_padded_full(dy2, np_) if np_ != n else None
        if full is None and not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            if full is not None:
                # K = Np: the zero pad columns of dY meet the zero pad rows of W
                dx = _pk_mm(full, grad_accum.cached_transpose(w, w.dtype)) if _pk_ok(full, w.shape[1], np_, "dgrad") \
                    else torch.mm(full, w)
            elif _pk_ok(dy2, w.shape[1], n, "dgrad"):
                # dX = dY W as a KC . KC product against W^T, transposed once per optimizer step
                dx = _pk_mm(dy2, grad_accum.cached_transpose(ctx.param, w.dtype))
            else:
                dx = torch.mm(dy2, w[:n])
        dw = None
        if ctx.needs_input_grad[1]:
            p = ctx.param
            if _native_ok(dy2, x2):
                dw = _wgrad_native(p, dy2, x2)
                if dw is not None:
                    dw = grad_accum.defer(p, dw.to(ctx.wdtype))
            else:
                dw = grad_accum.defer(p, torch.mm(dy2.t(), x2).to(ctx.wdtype))
        return (dx.view(ctx.xshape) if dx is not None else None), dw, None, None


def _pad_enabled() -> bool:
    import os
    return os.environ.get("MAMBA_AMD_PAD_PROJ", "1") != "0"


def linear(x: torch.Tensor, layer: torch.nn.Linear, pad: bool = False) -> torch.Tensor:
    """``layer(x)`` for a bias-free nn.Linear, native weight gradient on the GPU.  ``pad``: compute into rows
    padded to a multiple of 64 and return the column view (see register_zero_padded_grad)."""
    if layer.bias is None and _ext.use_native(x):
        pad = pad and _pad_enabled() and layer.weight.shape[0] % 64 != 0
        return _ProjFn.apply(x, layer.weight, _compute_dtype(x), pad)
    return layer(x)
