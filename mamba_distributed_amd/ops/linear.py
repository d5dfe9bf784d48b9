"""Bias-free projection (nn.Linear without bias) with a native weight-gradient GEMM.

Forward and input-gradient GEMMs are plain GEMMs (no fusion) on hipBLASLt with the pinned TunableOp table
(``utils/gemm_tuning``), measured faster at these shapes than the native engine, whose 256 x 192 tile for the
d_model-wide outputs stays available as an opt-in (``_narrow_native``).  The weight
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


def _wgrad_native(p, dy2: torch.Tensor, x2: torch.Tensor):
    """dW = dy2^T x2 (fp32) on the native engine; None when deferred to the sync micro-step."""
    ops = _ext.ops()
    T, P, Q = dy2.shape[0], dy2.shape[1], x2.shape[1]
    S = ops.gp_splits(P, Q, T)
    d = grad_accum.deferred(p, "wgrad", (S, P, Q), dy2.device)
    if d is None:  # outside an accumulation scope: transient slabs, reduce now
        part = ops.gp_mm(dy2, x2, None, 1, 1, 1, S, 256)
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
            ops.gp_mm(dy2, x2, buf, 1, 1, slab_mode, S, 256)
        else:
            side.wait_stream(torch.cuda.current_stream(dy2.device))
            with torch.cuda.stream(side):
                ops.gp_mm(dy2, x2, buf, 1, 1, slab_mode, S, 256)
            dy2.record_stream(side)
            x2.record_stream(side)
        return None
    ops.gp_mm(dy2, x2, buf, 1, 1, slab_mode, S, 256)
    dw = torch.empty(P, Q, device=dy2.device, dtype=torch.float32)
    ops.gp_reduce(buf, dw, False)
    return dw


def _native_dgrad_ok(dy2: torch.Tensor, w: torch.Tensor) -> bool:
    """Opt-in (MAMBA_AMD_NATIVE_DGRAD=1): the input gradient dX = dY W on the native pipelined engine for
    short contractions (K = out_features <= 1024, the out_proj of the d_model=768 models).  In isolation it
    is 3% faster than the tuned hipBLASLt solution (91.6-94 vs 94-97 us, profiles/r2_v3_gemm_pipe_bench.log)
    but the whole 280M step is 1% slower with it (276.6k vs 279.3k tok/s, interleaved A/B,
    profiles/r2_v5_ab_native_dgrad.txt: its 128 KB-LDS workgroups crowd the overlapped micro-batch's
    kernels), so hipBLASLt stays the default."""
    import os
    return (os.environ.get("MAMBA_AMD_NATIVE_DGRAD", "0") == "1" and dy2.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and dy2.is_cuda and w.is_contiguous() and w.shape[0] <= 1024
            and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0 and dy2.shape[0] >= 4096)


def _dgrad_native(dy2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dX (T, in) = dY (T, out) . W (out, in): A k-contiguous, B (k rows, n contiguous), bf16 epilogue."""
    return _ext.ops().gp_mm(dy2, w, None, 0, 1, 0, 1, 256)


def _narrow_native() -> bool:
    """MAMBA_AMD_NATIVE_NARROW=1 (opt-in; default off): GEMMs whose OUTPUT is d_model <= 1024 wide -- the out_proj
    forward and the in_proj input gradient of the 280M models -- on the native engine's 256 x 192 tile
    (gemm_pipe.hip, tile code 192): N = 768 makes 4 column tiles, so 32768 rows are 512 tiles = exactly two
    rounds of 256 CUs, where 256-wide tiles (ours or the library's) leave the second round half empty.  The
    input gradient reads W^T as a k-contiguous operand, transposed once per optimizer step
    (grad_accum.cached_transpose).  Measured on one MI355X (profiles/r2_v7_narrow_tile_ab.txt): the out_proj
    forward 71.4 us against hipBLASLt's 69.5 (256 x 256: 79.7), the in_proj input gradient 203 against 167,
    whole 280M step -2.2 % (277.5k vs 283.6k tok/s, interleaved), so the library stays the default."""
    import os
    return os.environ.get("MAMBA_AMD_NATIVE_NARROW", "0") == "1"


def _narrow_ok(a: torch.Tensor, n_out: int, k: int) -> bool:
    return (a.is_cuda and a.dtype == torch.bfloat16 and a.dim() == 2 and a.stride(-1) == 1
            and a.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0 and a.shape[0] >= 8192
            and 384 <= n_out <= 1024 and n_out % 8 == 0 and k % 8 == 0 and _narrow_native())


class _ProjFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, cd):
        x2 = x.reshape(-1, x.shape[-1]).to(cd)
        w = grad_accum.cached_cast(weight, cd)
        if _narrow_ok(x2, w.shape[0], w.shape[1]) and w.is_contiguous():
            y = _ext.ops().gp_mm(x2, w, None, 0, 0, 0, 1, 192)
        else:
            y = F.linear(x2, w)
        ctx.save_for_backward(x2, w)
        ctx.param = weight
        ctx.wdtype = weight.dtype
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != w.dtype:
            dy2 = dy2.to(w.dtype)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            if _narrow_ok(dy2, w.shape[1], w.shape[0]):
                dx = _ext.ops().gp_mm(dy2, grad_accum.cached_transpose(ctx.param, w.dtype), None, 0, 0, 0, 1, 192)
            elif _native_dgrad_ok(dy2, w):
                dx = _dgrad_native(dy2, w)
            else:
                dx = torch.mm(dy2, w)
        dw = None
        if ctx.needs_input_grad[1]:
            p = ctx.param
            if _native_ok(dy2, x2):
                dw = _wgrad_native(p, dy2, x2)
                if dw is not None:
                    dw = grad_accum.defer(p, dw.to(ctx.wdtype))
            else:
                dw = grad_accum.defer(p, torch.mm(dy2.t(), x2).to(ctx.wdtype))
        return (dx.view(ctx.xshape) if dx is not None else None), dw, None


def linear(x: torch.Tensor, layer: torch.nn.Linear) -> torch.Tensor:
    """``layer(x)`` for a bias-free nn.Linear, native weight gradient on the GPU."""
    if layer.bias is None and _ext.use_native(x):
        return _ProjFn.apply(x, layer.weight, _compute_dtype(x))
    return layer(x)
