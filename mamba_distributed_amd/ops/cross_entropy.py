"""Cross-entropy for the LM head.

The reference computes ``F.cross_entropy(logits.view(-1, V), targets.view(-1))`` on the
(B*T, 50304) bf16 logits under autocast, which upcasts to a 6.6 GB fp32 copy and writes a second
fp32 gradient (model.py:44-46).  Here the HIP kernel ``ce_fwd`` (csrc/kernels/cross_entropy.hip)
reads each bf16 logit row exactly once (the row lives in registers of one 512-thread workgroup),
computes the log-sum-exp and the loss, and — when a gradient is needed — writes
d(loss)/d(logits) = (softmax - onehot) / n_valid as bf16 in the same pass.

Two entry points:
  * ``cross_entropy(logits, targets)``            — drop-in loss, logits preserved, bf16 grad buffer.
  * ``fused_linear_cross_entropy(h, W, targets)`` — lm_head GEMMs + CE in one autograd node over row chunks
    of the logits (the whole (B*T, V) tensor never exists; dh and dW are produced in the forward pass).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext, grad_accum


def _inv_count(targets, ignore_index):
    return 1.0 / (targets != ignore_index).sum().clamp(min=1).to(torch.float32)


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, ignore_index):
        shape = logits.shape
        l2 = logits.reshape(-1, shape[-1])
        t = targets.reshape(-1)
        inv = _inv_count(t, ignore_index)
        need_grad = ctx.needs_input_grad[0]
        grad = torch.empty_like(l2) if need_grad else None
        losses = _ext.ops().ce_fwd(l2, t, ignore_index, inv, grad)
        loss = losses.sum() * inv
        ctx.save_for_backward(grad if need_grad else None)
        ctx.shape = shape
        return loss

    @staticmethod
    def backward(ctx, gloss):
        (grad,) = ctx.saved_tensors
        return (grad * gloss.to(grad.dtype)).view(ctx.shape), None, None


def cross_entropy(logits, targets, ignore_index=-100):
    if _ext.use_native(logits) and logits.dtype in (torch.bfloat16, torch.float16, torch.float32):
        return _CrossEntropyFn.apply(logits, targets, ignore_index)
    return F.cross_entropy(logits.float().view(-1, logits.size(-1)), targets.view(-1),
                           ignore_index=ignore_index)


class _FusedLinearCEFn(torch.autograd.Function):
    """loss = CE(h @ W^T, targets), with both gradients produced in the forward pass.

    The tokens are processed in row chunks (``_row_chunk``: <= 16384 rows, i.e. a 1.65 GB bf16 logits tile at
    V = 50304).  Per chunk:
      logits_c = h_c W^T                         native persistent GEMM (gp_pk)
      loss_c, dlogits_c (in place, / n_valid)    ce_fwd (one read of the tile)
      dh_c     = dlogits_c W                     gp_pk against W^T (cached once per optimizer step)
      dW      += dlogits_c^T h_c                 split-K engine (gp_mm), fp32 K-split slabs summed once per node
    (MAMBA_AMD_LMHEAD=lib puts all three products on hipBLASLt, fp32 output + accumulate for dW: A/B only)
    so the (B*T, V) logits never exist whole (6.6 GB at 64 x 1024 tokens) and nothing of the lm_head is kept
    for the backward but dh and dW, which the backward scales by d(loss).  Engines (MAMBA_AMD_LMHEAD=native|lib):
    native by default (round 3 measured the whole node at 64k tokens 19.0 ms all native vs 17.0 on hipBLASLt,
    profiles/r3/lm_head_chunk_products.log; the library stays as an A/B switch).
    The reference materialises the full fp32 logits (model.py:44-46)."""

    @staticmethod
    def forward(ctx, h, weight, targets, ignore_index, compute_dtype, row_chunk, grad_enabled):
        h2 = h.reshape(-1, h.shape[-1]).to(compute_dtype)
        w = grad_accum.cached_cast(weight, compute_dtype)        # once per optimizer step
        t = targets.reshape(-1)
        M, K = h2.shape
        V = w.shape[0]
        inv = _inv_count(t, ignore_index)
        # needs_input_grad reflects requires_grad even under no_grad (validation): skip the dh / dW products then
        need_h = ctx.needs_input_grad[0] and grad_enabled
        need_w = ctx.needs_input_grad[1] and grad_enabled
        nat_f, nat_h, nat_w = _lm_engines(h2, w)
        R = _row_chunk(M, V, row_chunk)
        buf = torch.empty(min(R, M), V, device=h2.device, dtype=compute_dtype)
        losses = torch.empty(M, device=h2.device, dtype=torch.float32)
        dh = torch.empty(M, K, device=h2.device, dtype=compute_dtype) if need_h else None
        # native dW: fp32 K-split slabs kept across the row chunks (each chunk adds into them), summed once at the end
        S = _lm_dw_splits(V, K, h2.device) if (need_w and nat_w) else 1
        dw = torch.empty(S, V, K, device=h2.device, dtype=torch.float32) if need_w else None
        wt = grad_accum.cached_transpose(weight, compute_dtype) if (need_h and nat_h) else None
        ops = _ext.ops()
        for r0 in range(0, M, R):
            r1 = min(M, r0 + R)
            hc, lg = h2[r0:r1], buf[:r1 - r0]
            if nat_f:
                ops.gp_pk(hc, w, lg)
            else:
                torch.mm(hc, w.t(), out=lg)
            losses[r0:r1] = ops.ce_fwd(lg, t[r0:r1], ignore_index, inv, lg if (need_h or need_w) else None)
            if need_h:
                if nat_h:
                    ops.gp_pk(lg, wt, dh[r0:r1])
                else:
                    torch.mm(lg, w, out=dh[r0:r1])
            if need_w:
                if nat_w:
                    ops.gp_mm(lg, hc, dw, 1, 1, 1 if r0 == 0 else 2, S, 256)
                else:
                    _lib_wgrad_acc(dw[0], lg, hc, r0 == 0)
        del buf
        if need_w and S > 1:
            dw1 = torch.empty(1, V, K, device=h2.device, dtype=torch.float32)
            ops.gp_reduce(dw, dw1[0], False)
            dw = dw1
        loss = losses.sum() * inv
        ctx.save_for_backward(dh, dw)
        ctx.hshape, ctx.hdtype, ctx.wdtype = h.shape, h.dtype, weight.dtype
        return loss

    @staticmethod
    def backward(ctx, gloss):
        dh_, dw_ = ctx.saved_tensors
        g = gloss.to(torch.float32)
        dh = dw = None
        # out of place: a second backward through the graph (retain_graph) must not scale the saved products twice
        if ctx.needs_input_grad[0] and dh_ is not None:
            dh = (dh_ * g.to(dh_.dtype)).view(ctx.hshape).to(ctx.hdtype)
        if ctx.needs_input_grad[1] and dw_ is not None:
            dw = (dw_[0] * g).to(ctx.wdtype)
        return dh, dw, None, None, None, None, None


def _lm_dw_splits(V: int, K: int, device) -> int:
    """K splits of the native dW = dlogits^T h product (gemm_pipe_k, 256 x 256 tiles, one workgroup per CU): the
    (V/256) x (K/256) tiles alone fill whole rounds of the CUs badly (V = 50304, K = 768: 591 tiles = 2.3 rounds of
    256, i.e. 3 rounds of work for 2.3 of tiles); S splits give S times the tiles at 1/S the depth: pick S <= 4 (and <= 1 GB of
    slabs) with the least ceil(tiles S / CUs) / S (S = 3: 6.9 rounds -> 7 rounds of 1/3-depth tiles = 2.33 full-depth rounds)."""
    tiles = -(-V // 256) * -(-K // 256)
    ncu = torch.cuda.get_device_properties(device).multi_processor_count if device.type == "cuda" else 256
    smax = max(1, min(4, (1 << 30) // (V * K * 4)))  # at most ~1 GB of slabs (the lm_head runs at the activation peak)
    best, bs = None, 1
    for S in range(1, smax + 1):
        cost = -(-tiles * S // ncu) / S
        if best is None or cost < best - 1e-9:
            best, bs = cost, S
    return bs


_F32_OUT = [None]  # hipBLASLt bf16 x bf16 -> fp32 products (aten::mm.dtype / addmm.dtype) usable here


def _lib_wgrad_acc(dw: torch.Tensor, g: torch.Tensor, h: torch.Tensor, first: bool) -> None:
    """dw (fp32) (+)= g^T h on the library: fp32 output straight from the GEMM where torch exposes it (no bf16
    rounding of the chunk's product and no separate add), else a bf16 product added in fp32."""
    if _F32_OUT[0] is None:
        import os
        if os.environ.get("MAMBA_AMD_LM_DW_F32", "1") == "0":
            _F32_OUT[0] = False
            return _lib_wgrad_acc(dw, g, h, first)
        try:
            torch.mm(g[:8].t(), h[:8], out_dtype=torch.float32)
            _F32_OUT[0] = True
        except (RuntimeError, TypeError):
            _F32_OUT[0] = False
    if _F32_OUT[0]:
        if first:
            torch.mm(g.t(), h, out_dtype=torch.float32, out=dw)
        else:
            torch.addmm(dw, g.t(), h, out_dtype=torch.float32, out=dw)
    elif first:
        dw.copy_(g.t() @ h)
    else:
        dw.add_(g.t() @ h)


def _lm_native(h2: torch.Tensor, w: torch.Tensor) -> bool:
    """The shapes suit the native engines (persistent GEMM: K > 192, 8-aligned, 16-B aligned rows)."""
    return (h2.is_cuda and h2.dtype == torch.bfloat16 and h2.stride(-1) == 1 and h2.stride(0) % 8 == 0
            and h2.data_ptr() % 16 == 0 and h2.shape[1] > 192 and h2.shape[1] % 8 == 0 and w.shape[0] % 8 == 0
            and w.is_contiguous())


def _lm_engines(h2: torch.Tensor, w: torch.Tensor):
    """(logits, dh, dW) on the native engines?  MAMBA_AMD_LMHEAD=native (default): all three; lib: none."""
    import os
    nat = os.environ.get("MAMBA_AMD_LMHEAD", "native") == "native" and _lm_native(h2, w)
    return nat, nat, nat


_ROW_CAP = 16384


def _row_chunk(M: int, V: int, row_chunk=None) -> int:
    """Rows per logits tile: at most 16384 (a 1.65 GB bf16 tile at V = 50304, under the persistent GEMM's 4 GB
    operand limit), balanced over the chunks and rounded up to whole 256-row GEMM tiles."""
    if row_chunk:
        return min(M, int(row_chunk))
    cap = max(256, min(_ROW_CAP, (1 << 31) // max(1, 2 * V) // 256 * 256))
    n = -(-M // cap)
    per = -(-M // n)
    return min(M, -(-per // 256) * 256)


def fused_linear_cross_entropy(h, weight, targets, ignore_index=-100, compute_dtype=torch.bfloat16, row_chunk=None):
    if _ext.use_native(h):
        return _FusedLinearCEFn.apply(h, weight, targets, ignore_index, compute_dtype, row_chunk,
                                      torch.is_grad_enabled())
    logits = F.linear(h, weight.to(h.dtype))
    return F.cross_entropy(logits.float().view(-1, logits.size(-1)), targets.view(-1),
                           ignore_index=ignore_index)
