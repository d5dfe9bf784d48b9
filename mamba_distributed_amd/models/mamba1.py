"""Mamba-1 (S6) mixer.

Parameter names, shapes and init follow upstream ``mamba_ssm/modules/mamba_simple.py::Mamba``
so checkpoints are interchangeable with the reference.

Layout choice (MI355X-first, not upstream's): the whole inner path runs channel-major with the
batch folded inside, i.e. tensors of logical shape (b, d, l) live in memory as (d, b, l).  Every
projection is then ONE plain 2-D GEMM on the native engines (csrc/kernels/gemm_pipe.hip persistent /
split-K, gemm.hip skinny; hipBLASLt only under the MAMBA_AMD_PROJ_GEMM=lib A/B switch) —
  xz    = W_in  @ h^T           (2di, b*l)
  x_dbl = W_x   @ conv_out      (R+2N, b*l)
  delta = W_dt  @ x_dbl[:R]     (di, b*l)
  out   = y^T   @ W_out^T       (b*l, d)
— and the HIP conv / scan kernels see unit stride along time, which is what their time-tiled
wavefront layout wants.  The backward writes d(xz) as one buffer (no slice-gradient
materialisation), like upstream's MambaInnerFn.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import _ext, grad_accum
from ..ops.conv1d import causal_conv1d_fn, causal_conv1d_update
from ..ops.linear import _wgrad_inplace, mm_nt
from ..ops.reference import causal_conv1d_ref, selective_scan_ref, softplus_inverse
from ..ops.selective_scan import selective_scan_fn, selective_state_update


def _cm(t2d: torch.Tensor, b: int, l: int) -> torch.Tensor:
    """(d, b*l) -> logical (b, d, l) view over the same memory."""
    return t2d.view(t2d.shape[0], b, l).permute(1, 0, 2)


def _flat(t: torch.Tensor) -> torch.Tensor:
    """logical (b, d, l) stored (d, b, l) -> (d, b*l) view."""
    return t.permute(1, 0, 2).reshape(t.shape[1], -1)


def _mm_cm(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False):
    """``out (+)= A @ B`` for a small weight ``A`` (N, K) and a channel-major activation ``B`` (K, M):
    the native streaming kernel (csrc/kernels/gemm.hip::gemm_skinny_k) for wide short-K products when
    the layout allows it, torch.mm otherwise.  Used for x_proj / dt_proj and their input gradients."""
    M = B.shape[1]
    # the streaming kernel only for the wide, short-K products (delta = W_dt x_dbl[:R], dconv += W_x^T dx_dbl);
    # the narrow long-K ones (x_dbl, dx_dbl[:R]) take the split-K engine's 128-row tile form below
    ok = (A.shape[0] >= 256 and A.shape[1] <= 128 and A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16 and A.is_cuda and B.stride(1) == 1
          and A.shape[1] % 8 == 0 and M % 8 == 0 and B.stride(0) % 8 == 0 and B.data_ptr() % 16 == 0
          and (out is None or (out.stride(1) == 1 and out.stride(0) % 8 == 0 and out.data_ptr() % 16 == 0)))
    if ok:
        A = A.contiguous()
        return _ext.ops().gemm_skinny(A, B, out, accumulate)
    if not accumulate and _narrow_native_ok(A, B, out):
        # the narrow long-K products (x_dbl = W_x conv_out: 80 rows; d x_dbl[:R] = W_dt^T ddelta: 48 rows) on the
        # split-K engine: A as stored (KC rows, or XC for the transposed W_dt view), B channel-major (XC), one
        # 128-row tile (gemm_pipe_k with MI = 4) of which only the weight rows are live (hipBLASLt:
        # MAMBA_AMD_PROJ_GEMM=lib)
        la = 0 if A.stride(1) == 1 else 1
        a_ = A if la == 0 else A.t()
        return _ext.ops().gp_mm(a_, B, out, la, 1, 0, 1, 128 if A.shape[0] <= 128 else 256)
    if accumulate:
        return out.addmm_(A, B)
    return torch.mm(A, B, out=out) if out is not None else torch.mm(A, B)


class _NegExpFn(torch.autograd.Function):
    """A = -exp(A_log) (fp32), computed once per optimizer step inside an accumulation scope
    (ops/grad_accum.cached_value) instead of two elementwise launches per layer and micro-batch."""

    @staticmethod
    def forward(ctx, A_log):
        A = grad_accum.cached_value(A_log, "negexp", lambda t: -torch.exp(t.float()))
        ctx.save_for_backward(A)
        ctx.dtype = A_log.dtype
        return A.view_as(A)

    @staticmethod
    def backward(ctx, dA):
        (A,) = ctx.saved_tensors
        return (dA * A).to(ctx.dtype)


class _InProjCMFn(torch.autograd.Function):
    """xz (2di, b*l) = W_in h^T, channel-major (the Mamba-1 in_proj).  The bf16 weight cast is cached
    for the optimizer step (ops/grad_accum.py) and the weight gradient dW = d(xz) h runs on the native
    channel-major wgrad GEMM (csrc/kernels/gemm.hip, CM variant): fp32 out, added in place into
    ``.grad`` on the no-sync micro-steps (side stream), no bf16 -> fp32 cast."""

    @staticmethod
    def forward(ctx, h2, weight, cd):
        w = grad_accum.cached_cast(weight, cd)
        ctx.save_for_backward(h2, w)
        ctx.param = weight
        return mm_nt(w, h2)  # (2di, b*l): the persistent native GEMM (ops/linear.py) or hipBLASLt

    @staticmethod
    def backward(ctx, dxz):
        h2, w = ctx.saved_tensors
        if dxz.stride(1) != 1:
            dxz = dxz.contiguous()
        dh = None
        if ctx.needs_input_grad[0]:
            # dh (b*l, d) = dxz^T W with both operands stored contraction-major ([2di][tokens], [2di][d]): the
            # native split-K engine's XC . XC product (csrc/kernels/gemm_pipe.hip), bf16 out, no K split
            if _gp_xc_ok(dxz, w):
                dh = _ext.ops().gp_mm(dxz, w, None, 1, 1, 0, 1, 256)
            else:
                dh = torch.mm(dxz.t(), w)
        dw = None
        if ctx.needs_input_grad[1]:
            p = ctx.param
            handled, dw = _wgrad_native(p, dxz, h2, True, False)
            if not handled:
                dw = grad_accum.defer(p, torch.mm(dxz, h2).to(p.dtype))
        return dh, dw, None


def _narrow_native_ok(A: torch.Tensor, B: torch.Tensor, out) -> bool:
    """A (N, K) narrow weight (KC, or the transpose of a row-contiguous (K, N) weight), B (K, M) channel-major, bf16
    out (N, M): the gemm_pipe_k layouts (gemm_pipe_supported) and the projection engine switch."""
    from ..ops.linear import _pk_wins
    N, K = A.shape
    M = B.shape[1]
    kc = A.stride(1) == 1 and A.stride(0) % 8 == 0 and K % 8 == 0
    xc = A.stride(0) == 1 and A.stride(1) % 8 == 0 and N % 8 == 0
    return (A.is_cuda and A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16 and (kc or xc) and N <= 256
            and K >= 256 and B.stride(1) == 1 and B.stride(0) % 8 == 0 and M % 8 == 0 and M >= 4096
            and A.data_ptr() % 16 == 0 and B.data_ptr() % 16 == 0
            and (out is None or (out.stride(1) == 1 and out.stride(0) % 4 == 0 and out.data_ptr() % 16 == 0))
            and _pk_wins(N, M, K) and _ext.use_native(B))


def _gp_xc_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    """a (K, M) and b (K, N), both rows contiguous: the native XC . XC product C = a^T b (gemm_pipe_supported)."""
    return (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 2
            and a.stride(1) == 1 and b.stride(1) == 1 and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
            and a.shape[1] % 8 == 0 and b.shape[1] % 8 == 0 and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and a.shape[1] >= 4096 and _pk_wins_xc(a.shape[1], b.shape[1], a.shape[0]) and _ext.use_native(a))


def _pk_wins_xc(m: int, n: int, k: int) -> bool:
    """The projection-engine switch (MAMBA_AMD_PROJ_GEMM, ops/linear.py::_pk_wins) for the XC . XC input gradient."""
    from ..ops.linear import _pk_wins
    return _pk_wins(m, n, k, "dgrad_xc")


def _wgrad_native(p, dY, X, dy_cm, x_cm):
    """Weight gradient of a channel-major Mamba-1 projection: gemm_wgrad_cm (csrc/kernels/gemm.hip), its split-K
    slabs reduced every micro-step and added in place into ``p.grad`` on the no-sync micro-steps (weight-gradient
    side stream).  Returns (handled, dw); handled is False when the layout is not supported.
    Measured alternatives: the 256x256 pipelined engine with slabs deferred to the sync micro-step -0.7%
    (profiles/r2_v5_ab_m1_defer_wgrad.txt); keeping the
    slabs across micro-steps (gemm_wgrad_cm's ``part_mode`` add-into-slabs form) made the wgrad kernels
    read-modify-write their fp32 slabs (in_proj 190 -> 240 us, x/dt_proj 34 -> 60 us per call) for a 13 us
    reduce saved, and halved the overlapped step (profiles/r3/ab3_mamba1_deferral.txt)."""
    M = dY.shape[1] if dy_cm else dY.shape[0]
    ok = (dY.dtype == torch.bfloat16 and X.dtype == torch.bfloat16 and dY.stride(1) == 1 and X.stride(1) == 1
          and M % 64 == 0 and dY.stride(0) % 8 == 0 and X.stride(0) % 8 == 0 and dY.shape[0] % 8 == 0
          and X.shape[0] % 8 == 0 and dY.shape[1] % 8 == 0 and X.shape[1] % 8 == 0
          and dY.data_ptr() % 16 == 0 and X.data_ptr() % 16 == 0)
    if not ok:
        return False, None
    if grad_accum.sync_accumulable(p):  # sync micro-step, gradient in place: add into it (ops/grad_accum.py)
        _ext.ops().gemm_wgrad_cm(dY, X, p.grad, True, dy_cm, x_cm)
        return True, None
    if (grad_accum.accumulable(p) and p.grad.dtype == torch.float32 and p.grad.is_contiguous()
            and _wgrad_inplace(dY.device)):
        side = grad_accum.side_stream(dY.device)
        if side is None:
            _ext.ops().gemm_wgrad_cm(dY, X, p.grad, True, dy_cm, x_cm)
        else:
            side.wait_stream(torch.cuda.current_stream(dY.device))
            with torch.cuda.stream(side):
                _ext.ops().gemm_wgrad_cm(dY, X, p.grad, True, dy_cm, x_cm)
            grad_accum.side_keep(dY.device, dY, X)
        return True, None
    return True, grad_accum.defer(p, _ext.ops().gemm_wgrad_cm(dY, X, None, False, dy_cm, x_cm).to(p.dtype))


class _OutProjCMFn(torch.autograd.Function):
    """out (b*l, d) = y2^T W_out^T for the channel-major SSM output y2 (di, b*l), the Mamba-1 out_proj.
    Backward: d y2 comes out channel-major directly (W^T . dout^T), and dW = dout^T . y2^T runs on the native
    pipelined engine as fp32 split-K slabs (csrc/kernels/gemm_pipe.hip, dout token-major, y2 k-contiguous),
    deferred to the sync micro-step like the Mamba-2 projections (ops/linear.py::_wgrad_native)."""

    @staticmethod
    def forward(ctx, y2, weight, cd):
        w = grad_accum.cached_cast(weight, cd)
        ctx.save_for_backward(y2, w)
        ctx.param = weight
        T = y2.shape[1]
        if (y2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and y2.stride(1) == 1
                and y2.stride(0) % 8 == 0 and y2.data_ptr() % 16 == 0 and w.is_contiguous() and T % 8 == 0
                and w.shape[1] % 8 == 0 and T >= 4096):
            # y2 is channel-major (di, T): its transpose is the A operand as stored (k-rows of contiguous
            # tokens) on the pipelined engine; hipBLASLt's transposed-A solution ran 154 us here
            return _ext.ops().gp_mm(y2, w, None, 1, 0, 0, 1, 256)
        return F.linear(y2.t(), w)

    @staticmethod
    def backward(ctx, dout):
        from ..ops.linear import _native_ok, _wgrad_native
        y2, w = ctx.saved_tensors
        if dout.dtype != w.dtype:
            dout = dout.to(w.dtype)
        dout = dout.contiguous()
        dy2 = None
        if ctx.needs_input_grad[0]:
            dy2 = mm_nt(grad_accum.cached_transpose(ctx.param, w.dtype), dout)  # (di, b*l)
        dw = None
        if ctx.needs_input_grad[1]:
            p = ctx.param
            T = dout.shape[0]
            ok = (_native_ok(dout, dout) and y2.stride(1) == 1 and y2.stride(0) % 8 == 0 and y2.data_ptr() % 16 == 0
                  and y2.shape[0] % 8 == 0 and T % 8 == 0 and y2.dtype == torch.bfloat16)
            if ok:
                dw = _wgrad_native(p, dout, y2, lb=0)
                if dw is not None:
                    dw = grad_accum.defer(p, dw.to(p.dtype))
            else:
                dw = grad_accum.defer(p, torch.mm(dout.t(), y2.t()).to(p.dtype))
        return dy2, dw, None


class _Mamba1InnerFn(torch.autograd.Function):
    """conv1d+SiLU -> x_proj -> dt_proj -> selective scan(+D, *silu(z)) ; returns y as (di, b*l)."""

    @staticmethod
    def forward(ctx, xz, conv_w, conv_b, W_x, W_dt, dt_bias, A, D, b, l, compute_dtype):
        ops = _ext.ops()
        di = xz.shape[0] // 2
        R = W_dt.shape[1]
        N = A.shape[1]
        cd = compute_dtype
        xz3 = _cm(xz, b, l)
        x, z = xz3[:, :di], xz3[:, di:]
        w2 = conv_w.reshape(di, -1)
        conv_out = ops.conv1d_cf_fwd(x, w2, conv_b, True)                  # (b,di,l) in (di,b,l) memory
        co2 = _flat(conv_out)
        Wx, Wdt = grad_accum.cached_cast(W_x, cd), grad_accum.cached_cast(W_dt, cd)  # once per optimizer step
        x_dbl = _mm_cm(Wx, co2)                                             # (R+2N, b*l)
        Bm = _cm(x_dbl[R:R + N], b, l).unsqueeze(1)                         # (b,1,N,l)
        Cm = _cm(x_dbl[R + N:], b, l).unsqueeze(1)
        if _dt_fused_ok(b, l, di, N, Wdt, x_dbl, conv_out, z):
            # dt_proj inside the scan walk (MFMA per 16-step tile): delta is never written or re-read
            delta = None
            y, carries, _ = ops.selscan_fwd_dt(conv_out, Wdt, x_dbl[:R], A, Bm, Cm, D, z, dt_bias, True)
        else:
            delta = _mm_cm(Wdt, x_dbl[:R])                                  # (di, b*l)
            y, carries, _ = ops.selscan_fwd(conv_out, _cm(delta, b, l), A, Bm, Cm, D, z, dt_bias, True)
        ctx.save_for_backward(xz, w2, conv_b, Wx, Wdt, dt_bias, A, D, conv_out, x_dbl, delta, carries)
        ctx.meta = (b, l, conv_w.shape, W_x.dtype, W_dt.dtype)
        ctx.wparams = (W_x, W_dt)  # the parameters themselves (native weight gradients accumulate into .grad)
        # key of the deferred A / D / dt-bias partials: the dt bias parameter itself (fp32: .float() is the leaf)
        ctx.pkey = dt_bias if (dt_bias is not None and dt_bias.is_leaf and dt_bias.requires_grad) else None
        return _flat(y)

    @staticmethod
    def backward(ctx, dy2):
        xz, w2, conv_b, Wx, Wdt, dt_bias, A, D, conv_out, x_dbl, delta, carries = ctx.saved_tensors
        b, l, wshape, wx_dtype, wdt_dtype = ctx.meta
        ops = _ext.ops()
        di = xz.shape[0] // 2
        R = Wdt.shape[1]
        N = A.shape[1]
        xz3 = _cm(xz, b, l)
        x, z = xz3[:, :di], xz3[:, di:]
        dxz = torch.empty_like(xz)
        dxz3 = _cm(dxz, b, l)
        Bm = _cm(x_dbl[R:R + N], b, l).unsqueeze(1)
        Cm = _cm(x_dbl[R + N:], b, l).unsqueeze(1)
        dx_dbl = torch.empty_like(x_dbl)
        # the A / D / dt-bias gradient partials (B x D x (N + 2) fp32) are summed over the batch once per optimizer
        # step, even though Mamba-1 reduces its other partials every micro-step (microbatch.auto_defer_reduce):
        # per micro-step that reduction is a zero fill, two batch sums, casts and three small gradient adds
        d_s = (grad_accum.deferred(ctx.pkey, "selscan_small", (b * di * (N + 2),), xz.device, force=True)
               if ctx.pkey is not None else None)
        dyc = dy2.contiguous() if dy2.stride(-1) != 1 else dy2
        outs = (dxz3[:, di:], _cm(dx_dbl[R:R + N], b, l).unsqueeze(1), _cm(dx_dbl[R + N:], b, l).unsqueeze(1),
                *(d_s or (None, 0)))
        if delta is None:  # fused dt_proj forward: the backward walk recomputes delta the same way
            if dyc.data_ptr() % 16 or dyc.stride(0) % 8:
                dyc = dyc.contiguous().clone()
            du, ddelta, dA, dB, dC, dD, dz, ddt_bias = ops.selscan_bwd_dt_into(
                _cm(dyc, b, l), conv_out, Wdt, x_dbl[:R], A, Bm, Cm, D, z, dt_bias, carries, True, *outs)
        else:
            du, ddelta, dA, dB, dC, dD, dz, ddt_bias = ops.selscan_bwd_into(
                _cm(dyc, b, l), conv_out, _cm(delta, b, l), A, Bm, Cm, D, z, dt_bias, carries, True, *outs)
        nz = lambda t: t if t.numel() else None  # noqa: E731  (empty: deferred to the sync micro-step)
        dA, dD, ddt_bias = nz(dA), nz(dD), nz(ddt_bias)
        dd2 = _flat(ddelta)
        pWx, pWdt = ctx.wparams
        # both operands channel-major: (di, M) . (R, M)^T on the native wgrad GEMM
        ok_dt, dWdt = _wgrad_native(pWdt, dd2, x_dbl[:R], True, True)
        if not ok_dt:
            dWdt = torch.mm(dd2, x_dbl[:R].t()).to(wdt_dtype)                # (di, R)
        _mm_cm(Wdt.t(), dd2, out=dx_dbl[:R])                                # d x_dbl[:R]
        ok_x, dWx = _wgrad_native(pWx, dx_dbl, _flat(conv_out), True, True)
        if not ok_x:
            dWx = torch.mm(dx_dbl, _flat(conv_out).t()).to(wx_dtype)         # (R+2N, di)
        dco2 = _flat(du)
        _mm_cm(Wx.t(), dx_dbl, out=dco2, accumulate=True)                   # du + W_x^T dx_dbl
        _, dw, db = ops.conv1d_cf_bwd(x, w2, conv_b, _cm(dco2, b, l), True, dxz3[:, :di])
        return (dxz, dw.reshape(wshape).to(w2.dtype), db.to(conv_b.dtype) if conv_b is not None else None,
                dWx, dWdt, ddt_bias, dA, dD, None, None, None)


def _dt_fused_ok(b, l, di, N, Wdt, x_dbl, conv_out, z) -> bool:
    """dt_proj fused into the selective-scan walk (csrc/kernels/selective_scan.hip, DTF; selscan_dt_fusable mirrored
    here): the wave-per-state-group kernels (bf16, d_state 16, 64-channel groups, b * di >= 32768, l % 16 == 0) and a
    dt_rank the 4-step MFMA chain covers.  Opt-in (MAMBA_AMD_M1_DT_FUSED=1): it removes the delta GEMM (53 us per
    280M layer) and the saved (b, di, l) delta (12 GB of activations per 64k-token micro-batch at Mamba-1 280M), but
    the per-tile MFMA + extra barrier costs the forward walk 34 us and the backward walk 40 us, so the step is 0.5%
    slower (profiles/r5/m1_dt_fused_ab.txt).  Worth it where activation memory, not time, is the limit."""
    import os
    R = Wdt.shape[1]
    if os.environ.get("MAMBA_AMD_M1_DT_FUSED", "0") != "1":
        return False
    zok = z is None or (z.stride(0) % 8 == 0 and z.stride(1) % 8 == 0 and z.data_ptr() % 16 == 0)
    return (conv_out.dtype == torch.bfloat16 and x_dbl.dtype == torch.bfloat16 and Wdt.dtype == torch.bfloat16
            and Wdt.is_contiguous() and N == 16 and di % 64 == 0 and l % 16 == 0 and b * di >= 32768
            and 0 < R <= 128 and R % 8 == 0 and x_dbl.stride(1) == 1 and x_dbl.stride(0) % 8 == 0
            and x_dbl.data_ptr() % 16 == 0 and Wdt.data_ptr() % 16 == 0 and conv_out.stride(0) % 8 == 0
            and conv_out.stride(1) % 8 == 0 and conv_out.data_ptr() % 16 == 0 and zok)


def mamba1_inner_ref(xz3, conv_w, conv_b, W_x, W_dt, dt_bias, A, D):
    """Pure-torch composition of the same path (CPU / oracle).  xz3: (b, 2di, l)."""
    di = xz3.shape[1] // 2
    R = W_dt.shape[1]
    N = A.shape[1]
    x, z = xz3[:, :di], xz3[:, di:]
    conv_out = causal_conv1d_ref(x, conv_w.reshape(di, -1), conv_b, "silu")
    x_dbl = torch.einsum("rd,bdl->brl", W_x.to(conv_out.dtype), conv_out)
    delta = torch.einsum("dr,brl->bdl", W_dt.to(x_dbl.dtype), x_dbl[:, :R])
    Bm = x_dbl[:, R:R + N].unsqueeze(1)
    Cm = x_dbl[:, R + N:].unsqueeze(1)
    return selective_scan_ref(conv_out, delta, A, Bm, Cm, D, z, dt_bias, True)


class Mamba(nn.Module):
    def __init__(self, d_model, d_state=16, d_conv=4, expand=2, dt_rank="auto", dt_min=0.001,
                 dt_max=0.1, dt_init="random", dt_scale=1.0, dt_init_floor=1e-4, conv_bias=True,
                 bias=False, use_fast_path=True, layer_idx=None, device=None, dtype=None):
        factory = {"device": device, "dtype": dtype}
        super().__init__()
        self.d_model = d_model
        self.d_state = d_state
        self.d_conv = d_conv
        self.expand = expand
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16) if dt_rank == "auto" else dt_rank
        self.use_fast_path = use_fast_path
        self.layer_idx = layer_idx

        self.in_proj = nn.Linear(d_model, self.d_inner * 2, bias=bias, **factory)
        self.conv1d = nn.Conv1d(self.d_inner, self.d_inner, bias=conv_bias, kernel_size=d_conv,
                                groups=self.d_inner, padding=d_conv - 1, **factory)
        self.activation = "silu"
        self.act = nn.SiLU()
        self.x_proj = nn.Linear(self.d_inner, self.dt_rank + d_state * 2, bias=False, **factory)
        self.dt_proj = nn.Linear(self.dt_rank, self.d_inner, bias=True, **factory)

        dt_init_std = self.dt_rank ** -0.5 * dt_scale
        with torch.no_grad():
            if dt_init == "constant":
                nn.init.constant_(self.dt_proj.weight, dt_init_std)
            elif dt_init == "random":
                nn.init.uniform_(self.dt_proj.weight, -dt_init_std, dt_init_std)
            else:
                raise NotImplementedError(dt_init)
            dt = torch.exp(torch.rand(self.d_inner, **factory) * (math.log(dt_max) - math.log(dt_min))
                           + math.log(dt_min)).clamp(min=dt_init_floor)
            self.dt_proj.bias.copy_(softplus_inverse(dt))
        self.dt_proj.bias._no_reinit = True

        A = torch.arange(1, d_state + 1, dtype=torch.float32, device=device).repeat(self.d_inner, 1)
        self.A_log = nn.Parameter(torch.log(A))
        self.A_log._no_weight_decay = True
        self.D = nn.Parameter(torch.ones(self.d_inner, device=device))
        self.D._no_weight_decay = True
        self.out_proj = nn.Linear(self.d_inner, d_model, bias=bias, **factory)

    # ------------------------------------------------------------------
    def forward(self, hidden_states, inference_params=None):
        b, l, _ = hidden_states.shape
        if inference_params is not None:
            conv_state, ssm_state = self._get_states_from_cache(inference_params, b)
            if inference_params.seqlen_offset > 0:
                out, _, _ = self.step(hidden_states, conv_state, ssm_state)
                return out
        else:
            conv_state = ssm_state = None
        cd = torch.get_autocast_dtype("cuda") if (hidden_states.is_cuda and torch.is_autocast_enabled("cuda")) else hidden_states.dtype
        A = _NegExpFn.apply(self.A_log) if self.A_log.requires_grad else -torch.exp(self.A_log.float())
        h2 = hidden_states.reshape(b * l, -1).to(cd)
        if _ext.use_native(h2) and self.in_proj.weight.requires_grad:
            xz = _InProjCMFn.apply(h2, self.in_proj.weight, cd)            # (2di, b*l)
        else:
            xz = torch.mm(self.in_proj.weight.to(cd), h2.t())              # (2di, b*l)
        if self.in_proj.bias is not None:
            xz = xz + self.in_proj.bias.to(cd)[:, None]
        if conv_state is None and self.use_fast_path and _ext.use_native(xz):
            y2 = _Mamba1InnerFn.apply(xz, self.conv1d.weight, self.conv1d.bias, self.x_proj.weight,
                                      self.dt_proj.weight, self.dt_proj.bias.float(), A, self.D.float(),
                                      b, l, cd)
            if self.out_proj.bias is None and y2.dtype == cd:
                out = _OutProjCMFn.apply(y2, self.out_proj.weight, cd)
            else:
                out = F.linear(y2.t().to(cd), grad_accum.cached_cast(self.out_proj.weight, cd),
                               None if self.out_proj.bias is None else self.out_proj.bias.to(cd))
            return out.view(b, l, -1)
        xz3 = _cm(xz, b, l)
        if conv_state is not None:  # prefill: remember the last d_conv-1 inputs for decoding
            x = xz3[:, :self.d_inner]
            sl = conv_state.shape[-1]  # upstream layout: the last d_conv inputs
            conv_state.copy_(F.pad(x, (max(0, sl - l), 0))[..., -sl:])
            y, last = self._inner_with_state(xz3, A)
            ssm_state.copy_(last)
        else:
            y = mamba1_inner_ref(xz3, self.conv1d.weight, self.conv1d.bias, self.x_proj.weight,
                                 self.dt_proj.weight, self.dt_proj.bias.float(), A, self.D.float())
        out = F.linear(y.transpose(1, 2).to(cd), self.out_proj.weight.to(cd),
                       None if self.out_proj.bias is None else self.out_proj.bias.to(cd))
        return out

    def _inner_with_state(self, xz3, A):
        """Prompt pass that also returns the final SSM state (cache fill for decoding): native
        conv + scan kernels on a GPU (the scan returns its last state), oracles on the CPU."""
        di = self.d_inner
        R, N = self.dt_rank, self.d_state
        x, z = xz3[:, :di], xz3[:, di:]
        conv_out = causal_conv1d_fn(x, self.conv1d.weight.reshape(di, -1), self.conv1d.bias, "silu")
        x_dbl = torch.einsum("rd,bdl->brl", self.x_proj.weight.to(conv_out.dtype), conv_out)
        delta = torch.einsum("dr,brl->bdl", self.dt_proj.weight.to(x_dbl.dtype), x_dbl[:, :R])
        return selective_scan_fn(conv_out, delta, A, x_dbl[:, R:R + N].unsqueeze(1),
                                 x_dbl[:, R + N:].unsqueeze(1), self.D.float(), z,
                                 self.dt_proj.bias.float(), True, return_last_state=True)

    @torch.no_grad()
    def step(self, hidden_states, conv_state, ssm_state):
        """One decode token.  hidden_states (b, 1, d)."""
        dtype = hidden_states.dtype
        h = hidden_states.squeeze(1)
        xz = F.linear(h, self.in_proj.weight.to(h.dtype),
                      None if self.in_proj.bias is None else self.in_proj.bias.to(h.dtype))
        x, z = xz.chunk(2, dim=-1)
        x = causal_conv1d_update(x, conv_state, self.conv1d.weight, self.conv1d.bias, "silu")
        x_db = F.linear(x, self.x_proj.weight.to(x.dtype))
        dt, B, C = torch.split(x_db, [self.dt_rank, self.d_state, self.d_state], dim=-1)
        dt = F.linear(dt, self.dt_proj.weight.to(dt.dtype))
        A = -torch.exp(self.A_log.float())
        y = selective_state_update(ssm_state, x, dt, A, B, C, self.D.float(), z=z,
                                   dt_bias=self.dt_proj.bias.float(), dt_softplus=True)
        out = F.linear(y, self.out_proj.weight.to(y.dtype),
                       None if self.out_proj.bias is None else self.out_proj.bias.to(y.dtype))
        return out.unsqueeze(1).to(dtype), conv_state, ssm_state

    def allocate_inference_cache(self, batch_size, max_seqlen, dtype=None, **kwargs):
        device = self.out_proj.weight.device
        conv_dtype = self.conv1d.weight.dtype if dtype is None else dtype
        conv_state = torch.zeros(batch_size, self.d_inner, self.d_conv, device=device, dtype=conv_dtype)  # upstream width
        ssm_state = torch.zeros(batch_size, self.d_inner, self.d_state, device=device, dtype=torch.float32)
        return conv_state, ssm_state

    def _get_states_from_cache(self, inference_params, batch_size):
        assert self.layer_idx is not None
        if self.layer_idx not in inference_params.key_value_memory_dict:
            inference_params.key_value_memory_dict[self.layer_idx] = self.allocate_inference_cache(
                batch_size, inference_params.max_seqlen)
        return inference_params.key_value_memory_dict[self.layer_idx]
