"""Mamba-2 SSD (state-space duality) chunked scan — the Mamba-2 hot op.

Call surface mirrors upstream ``mamba_chunk_scan_combined`` / ``mamba_split_conv1d_scan_combined``
(SURVEY.md D11/D12, T1-T5, T8); the reference reaches them through ``Mamba2.forward``.

GPU implementation (csrc/kernels/ssd.hip; 64-step chunks on v_mfma_f32_16x16x32_bf16):
  fwd  1. ``ssd_cumsum``     wave per (b, h, chunk): dt = softplus(dt + bias) (clamped), in-chunk wave64
          inclusive scan of dt*A.
       2. ``ssd_fused_fwd``  one workgroup per (h, b) walks the chunks in order with the running state
          S (P x N) in MFMA accumulators: per chunk y = e^{cum} C S^T + (C B^T o L o dt) x + D x (the
          masked C B^T accumulator feeds the next MFMA as its operand) and S <- e^{cum_last} S + (w x)^T B;
          the state entering every chunk is saved (bf16) for the backward.
  bwd  3. ``ssd_dstate_bwd`` reverse chunk walk per (h, b): dS entering every chunk (bf16), dS_init.
       4. ``ssd_chunk_bwd``  workgroup per (chunk, head group, b): dM, M, dX, ddt (with the in-chunk
          reverse cumsum of dcum), dA / dD / dt_bias partial rows; head-summed dCB, dB_off, dC_off stay
          in registers across the heads of the group.
       5. ``ssd_dbc_bwd``    workgroup per (chunk, group, b): dC = sum dC_off + dCB B, dB = sum dB_off
          + dCB^T C.
  No float atomics: every cross-workgroup sum goes through fixed-order partials (bitwise deterministic).
CPU: ``reference.ssd_chunked_ref`` under autograd.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _ext, grad_accum
from .reference import ssd_chunked_ref, gated_rms_norm_ref, causal_conv1d_ref

_INF = float("inf")

# chunk length used by the HIP kernels (a pure implementation detail: results are identical up to
# fp rounding for any chunk size); 64 keeps every per-chunk tile MFMA/LDS friendly on gfx950.
NATIVE_CHUNK = 64


class _SSDFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dt, A, B, C, D, dt_bias, initial_states, dt_softplus, dt_min, dt_max,
                return_final_states, seq_idx=None):
        ops = _ext.ops()
        y, cum, dtp, states, final = ops.ssd_fwd(x, dt, A, B, C, D, dt_bias, initial_states,
                                                  NATIVE_CHUNK, dt_softplus, dt_min, dt_max, False, seq_idx)
        ctx.save_for_backward(x, dt, A, B, C, D, dt_bias, initial_states, cum, dtp, states)
        ctx.flags = (dt_softplus, dt_min, dt_max)
        ctx.return_final = return_final_states
        ctx.params = (A, D, dt_bias)
        ctx.set_materialize_grads(False)
        if return_final_states:
            return y, final
        return y

    @staticmethod
    def backward(ctx, dy, *rest):
        x, dt, A, B, C, D, dt_bias, init, cum, dtp, states = ctx.saved_tensors
        dfinal = rest[0] if ctx.return_final and len(rest) else None
        softplus, dt_min, dt_max = ctx.flags
        if dy is None:
            dy = torch.zeros_like(x)
        g = _ext.ops().ssd_bwd(dy.contiguous(), x, dt, A, B, C, D, dt_bias, init, cum, dtp, states,
                               dfinal, NATIVE_CHUNK, softplus, dt_min, dt_max, None, None, None, None)
        dx, ddt, dA, dB, dC, dD, ddt_bias, dinit = g
        pA, pD, pdtb = ctx.params
        d = grad_accum.defer
        return (dx, ddt, d(pA, dA), dB, dC,
                d(pD, dD) if D is not None else None,
                d(pdtb, ddt_bias) if dt_bias is not None else None,
                dinit if init is not None else None,
                None, None, None, None, None)


def _f32_eval_ok(x, dt, B, C, D, init, seq_idx) -> bool:
    """fp32 SSD forward on the native sequential kernel: fp32 operands, no autograd, headdim 64,
    d_state 64/128, per-head D, no packed sequences."""
    if x.dtype != torch.float32 or B.dtype != torch.float32 or C.dtype != torch.float32:
        return False
    if not _ext.use_native(x) or seq_idx is not None or x.shape[-1] != 64 or B.shape[-1] not in (64, 128):
        return False
    if D is not None and D.dim() != 1:
        return False
    ts = [t for t in (x, dt, B, C, D, init) if t is not None]
    return not (torch.is_grad_enabled() and any(t.requires_grad for t in ts))


def mamba_chunk_scan_combined(x, dt, A, B, C, chunk_size=256, D=None, z=None, dt_bias=None,
                              initial_states=None, seq_idx=None, dt_softplus=False,
                              dt_limit=(0.0, _INF), return_final_states=False):
    """x (b,l,h,p), dt (b,l,h), A (h), B/C (b,l,g,n) -> y (b,l,h,p) [, final_states (b,h,p,n)].

    ``seq_idx`` (b,l) int, non-decreasing per row: packed variable-length sequences; the scan state
    restarts at every change (native: the in-chunk cumsum gets a -256 offset at each sequence
    start, so every decay factor across the boundary is exactly 0 in fp32 -- the same masks as
    upstream, with unchanged gradients).  ``initial_states`` belong to the row's first sequence."""
    # native MFMA kernels are bf16 (the training/serving dtype); fp32 activations without autograd (the
    # reference's fp32 HellaSwag eval) run the native fp32 sequential forward
    if _f32_eval_ok(x, dt, B, C, D, initial_states, seq_idx):
        x, B, C = (t if t.stride(-1) == 1 else t.contiguous() for t in (x, B, C))
        y, fin = _ext.ops().ssd_fwd_f32(x, dt.float(), A, B, C, D, dt_bias,
                                        None if initial_states is None else initial_states.float(),
                                        dt_softplus, float(dt_limit[0]), float(dt_limit[1]), return_final_states)
        if z is not None:
            y = y * F.silu(z.float())
        y = y.to(x.dtype)
        return (y, fin) if return_final_states else y
    if x.dtype == torch.bfloat16 and _ext.use_native(x):
        hdim_D = D is not None and D.dim() == 2  # per-channel skip (h, p): added after the native scan
        out = _SSDFn.apply(x, dt, A, B, C, None if hdim_D else D, dt_bias, initial_states, dt_softplus,
                           float(dt_limit[0]), float(dt_limit[1]), return_final_states, seq_idx)
        if z is not None or hdim_D:  # upstream's (y + x D) * silu(z) (elementwise, fp32 math, autograd)
            y, fin = out if return_final_states else (out, None)
            yf = y.float()
            if hdim_D:
                yf = yf + x.float() * D.float()
            if z is not None:
                yf = yf * F.silu(z.float())
            y = yf.to(y.dtype)
            return (y, fin) if return_final_states else y
        return out
    return ssd_chunked_ref(x, dt, A, B, C, chunk_size, D=D, z=z, dt_bias=dt_bias,
                           dt_softplus=dt_softplus, dt_limit=dt_limit, initial_states=initial_states,
                           return_final_states=return_final_states, seq_idx=seq_idx)


# ----------------------------------------------------------------------------------------
# Fused Mamba-2 inner path: conv1d(xBC)+SiLU -> SSD -> gated RMSNorm   (out_proj stays outside, on the
# native persistent GEMM of ops/linear.py)
# ----------------------------------------------------------------------------------------
class _Mamba2InnerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, zxbcdt, conv_w, conv_b, dt_bias, A, D, norm_w, eps, headdim, ngroups, d_state,
                dt_min, dt_max, norm_before_gate, A_is_log=False, initial_states=None, seq_idx=None,
                return_final_states=False):
        ops = _ext.ops()
        b, l, dproj = zxbcdt.shape
        H = dt_bias.shape[0]
        di = H * headdim
        conv_dim = di + 2 * ngroups * d_state
        assert dproj == 2 * di + 2 * ngroups * d_state + H, "only d_mlp == 0 layouts are supported"
        if zxbcdt.stride(-1) != 1 or zxbcdt.stride(-2) % 8 or zxbcdt.stride(0) != l * zxbcdt.stride(-2):
            # the native conv / SSD / norm kernels want 16-B aligned rows: an odd width (nheads % 8 != 0 without
            # the padded in_proj) is copied into rows of a multiple of 8 columns
            full = torch.empty(b, l, (dproj + 7) // 8 * 8, device=zxbcdt.device, dtype=zxbcdt.dtype)
            full[..., :dproj].copy_(zxbcdt)
            zxbcdt = full[..., :dproj]
        z = zxbcdt[..., :di]
        xBC = zxbcdt[..., di:di + conv_dim]
        dt = zxbcdt[..., di + conv_dim:]
        w2 = conv_w.reshape(conv_dim, -1)
        if seq_idx is None:
            xBC_c = ops.conv1d_cl_fwd(xBC, w2, conv_b, True)                # (b, l, conv_dim)
        else:
            xBC_c, _ = ops.conv1d_cl_var_fwd(xBC, w2, conv_b, True, seq_idx, None, False)
        x = xBC_c[..., :di].unflatten(-1, (H, headdim))
        Bm = xBC_c[..., di:di + ngroups * d_state].unflatten(-1, (ngroups, d_state))
        Cm = xBC_c[..., di + ngroups * d_state:].unflatten(-1, (ngroups, d_state))
        y, cum, dtp, states, final = ops.ssd_fwd(x, dt, A, Bm, Cm, D, dt_bias, initial_states, NATIVE_CHUNK,
                                                 True, dt_min, dt_max, A_is_log, seq_idx)
        y2 = y.view(b * l, di)
        yn, rstd = ops.gated_rmsnorm_fwd(y2, z.flatten(0, 1), norm_w, eps, di // ngroups, norm_before_gate)
        ctx.save_for_backward(zxbcdt, w2, conv_b, dt_bias, A, D, norm_w, xBC_c, y, rstd, cum, dtp, states,
                              initial_states, seq_idx)
        ctx.meta = (eps, headdim, ngroups, d_state, dt_min, dt_max, norm_before_gate, A_is_log)
        ctx.wshape = conv_w.shape
        ctx.params = (conv_w, conv_b, dt_bias, A, D, norm_w)
        ctx.ret_final = return_final_states
        # unused outputs (final when not requested) must not get materialised zero gradients: that was a
        # 25 MB fill per layer per micro-step at the 280M shape
        ctx.set_materialize_grads(False)
        if not return_final_states:
            ctx.mark_non_differentiable(final)
        return yn.view(b, l, di), final

    @staticmethod
    def backward(ctx, dyn, dfinal):
        (zxbcdt, w2, conv_b, dt_bias, A, D, norm_w, xBC_c, y, rstd, cum, dtp, states, init,
         seq_idx) = ctx.saved_tensors
        if dyn is None:
            dyn = torch.zeros(zxbcdt.shape[0], zxbcdt.shape[1], dt_bias.shape[0] * ctx.meta[1],
                              device=zxbcdt.device, dtype=zxbcdt.dtype)
        eps, headdim, ngroups, d_state, dt_min, dt_max, nbg, a_log = ctx.meta
        ops = _ext.ops()
        b, l, dproj = zxbcdt.shape
        H = dt_bias.shape[0]
        di = H * headdim
        gn = ngroups * d_state
        conv_dim = di + 2 * gn
        rs = zxbcdt.stride(-2)
        # (the pad must start 16-B aligned and span whole 8-column groups for the chunk backward's zero fill:
        # dproj % 8 == 0, i.e. nheads % 8 == 0 at the default layout; other widths take the unpadded gradient)
        if rs > dproj and rs % 64 == 0 and dproj % 8 == 0 and zxbcdt.stride(0) == l * rs:
            # zxbcdt is the column view of a padded in_proj output (ops/linear.py): write d(zxbcdt) into the
            # same layout with zero pad columns, so the in_proj input gradient runs on 128-B aligned rows
            # (the pad columns are zeroed by the SSD chunk backward, beside the dt gradient it writes: ddt_zero_pad)
            dz_full = torch.empty(b, l, rs, device=zxbcdt.device, dtype=zxbcdt.dtype)
            dz_all = dz_full[..., :dproj]
        else:
            dz_full = None
            # rows of a multiple of 8 columns (16-B aligned) for the gated-norm / SSD / conv gradient writers
            dz_all = torch.empty(b, l, (dproj + 7) // 8 * 8, device=zxbcdt.device, dtype=zxbcdt.dtype)[..., :dproj]
        z = zxbcdt[..., :di]
        pw, pb, pdtb, pA, pD, pn = ctx.params
        dev = zxbcdt.device
        # parameter-gradient partials are reduced once per optimizer step (grad_accum.deferred)
        d_n = grad_accum.deferred(pn, "gated_rmsnorm", (ops.part_rows("gated_rmsnorm", b * l), di), dev)
        d_s = grad_accum.deferred(pA, "ssd_small", (b * ((l + NATIVE_CHUNK - 1) // NATIVE_CHUNK), 3, H), dev)
        ck = "conv_cl" if seq_idx is None else "conv_cl_var"
        # one tag for both conv kernels: their partial rows differ, so seq_idx appearing on only some micro-steps
        # of a step is refused by grad_accum.deferred instead of silently starting a second buffer
        d_c = grad_accum.deferred(pw, "conv_cl", (ops.part_rows(ck, b, l), conv_dim, w2.shape[1] + 1), dev)
        # sync micro-step: leave the three partial blocks unreduced and queue them for the batched late column sum
        # after the backward (ops/grad_accum.py::flush_late) instead of two launches each here
        late = (d_n is not None and d_s is not None and d_c is not None and d_n[1] >= 3 and d_s[1] >= 3
                and d_c[1] >= 3 and grad_accum.late_ok(pn, pA, pD, pdtb, pw, pb))
        if late:
            d_n, d_s, d_c = (d_n[0], d_n[1] - 2), (d_s[0], d_s[1] - 2), (d_c[0], d_c[1] - 2)
        # gated norm backward writes dz straight into its slice of d(zxbcdt)
        dy, _, dnorm_w = ops.gated_rmsnorm_bwd(dyn.reshape(b * l, di), y.view(b * l, di),
                                               z.flatten(0, 1), norm_w, rstd, di // ngroups, nbg,
                                               None, dz_all[..., :di].flatten(0, 1), *(d_n or (None, 0)))
        x = xBC_c[..., :di].unflatten(-1, (H, headdim))
        Bm = xBC_c[..., di:di + gn].unflatten(-1, (ngroups, d_state))
        Cm = xBC_c[..., di + gn:].unflatten(-1, (ngroups, d_state))
        dt = zxbcdt[..., di + conv_dim:]
        dxBC_c = torch.empty_like(xBC_c)
        g = ops.ssd_bwd(dy.view(b, l, H, headdim), x, dt, A, Bm, Cm, D, dt_bias, init, cum, dtp, states,
                        dfinal if ctx.ret_final else None, NATIVE_CHUNK, True, dt_min, dt_max,
                        dxBC_c[..., :di].unflatten(-1, (H, headdim)),
                        dz_all[..., di + conv_dim:],
                        dxBC_c[..., di:di + gn].unflatten(-1, (ngroups, d_state)),
                        dxBC_c[..., di + gn:].unflatten(-1, (ngroups, d_state)), a_log, *(d_s or (None, 0)),
                        (rs - dproj) if dz_full is not None else 0)
        _, _, dA, _, _, dD, ddt_bias, dinit = g
        xBC = zxbcdt[..., di:di + conv_dim]
        if seq_idx is None:
            _, dw, db = ops.conv1d_cl_bwd(xBC, w2, conv_b, dxBC_c, True, dz_all[..., di:di + conv_dim],
                                          *(d_c or (None, 0)))
        else:
            _, dw, db, _ = ops.conv1d_cl_var_bwd(xBC, w2, conv_b, dxBC_c, True, seq_idx, None, None,
                                                 dz_all[..., di:di + conv_dim], *(d_c or (None, 0)))
        d = grad_accum.defer
        nz = lambda t: t if t.numel() else None  # noqa: E731  (empty = deferred to the sync micro-step)
        dw = nz(dw)
        if late:
            grad_accum.late_colsum(d_n[0], 0, 0, [pn])
            grad_accum.late_colsum(d_s[0], 2, H, [pA, pD, pdtb])
            grad_accum.late_colsum(d_c[0], 1, w2.shape[1] + 1, [pw, pb])
        if dz_full is not None:
            from .linear import register_zero_padded_grad
            register_zero_padded_grad(dz_full)
        return (dz_all, d(pw, dw.reshape(ctx.wshape).to(w2.dtype)) if dw is not None else None,
                d(pb, nz(db).to(conv_b.dtype)) if (conv_b is not None and db.numel()) else None,
                d(pdtb, nz(ddt_bias)), d(pA, nz(dA)), d(pD, nz(dD)), d(pn, nz(dnorm_w)),
                None, None, None, None, None, None, None, None,
                dinit if init is not None else None, None, None)


def mamba2_inner_ref(zxbcdt, conv_w, conv_b, dt_bias, A, D, norm_w, eps, headdim, ngroups, d_state,
                     dt_limit=(0.0, _INF), norm_before_gate=False, chunk_size=64, initial_states=None,
                     seq_idx=None, return_final_states=False, native_ssd=False):
    """The composed reference (PyTorch ops); ``native_ssd``: the SSD step through
    ``mamba_chunk_scan_combined`` (fp32 inference -> the native fp32 forward)."""
    b, l, dproj = zxbcdt.shape
    H = dt_bias.shape[0]
    di = H * headdim
    gn = ngroups * d_state
    conv_dim = di + 2 * gn
    z, xBC, dt = torch.split(zxbcdt, [di, conv_dim, H], dim=-1)
    xBC = causal_conv1d_ref(xBC.transpose(1, 2), conv_w.reshape(conv_dim, -1), conv_b, "silu",
                            seq_idx=seq_idx).transpose(1, 2)
    x, Bm, Cm = torch.split(xBC, [di, gn, gn], dim=-1)
    ssd = mamba_chunk_scan_combined if native_ssd else ssd_chunked_ref
    y = ssd(x.unflatten(-1, (H, headdim)), dt, A, Bm.unflatten(-1, (ngroups, d_state)),
            Cm.unflatten(-1, (ngroups, d_state)), chunk_size, D=D, dt_bias=dt_bias,
            dt_softplus=True, dt_limit=dt_limit, initial_states=initial_states,
            return_final_states=return_final_states, seq_idx=seq_idx)
    y, final = y if return_final_states else (y, None)
    y = gated_rms_norm_ref(y.flatten(-2), z, norm_w, eps, di // ngroups, norm_before_gate)
    return (y, final) if return_final_states else y


def mamba2_inner_fn(zxbcdt, conv_w, conv_b, dt_bias, A, D, norm_w, eps, headdim, ngroups, d_state,
                    dt_limit=(0.0, _INF), norm_before_gate=False, ref_chunk_size=64, A_is_log=False,
                    initial_states=None, seq_idx=None, return_final_states=False):
    """conv1d+SiLU -> SSD -> gated RMSNorm on the in_proj output; returns (b, l, d_inner)
    [, final SSM states (b, h, p, n) fp32].
    ``A_is_log``: ``A`` is the A_log parameter; the kernels apply A = -exp(A_log) and return dA_log
    (saves the per-layer exp/neg launches and their backward).  ``initial_states`` (b, h, p, n) SSM
    states entering the sequence (gradients flow); ``seq_idx`` (b, l) packed variable-length rows
    (conv taps and the scan state never cross a change)."""
    if zxbcdt.dtype == torch.bfloat16 and _ext.use_native(zxbcdt):
        if seq_idx is not None:
            seq_idx = seq_idx.to(torch.int32).contiguous()
        if initial_states is not None:
            initial_states = initial_states.float().contiguous()
        y, final = _Mamba2InnerFn.apply(zxbcdt, conv_w, conv_b, dt_bias, A, D, norm_w, eps, headdim,
                                        ngroups, d_state, float(dt_limit[0]), float(dt_limit[1]),
                                        norm_before_gate, A_is_log, initial_states, seq_idx,
                                        return_final_states)
        return (y, final) if return_final_states else y
    if A_is_log:
        A = -torch.exp(A.float())
    return mamba2_inner_ref(zxbcdt, conv_w, conv_b, dt_bias, A, D, norm_w, eps, headdim, ngroups,
                            d_state, dt_limit, norm_before_gate, ref_chunk_size, initial_states,
                            seq_idx, return_final_states, native_ssd=True)


def _split_conv1d_scan_general(zxbcdt, conv1d_weight, conv1d_bias, dt_bias, A, D, chunk_size, initial_states,
                               seq_idx, dt_limit, return_final_states, rmsnorm_weight, rmsnorm_eps, headdim,
                               ngroups, d_state, norm_before_gate):
    """conv1d+SiLU -> SSD -> (+ x D per channel) -> silu(z) gate or gated RMSNorm, from the native ops."""
    from .conv1d import causal_conv1d_fn
    from .norm import rmsnorm_gated_fn
    b, l, _ = zxbcdt.shape
    H = dt_bias.shape[0]
    di, gn = H * headdim, ngroups * d_state
    z, xBC, dt = torch.split(zxbcdt, [di, di + 2 * gn, H], dim=-1)
    if zxbcdt.stride(-2) % 8:
        z, xBC, dt = z.contiguous(), xBC.contiguous(), dt.contiguous()
    xBC = causal_conv1d_fn(xBC.transpose(1, 2), conv1d_weight, conv1d_bias, "silu", seq_idx=seq_idx).transpose(1, 2)
    x, B, C = torch.split(xBC, [di, gn, gn], dim=-1)
    xh = x.unflatten(-1, (H, headdim))
    res = mamba_chunk_scan_combined(xh, dt, A, B.unflatten(-1, (ngroups, d_state)),
                                    C.unflatten(-1, (ngroups, d_state)), chunk_size,
                                    D=D if D.dim() == 1 else None, dt_bias=dt_bias, dt_softplus=True,
                                    dt_limit=dt_limit, seq_idx=seq_idx, initial_states=initial_states,
                                    return_final_states=return_final_states)
    y, final = res if return_final_states else (res, None)
    if D.dim() == 2:
        y = y + xh * D.to(y.dtype)
    y = y.flatten(-2)
    if rmsnorm_weight is None:
        y = y * F.silu(z)
    else:
        y = rmsnorm_gated_fn(y, z, rmsnorm_weight, rmsnorm_eps, di // ngroups, norm_before_gate)
    return (y, final) if return_final_states else y


def mamba_split_conv1d_scan_combined(zxbcdt, conv1d_weight, conv1d_bias, dt_bias, A, D, chunk_size,
                                     initial_states=None, seq_idx=None, dt_limit=(0.0, _INF),
                                     return_final_states=False, activation="silu",
                                     rmsnorm_weight=None, rmsnorm_eps=1e-6, outproj_weight=None,
                                     outproj_bias=None, headdim=None, ngroups=1, norm_before_gate=True):
    """Upstream-compatible entry point (D11).  ``initial_states`` (b, h, p, n), ``seq_idx`` (b, l) and
    ``return_final_states`` run through the fused native chain (conv1d_cl_var / ssd_fwd with seq_idx and
    initial states).  Upstream's other forms -- no norm (``rmsnorm_weight=None``: y * silu(z)) and a
    per-channel skip (``D`` of shape (h, p)) -- run the same native ops unfused."""
    assert activation in ("silu", "swish")
    if D.dim() == 2:
        headdim = D.shape[1]
    assert headdim is not None, "headdim is required with a per-head D"
    H = dt_bias.shape[0]
    d_state = (zxbcdt.shape[-1] - H - 2 * H * headdim) // (2 * ngroups)
    if rmsnorm_weight is None or D.dim() == 2:
        out = _split_conv1d_scan_general(zxbcdt, conv1d_weight, conv1d_bias, dt_bias, A, D, chunk_size,
                                         initial_states, seq_idx, dt_limit, return_final_states, rmsnorm_weight,
                                         rmsnorm_eps, headdim, ngroups, d_state, norm_before_gate)
        y, final = out if return_final_states else (out, None)
        if outproj_weight is not None:
            y = F.linear(y, outproj_weight, outproj_bias)
        return (y, final) if return_final_states else y
    out = mamba2_inner_fn(zxbcdt, conv1d_weight, conv1d_bias, dt_bias, A, D, rmsnorm_weight, rmsnorm_eps,
                          headdim, ngroups, d_state, dt_limit, norm_before_gate, chunk_size,
                          initial_states=initial_states, seq_idx=seq_idx,
                          return_final_states=return_final_states)
    y, final = out if return_final_states else (out, None)
    if outproj_weight is not None:
        y = F.linear(y, outproj_weight, outproj_bias)
    return (y, final) if return_final_states else y

