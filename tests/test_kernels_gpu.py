"""Native HIP kernels vs the PyTorch fp32 references (SURVEY.md §4 'Op oracles' / 'Autograd').

Every test runs the same bf16 inputs through (a) the gfx950 kernel path and (b) the reference
path (ops/reference.py, fp32 math), forward and backward, and compares with bf16 tolerances:
relative L2 error of the whole tensor, plus a max-abs bound.
"""
import math
import os

import pytest
import torch
import torch.nn.functional as F

from mamba_distributed_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def sharpen_logits(m, scale=4.0):
    """Scale the (tied) embedding / lm_head weight so the random-init logits are far from uniform: the loss then
    sits well above ln V (by ~scale^2 x its random-init excess), and a kernel bug that flattens the logits cannot
    hide inside the loss tolerance."""
    with torch.no_grad():
        m.lm_head.weight.mul_(scale)


def check_loss(ln, lr, vocab):
    """Native vs reference loss: within 2e-3 relative AND within 3% of the reference's distance from ln V (the
    loss of uniform logits), which must itself be substantial (see sharpen_logits)."""
    excess = abs(lr - math.log(vocab))
    assert excess > 0.5, ("loss too close to ln V for a meaningful check", lr, math.log(vocab))
    assert abs(ln - lr) < 2e-3 * abs(lr) and abs(ln - lr) < 0.03 * excess, (ln, lr, excess)


def leaf(t):
    return t.detach().clone().requires_grad_(True)


def run_both(fn_native, fn_ref, inputs, grad_seed=0):
    """Run fwd+bwd on cloned leaves; returns (out_n, out_r, grads_n, grads_r)."""
    xn = [leaf(t) if (t is not None and t.is_floating_point()) else t for t in inputs]
    xr = [leaf(t) if (t is not None and t.is_floating_point()) else t for t in inputs]
    on = fn_native(*xn)
    os.environ["MAMBA_AMD_FORCE_REFERENCE"] = "1"
    try:
        orf = fn_ref(*xr)
    finally:
        os.environ.pop("MAMBA_AMD_FORCE_REFERENCE")
    on_t = on if isinstance(on, torch.Tensor) else on[0]
    or_t = orf if isinstance(orf, torch.Tensor) else orf[0]
    g = torch.Generator(device=on_t.device).manual_seed(grad_seed)
    go = torch.randn(on_t.shape, generator=g, device=on_t.device, dtype=torch.float32).to(on_t.dtype)
    on_t.backward(go)
    or_t.backward(go.to(or_t.dtype))
    gn = [t.grad if isinstance(t, torch.Tensor) and t.requires_grad else None for t in xn]
    gr = [t.grad if isinstance(t, torch.Tensor) and t.requires_grad else None for t in xr]
    return on, orf, gn, gr


# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("D", [256, 768, 1040])
@pytest.mark.parametrize("with_res", [False, True])
@pytest.mark.parametrize("dts", ["bf16_f32res", "f32", "bf16_bf16res"])
def test_add_rmsnorm(cuda, D, with_res, dts):
    """bf16 activations + fp32 residual stream run the typed kernels (norm.hip add_rmsnorm_*_t_k); the other dtype
    combinations the dynamic-dtype ones.  D = 1040 leaves the last lane chunk partly past the row."""
    from mamba_distributed_amd.ops.norm import rms_norm_fn
    torch.manual_seed(0)
    M = 333
    xdt = torch.float32 if dts == "f32" else torch.bfloat16
    rdt = torch.bfloat16 if dts == "bf16_bf16res" else torch.float32
    x = torch.randn(M, D, device=cuda, dtype=xdt)
    r = torch.randn(M, D, device=cuda, dtype=rdt) if with_res else None
    w = torch.rand(D, device=cuda) + 0.5

    def f(x, w, r):
        y, res = rms_norm_fn(x, w, None, residual=r, prenorm=True, residual_in_fp32=rdt == torch.float32, eps=1e-5)
        return y.float() * 1.0 + res.float() * 0.37

    on, orf, gn, gr = run_both(f, f, [x, w, r])
    assert rel(on, orf) < 1e-2
    for a, b in zip(gn, gr):
        if b is not None:
            assert rel(a, b) < 2e-2, (rel(a, b))


@pytest.mark.parametrize("nbg", [False, True])
@pytest.mark.parametrize("D,G", [(1536, 1536), (512, 256)])
def test_gated_rmsnorm(cuda, nbg, D, G):
    from mamba_distributed_amd.ops.norm import rmsnorm_gated_fn
    torch.manual_seed(1)
    M = 257
    big = torch.randn(M, 2 * D + 64, device=cuda, dtype=torch.bfloat16)
    x = torch.randn(M, D, device=cuda, dtype=torch.bfloat16)
    w = torch.rand(D, device=cuda) + 0.5

    def f(x, zbig, w):
        return rmsnorm_gated_fn(x, zbig[:, 64:64 + D], w, 1e-5, G, nbg)

    on, orf, gn, gr = run_both(f, f, [x, big, w])
    assert rel(on, orf) < 1e-2
    for a, b in zip(gn, gr):
        assert rel(a, b) < 2e-2


@pytest.mark.parametrize("layout", ["cf", "cl"])
@pytest.mark.parametrize("L,d", [(1024, 384), (77, 384), (300, 1800)])
def test_conv1d(cuda, layout, L, d):
    """d = 1800: a channel-last width that is not a multiple of the 256 channels of a workgroup."""
    from mamba_distributed_amd.ops.conv1d import causal_conv1d_fn
    torch.manual_seed(2)
    b, W = 3, 4
    if layout == "cf":
        base = torch.randn(b, 2 * d, L, device=cuda, dtype=torch.bfloat16)   # x = first half of channels
    else:
        base = torch.randn(b, L, 2 * d + 40, device=cuda, dtype=torch.bfloat16)  # x = column slice
    w = torch.randn(d, 1, W, device=cuda) * 0.5
    bias = torch.randn(d, device=cuda) * 0.1

    def f(base, w, bias):
        x = base[:, :d] if layout == "cf" else base[:, :, 40:40 + d].transpose(1, 2)
        return causal_conv1d_fn(x, w, bias, "silu")

    on, orf, gn, gr = run_both(f, f, [base, w, bias])
    assert rel(on, orf) < 1e-2
    for a, b_ in zip(gn, gr):
        assert rel(a, b_) < 2e-2


@pytest.mark.parametrize("L,act", [(512, "silu"), (1536, None), (2048, "silu")])
def test_conv1d_channel_first_whole_chunks(cuda, L, act):
    """Channel-first rows of 1 / 3 / 4 whole 512-step chunks (the chunk carry and halo across chunk boundaries),
    with and without the SiLU."""
    from mamba_distributed_amd.ops.conv1d import causal_conv1d_fn
    torch.manual_seed(5)
    b, d, W = 2, 136, 4
    base = torch.randn(b, 2 * d, L, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(d, 1, W, device=cuda) * 0.5
    bias = torch.randn(d, device=cuda) * 0.1

    def f(base, w, bias):
        return causal_conv1d_fn(base[:, :d], w, bias, act)

    on, orf, gn, gr = run_both(f, f, [base, w, bias])
    assert rel(on, orf) < 1e-2
    for a, b_ in zip(gn, gr):
        assert rel(a, b_) < 2e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("b,d,L", [(3, 520, 1024), (2, 136, 1536), (2, 64, 2048), (5, 7, 48), (3, 40, 77)])
def test_conv1d_cf_row_order(cuda, dtype, b, d, L):
    """Channel-first rows numbered in memory order ((d, b, l) buffers: b fastest, the default) against b-major
    numbering, bitwise (same per-row math), including the accumulated per-row tap / bias partials; L = 77 takes the
    scalar (non-16-B) kernels."""
    from mamba_distributed_amd.ops import _ext
    ops = _ext.ops()
    torch.manual_seed(9)
    W = 4
    x = torch.randn(d, b, L, device=cuda).to(dtype).permute(1, 0, 2)
    go = torch.randn(d, b, L, device=cuda).to(dtype).permute(1, 0, 2)
    w = torch.randn(d, W, device=cuda) * 0.5
    bias = torch.randn(d, device=cuda) * 0.1
    part_init = torch.randn(b, d, W + 1, device=cuda)
    prev = ops.conv_cf_order(-1)
    outs = []
    try:
        for order in (0, 1):
            ops.conv_cf_order(order)
            y = ops.conv1d_cf_fwd(x, w, bias, True)
            dx, dw, db = ops.conv1d_cf_bwd(x, w, bias, go, True, None)
            p = part_init.clone()
            ops.conv1d_cf_bwd(x, w, bias, go, True, None, p, 2)  # accumulate into the per-row partials
            outs.append((y, dx, dw, db, p))
        torch.cuda.synchronize()
    finally:
        ops.conv_cf_order(prev)
    for u, v in zip(*outs):
        assert torch.equal(u, v)


def test_cross_entropy(cuda):
    from mamba_distributed_amd.ops.cross_entropy import cross_entropy, fused_linear_cross_entropy
    torch.manual_seed(3)
    M, V, d = 300, 50304, 64
    logits = (torch.randn(M, V, device=cuda) * 3).to(torch.bfloat16)
    t = torch.randint(0, V, (M,), device=cuda)
    t[::7] = -100
    on, orf, gn, gr = run_both(lambda l: cross_entropy(l, t), lambda l: cross_entropy(l, t), [logits])
    assert abs(on.item() - orf.item()) < 2e-3 * abs(orf.item())
    assert rel(gn[0], gr[0]) < 2e-2
    h = torch.randn(M, d, device=cuda, dtype=torch.bfloat16)
    W = torch.randn(V, d, device=cuda) * 0.05
    on, orf, gn, gr = run_both(lambda h, W: fused_linear_cross_entropy(h, W, t),
                               lambda h, W: fused_linear_cross_entropy(h, W, t), [h, W])
    assert abs(on.item() - orf.item()) < 5e-3 * abs(orf.item())
    assert rel(gn[0], gr[0]) < 3e-2 and rel(gn[1], gr[1]) < 3e-2


@pytest.mark.parametrize("engine", ["lib", "native"])
@pytest.mark.parametrize("row_chunk", [None, 2048])
def test_fused_lm_head_ce_native(cuda, row_chunk, engine, monkeypatch):
    """The row-chunked lm_head + CE at the 280M head shape (d 768, V 50304) against fp32 math: loss, dh and dW
    (row_chunk 2048: three chunks, the last one 404 rows, dW accumulated across them); engine "native" (the
    default): all three products on the native MFMA engines, "lib": the MAMBA_AMD_LMHEAD=lib A/B switch (hipBLASLt,
    fp32-output dW accumulation)."""
    import importlib
    monkeypatch.setenv("MAMBA_AMD_LMHEAD", engine)
    ce = importlib.import_module("mamba_distributed_amd.ops.cross_entropy")
    torch.manual_seed(4)
    M, d, V = 4500, 768, 50304
    h = torch.randn(M, d, device=cuda, dtype=torch.bfloat16)
    W = torch.randn(V, d, device=cuda) * 0.05
    t = torch.randint(0, V, (M,), device=cuda)
    t[::5] = -100
    assert ce._lm_native(h, W.to(torch.bfloat16))
    hn, Wn = leaf(h), leaf(W)
    loss = ce.fused_linear_cross_entropy(hn, Wn, t, row_chunk=row_chunk)
    (loss * 1.7).backward()
    hr, Wr = leaf(h.float()), leaf(W.to(torch.bfloat16).float())
    lr = F.cross_entropy(hr @ Wr.t(), t, ignore_index=-100)
    (lr * 1.7).backward()
    assert abs(loss.item() - lr.item()) < 2e-3 * abs(lr.item())
    assert rel(hn.grad, hr.grad) < 2e-2, rel(hn.grad, hr.grad)
    assert rel(Wn.grad, Wr.grad) < 2e-2, rel(Wn.grad, Wr.grad)
    assert hn.grad.dtype == torch.bfloat16 and Wn.grad.dtype == torch.float32


def _ssd_inputs(cuda, b, L, H, G, N, seed=0, strided=True):
    g = torch.Generator(device=cuda).manual_seed(seed)
    P = 64
    width = H * P + 2 * G * N + (24 if strided else 0)
    buf = torch.randn(b, L, width, generator=g, device=cuda).to(torch.bfloat16)
    off = 24 if strided else 0
    x = buf[..., off:off + H * P].unflatten(-1, (H, P))
    Bm = buf[..., off + H * P: off + H * P + G * N].unflatten(-1, (G, N)) * 0.5
    Cm = buf[..., off + H * P + G * N:].unflatten(-1, (G, N)) * 0.5
    dt = (torch.randn(b, L, H, generator=g, device=cuda) * 0.5 - 1.0).to(torch.bfloat16)
    A = -torch.rand(H, generator=g, device=cuda) * 8 - 0.5
    D = torch.randn(H, generator=g, device=cuda)
    dt_bias = torch.randn(H, generator=g, device=cuda) * 0.3
    return x.contiguous() if not strided else x, dt, A, Bm, Cm, D, dt_bias


@pytest.mark.parametrize("b,L,H,G,N", [(2, 256, 4, 1, 128), (1, 200, 8, 2, 64), (2, 70, 6, 1, 128),
                                       (4, 1024, 24, 1, 128),   # the 280M headline shape (16 chunks, 24 heads)
                                       (1, 8192, 8, 1, 128)])   # the 2.8B long-sequence shape (128 chunks)
def test_ssd_fwd_bwd(cuda, b, L, H, G, N):
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    x, dt, A, Bm, Cm, D, dt_bias = _ssd_inputs(cuda, b, L, H, G, N)

    def f(x, dt, A, Bm, Cm, D, dt_bias):
        return mamba_chunk_scan_combined(x, dt, A, Bm, Cm, 64, D=D, dt_bias=dt_bias, dt_softplus=True)

    on, orf, gn, gr = run_both(f, f, [x, dt, A, Bm, Cm, D, dt_bias])
    assert rel(on, orf) < 2e-2, rel(on, orf)
    names = ["x", "dt", "A", "B", "C", "D", "dt_bias"]
    for nm, a, b_ in zip(names, gn, gr):
        assert rel(a, b_) < 3e-2, (nm, rel(a, b_))


def test_ssd_fp32_dt_partial_chunk(cuda):
    """dt given in fp32 (two-halfword raw prefetch path) with a partial last chunk (clamped rows)."""
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    x, dt, A, Bm, Cm, D, dt_bias = _ssd_inputs(cuda, 2, 130, 8, 1, 128, seed=3)
    dt = dt.float()

    def f(x, dt, A, Bm, Cm, D, dt_bias):
        return mamba_chunk_scan_combined(x, dt, A, Bm, Cm, 64, D=D, dt_bias=dt_bias, dt_softplus=True)

    on, orf, gn, gr = run_both(f, f, [x, dt, A, Bm, Cm, D, dt_bias])
    assert rel(on, orf) < 2e-2, rel(on, orf)
    for nm, a, b_ in zip(["x", "dt", "A", "B", "C", "D", "dt_bias"], gn, gr):
        assert rel(a, b_) < 3e-2, (nm, rel(a, b_))


@pytest.mark.parametrize("hg", ["24", "12", "3"])
def test_ssd_head_groups(cuda, monkeypatch, hg):
    """chunk-bwd head groups larger than the 8-slot dt-gradient ring (flushed every 8 heads) and
    odd sizes; forced through the MAMBA_AMD_SSD_HG override, checked against the reference."""
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    monkeypatch.setenv("MAMBA_AMD_SSD_HG", hg)
    x, dt, A, Bm, Cm, D, dt_bias = _ssd_inputs(cuda, 2, 200, 24, 1, 128, seed=11)

    def f(x, dt, A, Bm, Cm, D, dt_bias):
        return mamba_chunk_scan_combined(x, dt, A, Bm, Cm, 64, D=D, dt_bias=dt_bias, dt_softplus=True)

    on, orf, gn, gr = run_both(f, f, [x, dt, A, Bm, Cm, D, dt_bias])
    assert rel(on, orf) < 2e-2, rel(on, orf)
    for nm, a, b_ in zip(["x", "dt", "A", "B", "C", "D", "dt_bias"], gn, gr):
        assert rel(a, b_) < 3e-2, (hg, nm, rel(a, b_))


@pytest.mark.parametrize("H,G", [(24, 1), (8, 2)])
def test_ssd_fused_dbc_bitwise(cuda, monkeypatch, H, G):
    """One head group per B/C group (HG == H / G, the 280M training shape): ssd_chunk_bwd_k finishes dB / dC
    itself instead of writing head-group partials for ssd_dbc_bwd_k.  Same math in the same order: every
    gradient is bitwise the unfused one (MAMBA_AMD_SSD_FUSE_DBC=0)."""
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    monkeypatch.setenv("MAMBA_AMD_SSD_HG", str(H // G))
    x, dt, A, Bm, Cm, D, dt_bias = _ssd_inputs(cuda, 2, 200, H, G, 128, seed=13)
    grads = {}
    for fuse in ("0", "1"):
        monkeypatch.setenv("MAMBA_AMD_SSD_FUSE_DBC", fuse)
        ins = [t.detach().clone().requires_grad_(True) for t in (x, dt, Bm, Cm)]
        y = mamba_chunk_scan_combined(ins[0], ins[1], A, ins[2], ins[3], 64, D=D, dt_bias=dt_bias, dt_softplus=True)
        y.float().square().mean().backward()
        grads[fuse] = [t.grad for t in ins]
    for nm, a, b_ in zip(["x", "dt", "B", "C"], grads["1"], grads["0"]):
        assert torch.equal(a, b_), nm


def test_ssd_initial_and_final_states(cuda):
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    x, dt, A, Bm, Cm, D, dt_bias = _ssd_inputs(cuda, 2, 192, 4, 1, 128, seed=5)
    init = torch.randn(2, 4, 64, 128, device=cuda) * 0.2

    def f(x, dt, Bm, Cm, init):
        y, fin = mamba_chunk_scan_combined(x, dt, A, Bm, Cm, 64, D=D, dt_bias=dt_bias, dt_softplus=True,
                                           initial_states=init, return_final_states=True)
        return y.float().sum(-1) * 0 + y.float().mean(-1) + fin.sum((-1, -2))[:, None, :].float() * 1e-2

    on, orf, gn, gr = run_both(f, f, [x, dt, Bm, Cm, init])
    assert rel(on, orf) < 2e-2
    for a, b_ in zip(gn, gr):
        assert rel(a, b_) < 3e-2


@pytest.mark.parametrize("b,L,H,S", [(1, 8192, 8, 1), (1, 8192, 8, 2), (1, 8192, 8, 4),  # the 2.8B sequence length
                                     (2, 1000, 8, 3), (2, 1000, 8, 16)])   # partial segments / chunk, 16 x 1 chunk
def test_ssd_segment_parallel(cuda, b, L, H, S):
    """Segment-parallel state walks (kernels/ssd.hip ssd_seg_state_k / ssd_seg_dstate_k / ssd_seg_combine_k): the
    forward and reverse walks split into S segments from carried-in states, forced through the ssd_segments
    override; y, the final state and every gradient (incl. initial_states and through the final state) against the
    fp32 reference, and against the one-segment walk."""
    from mamba_distributed_amd.ops import _ext
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    ops = _ext.ops()
    nc = (L + 63) // 64
    x, dt, A, Bm, Cm, D, dt_bias = _ssd_inputs(cuda, b, L, H, 1, 128, seed=17)
    # slow decay (a dt ~ -0.002 .. -0.008 per step): the carried-in state of a segment is far from negligible, so a
    # wrong combine shows (with _ssd_inputs' A the state forgets within a chunk)
    A = -(torch.rand(H, generator=torch.Generator(device=cuda).manual_seed(3), device=cuda) * 0.02 + 0.005)
    init = torch.randn(b, H, 64, 128, device=cuda) * 0.2

    def f(x, dt, Bm, Cm, init):
        y, fin = mamba_chunk_scan_combined(x, dt, A, Bm, Cm, 64, D=D, dt_bias=dt_bias, dt_softplus=True,
                                           initial_states=init, return_final_states=True)
        return y.float().mean(-1) + fin.sum((-1, -2))[:, None, :].float() * 1e-2

    try:
        got = int(ops.ssd_segments(S, b, H, nc))
        assert got == min(S, nc), got
        on, orf, gn, gr = run_both(f, f, [x, dt, Bm, Cm, init])
        ops.ssd_segments(1, b, H, nc)
        xs = [leaf(t) for t in (x, dt, Bm, Cm, init)]
        o1 = f(*xs)
        o1.backward(torch.randn(o1.shape, generator=torch.Generator(device=cuda).manual_seed(0), device=cuda))
    finally:
        ops.ssd_segments(0, 1, 1, 1)
    assert rel(on, orf) < 2e-2, rel(on, orf)
    assert rel(on, o1) < 5e-3, rel(on, o1)
    for nm, a, b_, c in zip(["x", "dt", "B", "C", "init"], gn, gr, [t.grad for t in xs]):
        assert rel(a, b_) < 3e-2, (nm, rel(a, b_))
        assert rel(a, c) < 1e-2, (nm, rel(a, c))


def test_ssd_segments_auto_pick(cuda):
    """The automatic segment count: one walk per (h, b) whenever b * H fills the CUs (every BASELINE training shape),
    a split below that (batch-1 / small-batch long prefill)."""
    from mamba_distributed_amd.ops import _ext
    ops = _ext.ops()
    ops.ssd_segments(0, 1, 1, 1)
    assert ops.ssd_segments(-1, 64, 24, 16) == 1      # 280M, micro-batch 64 x 1024
    assert ops.ssd_segments(-1, 32, 48, 16) == 1      # 1.4B, micro-batch 32 x 1024
    assert ops.ssd_segments(-1, 4, 80, 128) == 1      # 2.8B, micro-batch 4 x 8192: 320 walks, splitting measured no gain
    assert ops.ssd_segments(-1, 1, 24, 512) == 16     # batch-1 prefill of 32k tokens: 24 walks on 256 CUs
    assert ops.ssd_segments(-1, 1, 8, 128) == 16
    assert ops.ssd_segments(-1, 2, 80, 128) == 3      # <= 2 workgroups per CU


def test_ssd_deterministic(cuda):
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    x, dt, A, Bm, Cm, D, dt_bias = _ssd_inputs(cuda, 2, 256, 8, 1, 128, seed=7)
    outs = []
    for _ in range(2):
        xs = [leaf(t) for t in (x, dt, Bm, Cm)]
        y = mamba_chunk_scan_combined(xs[0], xs[1], A, xs[2], xs[3], 64, D=D, dt_bias=dt_bias, dt_softplus=True)
        y.float().square().sum().backward()
        outs.append([y] + [t.grad for t in xs])
    for a, b_ in zip(*outs):
        assert torch.equal(a, b_)


def test_mamba2_inner(cuda):
    from mamba_distributed_amd.ops.ssd import mamba2_inner_fn
    torch.manual_seed(4)
    b, L, H, P, N, G = 2, 300, 8, 64, 128, 1
    di = H * P
    dproj = 2 * di + 2 * G * N + H
    zx = torch.randn(b, L, dproj, device=cuda).to(torch.bfloat16)
    conv_w = torch.randn(di + 2 * G * N, 1, 4, device=cuda) * 0.3
    conv_b = torch.randn(di + 2 * G * N, device=cuda) * 0.1
    dt_bias = torch.randn(H, device=cuda) * 0.3
    A = -torch.rand(H, device=cuda) * 8 - 0.5
    D = torch.randn(H, device=cuda)
    nw = torch.rand(di, device=cuda) + 0.5

    def f(zx, conv_w, conv_b, dt_bias, A, D, nw):
        return mamba2_inner_fn(zx, conv_w, conv_b, dt_bias, A, D, nw, 1e-5, P, G, N)

    on, orf, gn, gr = run_both(f, f, [zx, conv_w, conv_b, dt_bias, A, D, nw])
    assert rel(on, orf) < 2e-2
    for i, (a, b_) in enumerate(zip(gn, gr)):
        assert rel(a, b_) < 3e-2, (i, rel(a, b_))


@pytest.mark.parametrize("L,n", [(512, 16), (700, 16), (2048, 16), (1500, 8), (256, 4)])
@pytest.mark.parametrize("with_z", [True, False])
def test_selective_scan(cuda, L, n, with_z):
    """vector path (L % 16 == 0), guarded path, several forward/backward tiles, N = 16/8/4."""
    from mamba_distributed_amd.ops.selective_scan import selective_scan_fn
    torch.manual_seed(5)
    b, d = 2, 96
    u = torch.randn(b, d, L, device=cuda).to(torch.bfloat16)
    delta = (torch.randn(b, d, L, device=cuda) * 0.5 - 1).to(torch.bfloat16)
    A = -torch.rand(d, n, device=cuda) * 4 - 0.1
    Bm = torch.randn(b, 1, n, L, device=cuda).to(torch.bfloat16)
    Cm = torch.randn(b, 1, n, L, device=cuda).to(torch.bfloat16)
    D = torch.randn(d, device=cuda)
    z = torch.randn(b, d, L, device=cuda).to(torch.bfloat16) if with_z else None
    db = torch.randn(d, device=cuda) * 0.3

    def f(u, delta, A, Bm, Cm, D, z, db):
        return selective_scan_fn(u, delta, A, Bm, Cm, D, z=z, delta_bias=db, delta_softplus=True)

    on, orf, gn, gr = run_both(f, f, [u, delta, A, Bm, Cm, D, z, db])
    assert rel(on, orf) < 2e-2, rel(on, orf)
    names = ["u", "delta", "A", "B", "C", "D", "z", "db"]
    for nm, a, b_ in zip(names, gn, gr):
        if b_ is not None:
            assert rel(a, b_) < 3e-2, (nm, rel(a, b_))


@pytest.mark.parametrize("layer", ["Mamba1", "Mamba2"])
def test_model_native_vs_reference(cuda, layer):
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=256, n_layer=2, vocab_size=1024, ssm_cfg={"layer": layer})
    m = LMHeadModel(cfg, device=cuda)
    sharpen_logits(m)
    x = torch.randint(0, 1024, (2, 192), device=cuda)
    y = torch.randint(0, 1024, (2, 192), device=cuda)

    def lossgrad(force_ref):
        if force_ref:
            os.environ["MAMBA_AMD_FORCE_REFERENCE"] = "1"
        try:
            m.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                _, loss = m(x, y)
            loss.backward()
            return loss.item(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        finally:
            os.environ.pop("MAMBA_AMD_FORCE_REFERENCE", None)

    ln, gn = lossgrad(False)
    lr, gr = lossgrad(True)
    check_loss(ln, lr, cfg.vocab_size)
    bad = {n: rel(gn[n], gr[n]) for n in gr if rel(gn[n], gr[n]) > 5e-2}
    assert not bad, bad


@pytest.mark.parametrize("engine", ["lib", "pk"])
@pytest.mark.parametrize("layer", ["Mamba1", "Mamba2"])
def test_model_native_vs_reference_headline_width(cuda, monkeypatch, layer, engine):
    """The 280M configs' layer width and sequence length (d_model 768, T=1024, 16 SSD chunks, 24 heads)
    through 2 layers: loss and every parameter gradient, native kernels vs the fp32 reference ops, with the
    projection forward and input-gradient GEMMs on hipBLASLt and on the persistent native engine.  8 x 1024
    tokens: enough rows for the persistent engine on every projection (Mamba-1's channel-major in_proj needs
    M * N >= 2^24), and a spy checks that it ran (pk) or did not (lib)."""
    monkeypatch.setenv("MAMBA_AMD_PROJ_GEMM", engine)
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.ops import linear as lin
    calls = []
    orig = lin._pk_mm

    def spy(a2, w):
        calls.append(tuple(a2.shape) + (w.shape[0],))
        return orig(a2, w)
    monkeypatch.setattr(lin, "_pk_mm", spy)
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=768, n_layer=2, vocab_size=4096, ssm_cfg={"layer": layer})
    m = LMHeadModel(cfg, device=cuda)
    sharpen_logits(m)
    x = torch.randint(0, 4096, (8, 1024), device=cuda)
    y = torch.randint(0, 4096, (8, 1024), device=cuda)

    def lossgrad(force_ref):
        if force_ref:
            os.environ["MAMBA_AMD_FORCE_REFERENCE"] = "1"
        try:
            m.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                _, loss = m(x, y)
            loss.backward()
            return loss.item(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        finally:
            os.environ.pop("MAMBA_AMD_FORCE_REFERENCE", None)

    ln, gn = lossgrad(False)
    # pk: every layer's in_proj / out_proj forward and input gradient (Mamba-1: in_proj fwd, out_proj dgrad... on
    # the engine where the layout is KC . KC); lib: none
    n_pk = len(calls)
    assert (n_pk >= 2 * cfg.n_layer) if engine == "pk" else (n_pk == 0), calls
    lr, gr = lossgrad(True)
    check_loss(ln, lr, cfg.vocab_size)
    bad = {n: rel(gn[n], gr[n]) for n in gr if rel(gn[n], gr[n]) > 5e-2}
    assert not bad, bad


@pytest.mark.parametrize("d_model", [2048, 2560])
def test_model_native_wide_vs_reference(cuda, monkeypatch, d_model):
    """The 1.4B / 2.8B layer widths (d_model 2048 / 2560: in_proj 8512 / 10576 -> padded 10624 wide, out_proj
    K = 4096 / 5120) through 2 Mamba-2 layers on the DEFAULT routing: every projection forward and input gradient on
    the hand-written persistent engine (a spy counts them: the wide long-K products that round 5 routed to hipBLASLt
    included), loss and every parameter gradient vs the fp32 reference ops."""
    monkeypatch.delenv("MAMBA_AMD_PROJ_GEMM", raising=False)
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.ops import linear as lin
    calls = []
    orig = lin._pk_mm

    def spy(a2, w):
        calls.append((a2.shape[0], w.shape[0], a2.shape[1]))
        return orig(a2, w)
    monkeypatch.setattr(lin, "_pk_mm", spy)
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=d_model, n_layer=2, vocab_size=4096, ssm_cfg={"layer": "Mamba2"})
    m = LMHeadModel(cfg, device=cuda)
    sharpen_logits(m)
    x = torch.randint(0, 4096, (4, 1024), device=cuda)
    y = torch.randint(0, 4096, (4, 1024), device=cuda)

    def lossgrad(force_ref):
        if force_ref:
            os.environ["MAMBA_AMD_FORCE_REFERENCE"] = "1"
        try:
            m.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                _, loss = m(x, y)
            loss.backward()
            return loss.item(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        finally:
            os.environ.pop("MAMBA_AMD_FORCE_REFERENCE", None)

    ln, gn = lossgrad(False)
    # per layer: in_proj fwd + dgrad, out_proj fwd + dgrad, all with K > 1024 or a >= 2048-wide output
    long_k = [c for c in calls if c[2] > 1024]
    assert len(calls) >= 4 * cfg.n_layer and len(long_k) >= 2 * cfg.n_layer, calls
    lr, gr = lossgrad(True)
    check_loss(ln, lr, cfg.vocab_size)
    bad = {n: rel(gn[n], gr[n]) for n in gr if rel(gn[n], gr[n]) > 5e-2}
    assert not bad, bad


@pytest.mark.parametrize("layer", ["Mamba1", "Mamba2"])
def test_bench_path_vs_reference(cuda, monkeypatch, layer):
    """The exact bench.py / trainer step path against the fp32 reference ops: fused lm_head + cross-entropy
    (return_logits=False) on the native engines, two micro-steps through parallel.microbatch.run_micro_batches
    inside grad_accum.accumulation_scope with the model's auto deferral policy, 8192-token micro-batches (every
    projection on the persistent GEMM), then loss and every parameter gradient.  Spies check that the native
    lm_head engines and the persistent projection GEMM actually ran."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    import importlib
    ce = importlib.import_module("mamba_distributed_amd.ops.cross_entropy")  # the module (ops exports a function of that name)
    from mamba_distributed_amd.ops import grad_accum
    from mamba_distributed_amd.ops import linear as lin
    from mamba_distributed_amd.parallel.microbatch import auto_defer_reduce, run_micro_batches
    pk_calls, lm_native = [], []
    orig_pk, orig_lm = lin._pk_mm, ce._lm_engines

    def spy_pk(a2, w):
        # the token side: a2's rows for the token-major Mamba-2 products, w's rows for Mamba-1's channel-major
        # mm_nt (W . h^T)
        pk_calls.append(max(a2.shape[0], w.shape[0]))
        return orig_pk(a2, w)

    def spy_lm(h2, w):
        r = orig_lm(h2, w)
        lm_native.append(r)
        return r
    monkeypatch.setattr(lin, "_pk_mm", spy_pk)
    monkeypatch.setattr(ce, "_lm_engines", spy_lm)
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=768, n_layer=2, vocab_size=50304, ssm_cfg={"layer": layer})
    m = LMHeadModel(cfg, device=cuda)
    sharpen_logits(m)
    g = torch.Generator(device=cuda).manual_seed(3)
    batches = [(torch.randint(0, 50304, (8, 1024), device=cuda, generator=g),
                torch.randint(0, 50304, (8, 1024), device=cuda, generator=g)) for _ in range(2)]

    def run(force_ref):
        if force_ref:
            os.environ["MAMBA_AMD_FORCE_REFERENCE"] = "1"
        try:
            m.zero_grad(set_to_none=True)
            it = iter(batches)

            def compute_loss(x, y):
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    _, loss = m(x, y, return_logits=False)
                return loss / 2
            with grad_accum.accumulation_scope(defer_reduce=auto_defer_reduce(cfg)):
                loss = run_micro_batches(m, lambda: next(it), 2, compute_loss, overlap=True)
            torch.cuda.synchronize()
            return loss.item(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}
        finally:
            os.environ.pop("MAMBA_AMD_FORCE_REFERENCE", None)

    ln, gn = run(False)
    assert lm_native and all(all(r) for r in lm_native), lm_native
    assert len(pk_calls) >= 2 * 2 * cfg.n_layer and min(pk_calls) >= 8192, pk_calls
    lr, gr = run(True)
    check_loss(ln, lr, cfg.vocab_size)
    bad = {n: rel(gn[n], gr[n]) for n in gr if rel(gn[n], gr[n]) > 5e-2}
    assert not bad, bad


@pytest.mark.parametrize("engine", ["lib", "auto"])
@pytest.mark.parametrize("pad", ["1", "0"])
def test_mamba2_padded_inproj_vs_reference(cuda, monkeypatch, engine, pad):
    """The Mamba-2 in_proj computed into 64-aligned padded rows (3352 -> 3392 at d_model 768) with d(zxbcdt)
    written by the fused chain into the same layout (zero pad columns) and the input gradient run as a K = 3392
    product: loss and every gradient vs the fp32 reference at 4096 tokens (large enough for the persistent
    engine), and the padded input-gradient path is the one taken."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.ops import linear as lin
    monkeypatch.setenv("MAMBA_AMD_PROJ_GEMM", engine)
    monkeypatch.setenv("MAMBA_AMD_PAD_PROJ", pad)
    hits = []
    orig = lin._zero_padded_full

    def spy(dy2, np_):
        r = orig(dy2, np_)
        hits.append(r is not None)
        return r
    monkeypatch.setattr(lin, "_zero_padded_full", spy)
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=768, n_layer=2, vocab_size=4096, ssm_cfg={"layer": "Mamba2"})
    m = LMHeadModel(cfg, device=cuda)
    sharpen_logits(m)
    x = torch.randint(0, 4096, (4, 1024), device=cuda)
    y = torch.randint(0, 4096, (4, 1024), device=cuda)

    def lossgrad(force_ref):
        if force_ref:
            os.environ["MAMBA_AMD_FORCE_REFERENCE"] = "1"
        try:
            m.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                _, loss = m(x, y)
            loss.backward()
            return loss.item(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        finally:
            os.environ.pop("MAMBA_AMD_FORCE_REFERENCE", None)

    ln, gn = lossgrad(False)
    assert hits == ([True] * 2 if pad == "1" else []), hits
    lr, gr = lossgrad(True)
    check_loss(ln, lr, cfg.vocab_size)
    bad = {n: rel(gn[n], gr[n]) for n in gr if rel(gn[n], gr[n]) > 5e-2}
    assert not bad, bad


@pytest.mark.gpu
def test_mamba2_odd_heads_padded_inproj_trains(cuda):
    """nheads % 8 != 0 (d_model 192, headdim 64: H = 6, in_proj width 1030, pad 58): the padded in_proj forward is
    taken, the fused backward falls back to the unpadded d(zxbcdt) layout (the chunk backward's pad fill needs
    8-column groups), and loss and gradients match the fp32 reference."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=192, n_layer=2, vocab_size=512, ssm_cfg={"layer": "Mamba2", "headdim": 64})
    m = LMHeadModel(cfg, device=cuda)
    sharpen_logits(m)
    x = torch.randint(0, 512, (2, 512), device=cuda)
    y = torch.randint(0, 512, (2, 512), device=cuda)

    def lossgrad(force_ref):
        if force_ref:
            os.environ["MAMBA_AMD_FORCE_REFERENCE"] = "1"
        try:
            m.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                _, loss = m(x, y)
            loss.backward()
            return loss.item(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        finally:
            os.environ.pop("MAMBA_AMD_FORCE_REFERENCE", None)

    ln, gn = lossgrad(False)
    lr, gr = lossgrad(True)
    check_loss(ln, lr, cfg.vocab_size)
    bad = {n: rel(gn[n], gr[n]) for n in gr if rel(gn[n], gr[n]) > 5e-2}
    assert not bad, bad


def test_padded_inproj_grad_pad_columns_zeroed_by_ssd_bwd(cuda, monkeypatch):
    """The padded in_proj gradient buffer's pad columns are written (zeros) by the SSD chunk backward
    (ddt_zero_pad), not by a separate fill: with the buffer allocated NaN-filled, the pad comes back exactly 0 and
    the d(zxbcdt) view equals the unpadded run's."""
    import importlib
    ssd_mod = importlib.import_module("mamba_distributed_amd.ops.ssd")
    lin = importlib.import_module("mamba_distributed_amd.ops.linear")
    torch.manual_seed(5)
    b, l, H, P, N = 2, 256, 24, 64, 128
    di = H * P
    dproj = 2 * di + 2 * N + H
    rs = (dproj + 63) // 64 * 64
    full = (torch.randn(b, l, rs, device=cuda) * 0.5).to(torch.bfloat16)
    zx_pad = full[..., :dproj]
    zx = zx_pad.contiguous()
    conv_w = torch.randn(di + 2 * N, 1, 4, device=cuda) * 0.3
    conv_b = torch.randn(di + 2 * N, device=cuda) * 0.1
    dt_bias = torch.randn(H, device=cuda) * 0.3
    A = -torch.rand(H, device=cuda) * 4 - 0.5
    D = torch.randn(H, device=cuda)
    nw = torch.rand(di, device=cuda) + 0.5
    seen = []
    monkeypatch.setattr(lin, "register_zero_padded_grad", lambda t: seen.append(t))

    class _NanEmpty:  # ssd.py's torch, with empty() NaN-filled
        def __getattr__(self, n):
            return getattr(torch, n)

        def empty(self, *size, **kw):
            return torch.full(size, float("nan"), **kw)
    monkeypatch.setattr(ssd_mod, "torch", _NanEmpty())
    grads = []
    for z in (zx_pad, zx):
        zl = z.detach().requires_grad_(True)
        y = ssd_mod.mamba2_inner_fn(zl, conv_w, conv_b, dt_bias, A, D, nw, 1e-5, P, 1, N)
        g = torch.randn(y.shape, device=cuda, generator=torch.Generator(device=cuda).manual_seed(1)).to(y.dtype)
        y.backward(g)
        grads.append(zl.grad)
    assert len(seen) == 1, len(seen)
    pad = seen[0][..., dproj:]
    assert pad.shape[-1] == rs - dproj and (pad == 0).all()
    assert torch.isfinite(grads[0].float()).all()
    assert torch.equal(grads[0], grads[1])


def test_decode_update_ops(cuda):
    from mamba_distributed_amd.ops.conv1d import causal_conv1d_update
    from mamba_distributed_amd.ops.selective_scan import selective_state_update
    torch.manual_seed(6)
    b, c = 3, 96
    x = torch.randn(b, c, device=cuda).to(torch.bfloat16)
    st = torch.randn(b, c, 3, device=cuda).to(torch.bfloat16)
    w = torch.randn(c, 1, 4, device=cuda)
    bias = torch.randn(c, device=cuda)
    st_r = st.clone()
    o = causal_conv1d_update(x, st, w, bias, "silu")
    o_r = R.causal_conv1d_update_ref(x, st_r, w.view(c, 4), bias, "silu")
    assert rel(o, o_r) < 1e-2 and torch.equal(st, st_r)
    # Mamba-2 form
    H, P, N, G = 4, 64, 128, 1
    s = torch.randn(b, H, P, N, device=cuda)
    s_r = s.clone()
    xx = torch.randn(b, H, P, device=cuda).to(torch.bfloat16)
    dt = torch.randn(b, H, device=cuda).to(torch.bfloat16)
    A = -torch.rand(H, device=cuda) * 4
    Bm = torch.randn(b, G, N, device=cuda).to(torch.bfloat16)
    Cm = torch.randn(b, G, N, device=cuda).to(torch.bfloat16)
    D = torch.randn(H, device=cuda)
    dtb = torch.randn(H, device=cuda)
    y = selective_state_update(s, xx, dt, A, Bm, Cm, D, None, dtb, True)
    y_r = R.selective_state_update_ref(s_r, xx, dt, A, Bm, Cm, D, None, dtb, True)
    assert rel(y, y_r) < 1e-2 and rel(s, s_r) < 1e-4


@pytest.mark.parametrize("layer", ["Mamba1", "Mamba2"])
def test_graphed_decode_matches_eager(cuda, layer):
    """HIP-graph replay of the whole-stack decode step == the eager cached step == full recompute."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.inference import GraphedDecoder
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=256, n_layer=3, vocab_size=1024, ssm_cfg={"layer": layer})
    m = LMHeadModel(cfg, device=cuda).eval()
    ids = torch.randint(0, 1024, (2, 40), device=cuda)
    g = GraphedDecoder(m, batch_size=2, max_seqlen=64, use_graph=True)
    e = GraphedDecoder(m, batch_size=2, max_seqlen=64, use_graph=False)
    lg, le = g.prefill(ids[:, :30]), e.prefill(ids[:, :30])
    torch.testing.assert_close(lg, le)
    for t in range(30, 40):
        lg, le = g.step(ids[:, t]), e.step(ids[:, t])
        torch.testing.assert_close(lg, le, rtol=1e-5, atol=1e-5)
    assert g.graph is not None
    with torch.no_grad():
        full = m(ids)[0][:, -1]
    assert rel(lg, full) < 1e-3


@pytest.mark.parametrize("batch", [1, 3, 9, 16])
def test_fused_decode_matches_unfused(cuda, batch):
    """The fused 3-kernel Mamba-2 decode layer (csrc/kernels/decode.hip), HIP-graph replayed, tracks the
    unfused cached step of a bf16 model (logits and SSM states) and the full bf16 recompute."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.inference import GraphedDecoder
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=256, n_layer=4, vocab_size=1024, ssm_cfg={"layer": "Mamba2"})
    m = LMHeadModel(cfg, device=cuda).to(torch.bfloat16).eval()
    ids = torch.randint(0, 1024, (batch, 48), device=cuda)
    f = GraphedDecoder(m, batch_size=batch, max_seqlen=64, use_graph=True)
    u = GraphedDecoder(m, batch_size=batch, max_seqlen=64, use_graph=False, fused=False)
    assert f.fused is not None and u.fused is None
    lf, lu = f.prefill(ids[:, :32]), u.prefill(ids[:, :32])
    torch.testing.assert_close(lf, lu)
    for t in range(32, 48):
        lf, lu = f.step(ids[:, t]), u.step(ids[:, t])
        assert rel(lf, lu) < 3e-2, (t, rel(lf, lu))
    assert f.graph is not None
    for (cf, sf), (cu, su) in zip(f.params.key_value_memory_dict.values(), u.params.key_value_memory_dict.values()):
        assert rel(sf, su) < 3e-2 and rel(cf, cu) < 3e-2
    with torch.no_grad():
        full = m(ids)[0][:, -1]
    assert rel(lf, full) < 5e-2


@pytest.mark.parametrize("layer", ["Mamba1", "Mamba2"])
def test_fp32_forward_on_gpu_matches_cpu(cuda, layer):
    """The reference's HellaSwag eval runs the model in fp32 without autocast: the GPU path must
    accept fp32 activations (bf16-only kernels defer to the fp32 reference ops)."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=128, n_layer=2, vocab_size=512, ssm_cfg={"layer": layer})
    m = LMHeadModel(cfg, device="cpu").eval()
    ids = torch.randint(0, 512, (2, 100))
    with torch.no_grad():
        ref = m(ids)[0]
        m.to(cuda)
        out = m(ids.to(cuda))[0]
    assert out.dtype == torch.float32
    assert rel(out.cpu(), ref) < 1e-4


@pytest.mark.parametrize("M,N,K", [(32768, 3352, 768), (4096, 768, 1536), (300, 200, 128), (129, 8, 64)])
def test_gemm_tn(cuda, M, N, K):
    """C = A B^T (bf16, fp32 accumulate) vs an fp32 matmul; ragged M/N tails and a strided output."""
    ops = torch.ops.mamba_amd
    torch.manual_seed(0)
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    B = torch.randn(N, K, device=cuda).to(torch.bfloat16)
    ref = A.float() @ B.float().t()
    C = ops.gemm_tn(A, B, None)
    assert rel(C.float(), ref) < 1e-2
    wide = torch.zeros(M, N + 24, device=cuda, dtype=torch.bfloat16)
    ops.gemm_tn(A, B, wide[:, 8:8 + N])
    assert rel(wide[:, 8:8 + N].float(), ref) < 1e-2
    assert wide[:, :8].abs().sum() == 0 and wide[:, 8 + N:].abs().sum() == 0


@pytest.mark.parametrize("M,P,Q", [(32768, 768, 1536), (32768, 3352, 768), (1000, 200, 136), (64, 8, 8),
                                   (8192, 4352, 4096)])
def test_gemm_wgrad(cuda, M, P, Q):
    """dW = dY^T X in fp32 (split over M, fixed-order reduction) vs fp32 matmul; accumulate mode.  The last shape
    has 272 output tiles, just past one round of 256 CUs: the persistent engine's rounds-aware split rule splits
    it (S = 1 before; this side-stream kernel keeps one round)."""
    ops = torch.ops.mamba_amd
    torch.manual_seed(1)
    if P * Q == 4352 * 4096:
        assert ops.gp_splits(P, Q, M) > 1
    dY = torch.randn(M, P, device=cuda).to(torch.bfloat16)
    X = torch.randn(M, Q, device=cuda).to(torch.bfloat16)
    ref = dY.float().t() @ X.float()
    C = ops.gemm_wgrad(dY, X, None, False)
    assert C.dtype == torch.float32 and rel(C, ref) < 1e-4
    acc = torch.ones(P, Q, device=cuda)
    ops.gemm_wgrad(dY, X, acc, True)
    assert rel(acc, ref + 1) < 1e-4
    C2 = ops.gemm_wgrad(dY, X, None, False)
    assert torch.equal(C, C2)  # deterministic


@pytest.mark.parametrize("R,C", [(3392, 768), (768, 3352), (40, 72), (8, 8)])
def test_transpose_bf16(cuda, R, C):
    """The native bf16 transpose behind grad_accum.cached_transpose (partial 64 x 64 tiles included) is exact."""
    from mamba_distributed_amd.ops import grad_accum
    x = torch.randn(R, C, device=cuda).to(torch.bfloat16)
    y = torch.ops.mamba_amd.transpose_bf16(x)
    assert y.shape == (C, R) and torch.equal(y, x.t())
    assert torch.equal(grad_accum.cached_transpose(x, torch.bfloat16), x.t())


@pytest.mark.parametrize("layer", ["Mamba1", "Mamba2"])
def test_in_place_grad_accumulation_matches_autograd(cuda, layer):
    """accumulation_scope (in-place split-K wgrad accumulation + one batched add for the small
    parameter grads on no-sync micro-steps) == plain autograd accumulation over 3 micro-batches."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.ops import grad_accum
    from mamba_distributed_amd.parallel import ddp as ddp_mod
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=256, n_layer=2, vocab_size=1024, ssm_cfg={"layer": layer})
    m = LMHeadModel(cfg, device=cuda)
    batches = [torch.randint(0, 1024, (2, 160), device=cuda) for _ in range(3)]

    def run(scoped):
        m.zero_grad(set_to_none=True)
        ctx = grad_accum.accumulation_scope() if scoped else torch.autograd.set_grad_enabled(True)
        with ctx:
            for i, ids in enumerate(batches):
                ddp_mod.set_grad_sync(m, i == len(batches) - 1)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    _, loss = m(ids[:, :-1].contiguous(), ids[:, 1:].contiguous(), return_logits=False)
                (loss / 3).backward()
        return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}

    ref = run(False)
    got = run(True)
    assert ref.keys() == got.keys()
    for n in ref:
        assert rel(got[n], ref[n]) < 1e-5, (n, rel(got[n], ref[n]))
    assert not grad_accum.in_scope() and not grad_accum.direct()


def test_context_parallel_split_matches_full_sequence(cuda):
    """The CP state hand-off (parallel/context_parallel.py) with the native SSD: scanning two halves from
    zero and folding the first half's final state into the second (ssd_state_correction) equals the
    native/reference scan of the whole sequence, forward and backward."""
    from mamba_distributed_amd.ops.reference import ssd_dt_transform
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    from mamba_distributed_amd.parallel.context_parallel import ssd_state_correction
    x, dt, A, Bm, Cm, D, dt_bias = _ssd_inputs(cuda, 2, 256, 8, 1, 128, seed=11)
    h = 128

    def split(x, dt, Bm, Cm):
        y1, s1 = mamba_chunk_scan_combined(x[:, :h], dt[:, :h], A, Bm[:, :h], Cm[:, :h], 64, D=D,
                                           dt_bias=dt_bias, dt_softplus=True, return_final_states=True)
        y2, _ = mamba_chunk_scan_combined(x[:, h:], dt[:, h:], A, Bm[:, h:], Cm[:, h:], 64, D=D,
                                          dt_bias=dt_bias, dt_softplus=True, return_final_states=True)
        cum2 = torch.cumsum(ssd_dt_transform(dt[:, h:], dt_bias) * A.float(), dim=1)
        y2 = ssd_state_correction(y2, cum2, Cm[:, h:], s1).to(y1.dtype)
        return torch.cat([y1, y2], 1)

    def full(x, dt, Bm, Cm):
        return mamba_chunk_scan_combined(x, dt, A, Bm, Cm, 64, D=D, dt_bias=dt_bias, dt_softplus=True)

    on, orf, gn, gr = run_both(split, full, [x, dt, Bm, Cm])
    assert rel(on, orf) < 2e-2, rel(on, orf)
    for nm, a, b_ in zip(["x", "dt", "B", "C"], gn, gr):
        assert rel(a, b_) < 3e-2, (nm, rel(a, b_))


def test_unfused_parallel_inner_matches_fused(cuda):
    """parallel.context_parallel.mamba2_inner_parallel (native conv1d / SSD / gated norm, unfused; the TP
    and CP building block) == the fused native mamba2_inner_fn, forward and backward."""
    from mamba_distributed_amd.ops.ssd import mamba2_inner_fn
    from mamba_distributed_amd.parallel.context_parallel import mamba2_inner_parallel
    torch.manual_seed(5)
    b, L, H, P, N, G = 2, 256, 8, 64, 128, 1
    di = H * P
    zx = torch.randn(b, L, 2 * di + 2 * G * N + H, device=cuda).to(torch.bfloat16)
    conv_w = torch.randn(di + 2 * G * N, 1, 4, device=cuda) * 0.3
    conv_b = torch.randn(di + 2 * G * N, device=cuda) * 0.1
    dt_bias = torch.randn(H, device=cuda) * 0.3
    A_log = torch.log(torch.rand(H, device=cuda) * 8 + 0.5)
    D = torch.randn(H, device=cuda)
    nw = torch.rand(di, device=cuda) + 0.5
    inputs = [zx, conv_w, conv_b, dt_bias, A_log, D, nw]
    xa = [leaf(t) for t in inputs]
    xb = [leaf(t) for t in inputs]
    ya = mamba2_inner_parallel(*xa, 1e-5, P, G, N)
    yb = mamba2_inner_fn(*xb, 1e-5, P, G, N, A_is_log=True)
    assert rel(ya, yb) < 1e-2, rel(ya, yb)
    go = torch.randn_like(yb.float()).to(yb.dtype)
    ya.backward(go)
    yb.backward(go)
    for i, (a, b_) in enumerate(zip(xa, xb)):
        assert rel(a.grad, b_.grad) < 2e-2, (i, rel(a.grad, b_.grad))


@pytest.mark.parametrize("layer", ["Mamba1", "Mamba2"])
def test_microbatch_overlap_is_bitwise_identical(cuda, layer):
    """parallel.microbatch: micro-batch k+1's forward on a second stream beside backward k (plus the
    side-stream in-place weight-gradient GEMMs) gives bitwise the same gradients and loss as the
    strictly sequential accumulation loop."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.ops import grad_accum
    from mamba_distributed_amd.parallel.microbatch import run_micro_batches
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=256, n_layer=4, vocab_size=1024, ssm_cfg={"layer": layer})
    m = LMHeadModel(cfg, device=cuda)
    accum = 5
    g = torch.Generator(device=cuda).manual_seed(1)
    data = [(torch.randint(0, 1024, (2, 256), device=cuda, generator=g),
             torch.randint(0, 1024, (2, 256), device=cuda, generator=g)) for _ in range(accum)]

    def run(overlap):
        m.zero_grad(set_to_none=True)
        it = iter(data)

        def loss_fn(x, y):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return m(x, y, return_logits=False)[1] / accum

        with grad_accum.accumulation_scope():
            loss = run_micro_batches(m, lambda: next(it), accum, loss_fn, overlap=overlap)
        torch.cuda.synchronize()
        return loss, {k: p.grad.clone() for k, p in m.named_parameters()}

    l0, g0 = run(False)
    l1, g1 = run(True)
    assert torch.equal(l0, l1), (l0, l1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k


@pytest.mark.parametrize("layer,comm,accum,impl", [
    ("Mamba2", "fp32", 3, "native"), ("Mamba1", "fp32", 3, "native"), ("Mamba2", "bf16", 3, "native"),
    # the 8-GPU per-rank regime (accum 2: forward 0 on the second stream) and the degenerate accum 1
    ("Mamba2", "fp32", 2, "native"), ("Mamba2", "fp32", 1, "native"), ("Mamba1", "fp32", 2, "native"),
    ("Mamba2", "fp32", 2, "ddp"), ("Mamba2", "fp32", 1, "ddp"),
    # four optimizer steps through clip_and_step: the native AdamW dividing the deferred average, a logged norm, then
    # a torch AdamW loaded from its state_dict
    ("Mamba2", "fp32", 1, "optim"), ("Mamba1", "fp32", 2, "optim")])
def test_native_reducer_two_ranks_one_gpu(cuda, layer, comm, accum, impl):
    """parallel/reducer.py (and torch DDP) on real HIP streams: two gloo ranks on cuda:0, overlapped
    micro-batches, tiny buckets; the averaged gradients match the single-process global-batch gradients
    (tests/reducer_worker.py), at accum 1, 2 (the 8-GPU per-rank regime) and 3; "optim": parameters after three
    clip + native-AdamW steps match a single process on torch's AdamW."""
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "tests", "reducer_worker.py"), "--layer", layer, "--comm-dtype", comm,
           "--accum", str(accum)] + (["--optim"] if impl == "optim" else ["--impl", impl])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="4"))
    if r.returncode != 0:  # the launcher's banner hides the worker's error at the end of stderr
        keep = [ln for ln in r.stderr.splitlines() if "Error" in ln or "assert" in ln or ln.startswith("  File")]
        pytest.fail("worker failed:\n" + r.stdout[-2000:] + "\n" + "\n".join(keep[-40:]))
    assert r.stdout.count("OK") == 2, r.stdout


@pytest.mark.parametrize("accum", [4, 5])
def test_microbatch_overlap_across_optimizer_steps(cuda, accum):
    """Several full optimizer steps (zero_grad -> overlapped micro-steps -> clip -> fused AdamW) with
    an even and an odd micro-step count: the parameters stay bitwise equal to the sequential loop's.
    With an even count forward 0 runs on the second stream, which must wait for the previous
    AdamW step (it reads the weights, and zero_grad has just released the gradient blocks)."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.ops import grad_accum
    from mamba_distributed_amd.parallel.microbatch import run_micro_batches
    cfg = MambaConfig(d_model=256, n_layer=4, vocab_size=1024, ssm_cfg={"layer": "Mamba2"})
    g = torch.Generator(device=cuda).manual_seed(1)
    steps = 4
    data = [(torch.randint(0, 1024, (2, 256), device=cuda, generator=g),
             torch.randint(0, 1024, (2, 256), device=cuda, generator=g)) for _ in range(accum * steps)]

    def train(overlap):
        torch.manual_seed(0)
        m = LMHeadModel(cfg, device=cuda)
        opt = m.configure_optimizers(0.1, 3e-3, "cuda", False)
        it = iter(data)

        def loss_fn(x, y):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return m(x, y, return_logits=False)[1] / accum

        losses = []
        for _ in range(steps):
            opt.zero_grad(set_to_none=True)
            with grad_accum.accumulation_scope():
                losses.append(run_micro_batches(m, lambda: next(it), accum, loss_fn, overlap=overlap))
            torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
            opt.step()
        torch.cuda.synchronize()
        return torch.stack(losses), {k: p.detach().clone() for k, p in m.named_parameters()}

    l0, p0 = train(False)
    l1, p1 = train(True)
    assert torch.isfinite(l0).all(), l0
    assert torch.equal(l0, l1), (l0, l1)
    for k in p0:
        assert torch.equal(p0[k], p1[k]), k


@pytest.mark.parametrize("layer", ["Mamba1", "Mamba2"])
def test_activation_checkpointing_bitwise_on_gpu(cuda, layer):
    """Per-block recompute (set_activation_checkpointing) with the native kernels, the two-stream
    micro-batch overlap and in-place gradient accumulation: loss and gradients bitwise unchanged."""
    import copy
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.ops import grad_accum
    from mamba_distributed_amd.parallel.microbatch import run_micro_batches
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=256, n_layer=4, vocab_size=1024, ssm_cfg={"layer": layer})
    m0 = LMHeadModel(cfg, device=cuda)
    m1 = copy.deepcopy(m0)
    m1.set_activation_checkpointing(1)
    accum = 4
    g = torch.Generator(device=cuda).manual_seed(1)
    data = [(torch.randint(0, 1024, (2, 256), device=cuda, generator=g),
             torch.randint(0, 1024, (2, 256), device=cuda, generator=g)) for _ in range(accum)]

    def run(m):
        it = iter(data)

        def loss_fn(x, y):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return m(x, y, return_logits=False)[1] / accum

        with grad_accum.accumulation_scope():
            loss = run_micro_batches(m, lambda: next(it), accum, loss_fn, overlap=True)
        torch.cuda.synchronize()
        return loss

    l0, l1 = run(m0), run(m1)
    assert torch.equal(l0, l1), (l0, l1)
    for (k, p), q in zip(m1.named_parameters(), m0.parameters()):
        assert torch.equal(p.grad, q.grad), k


@pytest.mark.parametrize("N,K,M", [(80, 1536, 32768), (1536, 48, 32768), (48, 1536, 4096), (1536, 80, 4096),
                                   (72, 40, 1000), (130, 24, 264), (300, 24, 1000)])
@pytest.mark.parametrize("acc", [False, True])
def test_gemm_skinny(cuda, N, K, M, acc):
    """gemm_skinny_k (channel-major Mamba-1 x_proj / dt_proj family) vs an fp32 matmul, including
    row-strided B / out views, N / K / M not multiples of the tiles, and accumulation into out."""
    from mamba_distributed_amd.ops import _ext
    g = torch.Generator(device=cuda).manual_seed(0)
    A = torch.randn(N, K, device=cuda, generator=g).to(torch.bfloat16)
    Bbig = torch.randn(K + 16, M, device=cuda, generator=g).to(torch.bfloat16)
    B = Bbig[:K]  # row-strided view like x_dbl[:R]
    C0 = torch.randn(N, M, device=cuda, generator=g).to(torch.bfloat16)
    out = C0.clone()
    r = _ext.ops().gemm_skinny(A, B, out, acc)
    ref = A.float() @ B.float() + (C0.float() if acc else 0)
    assert r.data_ptr() == out.data_ptr()
    assert rel(out, ref) < 8e-3, rel(out, ref)


@pytest.mark.parametrize("P,M,Q", [(3072, 32768, 768), (2048, 4096, 1024), (200, 1024, 136), (8, 64, 8)])
@pytest.mark.parametrize("acc", [False, True])
def test_gemm_wgrad_channel_major(cuda, P, M, Q, acc):
    """gemm_wgrad_cm (Mamba-1 in_proj dW = d(xz) h with a channel-major d(xz)) vs an fp32 matmul,
    fp32 output, accumulation into an existing gradient; P / Q not multiples of the 256 tiles."""
    from mamba_distributed_amd.ops import _ext
    g = torch.Generator(device=cuda).manual_seed(0)
    dY = torch.randn(P, M, device=cuda, generator=g).to(torch.bfloat16)
    X = torch.randn(M, Q, device=cuda, generator=g).to(torch.bfloat16)
    out = torch.randn(P, Q, device=cuda, generator=g)
    base = out.clone()
    r = _ext.ops().gemm_wgrad_cm(dY, X, out if acc else None, acc)
    ref = dY.float() @ X.float() + (base if acc else 0)
    assert r.dtype == torch.float32
    assert rel(r, ref) < 2e-3, rel(r, ref)


@pytest.mark.parametrize("dy_cm,x_cm", [(False, True), (True, True)])
@pytest.mark.parametrize("P,M,Q", [(768, 32768, 1536), (200, 1024, 136),
                                   # the Mamba-1 x_proj (80 rows: 128-row tiles) and dt_proj (48 columns: computed
                                   # transposed on 128-row tiles, added back transposed) weight gradients
                                   (80, 32768, 1536), (1536, 32768, 48), (1536, 4096, 80)])
def test_gemm_wgrad_channel_major_x(cuda, dy_cm, x_cm, P, M, Q):
    """gemm_wgrad_cm with a channel-major X (Mamba-1 out_proj dW = dout^T y^T from the (di, b*l) scan
    output) and with both operands channel-major, accumulating into fp32; deterministic run to run."""
    from mamba_distributed_amd.ops import _ext
    g = torch.Generator(device=cuda).manual_seed(1)
    dY = torch.randn(P, M, device=cuda, generator=g).to(torch.bfloat16)   # logical (P, M)
    X = torch.randn(Q, M, device=cuda, generator=g).to(torch.bfloat16)    # logical (Q, M)
    out = torch.randn(P, Q, device=cuda, generator=g)
    base = out.clone()
    dY_arg = dY if dy_cm else dY.t().contiguous()
    X_arg = X if x_cm else X.t().contiguous()
    _ext.ops().gemm_wgrad_cm(dY_arg, X_arg, out, True, dy_cm, x_cm)
    ref = dY.float() @ X.float().t() + base
    assert rel(out, ref) < 2e-3, rel(out, ref)
    again = base.clone()
    _ext.ops().gemm_wgrad_cm(dY_arg, X_arg, again, True, dy_cm, x_cm)
    assert torch.equal(again, out)


@pytest.mark.parametrize("sl_extra", [-1, 0, 3])
def test_conv_update_native_state_len(cuda, sl_extra):
    """Native conv1d_update with the upstream cache width (state_len = d_conv) and others vs the fp64
    reference: outputs and the rolled state."""
    from mamba_distributed_amd.ops import _ext
    from mamba_distributed_amd.ops.reference import causal_conv1d_update_ref
    torch.manual_seed(0)
    b, d, w = 3, 1792, 4
    sl = w + sl_extra
    st0 = torch.randn(b, d, sl, device=cuda).to(torch.bfloat16)
    wt = torch.randn(d, w, device=cuda) * 0.3
    bias = torch.randn(d, device=cuda)
    sn, sr = st0.clone(), st0.double()
    for t in range(5):
        x = torch.randn(b, d, device=cuda).to(torch.bfloat16)
        on = _ext.ops().conv1d_update(x, sn, wt, bias, True)
        orf = causal_conv1d_update_ref(x.double(), sr, wt.double(), bias.double(), "silu")
        assert rel(on, orf) < 1e-2, (t, rel(on, orf))
        sr.copy_(sr.to(torch.bfloat16).double())  # the native state is bf16
        assert torch.equal(sn, sr.to(torch.bfloat16)), t


def test_tuned_gemm_table_forces_highest_precision(cuda):
    """Regression: replaying the gfx950 TunableOp table under torch.set_float32_matmul_precision("high")
    (the reference's setting) produced garbage projections (280M forward at loss = ln V, NaN backward).
    enable_tuned_gemms must force "highest", and a 280M-shaped block must match the untuned forward."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.utils import gemm_tuning
    prev = torch.get_float32_matmul_precision()
    try:
        torch.set_float32_matmul_precision("high")
        with pytest.warns(UserWarning):
            on = gemm_tuning.enable_tuned_gemms()
        assert torch.get_float32_matmul_precision() == "highest"
        torch.manual_seed(0)
        m = LMHeadModel(MambaConfig(d_model=768, n_layer=1, vocab_size=50304, ssm_cfg={"layer": "Mamba2"}),
                        device=cuda)
        ids = torch.randint(0, 50304, (32, 1025), device=cuda)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            _, l_tuned = m(ids[:, :-1], ids[:, 1:], return_logits=False)
            torch.cuda.tunable.enable(False)
            _, l_plain = m(ids[:, :-1], ids[:, 1:], return_logits=False)
        assert torch.isfinite(l_tuned) and abs(l_tuned.item() - l_plain.item()) < 1e-2, (l_tuned, l_plain, on)
    finally:
        torch.cuda.tunable.enable(False)
        torch.set_float32_matmul_precision(prev)


@pytest.mark.parametrize("L,with_z", [(256, True), (1008, False)])
def test_selective_scan_channel_walk(cuda, monkeypatch, L, with_z):
    """Forward at a channel count that selects the sequential-time walk (B * D / 16 >= 2048):
    against the fp32 reference and bitwise-stable vs the time-parallel kernel's saved carries (the
    backward consumes them), including a partial last 32-step tile (L = 1008) and the last state."""
    from mamba_distributed_amd.ops.selective_scan import selective_scan_fn
    torch.manual_seed(6)
    b, d, n = 8, 4096, 16
    u = torch.randn(b, d, L, device=cuda).to(torch.bfloat16)
    delta = (torch.randn(b, d, L, device=cuda) * 0.5 - 1).to(torch.bfloat16)
    A = -torch.rand(d, n, device=cuda) * 4 - 0.1
    Bm = torch.randn(b, 1, n, L, device=cuda).to(torch.bfloat16)
    Cm = torch.randn(b, 1, n, L, device=cuda).to(torch.bfloat16)
    D = torch.randn(d, device=cuda)
    z = torch.randn(b, d, L, device=cuda).to(torch.bfloat16) if with_z else None
    db = torch.randn(d, device=cuda) * 0.3
    ops = torch.ops.mamba_amd
    out, carries, last = ops.selscan_fwd(u, delta, A, Bm, Cm, D, z, db, True)
    y_ref = R.selective_scan_ref(u, delta, A, Bm, Cm, D, z=z, delta_bias=db, delta_softplus=True)
    assert rel(out, y_ref) < 2e-2
    # the walk saves its state every 16 steps (for the sequential backward); the last carry row holds the
    # state after step 16 * (rows - 1) + 15, whose continuation to L is the returned last state
    assert carries.shape[2] == (L + 15) // 16 and torch.isfinite(last).all()
    y = selective_scan_fn(u, delta, A, Bm, Cm, D, z=z, delta_bias=db, delta_softplus=True)
    assert rel(y, y_ref) < 2e-2


@pytest.mark.parametrize("b,d,L,G,with_z", [(32, 1536, 256, 1, True), (16, 2048, 160, 2, False)])
def test_selective_scan_sequential_backward(cuda, monkeypatch, b, d, L, G, with_z):
    """The sequential-time backward (selscan_bwd_sg_k, 16-step carries, lane-butterfly dB/dC) at the
    Mamba-1 280M channel count: every gradient vs the fp32 reference and vs the time-parallel backward."""
    from mamba_distributed_amd.ops.selective_scan import selective_scan_fn
    torch.manual_seed(8)
    n = 16
    u = torch.randn(b, d, L, device=cuda).to(torch.bfloat16)
    delta = (torch.randn(b, d, L, device=cuda) * 0.5 - 1).to(torch.bfloat16)
    A = -torch.rand(d, n, device=cuda) * 4 - 0.1
    Bm = torch.randn(b, G, n, L, device=cuda).to(torch.bfloat16)
    Cm = torch.randn(b, G, n, L, device=cuda).to(torch.bfloat16)
    D = torch.randn(d, device=cuda)
    z = torch.randn(b, d, L, device=cuda).to(torch.bfloat16) if with_z else None
    db = torch.randn(d, device=cuda) * 0.3
    ops = torch.ops.mamba_amd
    assert ops.selscan_fwd(u, delta, A, Bm, Cm, D, z, db, True)[1].shape[2] == L // 16  # 16-step carries

    def f(u, delta, A, Bm, Cm, D, z, db):
        return selective_scan_fn(u, delta, A, Bm, Cm, D, z=z, delta_bias=db, delta_softplus=True)

    ins = [u, delta, A, Bm, Cm, D, z, db]
    on, orf, gn, gr = run_both(f, f, ins)
    assert rel(on, orf) < 2e-2, rel(on, orf)
    names = ["u", "delta", "A", "B", "C", "D", "z", "db"]
    for nm, a_, b_ in zip(names, gn, gr):
        if b_ is not None:
            assert rel(a_, b_) < 3e-2, (nm, rel(a_, b_))
    # 16-step carries consumed by the time-parallel backward (a dout that is not 16-B aligned keeps the
    # sequential kernel out): same gradients
    out, carries, _ = ops.selscan_fwd(u, delta, A, Bm, Cm, D, z, db, True)
    go = torch.randn_like(out)
    ref_g = ops.selscan_bwd(go, u, delta, A, Bm, Cm, D, z, db, carries, True)
    buf = torch.empty(go.numel() + 1, device=cuda, dtype=go.dtype)
    go_mis = buf[1:].view(go.shape)
    go_mis.copy_(go)
    mis_g = ops.selscan_bwd(go_mis, u, delta, A, Bm, Cm, D, z, db, carries, True)
    for nm, a_, b_ in zip(["du", "ddelta", "dA", "dB", "dC", "dD", "dz", "dbias"], mis_g, ref_g):
        if b_.numel():
            assert rel(a_, b_) < 1e-2, (nm, rel(a_, b_))


@pytest.mark.parametrize("preset", [False, True])
def test_late_colsum(cuda, preset):
    """The batched late column sum (ops/grad_accum.py::flush_late, kernels/norm.hip late_colsum_*): the three
    destination layouts (plain, conv taps | bias per channel, A | D | bias), stored into fresh .grad views or added
    into existing gradients; against fp64 column sums, and bitwise repeatable."""
    from mamba_distributed_amd.ops import grad_accum
    g = torch.Generator(device=cuda).manual_seed(3)
    P = lambda *s: torch.nn.Parameter(torch.zeros(*s, device=cuda))  # noqa: E731
    pn, pA, pD, pb_, pw, pb = P(1536), P(24), P(24), P(24), P(1792, 1, 4), P(1792)
    parts = [torch.randn(2048, 1536, device=cuda, generator=g), torch.randn(1024, 3, 24, device=cuda, generator=g),
             torch.randn(300, 1792, 5, device=cuda, generator=g), torch.randn(7, 1536, device=cuda, generator=g)]
    pn2 = P(1536)
    sums = [t.double().sum(0) for t in parts]
    base = {}
    for p in (pn, pA, pD, pb_, pw, pb, pn2):
        if preset:
            p.grad = torch.randn(p.shape, device=cuda, generator=g)
            base[id(p)] = p.grad.clone()

    def run():
        work = [t.clone() for t in parts]
        with grad_accum.accumulation_scope():
            grad_accum.set_late(True)
            grad_accum.late_colsum(work[0], 0, 0, [pn])
            grad_accum.late_colsum(work[1], 2, 24, [pA, pD, pb_])
            grad_accum.late_colsum(work[2], 1, 5, [pw, pb])
            grad_accum.late_colsum(work[3], 0, 0, [pn2])
            grad_accum.flush_late()
        torch.cuda.synchronize()
        return [p.grad.clone() for p in (pn, pA, pD, pb_, pw, pb, pn2)]

    got = run()
    want = [sums[0], sums[1][0], sums[1][1], sums[1][2], sums[2][:, :4].reshape(1792, 1, 4), sums[2][:, 4], sums[3]]
    for i, (a_, w_) in enumerate(zip(got, want)):
        p = (pn, pA, pD, pb_, pw, pb, pn2)[i]
        ref = w_ + (base[id(p)].double() if preset else 0)
        assert a_.shape == p.shape
        assert ((a_.double() - ref).abs().max() / (ref.abs().max() + 1e-9)).item() < 1e-5, i
    if preset:
        for p in (pn, pA, pD, pb_, pw, pb, pn2):
            p.grad = base[id(p)].clone()
    else:
        for p in (pn, pA, pD, pb_, pw, pb, pn2):
            p.grad = None
    again = run()
    for a_, b_ in zip(got, again):
        assert torch.equal(a_, b_)


@pytest.mark.parametrize("fused", [True, False])
def test_selective_scan_walk_order(cuda, fused):
    """The sequential walks with workgroups numbered b-fastest (MAMBA_AMD_SELSCAN_ORDER=1, for (d, b, l) memory) against
    the default b-major numbering: bitwise-equal outputs, carries, last state and every gradient (each workgroup's math is unchanged)."""
    torch.manual_seed(13)
    b, d, L, Rk, n = 40, 1536, 128, 48, 16
    ops = torch.ops.mamba_amd
    M = b * L
    cm = lambda t2: t2.view(t2.shape[0], b, L).permute(1, 0, 2)  # noqa: E731
    u, z = cm(torch.randn(d, M, device=cuda).to(torch.bfloat16)), cm(torch.randn(d, M, device=cuda).to(torch.bfloat16))
    x_dbl = torch.randn(Rk + 2 * n, M, device=cuda).to(torch.bfloat16)
    W = (torch.randn(d, Rk, device=cuda) * Rk ** -0.5).to(torch.bfloat16)
    A = -torch.rand(d, n, device=cuda) * 4 - 0.1
    D = torch.randn(d, device=cuda)
    db = torch.randn(d, device=cuda) * 0.3 - 1.0
    delta = cm((W.float() @ x_dbl[:Rk].float()).to(torch.bfloat16))
    Bm, Cm = cm(x_dbl[Rk:Rk + n]).unsqueeze(1), cm(x_dbl[Rk + n:]).unsqueeze(1)
    go2 = torch.randn(d, M, device=cuda).to(torch.bfloat16)

    def run():
        if fused:
            y, car, last = ops.selscan_fwd_dt(u, W, x_dbl[:Rk], A, Bm, Cm, D, z, db, True)
        else:
            y, car, last = ops.selscan_fwd(u, delta, A, Bm, Cm, D, z, db, True)
        dz2 = torch.empty(d, M, device=cuda, dtype=torch.bfloat16)
        dx = torch.empty(2 * n, M, device=cuda, dtype=torch.bfloat16)
        outs = (cm(dz2), cm(dx[:n]).unsqueeze(1), cm(dx[n:]).unsqueeze(1))
        if fused:
            g = ops.selscan_bwd_dt_into(cm(go2), u, W, x_dbl[:Rk], A, Bm, Cm, D, z, db, car, True, *outs)
        else:
            g = ops.selscan_bwd_into(cm(go2), u, delta, A, Bm, Cm, D, z, db, car, True, *outs)
        return [y, car, last, dz2, dx] + [t for t in g if t is not None]

    prev = ops.selscan_order(-1)
    try:
        ops.selscan_order(0)
        ref = run()
        ops.selscan_order(1)
        got = run()
        torch.cuda.synchronize()
    finally:
        ops.selscan_order(prev)
    for i, (a_, b_) in enumerate(zip(got, ref)):
        assert torch.equal(a_, b_), i


@pytest.mark.parametrize("b,d,L,Rk,with_z", [(32, 1536, 256, 48, True), (32, 1024, 128, 64, False),
                                              (24, 2048, 64, 96, True), (64, 512, 64, 16, True)])
def test_selective_scan_fused_dt(cuda, b, d, L, Rk, with_z):
    """dt_proj fused into the sequential scan walks (selscan_fwd_dt / selscan_bwd_dt_into, kernels/selective_scan.hip
    DTF): delta_raw = W_dt x_dbl[:R] per 16-step tile on MFMA inside the kernels, in the Mamba-1 channel-major layout
    (u, z as (d, b, l) memory; B / C / x as rows of one x_dbl).  Forward and every gradient vs the fp32 reference
    with the fp32 delta, and vs the unfused kernels fed the bf16-rounded delta; dt_rank 16 exercises the zero-padded
    K-step."""
    torch.manual_seed(12)
    n = 16
    ops = torch.ops.mamba_amd
    M = b * L
    cm = lambda t2: t2.view(t2.shape[0], b, L).permute(1, 0, 2)  # noqa: E731  (rows, b*L) -> (b, rows, L)
    u2 = torch.randn(d, M, device=cuda).to(torch.bfloat16)
    z2 = torch.randn(d, M, device=cuda).to(torch.bfloat16) if with_z else None
    x_dbl = (torch.randn(Rk + 2 * n, M, device=cuda)).to(torch.bfloat16)
    W = (torch.randn(d, Rk, device=cuda) * Rk ** -0.5).to(torch.bfloat16)
    A = -torch.rand(d, n, device=cuda) * 4 - 0.1
    D = torch.randn(d, device=cuda)
    db = torch.randn(d, device=cuda) * 0.3 - 1.0
    u, z = cm(u2), (cm(z2) if with_z else None)
    Bm, Cm = cm(x_dbl[Rk:Rk + n]).unsqueeze(1), cm(x_dbl[Rk + n:]).unsqueeze(1)
    d32 = W.float() @ x_dbl[:Rk].float()                       # (d, b*L) fp32 delta_raw
    y, carries, last = ops.selscan_fwd_dt(u, W, x_dbl[:Rk], A, Bm, Cm, D, z, db, True)
    assert carries.shape[2] == L // 16
    y_u, car_u, _ = ops.selscan_fwd(u, cm(d32.to(torch.bfloat16)), A, Bm, Cm, D, z, db, True)
    # fp32 reference with autograd for the gradients
    leaves = [t.detach().float().clone().requires_grad_(True) for t in (u, cm(d32), A, Bm, Cm, D, db)]
    zr = z.float() if with_z else None
    y_ref = R.selective_scan_ref(leaves[0], leaves[1], leaves[2], leaves[3], leaves[4], leaves[5], z=zr,
                                 delta_bias=leaves[6], delta_softplus=True)
    assert rel(y, y_ref) < 2e-2, rel(y, y_ref)
    assert rel(y, y_u) < 2e-2, rel(y, y_u)
    go = torch.randn_like(y_ref)
    y_ref.backward(go)
    gob = go.to(torch.bfloat16)
    go2 = torch.empty(d, M, device=cuda, dtype=torch.bfloat16)
    cm(go2).copy_(gob)

    def bwd(fused):
        dz2 = torch.empty(d, M, device=cuda, dtype=torch.bfloat16)
        dx = torch.empty(2 * n, M, device=cuda, dtype=torch.bfloat16)
        outs = (cm(dz2) if with_z else torch.empty(0, device=cuda, dtype=torch.bfloat16),
                cm(dx[:n]).unsqueeze(1), cm(dx[n:]).unsqueeze(1))
        if fused:
            return ops.selscan_bwd_dt_into(cm(go2), u, W, x_dbl[:Rk], A, Bm, Cm, D, z, db, carries, True, *outs)
        return ops.selscan_bwd_into(cm(go2), u, cm(d32.to(torch.bfloat16)), A, Bm, Cm, D, z, db, car_u, True, *outs)

    gf, gu = bwd(True), bwd(False)
    names = ["du", "ddelta", "dA", "dB", "dC", "dD", "dz", "dbias"]
    refs = [leaves[0].grad, leaves[1].grad, leaves[2].grad, leaves[3].grad, leaves[4].grad, leaves[5].grad,
            None, leaves[6].grad]
    for nm, a_, b_, r_ in zip(names, gf, gu, refs):
        if not a_.numel():
            continue
        assert torch.isfinite(a_.float()).all(), nm
        assert rel(a_, b_) < 3e-2, (nm, rel(a_, b_))
        if r_ is not None:
            assert rel(a_, r_) < 3e-2, (nm, rel(a_, r_))
    # determinism: the backward's recomputed delta is the forward's (same operands and instruction sequence)
    gf2 = bwd(True)
    for nm, a_, b_ in zip(names, gf, gf2):
        if a_.numel():
            assert torch.equal(a_, b_), nm


def test_mamba1_fused_dt_model(cuda, monkeypatch):
    """A Mamba-1 model at a shape that takes the fused dt_proj scan (b * d_inner >= 32768; opt-in
    MAMBA_AMD_M1_DT_FUSED=1): loss and every parameter gradient vs the fp32 reference ops and vs the unfused path
    (MAMBA_AMD_M1_DT_FUSED=0); a spy checks the fused op ran."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    calls = []
    ops = torch.ops.mamba_amd
    orig = ops.selscan_fwd_dt

    class Spy:
        def __getattr__(self, k):
            if k == "selscan_fwd_dt":
                def f(*a):
                    calls.append(1)
                    return orig(*a)
                return f
            return getattr(ops, k)
    from mamba_distributed_amd.ops import _ext
    real = _ext.ops
    monkeypatch.setattr(_ext, "ops", lambda: Spy())
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=768, n_layer=2, vocab_size=4096, ssm_cfg={"layer": "Mamba1"})
    m = LMHeadModel(cfg, device=cuda)
    sharpen_logits(m)
    x = torch.randint(0, 4096, (32, 256), device=cuda)
    y = torch.randint(0, 4096, (32, 256), device=cuda)

    def lossgrad(force_ref=False, fused=True):
        os.environ["MAMBA_AMD_M1_DT_FUSED"] = "1" if fused else "0"
        if force_ref:
            os.environ["MAMBA_AMD_FORCE_REFERENCE"] = "1"
        try:
            m.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                _, loss = m(x, y)
            loss.backward()
            return loss.item(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        finally:
            os.environ.pop("MAMBA_AMD_FORCE_REFERENCE", None)
            os.environ.pop("MAMBA_AMD_M1_DT_FUSED", None)

    ln, gn = lossgrad()
    assert len(calls) == cfg.n_layer, calls
    lu, gu = lossgrad(fused=False)
    assert len(calls) == cfg.n_layer
    monkeypatch.setattr(_ext, "ops", real)
    lr, gr = lossgrad(force_ref=True)
    check_loss(ln, lr, cfg.vocab_size)
    assert abs(ln - lu) < 2e-3 * abs(lu), (ln, lu)
    bad = {n: rel(gn[n], gr[n]) for n in gr if rel(gn[n], gr[n]) > 5e-2}
    assert not bad, bad
    bad = {n: rel(gn[n], gu[n]) for n in gu if rel(gn[n], gu[n]) > 3e-2}
    assert not bad, bad


@pytest.mark.parametrize("b,L,H,G,N,with_init", [(2, 200, 8, 1, 128, True), (1, 64, 4, 2, 64, False),
                                                 (3, 1030, 24, 1, 128, False)])
def test_ssd_fp32_native_forward(cuda, b, L, H, G, N, with_init):
    """fp32 inference (the reference's fp32 HellaSwag protocol) runs the native fp32 sequential SSD
    forward: y and the final state vs the fp32 chunked reference, incl. z gate and dt limits."""
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    g = torch.Generator(device=cuda).manual_seed(40)
    x = torch.randn(b, L, H, 64, generator=g, device=cuda)
    dt = torch.randn(b, L, H, generator=g, device=cuda) * 0.5 - 1
    A = -torch.rand(H, generator=g, device=cuda) * 4 - 0.2
    Bm = torch.randn(b, L, G, N, generator=g, device=cuda) * 0.5
    Cm = torch.randn(b, L, G, N, generator=g, device=cuda) * 0.5
    D = torch.randn(H, generator=g, device=cuda)
    dtb = torch.randn(H, generator=g, device=cuda) * 0.3
    z = torch.randn(b, L, H, 64, generator=g, device=cuda)
    init = torch.randn(b, H, 64, N, generator=g, device=cuda) * 0.3 if with_init else None
    ops = torch.ops.mamba_amd
    kw = dict(D=D, z=z, dt_bias=dtb, initial_states=init, dt_softplus=True, dt_limit=(0.01, 3.0),
              return_final_states=True)
    with torch.no_grad():
        y, fin = mamba_chunk_scan_combined(x, dt, A, Bm, Cm, 64, **kw)
        y2, fin2 = R.ssd_chunked_ref(x.double(), dt.double(), A.double(), Bm.double(), Cm.double(), 64,
                                     D=D.double(), z=z.double(), dt_bias=dtb.double(),
                                     initial_states=None if init is None else init.double(), dt_softplus=True,
                                     dt_limit=(0.01, 3.0), return_final_states=True)
        yn, finn = ops.ssd_fwd_f32(x, dt, A, Bm, Cm, D, dtb, init, True, 0.01, 3.0, True)
    assert y.dtype == torch.float32
    assert rel(y, y2) < 1e-4, rel(y, y2)
    assert rel(fin, fin2) < 1e-4, rel(fin, fin2)
    assert rel(yn * torch.nn.functional.silu(z), y) < 1e-6


def test_mamba2_layer_fp32_eval_uses_native_ssd(cuda, monkeypatch):
    """Mamba-2 layer in fp32 under no_grad: the SSD step runs ssd_fwd_f32 (native) and matches the
    all-reference forward."""
    from mamba_distributed_amd.models.mamba2 import Mamba2
    from mamba_distributed_amd.ops import ssd as ssd_mod
    torch.manual_seed(9)
    layer = Mamba2(256, d_state=128, headdim=64, device=cuda).float().eval()
    u = torch.randn(2, 150, 256, device=cuda)
    used = []
    orig = ssd_mod._f32_eval_ok

    def spy(*a, **k):
        r = orig(*a, **k)
        used.append(r)
        return r
    monkeypatch.setattr(ssd_mod, "_f32_eval_ok", spy)
    with torch.no_grad():
        y = layer(u)
    assert used and all(used)
    monkeypatch.setenv("MAMBA_AMD_FORCE_REFERENCE", "1")
    with torch.no_grad():
        yr = layer(u)
    assert rel(y, yr) < 1e-4, rel(y, yr)
