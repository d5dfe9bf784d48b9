"""Native varlen / state hand-off interfaces vs the fp32 references.

  * ``causal_conv1d_fn`` with seq_idx / initial_states / return_final_states -> HIP conv1d_cl_var
  * ``mamba_chunk_scan_combined`` with seq_idx (and initial states) -> HIP ssd_fwd/bwd
  * ``mamba_split_conv1d_scan_combined`` with initial_states / return_final_states / seq_idx (fused chain)
  * a packed two-sequence batch through the Mamba-2 layer == the two sequences run separately
"""
import pytest
import torch

from test_kernels_gpu import rel, run_both, _ssd_inputs

pytestmark = pytest.mark.gpu


def _seq(lens, device, b=1):
    s = torch.cat([torch.full((n,), i, dtype=torch.int32) for i, n in enumerate(lens)])
    return s[None].expand(b, -1).contiguous().to(device)


@pytest.mark.parametrize("layout", ["cl", "cf"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("W", [4, 2])
def test_conv_var_seq_init_final(cuda, layout, dtype, W):
    from mamba_distributed_amd.ops.conv1d import causal_conv1d_fn
    torch.manual_seed(0)
    lens = [1, 37, 2, 200, 60]
    b, d, L = 2, 200, sum(lens)
    if layout == "cl":
        x = torch.randn(b, L, d, device=cuda).to(dtype).transpose(1, 2)
    else:
        x = torch.randn(b, d, L, device=cuda).to(dtype)
    w = torch.randn(d, W, device=cuda) * 0.4
    bias = torch.randn(d, device=cuda) * 0.1
    init = (torch.randn(b, d, W - 1, device=cuda) * 0.5).to(dtype)
    sq = _seq(lens, cuda, b)

    def f(x, w, bias, init):
        out, fin = causal_conv1d_fn(x, w, bias, "silu", initial_states=init, return_final_states=True, seq_idx=sq)
        return out.float() + fin.float().mean(-1, keepdim=True)

    on, orf, gn, gr = run_both(f, f, [x, w, bias, init])
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert rel(on, orf) < tol
    for nm, a, b_ in zip(["x", "w", "bias", "init"], gn, gr):
        assert rel(a, b_) < 1.5 * tol, (nm, rel(a, b_))


def test_conv_var_native_matches_separate_sequences(cuda):
    """The native seq_idx conv equals convolving each packed sequence on its own (bitwise: same taps)."""
    from mamba_distributed_amd.ops.conv1d import causal_conv1d_fn
    torch.manual_seed(1)
    lens = [63, 1, 130]
    d = 96
    x = torch.randn(1, sum(lens), d, device=cuda).to(torch.bfloat16).transpose(1, 2)
    w = torch.randn(d, 4, device=cuda) * 0.4
    out = causal_conv1d_fn(x, w, None, "silu", seq_idx=_seq(lens, cuda))
    s = 0
    for n in lens:
        ref = causal_conv1d_fn(x[..., s:s + n], w, None, "silu", initial_states=torch.zeros(1, d, 3, device=cuda,
                                                                                              dtype=x.dtype))
        torch.testing.assert_close(out[..., s:s + n], ref, rtol=0, atol=0)
        s += n


@pytest.mark.parametrize("lens", [[64, 64, 100], [5, 1, 120, 70, 32], [300]])
def test_ssd_seq_idx(cuda, lens):
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    b, L, H = 2, sum(lens), 8
    x, dt, A, Bm, Cm, D, dt_bias = _ssd_inputs(cuda, b, L, H, 1, 128, seed=21)
    sq = _seq(lens, cuda, b)
    init = torch.randn(b, H, 64, 128, device=cuda) * 0.2

    def f(x, dt, A, Bm, Cm, D, dt_bias, init):
        y, fin = mamba_chunk_scan_combined(x, dt, A, Bm, Cm, 64, D=D, dt_bias=dt_bias, dt_softplus=True,
                                           initial_states=init, return_final_states=True, seq_idx=sq)
        return y.float() + fin.float().mean((-1, -2))[:, None, :, None] * 0.1

    on, orf, gn, gr = run_both(f, f, [x, dt, A, Bm, Cm, D, dt_bias, init])
    assert rel(on, orf) < 2e-2, rel(on, orf)
    for nm, a, b_ in zip(["x", "dt", "A", "B", "C", "D", "dt_bias", "init"], gn, gr):
        assert rel(a, b_) < 3e-2, (nm, rel(a, b_))


def _inner_inputs(cuda, b, L, H=8, G=1, N=128, seed=4):
    g = torch.Generator(device=cuda).manual_seed(seed)
    P = 64
    di = H * P
    dproj = 2 * di + 2 * G * N + H
    zx = torch.randn(b, L, dproj, generator=g, device=cuda).to(torch.bfloat16)
    conv_w = torch.randn(di + 2 * G * N, 1, 4, generator=g, device=cuda) * 0.3
    conv_b = torch.randn(di + 2 * G * N, generator=g, device=cuda) * 0.1
    dt_bias = torch.randn(H, generator=g, device=cuda) * 0.3
    A_log = torch.rand(H, generator=g, device=cuda) * 2
    D = torch.randn(H, generator=g, device=cuda)
    nw = torch.rand(di, generator=g, device=cuda) + 0.5
    return zx, conv_w, conv_b, dt_bias, A_log, D, nw


@pytest.mark.parametrize("with_seq", [False, True])
def test_split_conv1d_scan_combined_states(cuda, with_seq):
    """initial_states / return_final_states / seq_idx through the fused native chain, fwd + bwd."""
    from mamba_distributed_amd.ops.ssd import mamba_split_conv1d_scan_combined
    b, L, H = 2, 250, 8
    zx, conv_w, conv_b, dt_bias, A_log, D, nw = _inner_inputs(cuda, b, L, H)
    init = torch.randn(b, H, 64, 128, device=cuda) * 0.2
    sq = _seq([100, 3, 147], cuda, b) if with_seq else None

    def f(zx, conv_w, conv_b, dt_bias, A_log, D, nw, init):
        A = -torch.exp(A_log.float())
        y, fin = mamba_split_conv1d_scan_combined(zx, conv_w, conv_b, dt_bias, A, D, 64, initial_states=init,
                                                  seq_idx=sq, return_final_states=True, rmsnorm_weight=nw,
                                                  rmsnorm_eps=1e-5, headdim=64, ngroups=1,
                                                  norm_before_gate=False)
        return y.float() + fin.float().mean((-1, -2)).sum(-1)[:, None, None] * 0.1

    on, orf, gn, gr = run_both(f, f, [zx, conv_w, conv_b, dt_bias, A_log, D, nw, init])
    assert rel(on, orf) < 2e-2, rel(on, orf)
    for nm, a, b_ in zip(["zx", "conv_w", "conv_b", "dt_bias", "A_log", "D", "nw", "init"], gn, gr):
        assert rel(a, b_) < 3e-2, (nm, rel(a, b_))


def test_packed_two_sequence_batch_matches_separate(cuda):
    """Mamba-2 layer on one packed row (cu_seqlens) == each sequence run alone, fwd and input grads."""
    from mamba_distributed_amd.models.mamba2 import Mamba2
    torch.manual_seed(3)
    d_model, l1, l2 = 256, 150, 91
    layer = Mamba2(d_model, d_state=128, headdim=64, device=cuda).to(torch.bfloat16)
    u = torch.randn(1, l1 + l2, d_model, device=cuda).to(torch.bfloat16)
    up = u.clone().requires_grad_(True)
    yp = layer(up, cu_seqlens=torch.tensor([0, l1, l1 + l2], device=cuda))
    go = torch.randn_like(yp)
    yp.backward(go)
    ys, gs = [], []
    for s, e in ((0, l1), (l1, l1 + l2)):
        ui = u[:, s:e].clone().requires_grad_(True)
        yi = layer(ui)
        yi.backward(go[:, s:e])
        ys.append(yi)
        gs.append(ui.grad)
    assert rel(yp, torch.cat(ys, 1)) < 1e-2
    assert rel(up.grad, torch.cat(gs, 1)) < 2e-2


def test_chunk_scan_combined_with_z_native(cuda):
    """mamba_chunk_scan_combined(z=...) runs the native SSD (plus the elementwise gate), fwd and bwd vs fp32."""
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    b, L, H = 2, 200, 8
    x, dt, A, Bm, Cm, D, dt_bias = _ssd_inputs(cuda, b, L, H, 1, 128, seed=31)
    z = torch.randn(b, L, H, 64, device=cuda).to(torch.bfloat16)

    def f(x, dt, Bm, Cm, z):
        return mamba_chunk_scan_combined(x, dt, A, Bm, Cm, 64, D=D, z=z, dt_bias=dt_bias, dt_softplus=True)

    on, orf, gn, gr = run_both(f, f, [x, dt, Bm, Cm, z])
    assert rel(on, orf) < 2e-2
    for nm, a, b_ in zip(["x", "dt", "B", "C", "z"], gn, gr):
        assert rel(a, b_) < 3e-2, (nm, rel(a, b_))
