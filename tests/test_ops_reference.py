"""Reference-op oracles (CPU, fp64): chunked == sequential, layout/chunk invariance, gradcheck,
and parity with the transformers pure-PyTorch Mamba / Mamba-2 mixers (SURVEY.md [oracle])."""
import pytest
import torch
import torch.nn.functional as F

from mamba_distributed_amd.ops import reference as R

DT = torch.float64


def _ssd_inputs(b=2, l=37, h=4, p=8, g=2, n=6, seed=0):
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(b, l, h, p, generator=gen, dtype=DT)
    dt = torch.randn(b, l, h, generator=gen, dtype=DT) * 0.5
    A = -torch.rand(h, generator=gen, dtype=DT) * 3 - 0.1
    B = torch.randn(b, l, g, n, generator=gen, dtype=DT)
    C = torch.randn(b, l, g, n, generator=gen, dtype=DT)
    D = torch.randn(h, generator=gen, dtype=DT)
    dt_bias = torch.randn(h, generator=gen, dtype=DT) * 0.2
    return x, dt, A, B, C, D, dt_bias


@pytest.mark.parametrize("chunk", [8, 16, 64])
def test_ssd_chunked_equals_sequential(chunk):
    x, dt, A, B, C, D, dtb = _ssd_inputs()
    init = torch.randn(2, 4, 8, 6, dtype=DT) * 0.3
    y1, s1 = R.ssd_chunked_ref(x, dt, A, B, C, chunk, D=D, dt_bias=dtb, initial_states=init, return_final_states=True)
    y2, s2 = R.ssd_sequential_ref(x, dt, A, B, C, D=D, dt_bias=dtb, initial_states=init, return_final_states=True)
    torch.testing.assert_close(y1, y2, rtol=1e-9, atol=1e-9)
    torch.testing.assert_close(s1, s2, rtol=1e-9, atol=1e-9)


def test_ssd_gradcheck():
    x, dt, A, B, C, D, dtb = _ssd_inputs(b=1, l=9, h=2, p=3, g=1, n=2)
    args = [t.requires_grad_() for t in (x, dt, A, B, C, D, dtb)]
    f = lambda x, dt, A, B, C, D, dtb: R.ssd_chunked_ref(x, dt, A, B, C, 4, D=D, dt_bias=dtb)
    assert torch.autograd.gradcheck(f, args, eps=1e-6, atol=1e-5)


@pytest.mark.parametrize("chunk", [4, 32])
def test_selective_scan_chunked_equals_sequential(chunk):
    gen = torch.Generator().manual_seed(1)
    b, d, l, n = 2, 5, 23, 4
    u = torch.randn(b, d, l, generator=gen, dtype=DT)
    delta = torch.randn(b, d, l, generator=gen, dtype=DT) * 0.5
    A = -torch.rand(d, n, generator=gen, dtype=DT) * 2
    B = torch.randn(b, 1, n, l, generator=gen, dtype=DT)
    C = torch.randn(b, 1, n, l, generator=gen, dtype=DT)
    D = torch.randn(d, generator=gen, dtype=DT)
    z = torch.randn(b, d, l, generator=gen, dtype=DT)
    db = torch.randn(d, generator=gen, dtype=DT)
    y1, h1 = R.selective_scan_ref(u, delta, A, B, C, D, z, db, True, return_last_state=True, chunk=chunk)
    y2, h2 = R.selective_scan_sequential_ref(u, delta, A, B, C, D, z, db, True, return_last_state=True)
    torch.testing.assert_close(y1, y2, rtol=1e-9, atol=1e-9)
    torch.testing.assert_close(h1, h2, rtol=1e-9, atol=1e-9)


def test_conv1d_ref_and_update():
    gen = torch.Generator().manual_seed(2)
    b, d, l, w = 2, 6, 11, 4
    x = torch.randn(b, d, l, generator=gen, dtype=DT)
    wt = torch.randn(d, w, generator=gen, dtype=DT)
    bias = torch.randn(d, generator=gen, dtype=DT)
    out = R.causal_conv1d_ref(x, wt, bias, "silu")
    exp = F.silu(F.conv1d(x, wt.unsqueeze(1), bias, padding=w - 1, groups=d)[..., :l])
    torch.testing.assert_close(out, exp)
    # streaming one token at a time reproduces the full convolution
    state = torch.zeros(b, d, w - 1, dtype=DT)
    ys = [R.causal_conv1d_update_ref(x[..., t], state, wt, bias, "silu") for t in range(l)]
    torch.testing.assert_close(torch.stack(ys, -1), out)
    # initial states == prefix
    full = R.causal_conv1d_ref(torch.cat([x, x], -1), wt, bias, None)
    tail = R.causal_conv1d_ref(x, wt, bias, None, initial_states=x[..., -(w - 1):])
    torch.testing.assert_close(full[..., l:], tail)


def test_state_update_matches_scan():
    gen = torch.Generator().manual_seed(3)
    b, l, h, p, g, n = 2, 7, 4, 3, 2, 5
    x, dt, A, B, C, D, dtb = _ssd_inputs(b, l, h, p, g, n, seed=3)
    y = R.ssd_sequential_ref(x, dt, A, B, C, D=D, dt_bias=dtb)
    st = torch.zeros(b, h, p, n, dtype=DT)
    ys = [R.selective_state_update_ref(st, x[:, t], dt[:, t], A, B[:, t], C[:, t], D, None, dtb, True) for t in range(l)]
    torch.testing.assert_close(torch.stack(ys, 1), y)


def test_norms_match_definitions():
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(5, 16, generator=gen, dtype=DT)
    r = torch.randn(5, 16, generator=gen, dtype=DT)
    w = torch.randn(16, generator=gen, dtype=DT)
    y, res = R.add_rms_norm_ref(x, w, r, eps=1e-5, prenorm=True, residual_in_fp32=True)
    s = x + r
    torch.testing.assert_close(res, s.float())
    torch.testing.assert_close(y, s * torch.rsqrt(s.pow(2).mean(-1, keepdim=True) + 1e-5) * w)
    from transformers.models.mamba2.modeling_mamba2 import MambaRMSNormGated
    hf = MambaRMSNormGated(16, eps=1e-5).double()
    hf.weight.data.copy_(w)
    z = torch.randn(5, 16, generator=gen, dtype=DT)
    torch.testing.assert_close(R.gated_rms_norm_ref(x, z, w, 1e-5), hf(x, z))


def test_mamba2_mixer_matches_transformers_oracle():
    """Our Mamba2 mixer (CPU reference path) vs transformers' Mamba2Mixer.torch_forward."""
    from transformers import Mamba2Config
    from transformers.models.mamba2.modeling_mamba2 import Mamba2Mixer
    from mamba_distributed_amd.models.mamba2 import Mamba2
    torch.manual_seed(0)
    d, hd, n, g = 64, 16, 16, 1  # HF normalises the gated norm over all groups; g=1 is unambiguous
    ours = Mamba2(d, d_state=n, headdim=hd, ngroups=g, chunk_size=8).double()
    cfg = Mamba2Config(hidden_size=d, state_size=n, head_dim=hd, num_heads=2 * d // hd, n_groups=g, expand=2,
                       conv_kernel=4, chunk_size=8, use_bias=False, use_conv_bias=True, layer_norm_epsilon=1e-5,
                       rms_norm=True, time_step_limit=(0.0, float("inf")))
    hf = Mamba2Mixer(cfg, layer_idx=0).double()
    sd = {"in_proj.weight": ours.in_proj.weight, "conv1d.weight": ours.conv1d.weight, "conv1d.bias": ours.conv1d.bias,
          "dt_bias": ours.dt_bias, "A_log": ours.A_log, "D": ours.D, "norm.weight": ours.norm.weight,
          "out_proj.weight": ours.out_proj.weight}
    hf.load_state_dict({k: v.detach().clone() for k, v in sd.items()}, strict=True)
    u = torch.randn(2, 21, d, dtype=DT)
    out = hf.eval()(u)
    out = out[0] if isinstance(out, tuple) else out
    torch.testing.assert_close(ours(u), out, rtol=1e-5, atol=1e-6)  # HF keeps some fp32 casts


def test_mamba1_mixer_matches_transformers_oracle():
    from transformers import MambaConfig as HFMambaConfig
    from transformers.models.mamba.modeling_mamba import MambaMixer
    from mamba_distributed_amd.models.mamba1 import Mamba
    torch.manual_seed(0)
    d = 32
    ours = Mamba(d, d_state=8).double()
    cfg = HFMambaConfig(hidden_size=d, state_size=8, expand=2, conv_kernel=4, time_step_rank=ours.dt_rank,
                        use_bias=False, use_conv_bias=True, hidden_act="silu")
    hf = MambaMixer(cfg, layer_idx=0).double()
    hf.load_state_dict({k: v.detach().clone() for k, v in ours.state_dict().items()}, strict=True)
    u = torch.randn(2, 19, d, dtype=DT)
    out = hf.eval()(u)
    out = out[0] if isinstance(out, tuple) else out
    torch.testing.assert_close(ours(u), out, rtol=1e-7, atol=1e-8)


@pytest.mark.parametrize("extra", [-1, 0, 2])
def test_conv_update_state_len_semantics(extra):
    """causal-conv1d >= 1.4 update semantics for any state_len >= w-1 (upstream Mamba / Mamba2 caches use
    state_len = d_conv): stepping token by token reproduces the full causal conv, and the state holds the
    last state_len inputs (zero-padded at the start)."""
    from mamba_distributed_amd.ops.reference import causal_conv1d_ref, causal_conv1d_update_ref
    torch.manual_seed(0)
    b, d, L, w = 2, 5, 9, 4
    sl = w + extra
    x = torch.randn(b, d, L, dtype=torch.float64)
    wt = torch.randn(d, w, dtype=torch.float64)
    bias = torch.randn(d, dtype=torch.float64)
    full = causal_conv1d_ref(x, wt, bias, "silu")
    state = torch.zeros(b, d, sl, dtype=torch.float64)
    outs = [causal_conv1d_update_ref(x[..., t], state, wt, bias, "silu") for t in range(L)]
    torch.testing.assert_close(torch.stack(outs, -1), full)
    torch.testing.assert_close(state, x[..., L - sl:])


# ------------------------------------------------------------------------------------------
# packed variable-length sequences (seq_idx) — references vs running each sequence on its own
# ------------------------------------------------------------------------------------------
def _seq_idx(lens):
    return torch.cat([torch.full((n,), i, dtype=torch.int32) for i, n in enumerate(lens)])[None]


def test_conv_ref_seq_idx_matches_separate_sequences():
    torch.manual_seed(0)
    lens = [5, 1, 9, 3]
    d, w = 6, 4
    x = torch.randn(1, d, sum(lens), dtype=torch.float64)
    wt = torch.randn(d, w, dtype=torch.float64)
    bias = torch.randn(d, dtype=torch.float64)
    init = torch.randn(1, d, w - 1, dtype=torch.float64)
    out, fin = R.causal_conv1d_ref(x, wt, bias, "silu", initial_states=init, return_final_states=True,
                                   seq_idx=_seq_idx(lens))
    parts, s = [], 0
    for i, n in enumerate(lens):
        parts.append(R.causal_conv1d_ref(x[..., s:s + n], wt, bias, "silu", initial_states=init if i == 0 else None))
        s += n
    torch.testing.assert_close(out, torch.cat(parts, -1))
    torch.testing.assert_close(fin, x[..., -(w - 1):])


@pytest.mark.parametrize("lens", [[70, 58], [64, 64, 3], [10, 1, 100, 17]])
def test_ssd_ref_seq_idx_matches_separate_sequences(lens):
    torch.manual_seed(1)
    b, h, p, g, n = 1, 4, 8, 2, 16
    L = sum(lens)
    x = torch.randn(b, L, h, p, dtype=torch.float64)
    dt = torch.randn(b, L, h, dtype=torch.float64) * 0.5
    A = -torch.rand(h, dtype=torch.float64) * 2 - 0.1
    B = torch.randn(b, L, g, n, dtype=torch.float64)
    C = torch.randn(b, L, g, n, dtype=torch.float64)
    D = torch.randn(h, dtype=torch.float64)
    init = torch.randn(b, h, p, n, dtype=torch.float64)
    sq = _seq_idx(lens)
    y, fin = R.ssd_chunked_ref(x, dt, A, B, C, 32, D=D, initial_states=init, return_final_states=True, seq_idx=sq)
    ys, fs = R.ssd_sequential_ref(x, dt, A, B, C, D=D, initial_states=init, return_final_states=True, seq_idx=sq)
    torch.testing.assert_close(y, ys)
    torch.testing.assert_close(fin, fs)
    parts, s = [], 0
    for i, m in enumerate(lens):
        yi, fi = R.ssd_sequential_ref(x[:, s:s + m], dt[:, s:s + m], A, B[:, s:s + m], C[:, s:s + m], D=D,
                                      initial_states=init if i == 0 else None, return_final_states=True)
        parts.append(yi)
        s += m
    torch.testing.assert_close(y, torch.cat(parts, 1))
    torch.testing.assert_close(fin, fi)


def test_seq_idx_from_cu_seqlens():
    from mamba_distributed_amd.models.mamba2 import seq_idx_from_cu_seqlens
    sq = seq_idx_from_cu_seqlens(torch.tensor([0, 3, 4, 9]), 9)
    assert sq.tolist() == [[0, 0, 0, 1, 2, 2, 2, 2, 2]] and sq.dtype == torch.int32
