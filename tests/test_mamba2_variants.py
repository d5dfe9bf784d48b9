"""Upstream Mamba2 variants (mamba_ssm/modules/mamba2.py): rmsnorm=False (gate only), D_has_hdim
(per-channel skip), d_ssm < d_inner (gated-MLP branch beside the SSM).  Checked against an explicit
sequential fp64 recurrence of the same parameters, for the training forward, the gradients' existence,
and the cached decode (prefill + token steps == full forward)."""
import pytest
import torch
import torch.nn.functional as F

from mamba_distributed_amd.models.mamba2 import Mamba2

VARIANTS = [dict(rmsnorm=False), dict(D_has_hdim=True), dict(d_ssm=64), dict(rmsnorm=False, D_has_hdim=True, d_ssm=64)]


def _oracle(m, u):
    """Sequential recurrence in fp64 (the definition, no chunking)."""
    b, l, _ = u.shape
    zx = F.linear(u.double(), m.in_proj.weight.double())
    di, gn, H, P, N, G = m.d_ssm, m.ngroups * m.d_state, m.nheads, m.headdim, m.d_state, m.ngroups
    z0, x0, z, xBC, dt = torch.split(zx, [m.d_mlp, m.d_mlp, di, di + 2 * gn, H], dim=-1)
    w = m.conv1d.weight.double().squeeze(1)
    xt = F.pad(xBC.transpose(1, 2), (w.shape[1] - 1, 0))
    conv = torch.stack([(xt[..., t:t + w.shape[1]] * w).sum(-1) for t in range(l)], -1) + m.conv1d.bias.double()[:, None]
    xBC = F.silu(conv).transpose(1, 2)
    x, B, C = torch.split(xBC, [di, gn, gn], dim=-1)
    x = x.view(b, l, H, P)
    B = B.view(b, l, G, N).repeat_interleave(H // G, 2)
    C = C.view(b, l, G, N).repeat_interleave(H // G, 2)
    dt = F.softplus(dt + m.dt_bias.double())
    A = -torch.exp(m.A_log.double())
    S = torch.zeros(b, H, P, N, dtype=torch.float64)
    ys = []
    for t in range(l):
        S = S * torch.exp(dt[:, t] * A)[:, :, None, None] + (dt[:, t, :, None] * x[:, t])[..., None] * B[:, t, :, None, :]
        ys.append((S * C[:, t, :, None, :]).sum(-1))
    y = torch.stack(ys, 1)
    Dd = m.D.double()
    y = y + x * (Dd.view(H, P) if m.D_has_hdim else Dd[:, None])
    y = y.reshape(b, l, di)
    if m.rmsnorm:
        g = y * F.silu(z)
        y = g * torch.rsqrt(g.square().mean(-1, keepdim=True) + m.norm.eps) * m.norm.weight.double()
    else:
        y = y * F.silu(z)
    if m.d_mlp > 0:
        y = torch.cat([F.silu(z0) * x0, y], -1)
    return F.linear(y, m.out_proj.weight.double())


@pytest.mark.parametrize("kw", VARIANTS)
def test_variant_forward_matches_recurrence(kw):
    torch.manual_seed(0)
    m = Mamba2(64, d_state=16, headdim=16, expand=2, chunk_size=64, layer_idx=0, **kw)
    with torch.no_grad():
        m.D.uniform_(0.5, 1.5)
        if m.rmsnorm:
            m.norm.weight.uniform_(0.5, 1.5)
    assert m._general and (m.d_mlp > 0) == ("d_ssm" in kw)
    if not kw.get("rmsnorm", True):
        assert not hasattr(m, "norm")
    u = torch.randn(2, 40, 64)
    y = m(u)
    ref = _oracle(m, u)
    assert ((y.double() - ref).norm() / ref.norm()).item() < 1e-4
    y.square().mean().backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


@pytest.mark.parametrize("kw", VARIANTS)
def test_variant_cached_decode_matches_forward(kw):
    from mamba_distributed_amd.models.mixer_seq import InferenceParams
    torch.manual_seed(1)
    m = Mamba2(64, d_state=16, headdim=16, expand=2, chunk_size=64, layer_idx=0, **kw)
    u = torch.randn(2, 24, 64)
    with torch.no_grad():
        full = m(u)
        params = InferenceParams(max_seqlen=32, max_batch_size=2)
        out = [m(u[:, :16], inference_params=params)]
        params.seqlen_offset = 16
        for t in range(16, 24):
            out.append(m(u[:, t:t + 1], inference_params=params))
            params.seqlen_offset += 1
    got = torch.cat(out, 1)
    assert ((got - full).norm() / full.norm()).item() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("kw", VARIANTS)
def test_variant_native_gpu(kw):
    """The same variants through the native HIP ops (bf16 autocast) vs the fp64 recurrence, forward,
    backward and cached decode."""
    from mamba_distributed_amd.models.mixer_seq import InferenceParams
    from mamba_distributed_amd.ops import _ext
    assert _ext.load(), _ext.error()
    torch.manual_seed(2)
    m = Mamba2(256, d_state=64, headdim=64, expand=2, chunk_size=64, layer_idx=0, **kw)
    with torch.no_grad():
        m.D.uniform_(0.5, 1.5)
    u = torch.randn(2, 200, 256)
    ref = _oracle(m, u)
    m = m.cuda()
    uc = u.cuda()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(uc)
    assert ((y.double().cpu() - ref).norm() / ref.norm()).item() < 3e-2
    y.float().square().mean().backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        params = InferenceParams(max_seqlen=256, max_batch_size=2)
        params.key_value_memory_dict[0] = m.allocate_inference_cache(2, 256, dtype=torch.bfloat16)  # as generate()
        out = [m(uc[:, :192], inference_params=params)]
        params.seqlen_offset = 192
        for t in range(192, 200):
            out.append(m(uc[:, t:t + 1], inference_params=params))
            params.seqlen_offset += 1
    got = torch.cat(out, 1).double().cpu()
    assert ((got - ref).norm() / ref.norm()).item() < 3e-2


@pytest.mark.parametrize("form", ["default", "no_norm", "hdim_D", "hdim_D_no_norm"])
def test_split_conv1d_scan_combined_forms(form):
    """Upstream's mamba_split_conv1d_scan_combined forms (D11): the functional entry point equals the
    Mamba2 module with the matching options (whose forward is checked against the fp64 recurrence)."""
    from mamba_distributed_amd.ops.ssd import mamba_split_conv1d_scan_combined
    torch.manual_seed(3)
    kw = dict(rmsnorm="no_norm" not in form, D_has_hdim="hdim" in form)
    m = Mamba2(64, d_state=16, headdim=16, expand=2, chunk_size=64, layer_idx=0, **kw)
    with torch.no_grad():
        m.D.uniform_(0.5, 1.5)
    u = torch.randn(2, 40, 64)
    zxbcdt = F.linear(u, m.in_proj.weight)
    D = m.D.view(m.nheads, m.headdim) if m.D_has_hdim else m.D
    y = mamba_split_conv1d_scan_combined(
        zxbcdt, m.conv1d.weight.squeeze(1), m.conv1d.bias, m.dt_bias, -torch.exp(m.A_log), D, 64,
        rmsnorm_weight=m.norm.weight if m.rmsnorm else None, rmsnorm_eps=1e-5, outproj_weight=m.out_proj.weight,
        headdim=m.headdim, ngroups=m.ngroups, norm_before_gate=False)
    ref = _oracle(m, u)
    assert ((y.double() - ref).norm() / ref.norm()).item() < 1e-4


@pytest.mark.gpu
def test_chunk_scan_hdim_D_and_z_native(cuda):
    """mamba_chunk_scan_combined with D of shape (h, p) and z: native scan + elementwise skip/gate on the
    GPU vs the fp32 chunked reference."""
    from mamba_distributed_amd.ops import reference as R
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    g = torch.Generator(device=cuda).manual_seed(4)
    b, l, h, p, n = 2, 192, 4, 64, 64
    rnd = lambda *s: torch.randn(*s, device=cuda, generator=g)  # noqa: E731
    x, z = rnd(b, l, h, p).bfloat16(), rnd(b, l, h, p).bfloat16()
    dt = (rnd(b, l, h) * 0.5 - 1).bfloat16()
    A = -torch.rand(h, device=cuda, generator=g) * 4 - 0.5
    B, C = rnd(b, l, 1, n).bfloat16(), rnd(b, l, 1, n).bfloat16()
    D, dt_bias = rnd(h, p), rnd(h) * 0.1
    y = mamba_chunk_scan_combined(x, dt, A, B, C, 64, D=D, z=z, dt_bias=dt_bias, dt_softplus=True)
    ref = R.ssd_chunked_ref(x, dt, A, B, C, 64, D=D, z=z, dt_bias=dt_bias, dt_softplus=True)
    assert ((y.float() - ref.float()).norm() / ref.float().norm()).item() < 2e-2
