"""MHA extras from upstream (mamba_ssm/modules/mha.py): the causal depthwise conv over q/k/v (d_conv) and
the gated-MLP branch sharing in_proj / out_proj (mlp_dim).  Full forward vs a direct torch composition,
and prefill + token-by-token decode vs the full forward."""
import pytest
import torch
import torch.nn.functional as F

from mamba_distributed_amd.models.layers import MHA
from mamba_distributed_amd.models.mixer_seq import InferenceParams


def _direct(m, x):
    qkv = F.linear(x, m.in_proj.weight, m.in_proj.bias)
    mlp = None
    if m.mlp_dim:
        qkv, xm = qkv.split([qkv.shape[-1] - m.mlp_dim, m.mlp_dim], -1)
        up, gate = xm.chunk(2, -1)
        mlp = up * F.silu(gate)
    if m.d_conv:
        qkv = m.conv1d(qkv.transpose(1, 2))[..., :qkv.shape[1]].transpose(1, 2)
    b, l, _ = x.shape
    hq, hk, hd = m.num_heads, m.num_heads_kv, m.head_dim
    q, k, v = torch.split(qkv, [hq * hd, hk * hd, hk * hd], -1)
    q, k, v = (t.view(b, l, -1, hd).transpose(1, 2) for t in (q, k, v))
    rep = hq // hk
    o = F.scaled_dot_product_attention(q, k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1), is_causal=True)
    o = o.transpose(1, 2).reshape(b, l, hq * hd)
    if mlp is not None:
        o = torch.cat([o, mlp], -1)
    return F.linear(o, m.out_proj.weight, m.out_proj.bias)


@pytest.mark.parametrize("d_conv,mlp_dim", [(4, 0), (0, 100), (4, 300)])
def test_mha_conv_mlp(d_conv, mlp_dim):
    torch.manual_seed(0)
    m = MHA(64, 4, num_heads_kv=2, d_conv=d_conv, mlp_dim=mlp_dim, layer_idx=0)
    assert m.mlp_dim % 256 == 0 and m.mlp_dim >= mlp_dim
    x = torch.randn(2, 20, 64)
    y = m(x)
    assert torch.allclose(y, _direct(m, x), atol=1e-5, rtol=1e-4)
    with torch.no_grad():
        p = InferenceParams(max_seqlen=32, max_batch_size=2)
        out = [m(x[:, :13], inference_params=p)]
        p.seqlen_offset = 13
        for t in range(13, 20):
            out.append(m(x[:, t:t + 1], inference_params=p))
            p.seqlen_offset += 1
    assert torch.allclose(torch.cat(out, 1), y, atol=1e-5, rtol=1e-4)


@pytest.mark.gpu
def test_mha_conv_mlp_gpu():
    """Same on the GPU under bf16 autocast (native causal conv / conv update), vs the fp32 composition."""
    torch.manual_seed(1)
    m = MHA(128, 4, num_heads_kv=2, d_conv=4, mlp_dim=256, layer_idx=0)
    x = torch.randn(2, 48, 128)
    ref = _direct(m, x)
    m, xc = m.cuda(), x.cuda()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(xc)
        with torch.no_grad():
            p = InferenceParams(max_seqlen=64, max_batch_size=2)
            p.key_value_memory_dict[0] = m.allocate_inference_cache(2, 64, dtype=torch.bfloat16)
            out = [m(xc[:, :40], inference_params=p)]
            p.seqlen_offset = 40
            for t in range(40, 48):
                out.append(m(xc[:, t:t + 1], inference_params=p))
                p.seqlen_offset += 1
    rel = lambda a, b: ((a.float().cpu() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(y, ref) < 2e-2
    assert rel(torch.cat(out, 1), ref) < 2e-2
