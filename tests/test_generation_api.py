"""mamba-ssm-compatible MambaLMHeadModel.generate (utils/generation.py): greedy decoding equals an
uncached argmax loop over full forwards, plus upstream's length / eos / teacher / scores semantics and
the sampling filters."""
import pytest
import torch

from mamba_distributed_amd import preset
from mamba_distributed_amd.models.mixer_seq import MambaLMHeadModel
from mamba_distributed_amd.utils.generation import (modify_logit_for_repetition_penalty,
                                                    modify_logits_for_top_p_filtering, sample)


def _tiny(layer):
    torch.manual_seed(0)
    cfg = preset("mamba2-tiny" if layer == "Mamba2" else "mamba1-tiny", vocab_size=256)
    return MambaLMHeadModel(cfg).eval()


@pytest.mark.parametrize("layer", ["Mamba2", "Mamba1"])
def test_greedy_generate_equals_uncached_argmax(layer):
    m = _tiny(layer)
    prompt = torch.randint(0, 256, (2, 7))
    out = m.generate(prompt, max_length=15)
    assert out.shape == (2, 15) and torch.equal(out[:, :7], prompt)
    seq = prompt
    with torch.no_grad():
        for _ in range(8):
            nxt = m(seq).logits[:, -1].argmax(-1, keepdim=True)
            seq = torch.cat([seq, nxt], 1)
    assert torch.equal(out, seq)


def test_eos_teacher_scores():
    m = _tiny("Mamba2")
    prompt = torch.randint(0, 256, (1, 5))
    teacher = torch.cat([prompt, torch.tensor([[3, 4, 5, 6, 7, 8, 9, 10]])], 1)
    res = m.generate(prompt, max_length=13, teacher_outputs=teacher, return_dict_in_generate=True,
                     output_scores=True)
    assert torch.equal(res.sequences, teacher) and len(res.scores) == 8 and res.scores[0].shape == (1, 256)
    res = m.generate(prompt, max_length=13, teacher_outputs=teacher, eos_token_id=5)
    assert res.shape == (1, 8) and res[0, -1].item() == 5   # stopped at the eos token


def test_sampling_filters():
    torch.manual_seed(0)
    logits = torch.tensor([[4.0, 3.0, 2.0, -10.0, -10.0]])
    t = logits.clone()
    modify_logits_for_top_p_filtering(t, 0.9)
    assert torch.isinf(t[0, 3:]).all() and torch.isfinite(t[0, :2]).all()
    draws = torch.stack([sample(logits.clone(), top_k=2) for _ in range(200)])
    assert set(draws.flatten().tolist()) <= {0, 1}
    assert sample(logits, top_k=1).item() == 0
    pen = modify_logit_for_repetition_penalty(logits.clone(), torch.tensor([[0, 3]]), 2.0)
    assert pen[0, 0].item() == 2.0 and pen[0, 3].item() == -20.0


@pytest.mark.gpu
def test_generate_graph_matches_eager_gpu():
    """cg=True (whole-stack HIP graph of the fused decode step) generates the same tokens as cg=False."""
    torch.manual_seed(0)
    m = MambaLMHeadModel(preset("mamba2-tiny"), device="cuda", dtype=torch.bfloat16).eval()
    prompt = torch.randint(0, 50304, (2, 33), device="cuda")
    a = m.generate(prompt, max_length=64, cg=True)
    b = m.generate(prompt, max_length=64, cg=False)
    assert a.shape == (2, 64) and torch.equal(a, b)
    torch.manual_seed(5)
    s1 = m.generate(prompt, max_length=48, top_k=20, top_p=0.9, temperature=0.8, cg=True)
    torch.manual_seed(5)
    s2 = m.generate(prompt, max_length=48, top_k=20, top_p=0.9, temperature=0.8, cg=True)
    assert torch.equal(s1, s2)


@pytest.mark.parametrize("layer", ["Mamba2", "Mamba1"])
def test_layernorm_config_with_fused_add_norm(layer):
    """MambaConfig(rms_norm=False, fused_add_norm=True) (upstream: fused LayerNorm add) builds, trains and
    decodes: same prenorm math as the unfused path; cached greedy decode equals the uncached loop."""
    torch.manual_seed(0)
    cfg = preset("mamba2-tiny" if layer == "Mamba2" else "mamba1-tiny", vocab_size=256, rms_norm=False)
    assert cfg.fused_add_norm
    m = MambaLMHeadModel(cfg)
    assert isinstance(m.backbone.norm_f, torch.nn.LayerNorm)
    x = torch.randint(0, 256, (2, 16))
    m(x).logits.float().square().mean().backward()
    assert all(p.grad is not None for p in m.parameters() if p.requires_grad)
    m.eval()
    out = m.generate(x[:, :6], max_length=12)
    seq = x[:, :6]
    with torch.no_grad():
        for _ in range(6):
            seq = torch.cat([seq, m(seq).logits[:, -1].argmax(-1, keepdim=True)], 1)
    assert torch.equal(out, seq)


def test_decoder_cache_released_with_model_and_rebuilt_on_new_storage():
    """The per-model decoder cache dies with the model (no module-level strong reference), and a parameter
    storage change (dtype cast) builds a fresh decoder instead of replaying one that reads the old buffers."""
    import gc
    import weakref
    m = _tiny("Mamba2")
    prompt = torch.randint(0, 256, (1, 4))
    a = m.generate(prompt, max_length=8)
    dec0 = m._amd_decoders[(1, 8, False, prompt.device)][1]
    assert torch.equal(m.generate(prompt, max_length=8), a)
    assert m._amd_decoders[(1, 8, False, prompt.device)][1] is dec0  # reused while the storage is unchanged
    m.double()
    b = m.generate(prompt, max_length=8)
    assert m._amd_decoders[(1, 8, False, prompt.device)][1] is not dec0 and torch.equal(a, b)
    ref = weakref.ref(m)
    del m, dec0
    gc.collect()
    assert ref() is None
