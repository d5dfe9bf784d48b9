"""Model/param contract (SURVEY.md §2.8, §4 'Module/model'): counts, keys, init, optimizer groups."""
import math

import pytest
import torch

from mamba_distributed_amd import LMHeadModel, MambaConfig, preset


def meta_model(cfg):
    with torch.device("meta"):
        return LMHeadModel(cfg, device="meta", enc=object())


def test_param_counts_match_reference():
    m1 = meta_model(MambaConfig(d_model=768, vocab_size=50304))
    assert sum(p.numel() for p in m1.parameters()) == 280_019_712   # reference prints "280M"
    m2 = meta_model(MambaConfig(d_model=768, vocab_size=50304, ssm_cfg={"layer": "Mamba2"}))
    assert sum(p.numel() for p in m2.parameters()) == 279_614_720


def test_state_dict_keys_and_shapes():
    sd = meta_model(MambaConfig(d_model=768, vocab_size=50304)).state_dict()
    assert sd["backbone.embedding.weight"].shape == (50304, 768)
    assert sd["lm_head.weight"].shape == (50304, 768)
    assert sd["backbone.norm_f.weight"].shape == (768,)
    L0 = "backbone.layers.0."
    exp = {"norm.weight": (768,), "mixer.in_proj.weight": (3072, 768), "mixer.conv1d.weight": (1536, 1, 4),
           "mixer.conv1d.bias": (1536,), "mixer.x_proj.weight": (80, 1536), "mixer.dt_proj.weight": (1536, 48),
           "mixer.dt_proj.bias": (1536,), "mixer.A_log": (1536, 16), "mixer.D": (1536,),
           "mixer.out_proj.weight": (768, 1536)}
    for k, s in exp.items():
        assert tuple(sd[L0 + k].shape) == s, k
    assert len([k for k in sd if k.startswith(L0)]) == len(exp)
    sd2 = meta_model(MambaConfig(d_model=768, vocab_size=50304, ssm_cfg={"layer": "Mamba2"})).state_dict()
    exp2 = {"norm.weight": (768,), "mixer.in_proj.weight": (3352, 768), "mixer.conv1d.weight": (1792, 1, 4),
            "mixer.conv1d.bias": (1792,), "mixer.dt_bias": (24,), "mixer.A_log": (24,), "mixer.D": (24,),
            "mixer.norm.weight": (1536,), "mixer.out_proj.weight": (768, 1536)}
    for k, s in exp2.items():
        assert tuple(sd2[L0 + k].shape) == s, k
    assert len([k for k in sd2 if k.startswith(L0)]) == len(exp2)
    assert sum(1 for k in sd2 if k.startswith("backbone.layers.") and k.endswith("norm.weight")
               and "mixer" not in k) == 64


def test_optimizer_groups_match_reference(capsys):
    m1 = meta_model(MambaConfig(d_model=768, vocab_size=50304))
    opt = m1.configure_optimizers(0.1, 6e-4, "cpu", True)
    out = capsys.readouterr().out
    assert "num decayed parameter tensors: 385, with 279,674,880 parameters" in out
    assert "num non-decayed parameter tensors: 257, with 344,832 parameters" in out
    assert opt.param_groups[0]["weight_decay"] == 0.1 and opt.param_groups[1]["weight_decay"] == 0.0
    m2 = meta_model(MambaConfig(d_model=768, vocab_size=50304, ssm_cfg={"layer": "Mamba2"}))
    m2.configure_optimizers(0.1, 6e-4, "cpu", True)
    out = capsys.readouterr().out
    assert "num decayed parameter tensors: 193" in out and "num non-decayed parameter tensors: 385" in out


@pytest.mark.parametrize("name", ["mamba1-tiny", "mamba2-tiny"])
def test_init_and_loss_at_init(name):
    torch.manual_seed(0)
    m = LMHeadModel(preset(name), device="cpu")
    assert m.lm_head.weight is m.backbone.embedding.weight
    assert abs(m.backbone.embedding.weight.std().item() - 0.02) < 2e-3
    mix = m.backbone.layers[0].mixer
    if name.startswith("mamba2"):
        dt = torch.nn.functional.softplus(mix.dt_bias)
        assert dt.min() >= 1e-4 - 1e-7 and dt.max() <= 0.1 + 1e-6
        A = torch.exp(mix.A_log)
        assert A.min() >= 1 and A.max() <= 16
    else:
        dt = torch.nn.functional.softplus(mix.dt_proj.bias)
        assert dt.min() >= 1e-4 - 1e-7 and dt.max() <= 0.1 + 1e-6
        assert torch.allclose(torch.exp(mix.A_log[0]), torch.arange(1, 17, dtype=torch.float32))
    # out_proj rescaled by 1/sqrt(n_layer): kaiming-uniform bound / sqrt(2)
    fan_in = mix.out_proj.weight.shape[1]
    bound = 1 / math.sqrt(fan_in) / math.sqrt(2)
    assert mix.out_proj.weight.abs().max() <= bound + 1e-6
    x = torch.randint(0, 50304, (2, 64))
    y = torch.randint(0, 50304, (2, 64))
    _, loss = m(x, y)
    assert abs(loss.item() - math.log(50304)) < 0.3   # reference log line 1: 10.9911


def test_hybrid_config_builds_and_runs():
    cfg = MambaConfig(d_model=128, n_layer=3, vocab_size=512, d_intermediate=256, attn_layer_idx=[1],
                      attn_cfg={"num_heads": 4, "rotary_emb_dim": 16}, ssm_cfg={"layer": "Mamba2", "headdim": 32,
                                                                                "d_state": 32})
    m = LMHeadModel(cfg, device="cpu", enc=object())
    x = torch.randint(0, 512, (2, 40))
    logits, loss = m(x, x)
    loss.backward()
    assert logits.shape == (2, 40, 512)
    assert m.backbone.layers[1].mixer.__class__.__name__ == "MHA"


@pytest.mark.parametrize("every", [1, 2])
def test_activation_checkpointing_same_loss_and_grads(every):
    """MambaLMHeadModel.set_activation_checkpointing: recomputing blocks in the backward leaves the
    loss and every gradient unchanged (reference ops, fp32)."""
    import copy
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=64, n_layer=3, vocab_size=128, ssm_cfg={"layer": "Mamba2", "headdim": 16})
    m0 = LMHeadModel(cfg, device="cpu", enc=object())
    m1 = copy.deepcopy(m0)
    m1.set_activation_checkpointing(every)
    x = torch.randint(0, 128, (2, 40))
    y = torch.randint(0, 128, (2, 40))
    l0 = m0(x, y)[1]
    l1 = m1(x, y)[1]
    l0.backward()
    l1.backward()
    torch.testing.assert_close(l1, l0, rtol=0, atol=0)
    for (k, p), q in zip(m1.named_parameters(), m0.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-6, atol=1e-7, msg=k)
