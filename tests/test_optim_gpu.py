"""Native AdamW (ops/optim.py, csrc/kernels/optim.hip) against torch.optim.AdamW (fp32 reference of the same update),
the folded gradient clip and 1/world average, the bf16 weight images it writes for the next step's GEMMs, and
state_dict round trips with torch's optimizer."""
import copy
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _params(seed=0, shapes=((96, 64), (3392, 768), (768,), (17, 5), (1, 1))):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(*s, device="cuda", generator=g)) for s in shapes]


def _grads(ps, seed):
    g = torch.Generator(device="cuda").manual_seed(1000 + seed)
    for p in ps:
        p.grad = torch.randn(p.shape, device="cuda", generator=g) * 3.0


def _groups(ps):
    return [{"params": [p for p in ps if p.dim() >= 2], "weight_decay": 0.1},
            {"params": [p for p in ps if p.dim() < 2], "weight_decay": 0.0}]


@pytest.mark.parametrize("clip", [None, 1.0, 1e6])
def test_native_adamw_matches_torch(clip):
    from mamba_distributed_amd.ops.optim import NativeAdamW
    pn, pr = _params(), _params()
    on = NativeAdamW(_groups(pn), lr=6e-4, betas=(0.9, 0.95), eps=1e-8)
    orf = torch.optim.AdamW(_groups(pr), lr=6e-4, betas=(0.9, 0.95), eps=1e-8)
    for step in range(5):
        _grads(pn, step)
        _grads(pr, step)
        for grp in on.param_groups + orf.param_groups:
            grp["lr"] = 6e-4 * (step + 1) / 5
        if clip is None:
            on.step()
            orf.step()
        else:
            nn_ = on.clip_and_step(clip)
            nr = torch.nn.utils.clip_grad_norm_(pr, clip)
            orf.step()
            assert abs(nn_.item() - nr.item()) <= 1e-5 * nr.item()
    for a, b in zip(pn, pr):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (a.shape, (a - b).abs().max().item())
    for a, b in zip(pn, pr):
        sa, sb = on.state[a], orf.state[b]
        # torch's lerp / addcmul round differently from one fma: ulp-level differences near zero
        assert torch.allclose(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-6), \
            (sa["exp_avg"] - sb["exp_avg"]).abs().max().item()
        assert torch.allclose(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-5, atol=1e-6), \
            (sa["exp_avg_sq"] - sb["exp_avg_sq"]).abs().max().item()
        assert float(sa["step"]) == float(sb["step"]) == 5.0


def test_native_adamw_nan_gradient_poisons_like_torch():
    """A NaN gradient element makes the total norm NaN; torch's clip_grad_norm_ then multiplies EVERY gradient by a
    NaN coefficient (clamp propagates it), so every parameter turns NaN after the step.  The native clip coefficient
    must propagate it the same way (a loss-spike / NaN detector relies on it), not clamp NaN to 1."""
    from mamba_distributed_amd.ops.optim import NativeAdamW
    pn, pr = _params(), _params()
    on = NativeAdamW(_groups(pn), lr=6e-4, betas=(0.9, 0.95), eps=1e-8)
    orf = torch.optim.AdamW(_groups(pr), lr=6e-4, betas=(0.9, 0.95), eps=1e-8)
    _grads(pn, 0)
    _grads(pr, 0)
    pn[0].grad[3, 5] = float("nan")
    pr[0].grad[3, 5] = float("nan")
    nn_ = on.clip_and_step(1.0)
    nr = torch.nn.utils.clip_grad_norm_(pr, 1.0)
    orf.step()
    assert math.isnan(nn_.item()) and math.isnan(nr.item())
    for a, b in zip(pn, pr):
        assert torch.isnan(b).all()
        assert torch.isnan(a).all(), (a.shape, torch.isnan(a).float().mean().item())


def test_native_adamw_fold_average():
    """Gradients summed over `world` ranks, stepped with grad_divisor = world, update exactly like averaged gradients
    (the divisor is an explicit per-call argument: the native reducer's grad_divisor, parallel/ddp.py)."""
    from mamba_distributed_amd.ops.optim import NativeAdamW
    pa, pb = _params(3), _params(3)
    oa = NativeAdamW(_groups(pa), lr=1e-3, betas=(0.9, 0.95))
    ob = NativeAdamW(_groups(pb), lr=1e-3, betas=(0.9, 0.95))
    for step in range(3):
        _grads(pa, step)
        _grads(pb, step)
        for p in pb:
            p.grad.mul_(8.0)
        na = oa.clip_and_step(1.0)
        nb = ob.clip_and_step(1.0, grad_divisor=8.0)
        assert abs(na.item() - nb.item()) <= 1e-5 * na.item()
    for a, b in zip(pa, pb):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7)


def test_native_adamw_writes_bf16_images():
    """Images the GEMMs asked for (plain cast, zero-padded rows) come out of the update as the bf16 of the new
    weights and are handed to the next scope; a manual write to the weight invalidates them."""
    from mamba_distributed_amd.ops import grad_accum
    from mamba_distributed_amd.ops.optim import NativeAdamW
    grad_accum.drop_images()
    ps = _params(5)
    w_cast, w_pad = ps[0], ps[1]
    opt = NativeAdamW(_groups(ps), lr=1e-3)
    # the ops take images inside their autograd Functions' forwards, where grad mode is off
    with grad_accum.accumulation_scope(), torch.no_grad():
        c0 = grad_accum.cached_cast(w_cast, torch.bfloat16)
        p0 = grad_accum.cached_value(w_pad, ("pad_rows", torch.bfloat16, 3456), lambda t: None)  # demand recorded
    assert c0.dtype == torch.bfloat16 and p0 is None
    _grads(ps, 0)
    opt.clip_and_step(1.0)
    with grad_accum.accumulation_scope():  # differentiable context: never an image (it would drop the gradient)
        assert grad_accum.cached_cast(w_cast, torch.bfloat16).grad_fn is not None
    with grad_accum.accumulation_scope(), torch.no_grad():
        c1 = grad_accum.cached_cast(w_cast, torch.bfloat16)
        p1 = grad_accum.cached_value(w_pad, ("pad_rows", torch.bfloat16, 3456), lambda t: None)
    assert torch.equal(c1, w_cast.detach().to(torch.bfloat16))
    assert p1.shape == (3456, 768)
    assert torch.equal(p1[:3392], w_pad.detach().to(torch.bfloat16))
    assert not p1[3392:].any()
    with torch.no_grad():
        w_cast.mul_(2.0)  # bumps the version: the image is stale
    with grad_accum.accumulation_scope(), torch.no_grad():
        c2 = grad_accum.cached_cast(w_cast, torch.bfloat16)
    assert torch.equal(c2, w_cast.detach().to(torch.bfloat16))
    grad_accum.drop_images()


def test_native_adamw_state_dict_roundtrip():
    from mamba_distributed_amd.ops.optim import NativeAdamW
    pa, pb, pc = _params(7), _params(7), _params(7)
    oa = NativeAdamW(_groups(pa), lr=1e-3, betas=(0.9, 0.95))
    for step in range(2):
        _grads(pa, step)
        oa.step()
    # native -> torch and native -> native, then one more identical step everywhere
    with torch.no_grad():
        for p, q, r in zip(pa, pb, pc):
            q.copy_(p)
            r.copy_(p)
    # deep copies, as a checkpoint file would hand over (the live state dict's tensors are views of oa's buffers)
    ot = torch.optim.AdamW(_groups(pb), lr=1e-3, betas=(0.9, 0.95))
    ot.load_state_dict(copy.deepcopy(oa.state_dict()))
    on = NativeAdamW(_groups(pc), lr=1e-3, betas=(0.9, 0.95))
    on.load_state_dict(copy.deepcopy(oa.state_dict()))
    for o, ps in ((oa, pa), (ot, pb), (on, pc)):
        _grads(ps, 9)
        o.step()
    for a, b, c in zip(pa, pb, pc):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)
        assert torch.equal(a, c)


def test_configure_optimizers_uses_native_on_gpu():
    from mamba_distributed_amd import LMHeadModel, preset
    from mamba_distributed_amd.ops.optim import NativeAdamW
    cfg = preset("mamba2-280m")
    cfg.n_layer = 2
    m = LMHeadModel(cfg, device="cuda")
    opt = m.configure_optimizers(0.1, 6e-4, "cuda", False)
    assert isinstance(opt, NativeAdamW)
    assert math.isclose(opt.param_groups[0]["weight_decay"], 0.1)
