"""The native reducer's deferred 1/world average as EXPLICIT state (parallel/reducer.py ``grad_divisor``,
parallel/ddp.py ``configure_grad_average`` / ``averaged_grads`` / ``clip_and_step``), two gloo ranks on the CPU
against a single-process run of the same global batch: the gradients a torch optimizer, a logged norm and the clip
see are the AVERAGE on every step, whether the reducer deferred the division or not (reference
train.py:221-227).  The native AdamW's own division (clip_and_step(grad_divisor=world)) is covered on the GPU by
tests/test_optim_gpu.py::test_native_adamw_fold_average and the two-ranks-one-GPU run of tests/reducer_worker.py."""
import copy
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _model():
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=64, n_layer=2, vocab_size=128, ssm_cfg={"layer": "Mamba2", "headdim": 16})
    return LMHeadModel(cfg, device="cpu", enc=object())


def _worker(rank, world, path, out_q):
    try:
        from mamba_distributed_amd.parallel import ddp as ddp_mod
        from mamba_distributed_amd.parallel.api import grad_norm
        from mamba_distributed_amd.parallel.reducer import wrap_reducer
        dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
        m = _model()
        ref = copy.deepcopy(m)
        dm = wrap_reducer(m, None, bucket_cap_mb=0.01)
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
        ropt = torch.optim.AdamW(ref.parameters(), lr=1e-3)
        # a torch optimizer never defers; force the deferral to exercise every consumer of the summed state
        assert not ddp_mod.configure_grad_average(dm, opt)
        dm.reducer.defer_average = True
        g = torch.Generator().manual_seed(1)
        data = [(torch.randint(0, 128, (2, 32), generator=g), torch.randint(0, 128, (2, 32), generator=g))
                for _ in range(world)]
        for step in range(3):
            ddp_mod.zero_grad(dm, opt)
            assert dm.reducer.grad_divisor == 1.0
            dm.reducer.arm()
            x, y = data[rank]
            dm(x, y)[1].backward()
            dm.reducer.finish()
            assert dm.reducer.grad_divisor == float(world)  # .grad holds the SUM now
            ref.zero_grad(set_to_none=True)
            for xx, yy in data:
                (ref(xx, yy)[1] / world).backward()
            nr = torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.5)
            ropt.step()
            if step == 1:
                ln = grad_norm(dm)  # a logged norm: materialises the average
                assert dm.reducer.grad_divisor == 1.0
                torch.testing.assert_close(ln, nr, rtol=1e-5, atol=1e-6)
            nd = ddp_mod.clip_and_step(dm, opt, 0.5)  # torch optimizer: clip_grad_norm_ materialises first
            torch.testing.assert_close(nd, nr, rtol=1e-5, atol=1e-6)
            for (k, p), q in zip(m.named_parameters(), ref.parameters()):
                torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6, msg=f"step {step} {k}")
        dist.destroy_process_group()
        out_q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported by the parent
        import traceback
        out_q.put((rank, traceback.format_exc()))


def test_deferred_average_is_explicit_two_ranks(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = str(tmp_path / "rdv")
    ps = [ctx.Process(target=_worker, args=(r, 2, path, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    bad = [r for r in res if r[1] != "ok"]
    assert not bad, bad


def test_held_buckets_only_late_parameters():
    """Only the small non-matrix parameters (norm weights, conv taps / bias, A_log / D / dt_bias) are held until
    finish(); small 2-D weights launch from the hooks; grad_accum.late_ok refuses everything else."""
    from mamba_distributed_amd import LMHeadModel, MambaConfig
    from mamba_distributed_amd.parallel.reducer import held_param
    cfg = MambaConfig(d_model=64, n_layer=1, vocab_size=128, ssm_cfg={"layer": "Mamba1"})
    m = LMHeadModel(cfg, device="cpu", enc=object())
    names = {n: held_param(p) for n, p in m.named_parameters()}
    # Mamba-1's small 2-D weights (x_proj, dt_proj, and A_log (d_inner, d_state)) come out of the backward itself
    for n in ("x_proj.weight", "dt_proj.weight", "A_log"):
        assert not names["backbone.layers.0.mixer." + n], n
    for n in ("backbone.layers.0.mixer.D", "backbone.layers.0.mixer.conv1d.weight", "backbone.layers.0.norm.weight"):
        assert names[n], n
    big = torch.nn.Parameter(torch.zeros(1 << 17))
    assert not held_param(big)
