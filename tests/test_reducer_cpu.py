"""parallel/reducer.py in one process (gloo, world size 1): gradient views into the flat buffer,
zero_grad, arm/finish, and the flat-buffer clip (parallel/ddp.py::clip_grad_norm_) against torch's."""
import copy

import pytest
import torch
import torch.distributed as dist

from mamba_distributed_amd import LMHeadModel, MambaConfig
from mamba_distributed_amd.parallel import ddp as ddp_mod
from mamba_distributed_amd.parallel.reducer import wrap_reducer


@pytest.fixture
def world1(tmp_path):
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("gloo", store=store, rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def _model():
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=64, n_layer=2, vocab_size=128, ssm_cfg={"layer": "Mamba2", "headdim": 16})
    return LMHeadModel(cfg, device="cpu", enc=object())


def test_reducer_flat_views_and_clip_match_torch(world1):
    m = _model()
    ref = copy.deepcopy(m)
    dm = wrap_reducer(m, None, bucket_cap_mb=0.01)
    assert len(dm.reducer.buckets) > 2
    x = torch.randint(0, 128, (2, 32))
    y = torch.randint(0, 128, (2, 32))
    for step in range(2):
        ddp_mod.zero_grad(dm, None)
        ref.zero_grad(set_to_none=True)
        flat = dm.reducer.flat
        for p in m.parameters():  # every gradient is a view into the flat buffer
            assert p.grad.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()
        assert float(flat.abs().sum()) == 0.0
        dm.reducer.arm()
        dm(x, y)[1].backward()
        dm.reducer.finish()
        ref(x, y)[1].backward()
        n0 = torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.5)
        n1 = ddp_mod.clip_grad_norm_(dm, 0.5)
        torch.testing.assert_close(n1, n0, rtol=1e-5, atol=1e-6)
        for (k, p), q in zip(m.named_parameters(), ref.parameters()):
            torch.testing.assert_close(p.grad, q.grad, rtol=1e-5, atol=1e-7, msg=k)


def test_wgrad_inplace_policy_follows_allocator_headroom(monkeypatch):
    """ops/linear.py::_wgrad_inplace (auto): the side-stream in-place weight gradient only while the allocated
    peak is < 70% of the device and the allocator never retried; re-checked every 64 calls; env forces either
    (profiles/r3/ab15_2.8b_regression_fix.txt). The CUDA queries are faked, so this runs on CPU."""
    import types
    from mamba_distributed_amd.ops import linear
    stats = {"allocated_bytes.all.peak": 100, "num_alloc_retries": 0}
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: types.SimpleNamespace(total_memory=1000))
    monkeypatch.setattr(torch.cuda, "memory_stats", lambda i: dict(stats))
    monkeypatch.setattr(linear, "_INPLACE_STATE", {})
    monkeypatch.delenv("MAMBA_AMD_WGRAD_INPLACE", raising=False)
    dev = torch.device("cuda", 0)
    assert linear._wgrad_inplace(dev)
    stats["allocated_bytes.all.peak"] = 800       # 80% of the device: slabs, but only after the re-check
    assert all(linear._wgrad_inplace(dev) for _ in range(63))
    assert not linear._wgrad_inplace(dev)
    monkeypatch.setattr(linear, "_INPLACE_STATE", {})
    stats["allocated_bytes.all.peak"] = 100
    stats["num_alloc_retries"] = 3                # any allocator retry turns it off
    assert not linear._wgrad_inplace(dev)
    monkeypatch.setenv("MAMBA_AMD_WGRAD_INPLACE", "1")
    assert linear._wgrad_inplace(dev)
    monkeypatch.setenv("MAMBA_AMD_WGRAD_INPLACE", "0")
    stats["num_alloc_retries"] = 0
    monkeypatch.setattr(linear, "_INPLACE_STATE", {})
    assert not linear._wgrad_inplace(dev)
