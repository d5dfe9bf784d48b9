"""parallel/reducer.py bucket layout: the small non-matrix parameters (norm weights, conv taps, A_log / D / dt_bias) are laid
out last in buckets of their own, which the per-parameter hooks never launch -- finish() does, after the batched
late column sums wrote their gradients (ops/grad_accum.py::flush_late).  Single-rank gloo on the CPU."""
import socket

import pytest
import torch
import torch.distributed as dist

from mamba_distributed_amd import LMHeadModel, MambaConfig
from mamba_distributed_amd.parallel.reducer import GradReducer, held_param


@pytest.fixture
def gloo_world1():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("layer", ["Mamba1", "Mamba2"])
def test_small_parameters_last_and_held(gloo_world1, layer):
    torch.manual_seed(0)
    m = LMHeadModel(MambaConfig(d_model=256, n_layer=2, vocab_size=1024, ssm_cfg={"layer": layer}))
    r = GradReducer(m, bucket_cap_mb=0.5)
    params = [p for p in m.parameters() if p.requires_grad]
    small = [p for p in params if held_param(p)]  # small non-matrix parameters (Mamba-1's 2-D x_proj is not held)
    big = [p for p in params if not held_param(p)]
    assert small and big
    assert max(r._offset[id(p)] for p in big) < min(r._offset[id(p)] for p in small)
    held = r._held_from
    assert all(r._bucket_of[id(p)] >= held for p in small)
    assert all(r._bucket_of[id(p)] < held for p in big)
    # every .grad is a view of the flat buffer at its offset
    for p in params:
        assert p.grad.data_ptr() == r.flat.data_ptr() + 4 * r._offset[id(p)]
    # hooks launch every bucket up to the held ones, finish() the rest
    r.arm()
    for p in reversed(params):
        r._hook(p)
    assert r._next == held
    r.finish()
    assert r._next == len(r.buckets)
    r.remove()
