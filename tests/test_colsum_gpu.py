"""Column sums of per-workgroup partial rows (csrc/kernels/norm.hip launch_colsum: split rows, then the split sums,
or one pass for short blocks), the reduction behind every norm / conv / SSD parameter gradient: against an fp64 sum,
bitwise run-to-run, and over many launches."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def ops():
    from mamba_distributed_amd.ops import _ext
    assert _ext.load(), _ext.error()
    return _ext.ops()


SHAPES = [(2048, 768), (512, 8960), (1024, 72), (40, 100), (4097, 1536), (300, 65)]


@pytest.mark.parametrize("rows,cols", SHAPES)
def test_colsum_matches_fp64_and_is_deterministic(ops, rows, cols):
    g = torch.Generator(device="cuda").manual_seed(rows * 7 + cols)
    part = torch.randn(rows, cols, device="cuda", generator=g)
    ref = part.double().sum(0)
    outs = [ops.colsum(part.clone()) for _ in range(3)]
    scale = part.double().abs().sum(0).clamp_min(1e-30)
    assert ((outs[0].double() - ref).abs() / scale).max().item() < 1e-6
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


def test_colsum_many_launches(ops):
    """Hundreds of launches in a row: every result identical (fixed-order reductions, no shared state)."""
    part = torch.randn(2048, 768, device="cuda")
    first = ops.colsum(part.clone())
    bad = 0
    for _ in range(200):
        bad += int(not torch.equal(ops.colsum(part.clone()), first))
    assert bad == 0

