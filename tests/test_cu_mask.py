"""CU-partitioned streams (utils/cu_mask.py): mask layout on CPU, a masked stream on the GPU."""
import pytest
import torch

from mamba_distributed_amd.utils.cu_mask import mask_words


@pytest.mark.parametrize("k", range(1, 9))
def test_mask_words_share_every_engine_evenly(k):
    words = mask_words(256, k)
    assert len(words) == 8
    bits = [(words[i // 32] >> (i % 32)) & 1 for i in range(256)]
    assert sum(bits) == 32 * k
    for w in range(8):  # 32 bits per XCD under one mapping
        assert sum(bits[32 * w:32 * w + 32]) == 4 * k
    for se in range(4):  # bit i -> shader engine i % 4 under the other
        assert sum(bits[se::4]) == 8 * k


def test_mask_words_ragged_and_bounds():
    assert mask_words(40, 8) == [0xffffffff, 0xff]
    with pytest.raises(ValueError):
        mask_words(256, 0)


@pytest.mark.gpu
def test_masked_stream_runs_native_kernels():
    from mamba_distributed_amd.ops import _ext
    from mamba_distributed_amd.utils.cu_mask import masked_stream
    assert _ext.load(), _ext.error()
    dev = torch.device("cuda", 0)
    s = masked_stream(0, 2)
    assert masked_stream(0, 2) is s
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn(4096, 768, device=dev, generator=g).to(torch.bfloat16)
    B = torch.randn(1024, 768, device=dev, generator=g).to(torch.bfloat16)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        C = _ext.ops().gp_mm(A, B, None, 0, 0, 0, 1, 256)
    torch.cuda.current_stream().wait_stream(s)
    ref = A.float() @ B.float().t()
    assert ((C.float() - ref).norm() / ref.norm()).item() < 8e-3
