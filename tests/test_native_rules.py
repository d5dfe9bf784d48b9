"""Host-side launch rules of the native kernels, checked on the CPU through the extension (no GPU needed):
the SSD segment-parallel walk count (kernels/ssd.hip ssd_pick_segments)."""
import pytest

from mamba_distributed_amd.ops import _ext


@pytest.fixture
def ops():
    if not _ext.load():
        pytest.skip("extension not built")
    o = _ext.ops()
    o.ssd_segments(0, 1, 1, 1)  # automatic
    yield o
    o.ssd_segments(0, 1, 1, 1)


def test_ssd_segments_training_shapes_keep_one_walk(ops):
    # every BASELINE training shape has b * H >= 256 walks (one per CU or more): no split
    assert ops.ssd_segments(-1, 64, 24, 16) == 1     # 280M, 64 x 1024
    assert ops.ssd_segments(-1, 32, 48, 16) == 1     # 1.4B, 32 x 1024
    assert ops.ssd_segments(-1, 4, 80, 128) == 1     # 2.8B, 4 x 8192 (measured: no gain, profiles/r6/ssd_segments.txt)


def test_ssd_segments_small_batch_long_sequence(ops):
    # fewer walks than CUs: as many segments as keep <= 2 workgroups per CU and >= 4 chunks per segment (cap 16)
    assert ops.ssd_segments(-1, 1, 24, 512) == 16    # batch-1 prefill of 32k tokens
    assert ops.ssd_segments(-1, 2, 80, 128) == 3     # 160 walks: 3 segments = 480 workgroups
    assert ops.ssd_segments(-1, 1, 8, 8) == 2        # 8 chunks: >= 4 chunks per segment
    assert ops.ssd_segments(-1, 1, 8, 7) == 2        # segments of 4 + 3 chunks
    assert ops.ssd_segments(-1, 1, 8, 6) == 1        # 3-chunk segments: not split


def test_ssd_segments_override(ops):
    assert ops.ssd_segments(4, 64, 24, 16) == 4      # forced, even at a training shape
    assert ops.ssd_segments(-1, 1, 8, 3) == 3        # clamped to the chunk count
    assert ops.ssd_segments(5, 1, 8, 16) == 4        # 16 chunks in 5 segments of 4: the empty fifth is dropped
