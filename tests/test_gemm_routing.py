"""Default projection-GEMM routing (ops/linear.py::_pk_wins): the native persistent engine for every forward /
input-gradient product of every BASELINE config; hipBLASLt only under the MAMBA_AMD_PROJ_GEMM A/B switches."""
import pytest

from mamba_distributed_amd import preset
from mamba_distributed_amd.ops import linear


@pytest.fixture(autouse=True)
def _default_engine(monkeypatch):
    monkeypatch.delenv("MAMBA_AMD_PROJ_GEMM", raising=False)


def test_default_keeps_headline_shapes_native():
    T = 65536
    # Mamba-2 280M: in_proj fwd (padded), out_proj fwd, in_proj dgrad, out_proj dgrad
    assert linear._pk_wins(T, 3392, 768, "fwd")
    assert linear._pk_wins(T, 768, 1536, "fwd")
    assert linear._pk_wins(T, 768, 3392, "dgrad")
    assert linear._pk_wins(T, 1536, 768, "dgrad")


def test_default_keeps_wide_long_k_native():
    T = 32768
    # Mamba-2 1.4B and 2.8B: every projection product has K > 1024 and a >= 2048-wide output (round 5 sent these to
    # hipBLASLt; round 6 keeps them on the hand-written engine)
    for n, k, role in ((8512, 2048, "fwd"), (2048, 4096, "fwd"), (2048, 8512, "dgrad"), (4096, 2048, "dgrad"),
                       (10624, 2560, "fwd"), (2560, 5120, "fwd"), (2560, 10624, "dgrad"), (5120, 2560, "dgrad")):
        assert linear._pk_wins(T, n, k, role), (n, k, role)
    # the Mamba-1 channel-major products
    assert linear._pk_wins(8192, T, 2048, "fwd_cm")
    assert linear._pk_wins(T, 2048, 8192, "dgrad_xc")


def test_library_table_only_under_the_ab_switches(monkeypatch):
    for name in ("mamba2-280m", "mamba1-280m", "mamba2-1.4b", "mamba2-2.8b", "mamba1-370m"):
        assert not linear.library_gemms_possible(preset(name)), name
    monkeypatch.setenv("MAMBA_AMD_PROJ_GEMM", "auto")
    assert linear.library_gemms_possible(preset("mamba2-1.4b"))
    assert not linear._pk_wins(32768, 8512, 2048, "fwd")  # auto: K > 1024 -> library
    assert not linear._pk_wins(32768, 2048, 4096, "fwd")
    monkeypatch.setenv("MAMBA_AMD_PROJ_GEMM", "lib")
    assert not linear._pk_wins(65536, 3392, 768, "fwd")
    monkeypatch.setenv("MAMBA_AMD_PROJ_GEMM", "fwd_short,dgrad")
    assert linear._pk_wins(65536, 768, 3072, "dgrad_xc")  # role lists see the Mamba-1 roles as fwd / dgrad


def test_split_k_rule_fills_a_round_for_narrow_outputs():
    """launchers.h split_k_count through ops.gp_splits (host code, no GPU needed): a narrow weight gradient (the
    Mamba-1 x_proj 80 x 1536 over 65536 tokens: 6 tiles) is split until one round of 256 CUs is nearly full
    (the old cap of 16 slices left 160 CUs idle); the projection shapes keep their split counts."""
    import pytest
    from mamba_distributed_amd.ops import _ext
    if not _ext.load():
        pytest.skip("extension not built")
    ops = _ext.ops()
    s = ops.gp_splits(80, 1536, 65536)
    assert 32 <= s <= 64 and 6 * s <= 256, s
    assert ops.gp_splits(3392, 768, 65536) == 6     # Mamba-2 280M in_proj weight gradient
    assert ops.gp_splits(768, 1536, 65536) == 14    # out_proj weight gradient
    assert ops.gp_splits(8512, 2048, 32768) == 7    # 1.4B in_proj
