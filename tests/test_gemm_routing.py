"""Default projection-GEMM routing (ops/linear.py::_pk_wins "route"): native persistent engine everywhere except the
long-K products of wide Mamba-2 models, which go to hipBLASLt (measured, profiles/r5/proj_engine_routing.txt)."""
import pytest

from mamba_distributed_amd import preset
from mamba_distributed_amd.ops import linear


@pytest.fixture(autouse=True)
def _default_engine(monkeypatch):
    monkeypatch.delenv("MAMBA_AMD_PROJ_GEMM", raising=False)


def test_route_keeps_headline_shapes_native():
    T = 65536
    # Mamba-2 280M: in_proj fwd (padded), out_proj fwd, in_proj dgrad, out_proj dgrad
    assert linear._pk_wins(T, 3392, 768, "fwd")
    assert linear._pk_wins(T, 768, 1536, "fwd")
    assert linear._pk_wins(T, 768, 3392, "dgrad")
    assert linear._pk_wins(T, 1536, 768, "dgrad")


def test_route_sends_wide_long_k_to_library():
    T = 32768
    # Mamba-2 1.4B: every projection product has K > 1024 and a >= 2048-wide output
    assert not linear._pk_wins(T, 8512, 2048, "fwd")
    assert not linear._pk_wins(T, 2048, 4096, "fwd")
    assert not linear._pk_wins(T, 2048, 8512, "dgrad")
    assert not linear._pk_wins(T, 4096, 2048, "dgrad")
    # the Mamba-1 channel-major products stay native at any width
    assert linear._pk_wins(8192, T, 2048, "fwd_cm")
    assert linear._pk_wins(T, 2048, 8192, "dgrad_xc")


def test_library_table_only_where_a_library_gemm_can_run(monkeypatch):
    assert not linear.library_gemms_possible(preset("mamba2-280m"))
    assert not linear.library_gemms_possible(preset("mamba1-280m"))
    assert linear.library_gemms_possible(preset("mamba2-1.4b"))
    assert linear.library_gemms_possible(preset("mamba2-2.8b"))
    monkeypatch.setenv("MAMBA_AMD_PROJ_GEMM", "pk")
    assert not linear.library_gemms_possible(preset("mamba2-1.4b"))
    assert linear._pk_wins(32768, 8512, 2048, "fwd")
    monkeypatch.setenv("MAMBA_AMD_PROJ_GEMM", "fwd_short,dgrad")
    assert linear._pk_wins(65536, 768, 3072, "dgrad_xc")  # role lists see the Mamba-1 roles as fwd / dgrad
