import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the native HIP kernels)")
    config.addinivalue_line("markers", "slow: multi-process / longer CPU tests")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mamba_distributed_amd.ops import _ext
    assert _ext.load(), f"native extension must load on a GPU box: {_ext.error()}"
    return torch.device("cuda:0")
