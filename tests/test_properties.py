"""Property-based tests (Hypothesis) over random shapes, the SURVEY.md §4 'op oracles' row: sequence
lengths that are not multiples of the chunk, several chunk sizes / state sizes / group counts.

CPU: the fp64 reference ops must agree with their sequential definitions for every drawn shape.
GPU (marked): the native SSD / selective-scan / conv kernels must agree with the fp32 references at
bf16 tolerances for drawn shapes inside each kernel's supported set.
"""
import pytest
import torch
import torch.nn.functional as F
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from mamba_distributed_amd.ops import reference as R

DT = torch.float64
# derandomize: the same drawn shapes on every run (the suites run unattended every round)
CPU_SETTINGS = settings(max_examples=25, deadline=None, derandomize=True,
                        suppress_health_check=[HealthCheck.too_slow])


@CPU_SETTINGS
@given(b=st.integers(1, 2), l=st.integers(1, 70), h=st.sampled_from([1, 2, 4]), g=st.sampled_from([1, 2]),
       p=st.integers(1, 6), n=st.integers(1, 6), chunk=st.sampled_from([4, 8, 16, 64]), seed=st.integers(0, 10_000),
       with_init=st.booleans())
def test_ssd_chunked_equals_sequential_any_shape(b, l, h, g, p, n, chunk, seed, with_init):
    if h % g:
        g = 1
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(b, l, h, p, generator=gen, dtype=DT)
    dt = torch.randn(b, l, h, generator=gen, dtype=DT) * 0.5
    A = -torch.rand(h, generator=gen, dtype=DT) * 3 - 0.1
    B = torch.randn(b, l, g, n, generator=gen, dtype=DT)
    C = torch.randn(b, l, g, n, generator=gen, dtype=DT)
    D = torch.randn(h, generator=gen, dtype=DT)
    init = torch.randn(b, h, p, n, generator=gen, dtype=DT) * 0.3 if with_init else None
    y1, s1 = R.ssd_chunked_ref(x, dt, A, B, C, chunk, D=D, initial_states=init, return_final_states=True)
    y2, s2 = R.ssd_sequential_ref(x, dt, A, B, C, D=D, initial_states=init, return_final_states=True)
    torch.testing.assert_close(y1, y2, rtol=1e-8, atol=1e-8)
    torch.testing.assert_close(s1, s2, rtol=1e-8, atol=1e-8)


@CPU_SETTINGS
@given(b=st.integers(1, 2), d=st.integers(1, 6), l=st.integers(1, 60), n=st.sampled_from([1, 2, 4, 8, 16]),
       chunk=st.sampled_from([4, 16, 64]), with_z=st.booleans(), seed=st.integers(0, 10_000))
def test_selective_scan_chunked_equals_sequential_any_shape(b, d, l, n, chunk, with_z, seed):
    gen = torch.Generator().manual_seed(seed)
    u = torch.randn(b, d, l, generator=gen, dtype=DT)
    delta = torch.randn(b, d, l, generator=gen, dtype=DT) * 0.5
    A = -torch.rand(d, n, generator=gen, dtype=DT) * 2
    B = torch.randn(b, 1, n, l, generator=gen, dtype=DT)
    C = torch.randn(b, 1, n, l, generator=gen, dtype=DT)
    D = torch.randn(d, generator=gen, dtype=DT)
    z = torch.randn(b, d, l, generator=gen, dtype=DT) if with_z else None
    y1, h1 = R.selective_scan_ref(u, delta, A, B, C, D, z, None, True, return_last_state=True, chunk=chunk)
    y2, h2 = R.selective_scan_sequential_ref(u, delta, A, B, C, D, z, None, True, return_last_state=True)
    torch.testing.assert_close(y1, y2, rtol=1e-8, atol=1e-8)
    torch.testing.assert_close(h1, h2, rtol=1e-8, atol=1e-8)


@CPU_SETTINGS
@given(b=st.integers(1, 3), c=st.integers(1, 9), l=st.integers(1, 40), w=st.sampled_from([2, 3, 4]),
       silu=st.booleans(), seed=st.integers(0, 10_000))
def test_causal_conv1d_ref_equals_conv1d_any_shape(b, c, l, w, silu, seed):
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(b, c, l, generator=gen, dtype=DT)
    wt = torch.randn(c, w, generator=gen, dtype=DT)
    bias = torch.randn(c, generator=gen, dtype=DT)
    ref = F.conv1d(x, wt.unsqueeze(1), bias, padding=w - 1, groups=c)[..., :l]
    if silu:
        ref = F.silu(ref)
    out = R.causal_conv1d_ref(x, wt, bias, "silu" if silu else None)
    torch.testing.assert_close(out, ref, rtol=1e-10, atol=1e-10)


# ------------------------------------------------------------------------------------------------
# native kernels vs references on drawn shapes (GPU)
GPU_SETTINGS = settings(max_examples=8, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))


def _rel(a, b):
    """Relative L2 error, with an absolute floor: a reference that is exactly zero (e.g. dA at L = 1,
    where every h_{t-1} is 0) is matched by fp32 rounding noise, not by a relative bound."""
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-4)).item()


@pytest.mark.gpu
@GPU_SETTINGS
@given(b=st.integers(1, 2), l=st.integers(1, 300), n=st.sampled_from([4, 8, 16]), with_z=st.booleans(),
       seed=st.integers(0, 10_000))
def test_native_selective_scan_any_length(b, l, n, with_z, seed):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mamba_distributed_amd.ops.selective_scan import selective_scan_fn
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(seed)
    d = 40
    u = torch.randn(b, d, l, device=dev, generator=g).to(torch.bfloat16)
    delta = (torch.randn(b, d, l, device=dev, generator=g) * 0.5 - 1).to(torch.bfloat16)
    A = -torch.rand(d, n, device=dev, generator=g) * 4 - 0.1
    Bm = torch.randn(b, 1, n, l, device=dev, generator=g).to(torch.bfloat16)
    Cm = torch.randn(b, 1, n, l, device=dev, generator=g).to(torch.bfloat16)
    D = torch.randn(d, device=dev, generator=g)
    z = torch.randn(b, d, l, device=dev, generator=g).to(torch.bfloat16) if with_z else None
    ins = [u, delta, A, Bm, Cm, D, z]
    xn = [t.detach().clone().requires_grad_(t.is_floating_point()) if t is not None else None for t in ins]
    xr = [t.detach().clone().float().requires_grad_(True) if t is not None else None for t in ins]
    yn = selective_scan_fn(*xn[:6], z=xn[6], delta_softplus=True)
    yr = R.selective_scan_ref(*xr[:6], xr[6], None, True)
    assert _rel(yn, yr) < 2e-2
    go = torch.randn(yr.shape, device=dev, generator=g)
    yn.backward(go.to(yn.dtype))
    yr.backward(go)
    for a, r_ in zip(xn, xr):
        if a is not None and a.grad is not None:
            assert _rel(a.grad, r_.grad) < 4e-2


@pytest.mark.gpu
@GPU_SETTINGS
@given(b=st.integers(1, 2), l=st.integers(1, 300), h=st.sampled_from([2, 4]), n=st.sampled_from([64, 128]),
       seed=st.integers(0, 10_000))
def test_native_ssd_any_length(b, l, h, n, seed):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mamba_distributed_amd.ops.ssd import mamba_chunk_scan_combined
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(seed)
    p = 64
    x = torch.randn(b, l, h, p, device=dev, generator=g).to(torch.bfloat16)
    dt = (torch.randn(b, l, h, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    A = -torch.rand(h, device=dev, generator=g) * 3 - 0.1
    Bm = torch.randn(b, l, 1, n, device=dev, generator=g).to(torch.bfloat16)
    Cm = torch.randn(b, l, 1, n, device=dev, generator=g).to(torch.bfloat16)
    D = torch.randn(h, device=dev, generator=g)
    dtb = torch.randn(h, device=dev, generator=g) * 0.2
    ins = [x, dt, A, Bm, Cm]
    xn = [t.detach().clone().requires_grad_(True) for t in ins]
    xr = [t.detach().clone().float().requires_grad_(True) for t in ins]
    yn = mamba_chunk_scan_combined(*xn, 64, D=D, dt_bias=dtb, dt_softplus=True)
    yr = R.ssd_chunked_ref(*xr, 64, D=D, dt_bias=dtb)
    assert _rel(yn, yr) < 2e-2
    go = torch.randn(yr.shape, device=dev, generator=g)
    yn.backward(go.to(yn.dtype))
    yr.backward(go)
    for a, r_ in zip(xn, xr):
        assert _rel(a.grad, r_.grad) < 4e-2
