"""Pipelined MFMA GEMM engine (csrc/kernels/gemm_pipe.hip) vs an fp32 torch reference.

Covers every operand layout the projections use (forward KC.KC, dgrad KC.XC, wgrad XC.XC), the bf16 /
fp32 / fp32-accumulate epilogues, K splits with the fixed-order reduction, ragged M / N / K tails
(zero-page DMA for k >= K, clamped rows), row-strided views, and the headline Mamba-2 280M shapes.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from mamba_distributed_amd.ops import _ext
    assert _ext.load(), _ext.error()
    return _ext.ops()


def _ref(A, B, la, lb):
    a = A.float() if la == 0 else A.float().t()
    b = B.float() if lb == 0 else B.float().t()
    return a @ b.t()


def _mk(rows, K, lay, dev, g):
    t = torch.randn(rows, K, device=dev, generator=g).to(torch.bfloat16)
    return t if lay == 0 else t.t().contiguous()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 1), (1, 0)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 768), (300, 264, 200), (1000, 3352, 96),
                                   (768, 520, 1544), (64, 8, 32), (512, 256, 1024)])
def test_gp_bf16(cuda, la, lb, M, N, K):
    if la == 1 and (M % 8):
        pytest.skip("XC A needs M % 8 == 0")
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(M * 7 + N * 3 + K)
    A, B = _mk(M, K, la, cuda, g), _mk(N, K, lb, cuda, g)
    C = ops.gp_mm(A, B, None, la, lb, 0, 1, 256)
    ref = _ref(A, B, la, lb)
    assert C.shape == (M, N) and C.dtype == torch.bfloat16
    assert torch.isfinite(C.float()).all()
    assert _rel(C, ref) < 8e-3, _rel(C, ref)


@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 1)])
def test_gp_fp32_modes_and_splits(cuda, la, lb):
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(1)
    M, N, K = 520, 776, 4160
    A, B = _mk(M, K, la, cuda, g), _mk(N, K, lb, cuda, g)
    ref = _ref(A, B, la, lb)
    C = ops.gp_mm(A, B, None, la, lb, 1, 1, 256)
    assert C.dtype == torch.float32 and C.shape == (1, M, N) and _rel(C[0], ref) < 1e-5
    acc = torch.randn(M, N, device=cuda, generator=g)
    acc0 = acc.clone()
    ops.gp_mm(A, B, acc, la, lb, 2, 1, 256)
    assert _rel(acc, acc0 + ref) < 1e-5
    for S in (2, 3, 7):
        part = ops.gp_mm(A, B, None, la, lb, 1, S, 256)
        assert part.shape == (S, M, N)
        out = torch.full((M, N), 0.5, device=cuda)
        ops.gp_reduce(part, out, True)
        assert _rel(out, ref + 0.5) < 1e-5, (S, _rel(out, ref + 0.5))
        # deterministic: identical bits on a second run
        part2 = ops.gp_mm(A, B, None, la, lb, 1, S, 256)
        assert torch.equal(part, part2)


def test_gp_xc_ragged_k(cuda):
    """Weight-gradient layout (both operands token-major) with a token count that is not a multiple of 8."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(4)
    for T in (318, 1, 65):
        A, B = _mk(264, T, 1, cuda, g), _mk(136, T, 1, cuda, g)
        part = ops.gp_mm(A, B, None, 1, 1, 1, 1, 256)
        out = torch.zeros(264, 136, device=cuda)
        ops.gp_reduce(part, out, False)
        assert _rel(out, _ref(A, B, 1, 1)) < 1e-5, T


def test_gp_strided_views(cuda):
    """A as a column slice of a wider buffer, C written into a column slice (row-strided views)."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(2)
    big = torch.randn(640, 1000, device=cuda, generator=g).to(torch.bfloat16)
    A = big[:, 8:8 + 768]
    W = torch.randn(264, 768, device=cuda, generator=g).to(torch.bfloat16)
    outbig = torch.zeros(640, 400, device=cuda, dtype=torch.bfloat16)
    C = outbig[:, 64:64 + 264]
    ops.gp_mm(A, W, C, 0, 0, 0, 1, 256)
    assert _rel(C, A.float() @ W.float().t()) < 8e-3
    assert (outbig[:, :64] == 0).all() and (outbig[:, 64 + 264:] == 0).all()


@pytest.mark.parametrize("which", ["in_fwd", "in_dgrad", "in_wgrad", "out_fwd", "out_dgrad", "out_wgrad"])
def test_gp_headline_shapes(cuda, which):
    """Mamba-2 280M projections at the bench micro-batch (32 x 1024 tokens), vs fp32."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(3)
    T, d, dp, di = 32768, 768, 3352, 1536
    rnd = lambda *s: (torch.randn(*s, device=cuda, generator=g) * 0.5).to(torch.bfloat16)  # noqa: E731
    if which == "in_fwd":
        A, B, la, lb = rnd(T, d), rnd(dp, d), 0, 0
    elif which == "in_dgrad":
        A, B, la, lb = rnd(T, dp), rnd(dp, d), 0, 1
    elif which == "out_fwd":
        A, B, la, lb = rnd(T, di), rnd(d, di), 0, 0
    elif which == "out_dgrad":
        A, B, la, lb = rnd(T, d), rnd(d, di), 0, 1
    elif which == "in_wgrad":
        A, B, la, lb = rnd(T, dp), rnd(T, d), 1, 1
    else:
        A, B, la, lb = rnd(T, d), rnd(T, di), 1, 1
    ref = _ref(A, B, la, lb)
    if which.endswith("wgrad"):
        M, N = ref.shape
        S = ops.gp_splits(M, N, T)
        part = ops.gp_mm(A, B, None, la, lb, 1, S, 256)
        out = torch.zeros(M, N, device=cuda)
        ops.gp_reduce(part, out, False)
        assert _rel(out, ref) < 1e-5
    else:
        C = ops.gp_mm(A, B, None, la, lb, 0, 1, 256)
        assert _rel(C, ref) < 8e-3


# ---- persistent engine (gp_pk: KC . KC, bf16 out, optional row scale) --------------------------------------
def _pmm(ops, eng, A, B, rs=None):
    return ops.gp_pk(A, B, None, 0, 0, 0, rs)


@pytest.mark.parametrize("eng", ["pk"])
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (512, 768, 768), (300, 264, 200), (1000, 3352, 776),
                                   (768, 520, 1544), (64, 8, 256), (4096, 392, 3352), (2048, 1000, 320),
                                   (70000, 136, 448)])
def test_gp_pk_bf16(cuda, eng, M, N, K):
    """Persistent tile walk: ragged M / N (rows past the descriptor read as zeros, stores into the sink),
    K tails (out-of-range offsets), more tiles than CUs (several tiles per workgroup), fewer tiles than CUs."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(M * 5 + N * 3 + K)
    A, B = _mk(M, K, 0, cuda, g), _mk(N, K, 0, cuda, g)
    C = _pmm(ops, eng, A, B)
    ref = _ref(A, B, 0, 0)
    assert C.shape == (M, N) and C.dtype == torch.bfloat16
    assert _rel(C, ref) < 8e-3, _rel(C, ref)
    assert torch.equal(C, _pmm(ops, eng, A, B)) and torch.isfinite(C.float()).all()
    rs = torch.rand(M, device=cuda, generator=g) + 0.5
    Cs = _pmm(ops, eng, A, B, rs)
    assert _rel(Cs, ref * rs[:, None]) < 8e-3
    # deterministic across launches, and every row / column written (no stale parked tile)
    assert torch.equal(C, _pmm(ops, eng, A, B))
    assert torch.isfinite(C.float()).all()


@pytest.mark.parametrize("eng", ["pk"])
def test_gp_pk_strided_out_and_unsupported(cuda, eng):
    """C written into a column slice of a wider buffer (neighbours untouched); K <= 192 is refused."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(9)
    A = torch.randn(640, 768, device=cuda, generator=g).to(torch.bfloat16)
    W = torch.randn(264, 768, device=cuda, generator=g).to(torch.bfloat16)
    outbig = torch.zeros(640, 400, device=cuda, dtype=torch.bfloat16)
    C = outbig[:, 64:64 + 264]
    ops.gp_pk(A, W, C)
    assert _rel(C, A.float() @ W.float().t()) < 8e-3
    assert (outbig[:, :64] == 0).all() and (outbig[:, 64 + 264:] == 0).all()
    with pytest.raises(RuntimeError):
        _pmm(ops, eng, A[:, :128], W[:, :128])


@pytest.mark.parametrize("eng", ["pk"])
@pytest.mark.parametrize("which", ["in_fwd", "in_dgrad", "out_fwd", "out_dgrad", "lm_fwd", "lm_dgrad"])
def test_gp_pk_headline_shapes(cuda, eng, which):
    """The persistent engine at the Mamba-2 280M bench micro-batch (32 x 1024 tokens), input gradients through
    the transposed weight (KC . KC), vs fp32.  The d_model-wide outputs (in_dgrad, out_fwd, lm_dgrad) take the
    256 x 192 tiles."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(3)
    T, d, dp, di = 32768, 768, 3352, 1536
    rnd = lambda *s: (torch.randn(*s, device=cuda, generator=g) * 0.5).to(torch.bfloat16)  # noqa: E731
    A, B = {"in_fwd": lambda: (rnd(T, d), rnd(dp, d)), "in_dgrad": lambda: (rnd(T, dp), rnd(d, dp)),
            "out_fwd": lambda: (rnd(T, di), rnd(d, di)), "out_dgrad": lambda: (rnd(T, d), rnd(di, d)),
            "lm_fwd": lambda: (rnd(8192, d), rnd(50304, d)), "lm_dgrad": lambda: (rnd(4096, 50304), rnd(d, 50304))}[which]()
    C = _pmm(ops, eng, A, B)
    assert _rel(C, A.float() @ B.float().t()) < 8e-3


def test_gp_pk_concurrent_streams(cuda):
    """Tile claims are per launch: many back-to-back launches on two streams (as under the micro-batch overlap)
    each produce the exact single-launch result."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(11)
    A1, B1 = _mk(4096, 768, 0, cuda, g), _mk(3352, 768, 0, cuda, g)
    A2, B2 = _mk(8192, 1536, 0, cuda, g), _mk(768, 1536, 0, cuda, g)
    r1, r2 = ops.gp_pk(A1, B1), ops.gp_pk(A2, B2)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for _ in range(20):
        with torch.cuda.stream(s1):
            o1 = ops.gp_pk(A1, B1)
        with torch.cuda.stream(s2):
            o2 = ops.gp_pk(A2, B2)
        outs.append((o1, o2))
    torch.cuda.synchronize()
    for o1, o2 in outs:
        assert torch.equal(o1, r1) and torch.equal(o2, r2)


@pytest.mark.parametrize("la,M", [(0, 80), (1, 48), (0, 128), (1, 120)])
def test_gp_narrow_128_row_tiles(cuda, la, M):
    """The split-K engine's 128-row tile form (gemm_pipe_k, MI = 4; bm=128): the Mamba-1 narrow long-K products
    x_dbl = W_x conv_out (KC weight, 80 rows) and d x_dbl[:R] = W_dt^T ddelta (the XC view of W_dt, 48 rows),
    channel-major B, bf16 out, written into a row slice of a wider buffer as in the mixer."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(M + 7 * la)
    K, N = 1536, 8192 + 64
    A = _mk(M, K, la, cuda, g)                     # la 1: stored (K, M), rows contiguous
    B = _mk(N, K, 1, cuda, g)                      # stored (K, N): channel-major activation
    out = torch.zeros(M + 32, N, device=cuda, dtype=torch.bfloat16)
    C = ops.gp_mm(A, B, out[:M], la, 1, 0, 1, 128)
    ref = _ref(A, B, la, 1)
    assert _rel(C, ref) < 8e-3, _rel(C, ref)
    assert (out[M:] == 0).all()
    assert torch.equal(C, ops.gp_mm(A, B, None, la, 1, 0, 1, 256))  # same K order as the 256-row tiles


# ---- split-K weight-gradient engine (gemm_wg_k: XC . XC, fp32 slabs, 32-deep stages in an NB-slot ring) -------
@pytest.fixture
def wg_engine():
    ops = _ops()
    old = ops.gp_wg_nb(-1)
    yield ops
    ops.gp_wg_nb(old)


@pytest.mark.parametrize("nb", [4, 5])
@pytest.mark.parametrize("M,N,T", [(264, 136, 318), (256, 256, 32), (520, 776, 4160), (3352, 768, 9000),
                                   (8, 8, 1), (776, 1536, 65)])
def test_gp_wg_engine(cuda, wg_engine, nb, M, N, T):
    """Ragged rows / columns / token counts (stages past K read zeros through the buffer descriptor), every split
    count the slab layout takes, fp32 store and += epilogues, bitwise determinism, and bitwise agreement with the
    gemm_pipe_k engine it replaces (same k order: one MFMA per 32 tokens, in sequence)."""
    ops = wg_engine
    g = torch.Generator(device=cuda).manual_seed(M + N + T)
    A, B = _mk(M, T, 1, cuda, g), _mk(N, T, 1, cuda, g)
    ref = _ref(A, B, 1, 1)
    for S in sorted({1, 2, 5, ops.gp_splits(M, N, T)}):
        ops.gp_wg_nb(0)
        base = ops.gp_mm(A, B, None, 1, 1, 1, S, 256)
        ops.gp_wg_nb(nb)
        assert ops.gp_wg_nb(-1) == nb
        part = ops.gp_mm(A, B, None, 1, 1, 1, S, 256)
        out = torch.zeros(M, N, device=cuda)
        ops.gp_reduce(part, out, False)
        assert _rel(out, ref) < 1e-5, (S, _rel(out, ref))
        assert torch.equal(part, ops.gp_mm(A, B, None, 1, 1, 1, S, 256)), S
        assert torch.equal(part, base), (S, (part - base).abs().max().item())
        acc = torch.randn(S, M, N, device=cuda, generator=g)
        acc0 = acc.clone()
        ops.gp_mm(A, B, acc, 1, 1, 2, S, 256)
        assert torch.equal(acc, acc0 + part), S


def test_gp_wg_engine_default_path(cuda):
    """The weight-gradient engine the process runs by default (MAMBA_AMD_WG_NB) on the headline in_proj shape."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(9)
    T, dp, d = 16384, 3392, 768
    A = (torch.randn(T, dp, device=cuda, generator=g) * 0.5).to(torch.bfloat16)
    B = (torch.randn(T, d, device=cuda, generator=g) * 0.5).to(torch.bfloat16)
    S = ops.gp_splits(dp, d, T)
    part = ops.gp_mm(A, B, None, 1, 1, 1, S, 256)
    out = torch.zeros(dp, d, device=cuda)
    ops.gp_reduce(part, out, False)
    assert _rel(out, _ref(A, B, 1, 1)) < 1e-5


@pytest.mark.parametrize("la,lb,mode", [(0, 1, 0), (0, 1, 1), (1, 0, 0), (1, 0, 2), (0, 0, 1), (0, 0, 2)])
@pytest.mark.parametrize("M,N,K,S,bm", [(256, 256, 32, 1, 256), (264, 136, 96, 1, 256), (520, 776, 200, 1, 256),
                                        (256, 512, 128, 1, 256), (768, 520, 1544, 3, 256), (3072, 768, 4160, 7, 256),
                                        (80, 1536, 2056, 4, 128), (128, 264, 288, 1, 128)])
def test_gp_wg_kc_pairs(cuda, la, lb, mode, M, N, K, S, bm):
    """gemm_wg_kp_k (paired 64-deep KC images, csrc/kernels/gemm_pipe.hip) against the 32-deep gemm_wg_k: the same
    fragments in the same MFMA order, so bitwise equal outputs -- over 1..4 stages (prologue only), odd stage counts,
    partial last stages, K splits, both tile heights and every epilogue -- and both against the fp32 reference."""
    ops = _ops()
    if la == 1 and M % 8 or lb == 1 and N % 8:
        pytest.skip("XC operands need 8-aligned rows")
    g = torch.Generator(device=cuda).manual_seed(M + 3 * N + 7 * K + la)
    A, B = _mk(M, K, la, cuda, g), _mk(N, K, lb, cuda, g)
    ref = _ref(A, B, la, lb)
    outs = {}
    old = ops.gp_wg_kcpair(-1)
    try:
        for kp in (0, 1):  # 1: forced on every KC operand (mode 2)
            assert ops.gp_wg_kcpair(2 * kp) == 2 * kp
            if mode == 2:
                acc = torch.full((M, N), 0.25, device=cuda)
                ops.gp_mm(A, B, acc, la, lb, 2, 1, bm)
                outs[kp] = acc
            elif mode == 1:
                outs[kp] = ops.gp_mm(A, B, None, la, lb, 1, S, bm)
            else:
                outs[kp] = ops.gp_mm(A, B, None, la, lb, 0, 1, bm)
    finally:
        ops.gp_wg_kcpair(old)
    assert torch.equal(outs[0], outs[1])
    got = outs[1].sum(0) if mode == 1 else outs[1]
    want = ref + 0.25 if mode == 2 else ref
    assert _rel(got, want) < (8e-3 if mode == 0 else 1e-5), _rel(got, want)


def test_gp_wg_kc_pairs_default_rule(cuda):
    """The default rule pairs a KC operand of >= 1536 rows over K >= 16384 (the Mamba-1 in_proj / out_proj weight
    gradients); either way the result is bitwise the unpaired engine's."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(5)
    A, B = _mk(1536, 16384, 0, cuda, g), _mk(768, 16384, 1, cuda, g)
    old = ops.gp_wg_kcpair(-1)
    try:
        ops.gp_wg_kcpair(1)
        p1 = ops.gp_mm(A, B, None, 0, 1, 1, 2, 256)
        ops.gp_wg_kcpair(0)
        p0 = ops.gp_mm(A, B, None, 0, 1, 1, 2, 256)
    finally:
        ops.gp_wg_kcpair(old)
    assert torch.equal(p0, p1)
    assert _rel(p1.sum(0), _ref(A, B, 0, 1)) < 1e-5


@pytest.mark.parametrize("S,n", [(42, 80 * 1536), (16, 48 * 1536), (7, 3072 * 768)])
def test_gp_reduce_forms(cuda, S, n):
    """gp_reduce over S fp32 slabs in fixed order: the slab-quarter form (many slabs, small output: the narrow weight
    gradients) and the float4 form give the fp64 sum, bitwise repeatably."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(S)
    part = torch.randn(S, n, device=cuda, generator=g)
    out = torch.full((n,), 0.5, device=cuda)
    ops.gp_reduce(part.view(S, 1, n), out.view(1, n), True)
    want = part.double().sum(0) + 0.5
    assert (out.double() - want).abs().max().item() < 1e-4
    out2 = torch.full((n,), 0.5, device=cuda)
    ops.gp_reduce(part.view(S, 1, n), out2.view(1, n), True)
    assert torch.equal(out, out2)
