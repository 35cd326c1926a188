"""Persistent 4-wave GEMM (csrc/gemm4.hip gemm_4w) through the uva_gemm C ABI: the K-contiguous
(ta = tb = 0) products with a bias-only epilogue that the dispatcher routes to it (asserted through
uva_gemm4_plan) -- the timm Block qkv / fc1 / fc2 forwards and the dX products through transposed
weights (mar_con_unified.py:201-249) at full and reduced token counts, ragged M / N edges (zero-filled
DMA past the descriptor range, masked stores), several tiles per workgroup (the substep stream running
across tile boundaries with the epilogue stores counted into the next tile's waits), fp32 / bf16
outputs, bias, alpha.  Reference: torch fp32 of the SAME bf16-rounded inputs; tolerance 5e-3 of the
output scale for fp32 outputs, 1e-2 for bf16 outputs (one extra rounding)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


@pytest.fixture(scope="module", autouse=True)
def _seed():
    from unified_video_action_amd.native import ops  # fails loudly without the .so
    torch.manual_seed(0)
    prev = ops.gemm4_set(1, -1)
    yield
    ops.gemm4_set(prev[0], prev[1])


# (M, N, K): the Block products at B = 32 (fwd qkv / fc1 / fc2, dX through transposed weights),
# ragged edges, fewer tiles than CUs, many tiles per workgroup, K = 256 (two substep groups)
CASES = [(32768, 2304, 768), (32768, 3072, 768), (32768, 768, 3072), (32768, 768, 768), (32768, 768, 2304),
         (4096, 768, 256), (1000, 776, 384), (300, 200, 512), (34816, 768, 768), (8192, 3072, 1024)]


@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K", CASES)
def test_gemm4_vs_fp32(odt, M, N, K):
    from unified_video_action_amd.native import ops
    plan = ops.gemm4_plan(M, N, K)
    assert plan is not None and plan[0] == 1, plan
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=odt)
    ops.linear(a, w, out, bias=bias)
    ref = a.float() @ w.float().t() + bias
    assert torch.isfinite(out).all()
    err = rel_err(out.float(), ref)
    assert err < (1e-2 if odt == torch.bfloat16 else 5e-3), err


def test_gemm4_no_bias_alpha_and_strides():
    """no bias, alpha != 1 (uva_gemm), operands inside wider rows (lda / ldb / ldc > K, N)"""
    from unified_video_action_amd.native import ops
    M, N, K = 2048, 1536, 512
    A = torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)
    B = torch.randn(N, K + 128, device=DEV).to(torch.bfloat16)
    C = torch.zeros(M, N + 256, device=DEV)
    ops.gemm(A, B, C, M, N, K, K + 64, K + 128, N + 256, 0, 0, alpha=0.5)
    ref = 0.5 * (A[:, :K].float() @ B[:, :K].float().t())
    assert rel_err(C[:, :N], ref) < 5e-3
    assert (C[:, N:] == 0).all()  # nothing written past N


def test_gemm4_matches_8ph_route():
    """the same product on the 4-wave kernel and on gemm_8ph agree to fp32-accumulation noise"""
    from unified_video_action_amd.native import ops
    M, N, K = 16384, 2304, 768
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    o4 = torch.empty(M, N, device=DEV)
    o8 = torch.empty(M, N, device=DEV)
    ops.linear(a, w, o4, bias=bias)
    prev = ops.gemm4_set(0)
    try:
        ops.linear(a, w, o8, bias=bias)
    finally:
        ops.gemm4_set(prev[0])
    assert rel_err(o4, o8) < 1e-5


def test_gemm4_repeatable():
    """deterministic: two launches give identical bits (no atomics, fixed summation order)"""
    from unified_video_action_amd.native import ops
    M, N, K = 32768, 768, 3072
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    o1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    o2 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.linear(a, w, o1)
    ops.linear(a, w, o2)
    assert torch.equal(o1, o2)


def test_gemm4_ineligible_shapes_fall_back():
    """K not a multiple of 128, K < 256, tiny M / N: not for this kernel (the 8-phase / 128x128 kernels
    take them) and still correct"""
    from unified_video_action_amd.native import ops
    for (M, N, K) in ((4096, 768, 200), (4096, 768, 128), (128, 768, 768), (4096, 64, 768)):
        assert ops.gemm4_plan(M, N, K) is None
        a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
        out = torch.empty(M, N, device=DEV)
        ops.linear(a, w, out)
        assert rel_err(out, a.float() @ w.float().t()) < 5e-3
