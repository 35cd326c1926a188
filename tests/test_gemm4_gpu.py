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


@pytest.mark.parametrize("M,N,K", [(32768, 2304, 768), (32768, 768, 3072), (32768, 3072, 768), (1000, 776, 384)])
def test_gemm4_fp32_pin_vs_fp64(M, N, K):
    """fp32 pin of the benched kernel itself: with fp32 outputs the only error left against exact (fp64)
    math on the same bf16 operands is fp32 accumulation -- held to 2e-5 of the output scale (the
    parity suite's 1e-4 loss pin runs the exact-f32 VALU GEMM; this is the MFMA kernel the bench runs)."""
    from unified_video_action_amd.native import ops
    plan = ops.gemm4_plan(M, N, K)
    assert plan is not None and plan[0] == 1, plan
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    out = torch.empty(M, N, device=DEV)
    ops.linear(a, w, out, bias=bias)
    ref = a.double() @ w.double().t() + bias.double()
    assert rel_err(out, ref) < 2e-5


@pytest.mark.parametrize("M,N,K", [(768, 768, 32768), (1000, 584, 4096)])
def test_gemm4_dw_fp32_pin_vs_fp64(M, N, K):
    """the same fp32 pin for the split-K dW form (fp32 slabs reduced in slice order)"""
    from unified_video_action_amd.native import ops
    assert ops.gemm4_plan_tt(M, N, K) is not None
    dy = torch.randn(K, M, device=DEV).to(torch.bfloat16)
    x = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    dw = torch.zeros(M, N, device=DEV)
    ops.linear_dw(dy, x, dw, beta=0.0)
    ref = dy.double().t() @ x.double()
    assert rel_err(dw, ref) < 2e-5


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


# dW products (ta = tb = 1: A = dY [tokens][out], B = X [tokens][in], fp32 gradient C[out][in]) routed
# to the 4-wave kernel (<= 16 tiles): the Block's proj at B = 32 (mar_con_unified.py:201-215), ragged
# edges, a K that does not split evenly, a single-slice case
TT_CASES = [(768, 768, 32768), (1000, 584, 4096), (300, 200, 512), (768, 768, 33280), (1024, 768, 256),
            (768, 960, 8192)]


@pytest.mark.parametrize("beta", [0.0, 1.0])
@pytest.mark.parametrize("M,N,K", TT_CASES)
def test_gemm4_dw_vs_fp32(M, N, K, beta):
    from unified_video_action_amd.native import ops
    plan = ops.gemm4_plan_tt(M, N, K)
    assert plan is not None, plan
    dy = torch.randn(K, M, device=DEV).to(torch.bfloat16)
    x = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    dw0 = torch.randn(M, N, device=DEV)
    dw = dw0.clone() if beta else torch.full((M, N), float("nan"), device=DEV)
    ops.linear_dw(dy, x, dw, beta=beta)
    ref = dy.float().t() @ x.float() + (dw0 if beta else 0.0)
    assert torch.isfinite(dw).all()
    err = rel_err(dw, ref)
    assert err < 5e-3, (err, plan)


def test_gemm4_dw_matches_8ph_and_repeatable():
    """the dW product on the 4-wave kernel agrees with the 8-phase route to fp32-accumulation noise and
    is bit-repeatable (slices reduced in a fixed order)"""
    from unified_video_action_amd.native import ops
    M, N, K = 768, 768, 32768
    dy = torch.randn(K, M, device=DEV).to(torch.bfloat16)
    x = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    o1 = torch.zeros(M, N, device=DEV)
    o2 = torch.zeros(M, N, device=DEV)
    o8 = torch.zeros(M, N, device=DEV)
    ops.linear_dw(dy, x, o1)
    ops.linear_dw(dy, x, o2)
    assert torch.equal(o1, o2)
    prev = ops.gemm4_set(0)
    try:
        ops.linear_dw(dy, x, o8)
    finally:
        ops.gemm4_set(prev[0])
    assert rel_err(o1, o8) < 1e-5


def test_gemm4_dw_strided_operands():
    """dY / X inside wider rows (the qkv slice of a fused buffer), ldc > N"""
    from unified_video_action_amd.native import ops
    M, N, K = 768, 768, 8192
    A = torch.randn(K, M + 64, device=DEV).to(torch.bfloat16)
    B = torch.randn(K, N + 128, device=DEV).to(torch.bfloat16)
    C = torch.zeros(M, N + 256, device=DEV)
    ops.gemm(A, B, C, M, N, K, M + 64, N + 128, N + 256, 1, 1, alpha=0.5)
    ref = 0.5 * (A[:, :M].float().t() @ B[:, :N].float())
    assert rel_err(C[:, :N], ref) < 5e-3
    assert (C[:, N:] == 0).all()


@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16])
def test_gemm4_output_past_descriptor_range(odt):
    """an output just past the 0x7fff0000-byte store-descriptor range (fp32: M = 699136 rows of 768;
    bf16: 1398272 rows) leaves gemm_4w (its 32-bit store offsets) for gemm_8ph: the rows at the very
    end are written and correct (they used to be dropped by the range check)"""
    from unified_video_action_amd.native import ops
    N, K = 768, 256
    M = 699136 if odt == torch.float32 else 1398272
    assert M * N * (4 if odt == torch.float32 else 2) > 0x7FFF0000
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=odt)
    ops.linear(a, w, out)
    for rows in (slice(0, 512), slice(M // 2, M // 2 + 512), slice(M - 512, M)):
        ref = a[rows].float() @ w.float().t()
        assert torch.isfinite(out[rows]).all()
        assert rel_err(out[rows].float(), ref) < (1e-2 if odt == torch.bfloat16 else 5e-3)
    del a, out
    torch.cuda.empty_cache()
