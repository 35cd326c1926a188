"""8-phase 256-row MFMA GEMM (csrc/gemm.hip gemm_8ph) at shapes the dispatcher routes to it
(asserted through the uva_gemm_plan query): all four operand layouts, ragged M/N edges and
K tails, both output dtypes, split-K dW, the fused Linear epilogues (bias, GELU + aux,
dropout, adaLN gate, residual, beta-accumulate) and the conv epilogue that also emits the
next GroupNorm's per-tile statistics.  Reference: torch fp32 of the SAME bf16-rounded inputs;
tolerance 5e-3 relative to the output scale for a bf16 input GEMM with fp32 accumulation
(1e-2 for bf16 outputs: one extra rounding)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


@pytest.fixture(scope="module", autouse=True)
def _seed():
    from unified_video_action_amd.native import ops  # fails loudly without the .so
    torch.manual_seed(0)
    # the K-contiguous bias-only products go to the 4-wave kernel by default (tests/test_gemm4_gpu.py);
    # this file pins gemm_8ph itself
    prev = ops.gemm4_set(0)
    yield
    ops.gemm4_set(prev[0])


def _stored(op, t_flag):
    return op.t().contiguous() if t_flag else op.contiguous()


CASES = [(5376, 3072, 328, 256), (5000, 3000, 136, 256), (6144, 2048, 200, 256),
         # > 256 tiles: several rounds of workgroups (ragged M, K tail)
         (16296, 3072, 328, 256), (16384, 3072, 256, 256),
         # N = 768: the 128x384 tile (ragged M and K tail; full tiles on the fast path)
         (32000, 768, 328, 384), (32768, 768, 3072, 384),
         # persistent form (gemm_8pp: full tiles, K % 64 == 0, K >= 128): 4.5 rounds of 256 workgroups
         # (the last round half full), and fewer tiles than CUs with K = 128 (two K-tiles)
         (32768, 2304, 768, 256), (4096, 2304, 128, 384)]


@pytest.fixture(params=[False, True], ids=["8ph", "8pp"])
def persist(request):
    """every case on gemm_8ph and on the persistent gemm_8pp (used where the shape is eligible: full
    tiles, K % 64 == 0, K >= 128, no row inputs in the epilogue)"""
    from unified_video_action_amd.native import ops
    prev = ops.gemm_set_persist(request.param)
    yield request.param
    ops.gemm_set_persist(prev)


@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K,bn", CASES)
def test_gemm8_layouts(odt, ta, tb, M, N, K, bn, persist):
    from unified_video_action_amd.native import ops
    assert ops.gemm_plan(M, N, K, ta, tb) == (3, bn, 1)
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    b = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    A, B = _stored(a, ta), _stored(b, tb)
    C = torch.full((M, N), float("nan"), device=DEV, dtype=odt)
    ops.gemm(A, B, C, M, N, K, A.stride(0), B.stride(0), C.stride(0), ta, tb)
    ref = a.float() @ b.float().t()
    assert torch.isfinite(C).all()
    assert rel_err(C.float(), ref) < (5e-3 if odt == torch.float32 else 1e-2)


@pytest.mark.parametrize("M,N,K,splits", [(768, 768, 16384, 26), (2304, 768, 8192, 9)])
def test_gemm8_splitk_dw_accumulate(M, N, K, splits):
    """dW = dY^T X accumulated into an fp32 grad (ta = tb = 1, K = tokens)."""
    from unified_video_action_amd.native import ops
    kern, bn, sp = ops.gemm_plan(M, N, K, 1, 1)
    assert kern == 3 and sp > 1, (kern, bn, sp)  # 8-phase kernel, split-K (tile width per the planner)
    dy = torch.randn(K, M, device=DEV).to(torch.bfloat16)
    x = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    g = torch.randn(M, N, device=DEV)
    g0 = g.clone()
    ops.linear_dw(dy, x, g)
    ref = g0.double() + dy.double().t() @ x.double()
    assert rel_err(g, ref) < 1e-4  # exact bf16 products, fp32 partial sums over 8-16k terms


@pytest.mark.parametrize("M,N,K,bn", [(5376, 3072, 256, 256), (16384, 3072, 256, 256),
                                      (32000, 768, 328, 384), (32768, 768, 768, 384), (32768, 2304, 768, 256)])
def test_gemm8_epilogues(M, N, K, bn, persist):
    from unified_video_action_amd.native import ops
    assert ops.gemm_plan(M, N, K) == (3, bn, 1)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.1).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    pre = x.float() @ w.float().t() + bias
    # bias + GELU + pre-activation aux, bf16 out
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    aux = torch.empty_like(out)
    ops.linear(x, w, out, bias=bias, act="gelu", aux=aux)
    assert rel_err(aux.float(), pre) < 1e-2
    assert rel_err(out.float(), F.gelu(pre)) < 1e-2
    # dropout: same keep pattern as the elementwise backward mask
    outd = torch.empty(M, N, device=DEV)
    ops.linear(x, w, outd, bias=bias, drop_p=0.1, seed=77)
    kept = outd != 0
    assert abs(kept.float().mean().item() - 0.9) < 0.005
    assert rel_err(outd[kept], pre[kept] / 0.9) < 5e-3
    dg = torch.empty(M, N, device=DEV)
    ops.act_bwd(None, torch.ones(M, N, device=DEV), dg, "none", drop_p=0.1, seed=77)
    # same keep pattern, except where acc + bias cancelled to exactly 0.0 (a kept zero reads as dropped:
    # ~1 element in 25M at these sizes)
    bad = (dg != 0) != kept
    assert int(bad.sum()) <= 4 and (pre[bad].abs() < 1e-4).all()
    # adaLN gate (bf16, strided) + fp32 residual, fp32 out
    gate_full = torch.randn(M, 3 * N, device=DEV).to(torch.bfloat16)
    gate = gate_full[:, 2 * N:]
    res = torch.randn(M, N, device=DEV)
    outg = torch.empty(M, N, device=DEV)
    ops.linear(x, w, outg, bias=bias, gate=gate, residual=res)
    assert rel_err(outg, res + gate.float() * pre) < 5e-3
    # bf16 residual, beta accumulate into bf16 C
    c = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    c0 = c.float()
    resb = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    ops.gemm(x, w, c, M, N, K, K, K, N, 0, 0, residual=resb, ldr=N, beta=1.0)
    assert rel_err(c.float(), c0 + resb.float() + x.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("residual", [False, True])
def test_conv8_with_groupnorm_stats(residual):
    """3x3 conv (NHWC implicit GEMM) + bias (+residual) through the 8-phase kernel, and the per-128-row
    GroupNorm(32) partial sums of its stored output -> finalize == GroupNorm of the output."""
    from unified_video_action_amd.native import ops
    n, H, W, Ci, Co = 16, 64, 64, 96, 256  # Ci % 64 != 0: not a halo-kernel shape (test_conv_halo_gpu.py)
    M = n * H * W
    assert ops.gemm_plan(M, Co, 9 * Ci, 2, 0, splitk=False) == (3, 256, 1)
    assert not ops.conv_fuses_gn(n, H, W, Ci, Co, 3, 1)
    x = torch.randn(n, H, W, Ci, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Co, 3, 3, Ci, device=DEV) * 0.05).to(torch.bfloat16)
    bias = torch.randn(Co, device=DEV) * 0.1
    res = torch.randn(n, H, W, Co, device=DEV).to(torch.bfloat16) if residual else None
    out = torch.empty(n, H, W, Co, device=DEV, dtype=torch.bfloat16)
    part = torch.empty(M // 128, 32, 2, device=DEV)
    ops.conv2d(x, w, out, n, H, W, Ci, Co, 3, 1, 1, 1, H, W, bias=bias, residual=res, gn_part=part)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias, padding=1).permute(0, 2, 3, 1)
    if residual:
        ref = ref + res.float()
    assert rel_err(out.float(), ref) < 1e-2
    gamma = torch.randn(Co, device=DEV)
    beta = torch.randn(Co, device=DEV)
    sc = torch.empty(n, Co, device=DEV)
    sh = torch.empty(n, Co, device=DEV)
    ops.groupnorm_finalize_tiles(part, n, H * W, Co, gamma, beta, sc, sh, eps=1e-6)
    o = out.double().reshape(n, H * W, 32, Co // 32)
    mean = o.mean(dim=(1, 3))
    var = o.var(dim=(1, 3), unbiased=False)
    rstd = (var + 1e-6).rsqrt()
    sc_ref = gamma.double()[None] * rstd.repeat_interleave(Co // 32, dim=1)
    sh_ref = beta.double()[None] - mean.repeat_interleave(Co // 32, dim=1) * sc_ref
    assert rel_err(sc, sc_ref) < 1e-4
    assert rel_err(sh, sh_ref) < 1e-4


@pytest.mark.parametrize("act", ["gelu", "silu"])
@pytest.mark.parametrize("M,N,K,p", [(4096, 768, 3072, 0.1), (1000, 1024, 1024, 0.0), (256, 64, 96, 0.1)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_linear_dx_act_matches_act_bwd(act, M, N, K, p, dtype):
    """Activation(+dropout) backward fused into the dX GEMM epilogue (act = 16 + kind) against the
    separate route: dX GEMM -> act_bwd (the same counter-hash keep bits, row * K + col) and against
    a plain fp32 torch reference of act'(pre) * keep / (1 - p) * (dy @ w).  Tolerance: bf16 -> 2e-2
    of the output scale (the separate route rounds dy @ w to bf16 first), fp32 -> 1e-5."""
    from unified_video_action_amd.native import ops
    torch.manual_seed(M + N + K)
    dy = (torch.randn(M, N, device=DEV) * 0.5).to(dtype)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(dtype)
    pre = (torch.randn(M, K, device=DEV) * 2).to(dtype)
    fused = torch.empty(M, K, device=DEV, dtype=dtype)
    ops.linear_dx_act(dy, w, fused, pre, act, drop_p=p, seed=77)
    da = torch.empty(M, K, device=DEV, dtype=dtype)
    ops.linear_dx(dy, w, da)
    split = torch.empty(M, K, device=DEV, dtype=dtype)
    ops.act_bwd(pre, da, split, act, drop_p=p, seed=77)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert rel_err(fused.float(), split.float()) < tol
    # fp32 reference with the kernels' own keep bits (recovered from the separate route on ones)
    keep = torch.ones(M, K, device=DEV)
    if p > 0:
        ones = torch.ones(M, K, device=DEV, dtype=dtype)
        kb = torch.empty(M, K, device=DEV, dtype=dtype)
        ops.act_bwd(None, ones, kb, "none", drop_p=p, seed=77)
        keep = kb.float()  # 0 or 1 / (1 - p)
        assert abs((keep > 0).float().mean().item() - (1 - p)) < 0.01
    x = pre.float().requires_grad_(True)
    y = F.gelu(x) if act == "gelu" else F.silu(x)
    g = (dy.float() @ w.float()) * keep
    (dx_ref,) = torch.autograd.grad(y, x, g)
    assert rel_err(fused.float(), dx_ref) < tol * 5
