"""Unit numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op
(or the oracle, for the diffusion math).  Tolerances are written per test:
fp32 kernels 1e-5..1e-4 relative; bf16-input kernels are compared with the fp32
reference of the SAME bf16-rounded inputs, tolerance 2e-2 relative to the output scale."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from unified_video_action_amd.native import ops  # noqa: F401 -- fails loudly without the .so
    torch.manual_seed(0)


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def _stored(op, t_flag):
    """stored layout of an [R, K] logical operand."""
    return op.t().contiguous() if t_flag else op.contiguous()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(256, 384, 192), (300, 200, 72), (130, 136, 520), (64, 48, 2)])
def test_gemm_layouts(dtype, ta, tb, M, N, K):
    """Every operand layout against fp32 torch; fp32 and bf16 outputs."""
    from unified_video_action_amd.native import ops
    if dtype == torch.bfloat16 and ((ta and M % 8) or (tb and N % 8)):
        pytest.skip("m-contiguous bf16 operands need 8-aligned dims (host pads these)")
    a = torch.randn(M, K, device=DEV).to(dtype)
    b = torch.randn(N, K, device=DEV).to(dtype)
    A, B = _stored(a, ta), _stored(b, tb)
    ref = a.float() @ b.float().t()
    for odt in ((torch.float32, torch.bfloat16) if dtype == torch.bfloat16 else (torch.float32,)):
        C = torch.empty(M, N, device=DEV, dtype=odt)
        ops.gemm(A, B, C, M, N, K, A.stride(0), B.stride(0), C.stride(0), ta, tb)
        tol = 1e-5 if dtype == torch.float32 else (5e-3 if odt == torch.float32 else 1e-2)
        assert rel_err(C, ref) < tol


@pytest.mark.parametrize("M,N,K", [(768, 768, 16384), (3072, 768, 8192), (32768, 768, 3072)])
def test_gemm_backward_shapes_accumulate(M, N, K):
    """The backward's products at MAR shapes: dW += dY^T X (ta = tb = 1, fp32 grad, beta = 1) and
    dX = dY W (tb = 1) agree with fp32 torch."""
    from unified_video_action_amd.native import ops
    torch.manual_seed(M + N + K)
    if K >= 8192:  # dW: A = dY stored [K tokens][M], B = X stored [K tokens][N]
        dy = torch.randn(K, M, device=DEV).to(torch.bfloat16)
        x = torch.randn(K, N, device=DEV).to(torch.bfloat16)
        C = torch.randn(M, N, device=DEV)
        ref = C.double() + dy.double().t() @ x.double()
        ops.gemm(dy, x, C, M, N, K, M, N, N, 1, 1, beta=1.0)
    else:  # dX: A = dY [M][K], B = W stored [K][N]
        dy = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        w = (torch.randn(K, N, device=DEV) * 0.05).to(torch.bfloat16)
        C = torch.empty(M, N, device=DEV)
        ref = dy.double() @ w.double()
        ops.gemm(dy, w, C, M, N, K, K, N, N, 0, 1)
    assert rel_err(C, ref) < 2e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogue_bias_gelu_aux_residual_beta(dtype):
    from unified_video_action_amd.native import ops
    M, N, K = 512, 256, 128
    x = torch.randn(M, K, device=DEV).to(dtype)
    w = torch.randn(N, K, device=DEV).to(dtype) * 0.1
    bias = torch.randn(N, device=DEV)
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    aux = torch.empty_like(out)
    ops.linear(x, w, out, bias=bias, act="gelu", aux=aux)
    pre = x.float() @ w.float().t() + bias
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel_err(aux.float(), pre) < tol
    assert rel_err(out.float(), torch.nn.functional.gelu(pre)) < tol
    # residual + beta accumulate, fp32 output
    res = torch.randn(M, N, device=DEV)
    c = torch.randn(M, N, device=DEV)
    c0 = c.clone()
    ops.gemm(x, w, c, M, N, K, K, K, N, 0, 0, residual=res, ldr=N, beta=1.0)
    assert rel_err(c, c0 + res + x.float() @ w.float().t()) < (1e-5 if dtype == torch.float32 else 1e-2)


def test_gemm_dropout_matches_act_bwd_mask():
    from unified_video_action_amd.native import ops
    M, N, K = 256, 512, 64
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV)
    out = torch.empty(M, N, device=DEV)
    ops.linear(x, w, out, drop_p=0.1, seed=1234)
    ref = x @ w.t()
    kept = out != 0
    frac = kept.float().mean().item()
    assert abs(frac - 0.9) < 0.01
    assert rel_err(out[kept], ref[kept] / 0.9) < 1e-5
    # backward mask (act none) reproduces the same keep pattern
    g = torch.ones(M, N, device=DEV)
    dg = torch.empty(M, N, device=DEV)
    ops.act_bwd(None, g, dg, "none", drop_p=0.1, seed=1234)
    assert torch.equal(dg != 0, kept)


def test_gemm_batched_two_level_strides():
    from unified_video_action_amd.native import ops
    Bn, H, N, Dh = 2, 3, 96, 64
    qkv = torch.randn(Bn, N, 3, H, Dh, device=DEV).to(torch.bfloat16)
    S = torch.empty(Bn, H, N, N, device=DEV, dtype=torch.float32)
    q = qkv[:, :, 0]
    k = qkv[:, :, 1]
    ld = 3 * H * Dh
    ops.gemm(q, k, S, N, N, Dh, ld, ld, N, 0, 0, batch=Bn * H, inner=H, sA=(N * ld, Dh), sB=(N * ld, Dh),
             sC=(H * N * N, N * N))
    ref = torch.einsum("bihd,bjhd->bhij", q.float(), k.float())
    assert rel_err(S, ref) < 5e-3


@pytest.mark.parametrize("D", [64, 128, 768, 1024])
@pytest.mark.parametrize("io", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16)])
def test_layernorm_affine_fwd_bwd(D, io):
    from unified_video_action_amd.native import ops
    tin, tout = io
    rows = 300
    x = torch.randn(rows, D, device=DEV).to(tin)
    w = torch.randn(D, device=DEV) * 0.1 + 1
    b = torch.randn(D, device=DEV) * 0.1
    y = torch.empty(rows, D, device=DEV, dtype=tout)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    ops.layernorm_fwd(x, w, b, y, mean, rstd)
    xr = x.float().clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (D,), wr, br, eps=1e-6)
    tol = 1e-5 if tout == torch.float32 else 1e-2
    assert rel_err(y.float(), yr) < tol
    dy = torch.randn(rows, D, device=DEV)
    yr.backward(dy)
    dx = torch.full((rows, D), 0.5, device=DEV)
    dw = torch.zeros(D, device=DEV)
    db = torch.zeros(D, device=DEV)
    ops.layernorm_bwd(x, w, dy, mean, rstd, dx, accum=True, dw=dw, db=db)
    assert rel_err(dx - 0.5, xr.grad) < 1e-4
    assert rel_err(dw, wr.grad) < 1e-4
    assert rel_err(db, br.grad) < 1e-4
    # bf16 dy (the consuming GEMM's bf16 dX) == fp32 dy holding the same bf16-rounded values
    dyb = dy.to(torch.bfloat16)
    dx1 = torch.empty(rows, D, device=DEV)
    dx2 = torch.empty(rows, D, device=DEV)
    ops.layernorm_bwd(x, w, dyb, mean, rstd, dx1, accum=False)
    ops.layernorm_bwd(x, w, dyb.float(), mean, rstd, dx2, accum=False)
    assert torch.equal(dx1, dx2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm_modulated_fwd_bwd(dtype):
    from unified_video_action_amd.native import ops
    rows, D = 257, 1024
    x = torch.randn(rows, D, device=DEV)
    mod = (torch.randn(rows, 3 * D, device=DEV) * 0.3).to(dtype)
    shift, scale = mod[:, :D], mod[:, D:2 * D]
    y = torch.empty(rows, D, device=DEV, dtype=dtype)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    ops.layernorm_fwd(x, None, None, y, mean, rstd, scale=scale, shift=shift, ldm=3 * D)
    xr = x.clone().requires_grad_(True)
    sc = scale.float().clone().requires_grad_(True)
    sh = shift.float().clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (D,), eps=1e-6) * (1 + sc) + sh
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(y.float(), yr) < tol
    dy = torch.randn(rows, D, device=DEV)
    yr.backward(dy)
    dx = torch.empty(rows, D, device=DEV)
    dmod = torch.zeros(rows, 3 * D, device=DEV, dtype=dtype)
    ops.layernorm_bwd(x, None, dy, mean, rstd, dx, accum=False, scale=scale, ldm=3 * D,
                      dscale=dmod[:, D:2 * D], dshift=dmod[:, :D])
    assert rel_err(dx, xr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)
    assert rel_err(dmod[:, D:2 * D].float(), sc.grad) < tol
    assert rel_err(dmod[:, :D].float(), sh.grad) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_softmax_fwd_bwd(dtype):
    from unified_video_action_amd.native import ops
    rows, L = 96, 1088
    S = torch.randn(rows, L, device=DEV).to(dtype) * 3
    P = torch.empty_like(S)
    ops.softmax_fwd(S, P, None, L, 0.125)
    Sr = S.float().clone().requires_grad_(True)
    Pr = torch.softmax(Sr * 0.125, dim=-1)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(P.float(), Pr) < tol
    dP = torch.randn(rows, L, device=DEV).to(dtype)
    Pr.backward(dP.float())
    dS = torch.empty_like(S)
    ops.softmax_bwd(P, dP, dS, L, 0.125)
    assert rel_err(dS.float(), Sr.grad) < (1e-4 if dtype == torch.float32 else 3e-2)


def test_colsum_and_cast():
    from unified_video_action_amd.native import ops
    x = torch.randn(5000, 300, device=DEV)
    out = torch.ones(300, device=DEV)
    ops.colsum(x, out, accum=True)
    assert rel_err(out - 1, x.sum(0)) < 1e-5
    xb = torch.empty(5000, 300, device=DEV, dtype=torch.bfloat16)
    ops.cast(x, xb)
    assert torch.equal(xb, x.to(torch.bfloat16))


@pytest.mark.parametrize("rows,cols", [(5000, 296), (33000, 768)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_colsum_vectorized_tall(rows, cols, dtype):
    from unified_video_action_amd.native import ops
    x = torch.randn(rows, cols, device=DEV).to(dtype)
    out = torch.full((cols,), 0.5, device=DEV)
    ops.colsum(x, out, accum=True)
    assert rel_err(out - 0.5, x.float().sum(0)) < 1e-5


@pytest.mark.parametrize("act,drop", [("none", 0.1), ("gelu", 0.1), ("silu", 0.0)])
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_act_bwd_bias_matches_act_bwd_plus_colsum(act, drop, gdt):
    """fused activation/dropout backward + bias gradient == act_bwd then colsum (same mask)."""
    from unified_video_action_amd.native import ops
    R, C = 1000, 520
    pre = torch.randn(R, C, device=DEV).to(torch.bfloat16)
    dy = torch.randn(R, C, device=DEV).to(gdt)
    ref = torch.empty(R, C, device=DEV, dtype=torch.bfloat16)
    ops.act_bwd(pre if act != "none" else None, dy, ref, act, drop_p=drop, seed=77)
    got = torch.empty_like(ref)
    db = torch.ones(C, device=DEV)
    ops.act_bwd_bias(pre if act != "none" else None, dy, got, db, act, drop_p=drop, seed=77)
    assert torch.equal(got, ref)
    assert rel_err(db - 1, ref.float().sum(0)) < 1e-5


def test_act_fwd_bwd():
    from unified_video_action_amd.native import ops
    x = torch.randn(1000, 64, device=DEV)
    for act, fn in (("silu", torch.nn.functional.silu), ("gelu", torch.nn.functional.gelu),
                    ("relu", torch.relu)):
        y = torch.empty_like(x)
        ops.act_fwd(x, y, act)
        assert rel_err(y, fn(x)) < 1e-5
        xr = x.clone().requires_grad_(True)
        dy = torch.randn_like(x)
        fn(xr).backward(dy)
        dx = torch.empty_like(x)
        ops.act_bwd(x, dy, dx, act)
        assert rel_err(dx, xr.grad) < 1e-5


def test_diffusion_loss_matches_oracle_golden():
    import cases
    import replay
    import uva_oracle as O
    from hashinit import hash_normal, hash_tensor
    from unified_video_action_amd.native import ops
    from unified_video_action_amd.model.autoregressive.diffusion import DiffusionSchedule
    g = replay.load("g3_diffusion_math.npz")
    sched = DiffusionSchedule(1000, DEV)
    for tag, C in (("video", 16), ("act", 2), ("act10", 10)):
        rows = 512
        x0 = torch.from_numpy(hash_tensor(f"dm/{tag}/x0", (rows, C))).to(DEV)
        out = torch.from_numpy(hash_tensor(f"dm/{tag}/out", (rows, 2 * C))).to(DEV)
        t = torch.from_numpy(cases.t_steps(f"dm/{tag}", rows)).to(DEV)
        noise = torch.from_numpy(hash_normal(f"dm/{tag}/noise", (rows, C))).to(DEV)
        lr = torch.empty(rows, device=DEV)
        dl = torch.empty(rows, 2 * C, device=DEV)
        ops.diffusion_loss(x0, noise, t, out, sched.tables, lr, dl)
        np.testing.assert_allclose(lr.cpu().numpy(), g[f"{tag}_loss"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(dl.cpu().numpy(), g[f"{tag}_gout"], rtol=1e-3, atol=1e-6)
        xt = torch.empty(rows, C, device=DEV)
        ops.q_sample(x0, noise, t, sched.tables, xt)
        tb = O.DiffusionTables(1000)
        ref = tb.gather("sqrt_ac", t.cpu()) * x0.cpu() + tb.gather("sqrt_1mac", t.cpu()) * noise.cpu()
        assert rel_err(xt.cpu(), ref) < 1e-6


def test_timestep_features():
    import uva_oracle as O
    from unified_video_action_amd.native import ops
    from unified_video_action_amd.model.autoregressive.diffusion import timestep_freqs
    t = torch.arange(0, 1000, 7, device=DEV)
    out = torch.empty(t.numel(), 256, device=DEV)
    ops.timestep_features(t, timestep_freqs(DEV), out)
    ref = O.timestep_features(t.cpu())
    assert (out.cpu() - ref).abs().max().item() < 2e-5


def test_adamw_ema_matches_torch():
    """one launch per param group region (16-B aligned; n = 6001 exercises the scalar tail),
    1/world gradient scaling, fused EMA, bf16 shadow; plus the standalone EMA kernel."""
    from unified_video_action_amd.native import ops
    n_a, n_b, off_b = 6001, 3999, 6016
    n = off_b + n_b
    p0 = torch.randn(n, device=DEV)
    pa, pb = p0[:n_a].clone(), p0[off_b:].clone()
    opt = torch.optim.AdamW([{"params": [pa], "weight_decay": 0.02},
                             {"params": [pb], "weight_decay": 0.0}], lr=1e-3, betas=(0.9, 0.95))
    p = p0.clone()
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    ema = p0.clone()
    pbf = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    ema_ref = p0.clone()
    regions = ((0, n_a, 0.02), (off_b, n_b, 0.0))
    for step in range(1, 4):
        g = torch.randn(n, device=DEV)
        pa.grad, pb.grad = g[:n_a].clone(), g[off_b:].clone()
        opt.step()
        for o, k, wd in regions:
            sl = slice(o, o + k)
            ops.adamw_ema(p[sl], (g * 2.0)[sl], m[sl], v[sl], ema[sl], pbf[sl], k if wd else 0, 1e-3, 0.9, 0.95,
                          1e-8, wd, step, 0.5, 0.7)
        ref = torch.cat([pa, p0[n_a:off_b], pb]).detach()
        ema_ref = ema_ref * 0.7 + ref * 0.3
        for o, k, _ in regions:
            assert rel_err(p[o:o + k], ref[o:o + k]) < 1e-6
    for o, k, _ in regions:
        assert rel_err(ema[o:o + k], ema_ref[o:o + k]) < 1e-6
        assert torch.equal(pbf[o:o + k], p[o:o + k].to(torch.bfloat16))
    e2 = ema.clone()
    ops.ema_update(e2, p, 0.25)
    assert rel_err(e2, ema * 0.25 + p * 0.75) < 1e-6
    with pytest.raises(RuntimeError):  # misaligned region
        ops.adamw_ema(p[1:5], g[1:5], m[1:5], v[1:5], None, None, 4, 1e-3, 0.9, 0.95, 1e-8, 0.0, 1, 1.0, 0.0)


@pytest.mark.parametrize("rows,cols", [(64, 3072), (1000, 768)])
def test_act_drop_fwd_matches_backward_mask_and_torch(rows, cols):
    """uva_act_drop_fwd (timm Mlp forward after bias-only GEMMs): GELU against torch's exact GELU, the
    dropout keep pattern identical to the one act_bwd regenerates (flat element index), residual add."""
    from unified_video_action_amd.native import ops
    torch.manual_seed(rows + cols)
    x = (torch.randn(rows, cols, device=DEV) * 2).to(torch.bfloat16)
    y = torch.empty_like(x)
    ops.act_drop_fwd(x, y, "gelu")
    ref = torch.nn.functional.gelu(x.float())
    assert rel_err(y.float(), ref) < 1e-2
    ones = torch.ones(rows, cols, device=DEV).to(torch.bfloat16)
    yd = torch.empty(rows, cols, device=DEV).to(torch.bfloat16)
    ops.act_drop_fwd(ones, yd, "none", drop_p=0.1, seed=77)
    g = torch.empty(rows, cols, device=DEV)
    ops.act_bwd(None, torch.ones(rows, cols, device=DEV), g, "none", drop_p=0.1, seed=77)
    assert torch.equal(yd.float() != 0, g != 0)
    assert abs((g != 0).float().mean().item() - 0.9) < 0.02
    res = torch.randn(rows, cols, device=DEV)
    out = torch.empty(rows, cols, device=DEV)
    ops.act_drop_fwd(x, out, "none", drop_p=0.1, seed=78, residual=res)
    keep = torch.empty(rows, cols, device=DEV)
    ops.act_bwd(None, torch.ones(rows, cols, device=DEV), keep, "none", drop_p=0.1, seed=78)
    assert torch.allclose(out, res + x.float() * keep, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("R,C", [(768, 2304), (2304, 768), (3072, 768), (768, 3072), (768, 768), (72, 136)])
def test_transpose_bf16_and_dx_through_transposed_weight(R, C):
    """uva_transpose_bf16 (64 x 64 LDS tiles, ragged edges) is an exact transpose, and the Block's dX
    through the transposed weight copy (functional.linear_dx_w: a forward-layout GEMM) equals the
    dX GEMM to bf16 output rounding (the same bf16 operands, fp32 accumulation in another order)."""
    from unified_video_action_amd.native import ops
    from unified_video_action_amd.model.autoregressive import functional as fn
    from unified_video_action_amd.runtime import RT
    torch.manual_seed(R + C)
    w = torch.randn(R, C, device="cuda").to(torch.bfloat16)
    t = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
    ops.transpose_bf16(w, t)
    assert torch.equal(t, w.t().contiguous())
    if R % 8:
        return
    # dX = dy @ W for nn.Linear(C -> R): W [R, C], dy [M, R], dX [M, C]; bf16 runs it through the
    # transposed copy (forward layout), fp32 through the stored weight (the dX layout)
    RT.set_precision("bf16")
    M = 2048
    p = torch.nn.Parameter((torch.randn(R, C, device="cuda") * 0.05))
    dy = (torch.randn(M, R, device="cuda")).to(torch.bfloat16)
    a = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
    b = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
    fn.linear_dx_w(dy, p, a)
    ops.linear_dx(dy, fn.compute_weight(p), b)
    ref = dy.float() @ p.detach().to(torch.bfloat16).float()
    scale = ref.abs().max().item()
    assert (a.float() - ref).abs().max().item() < 1e-2 * scale
    assert (a.float() - b.float()).abs().max().item() < 1e-2 * scale
