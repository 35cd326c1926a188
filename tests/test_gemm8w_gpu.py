"""8-wave GEMM (csrc/gemm8w.hip) and the fused timm Mlp products it carries (mar_con_unified.py:236-249:
Mlp.fc1 -> GELU -> drop -> fc2 -> drop, + the Block's residual add), through the C ABI:

* uva_linear_gelu_drop / uva_linear_drop_res / uva_linear_dgelu_drop against the split route they replace
  (bias-only GEMM + act_drop_fwd, dX GEMM + act_bwd_bias): the same rounding points and the same flat-index
  counter-hash dropout masks, so every stored tensor is compared BIT FOR BIT; the fused fc1 bias gradient
  (column partials reduced in another order) within 1e-5 of the split route's and of an fp64 column sum of
  the stored dpre;
* the plain 8-wave route (measurement switch) against gemm_4w, bit for bit (the same fp32 accumulation
  order per output);
* ragged M / N edges (masked stores, zero-filled operand rows), several tiles per workgroup, K = 256;
* a whole timm Block (functional.BlockFn) forward + backward with the fused routes (the defaults) against the
  split routes: output and every gradient bit-identical except fc1.bias (fp32 summation order, 1e-5).
Reference for the math: the split route, itself pinned to torch fp32 / the reference's goldens
(test_kernels_gpu.py, test_parity_gpu.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from unified_video_action_amd.native import ops  # fails loudly without the .so
    prev = ops.gemm8w_set(0, 0)
    yield
    ops.gemm8w_set(*prev)


# gemm_8w launch forms: 64 one 8-wave workgroup per CU (256 x 192 tiles), 32 two 4-wave workgroups per CU
# (128 x 192 tiles, bias from L2); the default (0) picks one of them per product
FORMS = [64, 32]


@pytest.fixture(params=FORMS)
def form(request):
    from unified_video_action_amd.native import ops
    prev = ops.gemm8w_set(-2, request.param)
    yield request.param
    ops.gemm8w_set(-2, prev[1])


def _rand(M, N, scale=1.0, dtype=torch.bfloat16, g=None):
    return ((torch.rand(M, N, device=DEV, generator=g) * 2 - 1) * scale).to(dtype)


SHAPES = [(32768, 3072, 768), (4096, 768, 3072), (1000, 776, 384), (300, 200, 256), (8192, 2304, 1024)]


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_fc1_gelu_drop_bit_exact_vs_split(M, N, K, p, form):
    from unified_video_action_amd.native import ops
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x, w = _rand(M, K, g=g), _rand(N, K, 0.1, g=g)
    b = torch.rand(N, device=DEV, generator=g) * 0.2 - 0.1
    pre_s, a_s = torch.empty(M, N, device=DEV, dtype=torch.bfloat16), torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.linear(x, w, pre_s, bias=b)
    ops.act_drop_fwd(pre_s, a_s, "gelu", drop_p=p, seed=1234)
    pre_f = torch.full_like(pre_s, float("nan"))
    a_f = torch.full_like(a_s, float("nan"))
    assert ops.linear_gelu_drop(x, w, b, pre_f, a_f, drop_p=p, seed=1234)
    assert torch.equal(pre_f, pre_s)
    assert torch.equal(a_f, a_s)
    if p > 0:
        frac = (a_f == 0).float().mean().item()
        assert abs(frac - p) < 0.02, frac


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("M,N,K", [(32768, 768, 3072), (32768, 768, 768), (1000, 776, 384), (300, 200, 256)])
def test_fc2_drop_residual_bit_exact_vs_split(M, N, K, p, form):
    from unified_video_action_amd.native import ops
    g = torch.Generator(device=DEV).manual_seed(7 * M + N + K)
    h, w = _rand(M, K, g=g), _rand(N, K, 0.05, g=g)
    b = torch.rand(N, device=DEV, generator=g) * 0.2
    res = torch.randn(M, N, device=DEV, generator=g)
    t = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    out_s = torch.empty(M, N, device=DEV)
    ops.linear(h, w, t, bias=b)
    ops.act_drop_fwd(t, out_s, "none", drop_p=p, seed=99, residual=res)
    out_f = torch.full_like(out_s, float("nan"))
    assert ops.linear_drop_res(h, w, b, res, out_f, drop_p=p, seed=99)
    assert torch.equal(out_f, out_s)


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("M,N,K", [(32768, 3072, 768), (1000, 776, 384), (300, 200, 256)])
def test_dgelu_drop_bit_exact_vs_split(M, N, K, p, form):
    """fc2's dX product with dropout + GELU' in the epilogue and the fc1 bias gradient as column partials"""
    from unified_video_action_amd.native import ops
    g = torch.Generator(device=DEV).manual_seed(3 * M + N + K)
    dy, wt = (torch.randn(M, K, device=DEV, generator=g) * 0.1).to(torch.bfloat16), _rand(N, K, 0.05, g=g)
    pre = (torch.randn(M, N, device=DEV, generator=g) * 1.5).to(torch.bfloat16)
    da = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    dp_s = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    db_s = torch.full((N,), 0.5, device=DEV)
    ops.linear(dy, wt, da)
    ops.act_bwd_bias(pre, da, dp_s, db_s, "gelu", drop_p=p, seed=4321)
    dp_f = torch.full_like(dp_s, float("nan"))
    db_f = torch.full((N,), 0.5, device=DEV)
    assert ops.linear_dgelu_drop(dy, wt, pre, dp_f, db_f, drop_p=p, seed=4321)
    ne = (dp_f != dp_s).nonzero()
    assert len(ne) == 0, (len(ne), ne[:4].tolist(), dp_f.isnan().sum().item(),
                          [(dp_f[r, c].item(), dp_s[r, c].item(), pre[r, c].item()) for r, c in ne[:4].tolist()])
    want = dp_f.double().sum(0) + 0.5
    scale = want.abs().max().item()
    assert (db_f.double() - want).abs().max().item() < 1e-5 * scale
    assert (db_f - db_s).abs().max().item() < 1e-5 * scale


@pytest.mark.parametrize("mode", [0, 2 | (4 << 2), 32])
@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K", SHAPES + [(32768, 768, 768)])
def test_plain_8w_bit_exact_vs_gemm4(M, N, K, odt, mode):
    """the plain product on the 8-wave kernel (64 x 96 immediate / 64 x 64 with all rows deferred into the next
    tile) vs the 4-wave kernel: the same per-output fp32 accumulation order -> the same bits"""
    from unified_video_action_amd.native import ops
    g = torch.Generator(device=DEV).manual_seed(M * 3 + N + K)
    x, w = _rand(M, K, g=g), _rand(N, K, g=g)
    b = torch.randn(N, device=DEV, generator=g)
    y4 = torch.empty(M, N, device=DEV, dtype=odt)
    ops.gemm8w_set(0, 0)
    ops.linear(x, w, y4, bias=b)
    y8 = torch.full((M, N), float("nan"), device=DEV, dtype=odt)
    try:
        ops.gemm8w_set(1, mode)
        ops.linear(x, w, y8, bias=b)
    finally:
        ops.gemm8w_set(0, 0)
    assert torch.equal(y8, y4)


def test_block_fused_routes_match_split_routes():
    """two chained timm Blocks (BlockFn) at a bench-geometry slice (B 4, N 1024, D 768, H 12, dropout 0.1) forward +
    backward with the fused routes (RT defaults: Mlp epilogues on the 8-wave GEMM, norm2 backward emitting the
    proj_drop backward, the second Block's norm1 backward emitting the first Block's fc2 dropout backward) and
    with the split routes, same seeds: output and every gradient bit-identical, the three bias gradients the
    fused routes sum in another order (fc1 / proj / fc2 bias) within 1e-5"""
    import copy
    from functools import partial

    import torch.nn as nn

    from unified_video_action_amd.model.autoregressive import functional as Fn
    from unified_video_action_amd.model.autoregressive.mar_con_unified import Block
    from unified_video_action_amd.runtime import RT

    RT.set_precision("bf16")
    torch.manual_seed(0)
    blocks = []
    for _ in range(2):
        blk = Block(768, 12, 4.0, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6), proj_drop=0.1,
                    attn_drop=0.1).to(DEV).train()
        with torch.no_grad():
            for n, p in blk.named_parameters():
                if n.endswith("bias") or "norm" in n:
                    p.add_(torch.randn_like(p) * 0.05)  # non-trivial biases / LayerNorm affines
        blocks.append(blk)
    B, N = 4, 1024
    x0 = torch.randn(B, N, 768, device=DEV)
    gy = torch.randn(B, N, 768, device=DEV)
    out = {}
    for split in (False, True):
        ms = [copy.deepcopy(b) for b in blocks]
        RT.mlp_split_epilogue, RT.act_bwd_in_gemm, RT.ln_bwd_drop = split, not split, not split
        RT.begin_forward()
        RT.seed(77)
        x = x0.clone().requires_grad_(True)
        y = Fn.block_forward(ms[1], Fn.block_forward(ms[0], x, B, N, 0.1, 0.1), B, N, 0.1, 0.1)
        y.backward(gy)
        torch.cuda.synchronize()
        out[split] = (y.detach(), x.grad, {f"{i}.{n}": p.grad.clone() for i, m in enumerate(ms)
                                           for n, p in m.named_parameters()})
    RT.mlp_split_epilogue, RT.act_bwd_in_gemm, RT.ln_bwd_drop = False, True, True
    (yf, gxf, gf), (ys, gxs, gs) = out[False], out[True]
    assert torch.equal(yf, ys)
    assert torch.equal(gxf, gxs)
    for n in gs:
        if n.endswith(("mlp.fc1.bias", "attn.proj.bias", "mlp.fc2.bias")):
            assert (gf[n] - gs[n]).abs().max().item() <= 1e-5 * gs[n].abs().max().item(), n
        else:
            assert torch.equal(gf[n], gs[n]), n


@pytest.mark.parametrize("n", [32 * 1000, 32768 * 768, 70])
def test_dropout_plane_matches_counter_hash(n):
    """keep-bit plane (uva_dropout_plane) == the mask act_drop_fwd applies (flat index, same seed)"""
    from unified_video_action_amd.native import ops
    p, seed = 0.1, 0xABCDEF12345
    plane = ops.dropout_plane(n, p, seed, DEV)
    ones = torch.ones(((n + 7) // 8) * 8, device=DEV, dtype=torch.bfloat16)
    y = torch.empty_like(ones)
    ops.act_drop_fwd(ones, y, "none", drop_p=p, seed=seed)
    keep = (y[:n] != 0)
    bits = ((plane.view(-1, 1) >> torch.arange(32, device=DEV, dtype=torch.int32).view(1, 32)) & 1).reshape(-1)[:n]
    assert torch.equal(bits.bool(), keep)


@pytest.mark.parametrize("which", ["fc1", "fc2", "dgelu"])
@pytest.mark.parametrize("M,N,K", [(32768, 3072, 768), (1000, 768, 384)])
def test_fused_with_plane_bit_exact_vs_hash(which, M, N, K):
    """the fused epilogues reading a precomputed keep-bit plane give the same bits as evaluating the hash"""
    from unified_video_action_amd.native import ops
    p, seed = 0.1, 4242
    g = torch.Generator(device=DEV).manual_seed(M + N)
    plane = ops.dropout_plane(M * N, p, seed, DEV)
    if which == "fc1":
        x, w = _rand(M, K, g=g), _rand(N, K, 0.1, g=g)
        b = torch.rand(N, device=DEV, generator=g) * 0.1
        pa, aa = torch.empty(M, N, device=DEV, dtype=torch.bfloat16), torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        pb, ab = torch.empty_like(pa), torch.empty_like(aa)
        assert ops.linear_gelu_drop(x, w, b, pa, aa, drop_p=p, seed=seed)
        assert ops.linear_gelu_drop(x, w, b, pb, ab, drop_p=p, seed=seed, plane=plane)
        assert torch.equal(pa, pb) and torch.equal(aa, ab)
    elif which == "fc2":
        x, w = _rand(M, K, g=g), _rand(N, K, 0.1, g=g)
        b = torch.rand(N, device=DEV, generator=g) * 0.1
        r = torch.randn(M, N, device=DEV, generator=g)
        oa, ob = torch.empty(M, N, device=DEV), torch.empty(M, N, device=DEV)
        assert ops.linear_drop_res(x, w, b, r, oa, drop_p=p, seed=seed)
        assert ops.linear_drop_res(x, w, b, r, ob, drop_p=p, seed=seed, plane=plane)
        assert torch.equal(oa, ob)
    else:
        dy, wt = (torch.randn(M, K, device=DEV, generator=g) * 0.1).to(torch.bfloat16), _rand(N, K, 0.05, g=g)
        pre = (torch.randn(M, N, device=DEV, generator=g) * 1.5).to(torch.bfloat16)
        da, db = torch.empty(M, N, device=DEV, dtype=torch.bfloat16), torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ga, gb = torch.zeros(N, device=DEV), torch.zeros(N, device=DEV)
        assert ops.linear_dgelu_drop(dy, wt, pre, da, ga, drop_p=p, seed=seed)
        assert ops.linear_dgelu_drop(dy, wt, pre, db, gb, drop_p=p, seed=seed, plane=plane)
        assert torch.equal(da, db) and torch.equal(ga, gb)


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("rows", [32768, 1000])
def test_layernorm_bwd_drop_matches_two_pass(rows, p):
    """norm2 backward with the proj_drop backward + proj bias gradient in the same pass (uva_layernorm_bwd_drop)
    vs layernorm_bwd then act_bwd_bias(none): dx, dropout output, LN dw / db bit-identical; the proj bias sum
    within 1e-5 (another summation order)"""
    from unified_video_action_amd.native import ops
    D = 768
    g = torch.Generator(device=DEV).manual_seed(rows)
    x = torch.randn(rows, D, device=DEV, generator=g)
    w = torch.rand(D, device=DEV, generator=g) + 0.5
    dy = (torch.randn(rows, D, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    base = torch.randn(rows, D, device=DEV, generator=g) * 0.1
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-6)
    res = []
    for fused in (True, False):
        dx = torch.empty(rows, D, device=DEV)
        dw, db, dbias = torch.full((D,), 0.25, device=DEV), torch.full((D,), 0.5, device=DEV), torch.full((D,), 1.0, device=DEV)
        out = torch.empty(rows, D, device=DEV, dtype=torch.bfloat16)
        if fused:
            assert ops.layernorm_bwd_drop(x, w, dy, mean, rstd, dx, dw, db, base, out, p, 99, dbias)
        else:
            ops.layernorm_bwd(x, w, dy, mean, rstd, dx, accum=False, dw=dw, db=db, dx_base=base)
            ops.act_bwd_bias(None, dx, out, dbias, "none", drop_p=p, seed=99)
        torch.cuda.synchronize()
        res.append((dx, out, dw, db, dbias))
    (a, b) = res
    for i in range(4):
        assert torch.equal(a[i], b[i]), i
    assert (a[4] - b[4]).abs().max().item() <= 1e-5 * b[4].abs().max().item()


@pytest.mark.parametrize("beta", [0.0, 1.0])
@pytest.mark.parametrize("M,N,K", [(768, 768, 32768), (2304, 768, 32768), (3072, 768, 32768), (768, 3072, 8192),
                                   (1000, 776, 1024), (256, 192, 256)])
def test_dw_8w_tt_vs_routes(M, N, K, beta):
    """the dW products (dw[M,N] (+)= dy[K,M]^T x[K,N], k-major operands) on gemm_8w (mode bit 7): bit-identical to
    gemm_4w's split-K form where that one takes the shape (the same plan, the same per-slice k order, the same
    slab reduce), and within 2e-6 of an fp64 product everywhere (fp32 accumulation over K)"""
    from unified_video_action_amd.native import ops
    g = torch.Generator(device=DEV).manual_seed(M + 7 * N + K)
    dy, x = _rand(K, M, g=g), _rand(K, N, g=g)
    init = torch.randn(M, N, device=DEV, generator=g)
    want = dy.double().t() @ x.double() + beta * init.double()
    prev = ops.gemm8w_set(-2, 128)
    try:
        d8 = init.clone()
        ops.linear_dw(dy, x, d8, beta=beta)
    finally:
        ops.gemm8w_set(-2, prev[1])
    d4 = init.clone()
    ops.linear_dw(dy, x, d4, beta=beta)  # gemm_4w (few tiles) or gemm_8ph
    torch.cuda.synchronize()
    scale = want.abs().max().item()
    assert (d8.double() - want).abs().max().item() < 2e-6 * scale * max(1.0, K / 8192)
    tiles = ((M + 255) // 256) * ((N + 191) // 192)
    if tiles <= 16 and K % 128 == 0 and K >= 256 and M >= 256 and N >= 192:
        assert torch.equal(d8, d4)
