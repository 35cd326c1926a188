"""Persistent 4-wave halo conv (csrc/conv4.hip conv3x3_4w) -- the Ci = Co = 128 3x3 / s1 / p1 convs with
the GroupNorm + SiLU prologue (KL-VAE ResnetBlock conv1 / conv2, vae/vaekl.py:56-113) -- against a
plain PyTorch fp32 reference of the same op on the SAME bf16-rounded activated input (1e-2 of the
output scale: bf16 operands and output), against the two-workgroup halo kernels it replaces (the
route switched off: same bf16 output up to fp32 accumulation order), and its fused GroupNorm(32)
partial sums against the statistics of its own output (1e-4).  Shapes: a single tile, fewer tiles
than CUs, several tiles per workgroup with a partial last round, the level-1 / level-0 production
shapes at reduced image counts, with and without the residual (tiles are 8 x 32 pixels)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def _case(n, H, W, residual, seed):
    torch.manual_seed(seed)
    x = torch.randn(n, H, W, 128, device=DEV).to(torch.bfloat16)
    w = (torch.randn(128, 3, 3, 128, device=DEV) * 0.05).to(torch.bfloat16)
    bias = torch.randn(128, device=DEV) * 0.1
    sc = torch.rand(n, 128, device=DEV) + 0.5
    sh = torch.randn(n, 128, device=DEV) * 0.3
    res = torch.randn(n, H, W, 128, device=DEV).to(torch.bfloat16) if residual else None
    return x, w, bias, sc, sh, res


def _run(x, w, bias, sc, sh, res, n, H, W):
    from unified_video_action_amd.native import ops
    out = torch.full((n, H, W, 128), float("nan"), device=DEV, dtype=torch.bfloat16)
    part = torch.full((n * H * W // 128, 32, 2), float("nan"), device=DEV)
    ops.conv2d(x, w, out, n, H, W, 128, 128, 3, 1, 1, 1, H, W, bias=bias, residual=res, gn_scale=sc, gn_shift=sh,
               gn_silu=True, gn_part=part)
    return out, part


@pytest.mark.parametrize("n,H,W", [(1, 8, 32), (3, 24, 64), (5, 128, 128), (2, 256, 256), (1, 64, 256)])
@pytest.mark.parametrize("residual", [False, True])
def test_conv4_matches_torch_and_stats(n, H, W, residual):
    from unified_video_action_amd.native import ops
    assert ops.conv4_ok(n, H, W, 128, 128)
    x, w, bias, sc, sh, res = _case(n, H, W, residual, n * 100 + H + W + int(residual))
    out, part = _run(x, w, bias, sc, sh, res, n, H, W)
    assert torch.isfinite(out.float()).all()
    a = F.silu(x.float() * sc[:, None, None, :] + sh[:, None, None, :]).to(torch.bfloat16).float()
    ref = F.conv2d(a.permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias, padding=1).permute(0, 2, 3, 1)
    if residual:
        ref = ref + res.float()
    assert rel_err(out.float(), ref) < 1e-2
    gamma = torch.randn(128, device=DEV)
    beta = torch.randn(128, device=DEV)
    gsc = torch.empty(n, 128, device=DEV)
    gsh = torch.empty(n, 128, device=DEV)
    ops.groupnorm_finalize_tiles(part, n, H * W, 128, gamma, beta, gsc, gsh, eps=1e-6)
    o = out.double().reshape(n, H * W, 32, 4)
    mean = o.mean(dim=(1, 3))
    var = o.var(dim=(1, 3), unbiased=False)
    rstd = (var + 1e-6).rsqrt()
    sc_ref = gamma.double()[None] * rstd.repeat_interleave(4, dim=1)
    sh_ref = beta.double()[None] - mean.repeat_interleave(4, dim=1) * sc_ref
    assert rel_err(gsc, sc_ref) < 1e-4
    assert rel_err(gsh, sh_ref) < 1e-4


@pytest.mark.parametrize("residual", [False, True])
def test_conv4_matches_previous_kernels(residual):
    """the 4-wave route and the two-workgroup halo kernels (route off) agree to fp32-accumulation-order
    noise on the bf16 output (<= 1 bf16 ulp of the output scale)"""
    from unified_video_action_amd.native import ops
    n, H, W = 3, 128, 128
    x, w, bias, sc, sh, res = _case(n, H, W, residual, 7 + int(residual))
    o4, p4 = _run(x, w, bias, sc, sh, res, n, H, W)
    prev = ops.conv4_set(0)
    try:
        assert not ops.conv4_ok(n, H, W, 128, 128)
        o8, p8 = _run(x, w, bias, sc, sh, res, n, H, W)
    finally:
        ops.conv4_set(prev)
    assert rel_err(o4.float(), o8.float()) < 8e-3
    # per-image statistics agree (the partial slots are laid out alike: 128-pixel slots per image)
    s4 = p4.reshape(n, -1, 32, 2).double().sum(1)
    s8 = p8.reshape(n, -1, 32, 2).double().sum(1)
    assert rel_err(s4, s8) < 1e-3


def test_conv4_repeatable():
    n, H, W = 2, 256, 256
    x, w, bias, sc, sh, res = _case(n, H, W, True, 3)
    o1, p1 = _run(x, w, bias, sc, sh, res, n, H, W)
    o2, p2 = _run(x, w, bias, sc, sh, res, n, H, W)
    assert torch.equal(o1, o2) and torch.equal(p1, p2)
