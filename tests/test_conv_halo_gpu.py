"""Direct 3x3 halo-tile convolution (csrc/conv.hip) against a plain PyTorch fp32 reference of the
same op: out = bias + residual + conv3x3(silu(x * scale + shift)) over NHWC bf16, zero padding
applied after the activation (F.conv2d of the activated tensor, vaekl.py:94-104), and the fused
per-128-pixel GroupNorm(32) partial sums of the stored output.  Tolerance: bf16 operands against
an fp32 reference on the SAME bf16-rounded activated input -> 1e-2 relative to the output scale;
GroupNorm scale/shift from the fused partials 1e-4."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


@pytest.mark.parametrize("n,H,W,Ci,Co", [(4, 32, 32, 128, 128), (2, 16, 16, 256, 512), (2, 64, 32, 64, 256),
                                         (1, 48, 16, 192, 128),
                                         # Ci = Co = 128 with GN and no residual: the persistent conv3x3_gn_pt
                                         # (two workgroups per CU walk 8 x 16 tiles); with a residual: the
                                         # single-tile conv3x3_halo (the strip form is compile-time off).
                                         # 6 / 30 tiles, and 640 tiles = 1.25 rounds of 2 x 256 CUs (the
                                         # persistent loop's last partial round)
                                         (3, 16, 16, 128, 128), (2, 80, 48, 128, 128), (5, 128, 128, 128, 128)])
@pytest.mark.parametrize("gn", [False, True])
@pytest.mark.parametrize("residual", [False, True])
def test_conv_halo_matches_torch(n, H, W, Ci, Co, gn, residual):
    from unified_video_action_amd.native import ops
    torch.manual_seed(n * 1000 + H + Ci + Co + int(gn) * 7 + int(residual))
    assert ops.conv_fuses_gn(n, H, W, Ci, Co, 3, 1)
    x = torch.randn(n, H, W, Ci, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Co, 3, 3, Ci, device=DEV) * 0.05).to(torch.bfloat16)
    bias = torch.randn(Co, device=DEV) * 0.1
    sc = (torch.rand(n, Ci, device=DEV) + 0.5) if gn else None
    sh = (torch.randn(n, Ci, device=DEV) * 0.3) if gn else None
    res = torch.randn(n, H, W, Co, device=DEV).to(torch.bfloat16) if residual else None
    out = torch.empty(n, H, W, Co, device=DEV, dtype=torch.bfloat16)
    part = torch.empty(n * H * W // 128, 32, 2, device=DEV)
    ops.conv2d(x, w, out, n, H, W, Ci, Co, 3, 1, 1, 1, H, W, bias=bias, residual=res, gn_scale=sc, gn_shift=sh,
               gn_silu=True, gn_part=part)
    a = x.float()
    if gn:
        a = F.silu(a * sc[:, None, None, :] + sh[:, None, None, :]).to(torch.bfloat16).float()
    ref = F.conv2d(a.permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias, padding=1).permute(0, 2, 3, 1)
    if residual:
        ref = ref + res.float()
    assert rel_err(out.float(), ref) < 1e-2
    # fused GroupNorm partials of the stored output -> finalize == GroupNorm statistics of `out`
    gamma = torch.randn(Co, device=DEV)
    beta = torch.randn(Co, device=DEV)
    gsc = torch.empty(n, Co, device=DEV)
    gsh = torch.empty(n, Co, device=DEV)
    ops.groupnorm_finalize_tiles(part, n, H * W, Co, gamma, beta, gsc, gsh, eps=1e-6)
    o = out.double().reshape(n, H * W, 32, Co // 32)
    mean = o.mean(dim=(1, 3))
    var = o.var(dim=(1, 3), unbiased=False)
    rstd = (var + 1e-6).rsqrt()
    sc_ref = gamma.double()[None] * rstd.repeat_interleave(Co // 32, dim=1)
    sh_ref = beta.double()[None] - mean.repeat_interleave(Co // 32, dim=1) * sc_ref
    assert rel_err(gsc, sc_ref) < 1e-4
    assert rel_err(gsh, sh_ref) < 1e-4


@pytest.mark.parametrize("n,H,W,Ci,Co", [(3, 16, 16, 128, 128), (2, 32, 32, 256, 256)])
@pytest.mark.parametrize("residual", [False, True])
def test_conv_halo_gn_without_silu(n, H, W, Ci, Co, residual):
    """GroupNorm prologue with gn_silu = 0 (the compile-time no-SiLU instantiations of the persistent and
    single-tile GN kernels): out = bias + residual + conv3x3(x * scale + shift)."""
    from unified_video_action_amd.native import ops
    torch.manual_seed(n + H + Ci + int(residual))
    x = torch.randn(n, H, W, Ci, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Co, 3, 3, Ci, device=DEV) * 0.05).to(torch.bfloat16)
    bias = torch.randn(Co, device=DEV) * 0.1
    sc = torch.rand(n, Ci, device=DEV) + 0.5
    sh = torch.randn(n, Ci, device=DEV) * 0.3
    res = torch.randn(n, H, W, Co, device=DEV).to(torch.bfloat16) if residual else None
    out = torch.empty(n, H, W, Co, device=DEV, dtype=torch.bfloat16)
    ops.conv2d(x, w, out, n, H, W, Ci, Co, 3, 1, 1, 1, H, W, bias=bias, residual=res, gn_scale=sc, gn_shift=sh,
               gn_silu=False)
    a = (x.float() * sc[:, None, None, :] + sh[:, None, None, :]).to(torch.bfloat16).float()
    ref = F.conv2d(a.permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias, padding=1).permute(0, 2, 3, 1)
    if residual:
        ref = ref + res.float()
    assert rel_err(out.float(), ref) < 1e-2


def test_conv_halo_eligibility():
    from unified_video_action_amd.native import ops
    assert ops.conv_fuses_gn(256, 256, 256, 128, 128, 3, 1)
    assert ops.conv_fuses_gn(256, 16, 16, 512, 512, 3, 1)
    assert not ops.conv_fuses_gn(256, 16, 16, 512, 32, 3, 1)    # conv_out: Co % 128
    assert not ops.conv_fuses_gn(256, 256, 256, 8, 128, 3, 1)   # conv_in: Ci % 64
    assert not ops.conv_fuses_gn(256, 256, 256, 128, 128, 3, 2)  # downsample
    assert not ops.conv_fuses_gn(4, 24, 24, 128, 128, 3, 1)     # 16 does not tile 24


@pytest.mark.parametrize("n,H,W", [(3, 32, 48), (1, 256, 256)])
def test_conv_in8_matches_torch(n, H, W):
    """Encoder.conv_in on the 8-channel padded frame (channels 3..7 zero, as uva_resize_select writes)."""
    from unified_video_action_amd.native import ops
    torch.manual_seed(5 + H)
    x = torch.zeros(n, H, W, 8, device=DEV)
    x[..., :3] = torch.rand(n, H, W, 3, device=DEV) * 2 - 1
    x = x.to(torch.bfloat16)
    w = torch.zeros(128, 3, 3, 8, device=DEV)
    w[..., :3] = torch.randn(128, 3, 3, 3, device=DEV) * 0.2
    w = w.to(torch.bfloat16)
    bias = torch.randn(128, device=DEV) * 0.1
    out = torch.empty(n, H, W, 128, device=DEV, dtype=torch.bfloat16)
    part = torch.empty(n * H * W // 128, 32, 2, device=DEV)
    ops.conv2d(x, w, out, n, H, W, 8, 128, 3, 1, 1, 1, H, W, bias=bias, gn_part=part)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias, padding=1).permute(0, 2, 3, 1)
    assert rel_err(out.float(), ref) < 1e-2
    gamma = torch.ones(128, device=DEV)
    beta = torch.zeros(128, device=DEV)
    gsc = torch.empty(n, 128, device=DEV)
    gsh = torch.empty(n, 128, device=DEV)
    ops.groupnorm_finalize_tiles(part, n, H * W, 128, gamma, beta, gsc, gsh, eps=1e-6)
    o = out.double().reshape(n, H * W, 32, 4)
    mean = o.mean(dim=(1, 3))
    rstd = (o.var(dim=(1, 3), unbiased=False) + 1e-6).rsqrt()
    assert rel_err(gsc, rstd.repeat_interleave(4, dim=1)) < 1e-4
    assert rel_err(gsh, -mean.repeat_interleave(4, dim=1) * rstd.repeat_interleave(4, dim=1)) < 1e-4


@pytest.mark.parametrize("n,H,W,Ci,Co", [(2, 32, 32, 128, 128), (1, 64, 32, 256, 256), (3, 16, 64, 64, 128),
                                         (1, 48, 96, 128, 256)])
@pytest.mark.parametrize("gn", [False, True])
def test_conv_s2_halo_matches_torch(n, H, W, Ci, Co, gn):
    """Downsample (vaekl.py Downsample with_conv): F.pad(x, (0, 1, 0, 1)) + 3x3 / stride 2 / pad 0,
    routed by uva_conv2d to the stride-2 halo kernel; also checked against the implicit-GEMM route."""
    from unified_video_action_amd.native import ops
    from unified_video_action_amd.native.lib import lib
    torch.manual_seed(3 * n + H + W + Ci + Co)
    assert lib().query("uva_conv3x3s2_ok", n, H, W, Ci, Co) > 0
    x = torch.randn(n, H, W, Ci, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Co, 3, 3, Ci, device=DEV) * 0.05).to(torch.bfloat16)
    bias = torch.randn(Co, device=DEV) * 0.1
    Ho, Wo = H // 2, W // 2
    out = torch.empty(n, Ho, Wo, Co, device=DEV, dtype=torch.bfloat16)
    part = torch.empty(n * Ho * Wo // 128, 32, 2, device=DEV) if gn else None
    ops.conv2d(x, w, out, n, H, W, Ci, Co, 3, 2, 0, 0, Ho, Wo, bias=bias, gn_part=part)
    xp = F.pad(x.float().permute(0, 3, 1, 2), (0, 1, 0, 1))
    ref = F.conv2d(xp, w.float().permute(0, 3, 1, 2), bias, stride=2).permute(0, 2, 3, 1)
    assert rel_err(out.float(), ref) < 1e-2
    gen = torch.empty_like(out)
    ops.conv2d(x, w, gen, n, H, W, Ci, Co, 3, 2, 0, 0, Ho, Wo, bias=bias, force_generic=True)
    assert rel_err(out.float(), gen.float()) < 1e-2
    if gn:
        gamma = torch.randn(Co, device=DEV)
        beta = torch.randn(Co, device=DEV)
        gsc = torch.empty(n, Co, device=DEV)
        gsh = torch.empty(n, Co, device=DEV)
        ops.groupnorm_finalize_tiles(part, n, Ho * Wo, Co, gamma, beta, gsc, gsh, eps=1e-6)
        o = out.double().reshape(n, Ho * Wo, 32, Co // 32)
        mean = o.mean(dim=(1, 3))
        rstd = (o.var(dim=(1, 3), unbiased=False) + 1e-6).rsqrt()
        sc_ref = gamma.double()[None] * rstd.repeat_interleave(Co // 32, dim=1)
        sh_ref = beta.double()[None] - mean.repeat_interleave(Co // 32, dim=1) * sc_ref
        assert rel_err(gsc, sc_ref) < 1e-4
        assert rel_err(gsh, sh_ref) < 1e-4


def test_conv_s2_halo_eligibility():
    from unified_video_action_amd.native.lib import lib
    q = lambda *a: lib().query("uva_conv3x3s2_ok", *a) > 0  # noqa: E731
    assert q(256, 256, 256, 128, 128) and q(256, 128, 128, 128, 128)
    assert q(256, 64, 64, 256, 256) and q(256, 32, 32, 256, 256)
    assert not q(4, 24, 32, 128, 128)   # Hin % 16
    assert not q(4, 32, 16, 128, 128)   # Win % 32
    assert not q(4, 32, 32, 32, 128)    # Ci % 64
    assert not q(4, 32, 32, 128, 64)    # Co % 128
