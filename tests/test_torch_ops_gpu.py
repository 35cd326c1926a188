"""The `uva::` torch.library custom ops on the MI355X against plain PyTorch fp32 references of the
same op (forward and autograd gradients), plus torch.library.opcheck of their registrations.
Tolerances: fp32 1e-4 relative to max; bf16 operands 2e-2 of max (fp32 reference on the same
bf16-rounded inputs)."""
import pytest
import torch
import torch.nn.functional as F

import unified_video_action_amd.native.torch_ops as T

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
def test_layer_norm_matches_torch(dtype, tol):
    torch.manual_seed(0)
    x = torch.randn(3, 100, 768, device=DEV).to(dtype).requires_grad_()
    w = (torch.randn(768, device=DEV) * 0.5 + 1).requires_grad_()
    b = (torch.randn(768, device=DEV) * 0.1).requires_grad_()
    y, mean, rstd = T.layer_norm(x, w, b, 1e-6)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    xr = x.detach().float().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    br = b.detach().clone().requires_grad_()
    yr = F.layer_norm(xr, (768,), wr, br, 1e-6)
    (yr * g.float()).sum().backward()
    assert rel(y, yr) < tol
    assert rel(x.grad, xr.grad) < tol
    assert rel(w.grad, wr.grad) < tol and rel(b.grad, br.grad) < tol
    assert rel(mean, xr.detach().mean(-1).reshape(-1)) < 1e-4


@pytest.mark.parametrize("act", ["none", "gelu", "silu"])
def test_linear_matches_torch(act):
    torch.manual_seed(1)
    x = (torch.randn(512, 768, device=DEV) * 0.5).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(1024, 768, device=DEV) * 0.03).to(torch.bfloat16).requires_grad_()
    b = (torch.randn(1024, device=DEV) * 0.1).requires_grad_()
    y, pre = T.linear(x, w, b, act, 0.0, 0)
    g = torch.randn(512, 1024, device=DEV)
    (y.float() * g).sum().backward()
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = xr @ wr.t() + br
    yr = {"none": lambda t: t, "gelu": F.gelu, "silu": F.silu}[act](yr)
    (yr * g).sum().backward()
    assert rel(y, yr) < 2e-2
    assert rel(x.grad, xr.grad) < 2e-2 and rel(w.grad, wr.grad) < 2e-2 and rel(b.grad, br.grad) < 2e-2


def test_linear_dropout_backward_uses_the_forward_mask():
    torch.manual_seed(2)
    p = 0.25
    x = torch.randn(256, 512, device=DEV).requires_grad_()
    w = (torch.randn(768, 512, device=DEV) * 0.05).requires_grad_()
    y, pre = T.linear(x, w, None, "gelu", p, 12345)
    y2, _ = T.linear(x, w, None, "gelu", p, 12345)
    assert torch.equal(y, y2)  # mask = f(seed, element)
    keep = (y != 0)
    assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    g = torch.randn_like(y)
    (y * g).sum().backward()
    pr = pre.detach().requires_grad_()
    (F.gelu(pr) * g * keep / (1 - p)).sum().backward()
    dx_ref = pr.grad @ w.detach()
    assert rel(x.grad, dx_ref) < 1e-4


def test_attention_matches_sdpa():
    torch.manual_seed(3)
    B, N, H = 2, 256, 4
    qkv = (torch.randn(B, N, 3 * H * 64, device=DEV) * 0.5).to(torch.bfloat16).requires_grad_()
    out, lse = T.attention(qkv, H, 0.0, 0)
    g = torch.randn(B, N, H * 64, device=DEV)
    (out.float() * g).sum().backward()
    qr = qkv.detach().float().requires_grad_()
    q, k, v = qr.view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, N, H * 64)
    (o * g).sum().backward()
    assert rel(out, o) < 2e-2
    assert rel(qkv.grad, qr.grad) < 2e-2


def test_attention_dropout_deterministic_per_seed():
    torch.manual_seed(4)
    qkv = torch.randn(1, 128, 3 * 2 * 64, device=DEV).to(torch.bfloat16)
    a, _ = T.attention(qkv, 2, 0.1, 5)
    b, _ = T.attention(qkv, 2, 0.1, 5)
    c, _ = T.attention(qkv, 2, 0.1, 6)
    assert torch.equal(a, b) and not torch.equal(a, c) and torch.isfinite(a.float()).all()


def test_conv3x3_matches_torch():
    torch.manual_seed(5)
    n, H, W, Ci, Co = 2, 32, 32, 128, 128
    x = torch.randn(n, H, W, Ci, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Co, 3, 3, Ci, device=DEV) * 0.05).to(torch.bfloat16)
    bias = torch.randn(Co, device=DEV) * 0.1
    sc = torch.rand(n, Ci, device=DEV) + 0.5
    sh = torch.randn(n, Ci, device=DEV) * 0.3
    res = torch.randn(n, H, W, Co, device=DEV).to(torch.bfloat16)
    y = T.conv3x3(x, w, bias, sc, sh, res)
    a = F.silu(x.float() * sc[:, None, None, :] + sh[:, None, None, :]).to(torch.bfloat16).float()
    ref = F.conv2d(a.permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias, padding=1).permute(0, 2, 3, 1)
    assert rel(y, ref + res.float()) < 1e-2


def test_opcheck_registrations():
    x = torch.randn(64, 256, device=DEV, requires_grad=True)
    w = torch.randn(256, device=DEV, requires_grad=True)
    b = torch.randn(256, device=DEV, requires_grad=True)
    utils = ("test_schema", "test_faketensor", "test_autograd_registration")
    torch.library.opcheck(torch.ops.uva.layer_norm.default, (x, w, b, 1e-6), test_utils=utils)
    lw = (torch.randn(128, 256, device=DEV) * 0.05).requires_grad_()
    torch.library.opcheck(torch.ops.uva.linear.default, (x, lw, None, "gelu", 0.0, 0), test_utils=utils)
    qkv = torch.randn(1, 128, 3 * 64, device=DEV).to(torch.bfloat16).requires_grad_()
    torch.library.opcheck(torch.ops.uva.attention.default, (qkv, 1, 0.0, 0), test_utils=utils)
