"""The `uva::` torch.library custom ops (native/torch_ops.py) without a GPU: every op is
registered with its schema, and the fake (meta) kernels + registered autograd formulas propagate
shapes / dtypes forward and backward (what FakeTensor / torch.compile tracing relies on)."""
import pytest
import torch

import unified_video_action_amd.native.torch_ops as T

META = "meta"


def test_ops_registered():
    for name in ("layer_norm", "layer_norm_backward", "linear", "linear_backward", "attention",
                 "attention_backward", "conv3x3"):
        assert hasattr(torch.ops.uva, name), name
    assert "Tensor? weight" in str(torch.ops.uva.layer_norm.default._schema)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layer_norm_meta_forward_backward(dtype):
    x = torch.empty(2, 5, 768, device=META, dtype=dtype, requires_grad=True)
    w = torch.empty(768, device=META, requires_grad=True)
    b = torch.empty(768, device=META, requires_grad=True)
    y, mean, rstd = T.layer_norm(x, w, b, 1e-6)
    assert y.shape == x.shape and y.dtype == dtype
    assert mean.shape == (10,) and rstd.dtype == torch.float32
    y.sum().backward()
    assert x.grad.shape == x.shape and x.grad.dtype == dtype
    assert w.grad.shape == (768,) and b.grad.shape == (768,)


def test_linear_meta_forward_backward():
    x = torch.empty(3, 7, 768, device=META, dtype=torch.bfloat16, requires_grad=True)
    w = torch.empty(3072, 768, device=META, dtype=torch.bfloat16, requires_grad=True)
    b = torch.empty(3072, device=META, requires_grad=True)
    y, pre = T.linear(x, w, b, "gelu", 0.1, 7)
    assert y.shape == (3, 7, 3072) and pre.shape == (21, 3072)
    y.float().sum().backward()
    assert x.grad.shape == x.shape and w.grad.shape == w.shape and w.grad.dtype == torch.bfloat16
    assert b.grad.shape == (3072,) and b.grad.dtype == torch.float32
    y2, pre2 = T.linear(x, w, None, "none", 0.0, 0)
    assert pre2.numel() == 0
    with pytest.raises(ValueError):
        T.linear(x, w, b, "tanh", 0.0, 0)


def test_attention_meta_forward_backward():
    qkv = torch.empty(2, 1024, 3 * 12 * 64, device=META, dtype=torch.bfloat16, requires_grad=True)
    out, lse = T.attention(qkv, 12, 0.1, 3)
    assert out.shape == (2, 1024, 768) and lse.shape == (2, 12, 1024) and lse.dtype == torch.float32
    out.float().sum().backward()
    assert qkv.grad.shape == qkv.shape
    with pytest.raises(ValueError):
        T.attention(torch.empty(2, 1000, 2304, device=META, dtype=torch.bfloat16), 12, 0.0, 0)


def test_conv3x3_meta():
    x = torch.empty(2, 32, 32, 128, device=META, dtype=torch.bfloat16)
    w = torch.empty(256, 3, 3, 128, device=META, dtype=torch.bfloat16)
    y = T.conv3x3(x, w, None, None, None, None)
    assert y.shape == (2, 32, 32, 256) and y.dtype == torch.bfloat16
