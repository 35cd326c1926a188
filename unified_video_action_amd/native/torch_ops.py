"""`torch.library` custom ops (namespace `uva`) over libuva_hip.so -- the op-level face of the
drop-in boundary (every hot-path op a custom op with a registered autograd formula
and a fake (meta) kernel, each calling the C ABI declared in include/uva_hip.h).

The training step itself runs the fused autograd Functions of model/autoregressive/functional.py
(one autograd node per timm Block / diffusion trunk, parameter gradients accumulated straight into
the optimizer's flat buffer by the GEMM epilogues).  These ops expose the same kernels
functionally -- fresh outputs, gradients returned, no flat-buffer side effects -- for code that
composes its own modules, for FakeTensor / torch.compile shape propagation (the fake kernels run
without a GPU) and for op-level parity tests (tests/test_torch_ops_cpu.py, tests/test_torch_ops_gpu.py).

  uva::layer_norm(x, weight?, bias?, eps) -> (y, mean, rstd)
      nn.LayerNorm (timm Block norm1 / norm2, encoder/decoder norms: mar_con_unified.py:198-249);
      y in x's dtype (fp32 or bf16), statistics fp32.
  uva::linear(x, weight, bias?, act, drop_p, seed) -> (y, pre)
      y = dropout(act(x @ weight^T + bias)) -- nn.Linear with the epilogues of timm Mlp / Attention.proj
      (act "none" | "gelu" | "silu" | "relu"; pre = the pre-activation, empty when act is "none").
  uva::attention(qkv, heads, drop_p, seed) -> (out, lse)
      F.scaled_dot_product_attention of timm Attention (mar_con_unified.py:201-215): qkv [B, N, 3*H*64]
      bf16 as the qkv Linear writes it, out [B, N, H*64], lse [B, H, N] (base-2 log-sum-exp).
  uva::conv3x3(x, weight, bias?, gn_scale?, gn_shift?, residual?) -> y
      KL-VAE ResnetBlock conv over NHWC bf16 with the GroupNorm-apply + SiLU prologue and the residual
      add fused (vaekl.py:56-113); forward only (the VAE is frozen on the training path).
Backward ops: uva::layer_norm_backward, uva::linear_backward, uva::attention_backward.
Dropout masks are the library's counter hash of (seed, element): the backward regenerates the
forward's mask from the same seed.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import ops

F32 = torch.float32
_ACTS = ("none", "gelu", "silu", "relu")


# ---- layer norm -------------------------------------------------------------------------------
@torch.library.custom_op("uva::layer_norm", mutates_args=(), device_types="cuda")
def layer_norm(x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor], eps: float) -> Tuple[Tensor, Tensor, Tensor]:
    D = x.shape[-1]
    x2 = x.contiguous().view(-1, D)
    M = x2.shape[0]
    y = torch.empty_like(x2)
    mean = torch.empty(M, dtype=F32, device=x.device)
    rstd = torch.empty(M, dtype=F32, device=x.device)
    ops.layernorm_fwd(x2, weight, bias, y, mean, rstd, eps)
    return y.view(x.shape), mean, rstd


@layer_norm.register_fake
def _layer_norm_fake(x, weight, bias, eps):
    M = x.numel() // x.shape[-1]
    return torch.empty_like(x), x.new_empty(M, dtype=F32), x.new_empty(M, dtype=F32)


@torch.library.custom_op("uva::layer_norm_backward", mutates_args=(), device_types="cuda")
def layer_norm_backward(x: Tensor, weight: Optional[Tensor], dy: Tensor, mean: Tensor,
                        rstd: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """-> (dx in x's dtype, dweight [D] fp32, dbias [D] fp32); dweight / dbias are zeros when the
    norm has no affine parameters."""
    D = x.shape[-1]
    x2 = x.contiguous().view(-1, D)
    dy2 = dy.contiguous().view(-1, D)
    if dy2.dtype not in (F32, torch.bfloat16):
        dy2 = dy2.float()
    dx = torch.empty(x2.shape, dtype=F32, device=x.device)
    dw = torch.zeros(D, dtype=F32, device=x.device)
    db = torch.zeros(D, dtype=F32, device=x.device)
    affine = weight is not None
    ops.layernorm_bwd(x2, weight, dy2, mean, rstd, dx, accum=False, dw=dw if affine else None,
                      db=db if affine else None)
    return dx.to(x.dtype).view(x.shape), dw, db


@layer_norm_backward.register_fake
def _layer_norm_backward_fake(x, weight, dy, mean, rstd):
    D = x.shape[-1]
    return torch.empty_like(x), x.new_empty(D, dtype=F32), x.new_empty(D, dtype=F32)


def _ln_setup(ctx, inputs, output):
    x, weight, bias, _ = inputs
    _, mean, rstd = output
    ctx.save_for_backward(x, weight, mean, rstd)
    ctx.wdt = None if weight is None else weight.dtype
    ctx.bdt = None if bias is None else bias.dtype


def _ln_backward(ctx, dy, _dmean, _drstd):
    x, weight, mean, rstd = ctx.saved_tensors
    dx, dw, db = layer_norm_backward(x, weight, dy, mean, rstd)
    return (dx, None if ctx.wdt is None else dw.to(ctx.wdt), None if ctx.bdt is None else db.to(ctx.bdt), None)


layer_norm.register_autograd(_ln_backward, setup_context=_ln_setup)


# ---- linear (+ activation + dropout epilogue) -------------------------------------------------
def _check_act(act: str):
    if act not in _ACTS:
        raise ValueError(f"uva::linear: act must be one of {_ACTS}, got {act!r}")


@torch.library.custom_op("uva::linear", mutates_args=(), device_types="cuda")
def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor], act: str, drop_p: float,
           seed: int) -> Tuple[Tensor, Tensor]:
    _check_act(act)
    K = x.shape[-1]
    N = weight.shape[0]
    x2 = x.contiguous().view(-1, K)
    w = weight.to(x.dtype).contiguous()
    y = torch.empty(x2.shape[0], N, dtype=x.dtype, device=x.device)
    pre = torch.empty(x2.shape[0], N, dtype=x.dtype, device=x.device) if act != "none" else x.new_empty(0)
    ops.linear(x2, w, y, bias=None if bias is None else bias.float().contiguous(), act=act,
               aux=pre if act != "none" else None, drop_p=drop_p, seed=seed)
    return y.view(*x.shape[:-1], N), pre


@linear.register_fake
def _linear_fake(x, weight, bias, act, drop_p, seed):
    _check_act(act)
    N = weight.shape[0]
    M = x.numel() // x.shape[-1]
    pre = x.new_empty(M, N) if act != "none" else x.new_empty(0)
    return x.new_empty(*x.shape[:-1], N), pre


@torch.library.custom_op("uva::linear_backward", mutates_args=(), device_types="cuda")
def linear_backward(dy: Tensor, x: Tensor, weight: Tensor, pre: Tensor, act: str, drop_p: float,
                    seed: int) -> Tuple[Tensor, Tensor, Tensor]:
    """-> (dx in x's dtype, dweight in weight's dtype, dbias [N] fp32)."""
    _check_act(act)
    K = x.shape[-1]
    N = weight.shape[0]
    x2 = x.contiguous().view(-1, K)
    w = weight.to(x.dtype).contiguous()
    g = dy.contiguous().view(-1, N)
    M = g.shape[0]
    if act != "none" or drop_p > 0:
        dpre = torch.empty(M, N, dtype=x.dtype, device=x.device)
        ops.act_bwd(pre if act != "none" else None, g, dpre, act, drop_p=drop_p, seed=seed)
    else:
        dpre = g.to(x.dtype).contiguous()
    dx = torch.empty(M, K, dtype=F32, device=x.device)
    ops.linear_dx(dpre, w, dx)
    dw = torch.zeros(N, K, dtype=F32, device=x.device)
    ops.linear_dw(dpre, x2, dw, beta=0.0)
    db = torch.zeros(N, dtype=F32, device=x.device)
    ops.colsum(dpre, db, accum=False)
    return dx.to(x.dtype).view(x.shape), dw.to(weight.dtype), db


@linear_backward.register_fake
def _linear_backward_fake(dy, x, weight, pre, act, drop_p, seed):
    _check_act(act)
    return torch.empty_like(x), torch.empty_like(weight), x.new_empty(weight.shape[0], dtype=F32)


def _lin_setup(ctx, inputs, output):
    x, weight, bias, act, drop_p, seed = inputs
    _, pre = output
    ctx.save_for_backward(x, weight, pre)
    ctx.cfg = (act, drop_p, seed, None if bias is None else bias.dtype)


def _lin_backward(ctx, dy, _dpre):
    x, weight, pre = ctx.saved_tensors
    act, drop_p, seed, bdt = ctx.cfg
    dx, dw, db = linear_backward(dy, x, weight, pre, act, drop_p, seed)
    return dx, dw, (None if bdt is None else db.to(bdt)), None, None, None


linear.register_autograd(_lin_backward, setup_context=_lin_setup)


# ---- attention ---------------------------------------------------------------------------------
def _attn_dims(qkv: Tensor, heads: int):
    if qkv.dim() != 3 or qkv.shape[-1] != 3 * heads * 64:
        raise ValueError(f"uva::attention: qkv must be [B, N, 3*heads*64], got {tuple(qkv.shape)} for {heads} heads")
    B, N = qkv.shape[0], qkv.shape[1]
    if N % 64:
        raise ValueError(f"uva::attention: N = {N} must be a multiple of 64")
    return B, N


@torch.library.custom_op("uva::attention", mutates_args=(), device_types="cuda")
def attention(qkv: Tensor, heads: int, drop_p: float, seed: int) -> Tuple[Tensor, Tensor]:
    B, N = _attn_dims(qkv, heads)
    q = qkv.to(torch.bfloat16).contiguous()
    out = torch.empty(B, N, heads * 64, dtype=torch.bfloat16, device=qkv.device)
    lse = torch.empty(B, heads, N, dtype=F32, device=qkv.device)
    ops.attn_fwd(q, out, lse, B, N, heads, 64 ** -0.5, drop_p=drop_p, seed=seed)
    return out, lse


@attention.register_fake
def _attention_fake(qkv, heads, drop_p, seed):
    B, N = _attn_dims(qkv, heads)
    return qkv.new_empty(B, N, heads * 64, dtype=torch.bfloat16), qkv.new_empty(B, heads, N, dtype=F32)


@torch.library.custom_op("uva::attention_backward", mutates_args=(), device_types="cuda")
def attention_backward(dout: Tensor, qkv: Tensor, out: Tensor, lse: Tensor, heads: int, drop_p: float,
                       seed: int) -> Tensor:
    B, N = _attn_dims(qkv, heads)
    q = qkv.to(torch.bfloat16).contiguous()
    dqkv = torch.empty(q.shape, dtype=torch.bfloat16, device=qkv.device)
    dvec = torch.empty(B, heads, N, dtype=F32, device=qkv.device)
    ops.attn_bwd(q, out.contiguous(), dout.to(torch.bfloat16).contiguous(), lse, dvec, dqkv, B, N, heads,
                 64 ** -0.5, drop_p=drop_p, seed=seed)
    return dqkv.to(qkv.dtype)


@attention_backward.register_fake
def _attention_backward_fake(dout, qkv, out, lse, heads, drop_p, seed):
    return torch.empty_like(qkv)


def _attn_setup(ctx, inputs, output):
    qkv, heads, drop_p, seed = inputs
    out, lse = output
    ctx.save_for_backward(qkv, out, lse)
    ctx.cfg = (heads, drop_p, seed)


def _attn_backward(ctx, dout, _dlse):
    qkv, out, lse = ctx.saved_tensors
    heads, drop_p, seed = ctx.cfg
    return attention_backward(dout, qkv, out, lse, heads, drop_p, seed), None, None, None


attention.register_autograd(_attn_backward, setup_context=_attn_setup)


# ---- VAE 3x3 convolution (forward only) --------------------------------------------------------
@torch.library.custom_op("uva::conv3x3", mutates_args=(), device_types="cuda")
def conv3x3(x: Tensor, weight: Tensor, bias: Optional[Tensor], gn_scale: Optional[Tensor],
            gn_shift: Optional[Tensor], residual: Optional[Tensor]) -> Tensor:
    """x NHWC bf16 [n, H, W, Ci], weight [Co, 3, 3, Ci] bf16, bias [Co] fp32; gn_scale / gn_shift
    [n, Ci] fp32 apply silu(x * scale + shift) to the input first (zero padding after it, as
    F.conv2d of the activated tensor); residual [n, H, W, Co] bf16 is added to the output."""
    n, H, W, Ci = x.shape
    Co = weight.shape[0]
    out = torch.empty(n, H, W, Co, dtype=x.dtype, device=x.device)
    ops.conv2d(x.contiguous(), weight.contiguous(), out, n, H, W, Ci, Co, 3, 1, 1, 1, H, W,
               bias=None if bias is None else bias.float().contiguous(),
               residual=None if residual is None else residual.contiguous(),
               gn_scale=gn_scale, gn_shift=gn_shift, gn_silu=True)
    return out


@conv3x3.register_fake
def _conv3x3_fake(x, weight, bias, gn_scale, gn_shift, residual):
    n, H, W, _ = x.shape
    return x.new_empty(n, H, W, weight.shape[0])
