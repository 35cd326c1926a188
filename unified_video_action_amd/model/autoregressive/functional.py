"""Autograd functions of the HIP path.  Forward and backward of every heavy op call
libuva_hip.so (native/ops.py); weight/bias gradients are written straight into the
fp32 `param.grad` buffers (views of the flat gradient buffer when a ParamStore owns the
model) by accumulating GEMM epilogues, so autograd never materialises per-parameter
gradient temporaries.

Dtype policy (mirrors the reference's fp16 autocast, with bf16 MFMA operands):
  * GEMM / attention operands in the compute dtype (runtime.RT.compute_dtype),
  * residual streams, LayerNorm statistics, losses and all gradients w.r.t. fp32 tensors
    in fp32,
  * fp32 master weights; compute-dtype shadows maintained by ParamStore.
"""
import math

import torch

from ...native import ops
from ...runtime import RT, cdt

F32 = torch.float32


def as_dtype(t, dtype):
    """Cast through the HIP cast kernel (contiguous result)."""
    if t.dtype == dtype and t.is_contiguous():
        return t
    t = t.contiguous()
    if t.dtype == dtype:
        return t
    out = torch.empty(t.shape, dtype=dtype, device=t.device)
    ops.cast(t, out)
    return out


def compute_weight(p):
    """compute-dtype version of an fp32 master parameter."""
    if cdt() == F32:
        return p.detach()
    sh = getattr(p, "_uva_shadow", None)
    if sh is not None and getattr(p, "_uva_shadow_owner", None) == id(p):
        return sh  # a view of the ParamStore's bf16 buffer, refreshed by the optimizer kernel
    # parameters rewritten by HIP kernels (an EMA model) do not bump _version: key on RT's generation
    key = (p._version, p.data_ptr(), RT.param_gen if getattr(p, "_uva_raw_updated", False) else 0)
    if sh is None or getattr(p, "_uva_shadow_ver", None) != key:
        sh = as_dtype(p.detach(), cdt())
        p._uva_shadow = sh
        p._uva_shadow_ver = key
    return sh


def compute_weight_t(p):
    """transposed compute-dtype copy [in, out] of an fp32 [out, in] weight, rebuilt once per
    parameter generation (the optimizer bumps RT.param_gen): the bf16 dX products run on it as
    forward-layout (K-contiguous) GEMMs.  A copy built ahead on RT's side stream (prefetch_weight_t) is
    waited for on first use."""
    ev = getattr(p, "_uva_t_event", None)
    if ev is not None:
        torch.cuda.current_stream().wait_event(ev)
        p._uva_t_event = None
    w = compute_weight(p)
    key = (p._version, p.data_ptr(), RT.param_gen)
    t = getattr(p, "_uva_shadow_t", None)
    if t is None or getattr(p, "_uva_shadow_t_ver", None) != key:
        if t is None or t.shape != (w.shape[1], w.shape[0]):
            t = torch.empty(w.shape[1], w.shape[0], dtype=w.dtype, device=w.device)
        ops.transpose_bf16(w, t)
        p._uva_shadow_t = t
        p._uva_shadow_t_ver = key
    return t


def prefetch_weight_t(params, side):
    """build this step's transposed bf16 weight copies on the side stream `side` (which already waits for the
    main stream's optimizer step), each with an event its first use waits on: the 4 transposes per Block
    (~5 us each) run under the VAE encode instead of on the backward's critical path"""
    if cdt() != torch.bfloat16:
        return
    todo = []
    for p in params:  # compute shadows (a cast only for parameters no ParamStore owns) and targets on main
        w = compute_weight(p)
        key = (p._version, p.data_ptr(), RT.param_gen)
        if getattr(p, "_uva_shadow_t_ver", None) == key and getattr(p, "_uva_t_event", None) is None:
            continue
        t = getattr(p, "_uva_shadow_t", None)
        if t is None or t.shape != (w.shape[1], w.shape[0]):
            t = torch.empty(w.shape[1], w.shape[0], dtype=w.dtype, device=w.device)  # persistent
            p._uva_shadow_t = t
        todo.append((p, w, t, key))
    side.wait_stream(torch.cuda.current_stream())
    for p, w, t, key in todo:
        with torch.cuda.stream(side):
            ops.transpose_bf16(w, t)
            ev = torch.cuda.Event()
            ev.record(side)
        p._uva_shadow_t_ver = key
        p._uva_t_event = ev


def linear_bias(x, p, b, out):
    """out = x W^T + b for an epilogue-free product (the bf16 ones run on the persistent 4-wave kernel,
    csrc/gemm4.hip)"""
    ops.linear(x, compute_weight(p), out, bias=b.detach())


def linear_dx_w(dy, p, dx):
    """dX = dy @ W of nn.Linear(W: [out, in]).  bf16: through the transposed weight copy as a
    forward-layout GEMM (both operands K-contiguous: the 4-wave kernel); fp32 (parity mode): the
    dX GEMM on the stored weight."""
    if cdt() == torch.bfloat16:
        ops.linear(dy, compute_weight_t(p), dx)
    else:
        ops.linear_dx(dy, compute_weight(p), dx)


def grad_buf(p):
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


def _seed():
    return RT.next_seed()


# --------------------------------------------------------------------------------------
class LinearFn(torch.autograd.Function):
    """out = residual + drop(act(x @ W^T + b))  (nn.Linear + fused epilogue).  A weight with more than two
    dims (a Conv1d [out, in, k] over im2col columns) is the [out, in*k] matrix of its contiguous layout."""

    @staticmethod
    def forward(ctx, x, weight, bias, act, drop_p, out_dtype, residual):
        xc = as_dtype(x, cdt())
        w = compute_weight(weight)
        if w.dim() != 2:
            w = w.reshape(w.shape[0], -1)
        M, N = xc.shape[0], weight.shape[0]
        out = torch.empty(M, N, dtype=out_dtype, device=x.device)
        aux = torch.empty(M, N, dtype=out_dtype, device=x.device) if act != "none" else None
        seed = _seed() if drop_p > 0 else 0
        ops.linear(xc, w, out, bias=None if bias is None else bias.detach(), act=act, aux=aux,
                   residual=residual, drop_p=drop_p, seed=seed)
        ctx.save_for_backward(xc, weight, bias, aux)
        ctx.cfg = (act, drop_p, seed, x.dtype, residual is not None)
        return out

    @staticmethod
    def backward(ctx, g):
        xc, weight, bias, aux = ctx.saved_tensors
        act, drop_p, seed, xdt, has_res = ctx.cfg
        M, N = g.shape
        fused_bias = False
        if act != "none" or drop_p > 0:
            dpre = torch.empty(M, N, dtype=cdt(), device=g.device)
            if bias is not None and N % 8 == 0:
                ops.act_bwd_bias(aux, g.contiguous(), dpre, grad_buf(bias), act, drop_p=drop_p, seed=seed)
                fused_bias = True
            else:
                ops.act_bwd(aux, g.contiguous(), dpre, act, drop_p=drop_p, seed=seed)
        else:
            dpre = as_dtype(g, cdt())
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty(M, xc.shape[1], dtype=F32, device=g.device)
            ops.linear_dx(dpre, compute_weight(weight).reshape(N, -1), gx)
            gx = as_dtype(gx, xdt)
        ops.linear_dw(dpre, xc, grad_buf(weight).view(N, -1))
        if bias is not None and not fused_bias:
            ops.colsum(dpre, grad_buf(bias), accum=True)
        return gx, None, None, None, None, None, (g if has_res else None)


def linear(x, layer, act="none", drop_p=0.0, out_dtype=F32, residual=None):
    shp = x.shape
    y = LinearFn.apply(x.reshape(-1, shp[-1]), layer.weight, layer.bias, act, drop_p, out_dtype,
                       None if residual is None else residual.reshape(-1, layer.weight.shape[0]))
    return y.reshape(*shp[:-1], layer.weight.shape[0])


# --------------------------------------------------------------------------------------
class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, out_dtype):
        x = x.contiguous()
        M, D = x.shape
        y = torch.empty(M, D, dtype=out_dtype, device=x.device)
        mean = torch.empty(M, dtype=F32, device=x.device)
        rstd = torch.empty(M, dtype=F32, device=x.device)
        ops.layernorm_fwd(x, None if weight is None else weight.detach(),
                          None if bias is None else bias.detach(), y, mean, rstd, eps)
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, g):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        dy = as_dtype(g, F32)
        dx = torch.empty(x.shape, dtype=F32, device=x.device)
        ops.layernorm_bwd(x, None if weight is None else weight.detach(), dy, mean, rstd, dx, accum=False,
                          dw=None if weight is None else grad_buf(weight),
                          db=None if bias is None else grad_buf(bias))
        return as_dtype(dx, x.dtype), None, None, None, None


def layer_norm(x, ln, out_dtype=F32):
    shp = x.shape
    y = LayerNormFn.apply(x.reshape(-1, shp[-1]), ln.weight, ln.bias, ln.eps, out_dtype)
    return y.reshape(shp)


class ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act, out_dtype):
        x = x.contiguous()
        y = torch.empty(x.shape, dtype=out_dtype, device=x.device)
        ops.act_fwd(x, y, act)
        ctx.save_for_backward(x)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        dx = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        ops.act_bwd(x.reshape(-1, x.shape[-1]), g.contiguous().reshape(-1, x.shape[-1]),
                    dx.reshape(-1, x.shape[-1]), ctx.act)
        return dx, None, None


# --------------------------------------------------------------------------------------
# attention
# --------------------------------------------------------------------------------------
def _attn_mat_fwd(qkv, B, N, H, scale, p, seed):
    """materialised attention in fp32 (parity path / head_dim != 64): S=QK^T, P=softmax, O=P V."""
    D = qkv.shape[1] // 3
    hd = D // H
    ld = 3 * D
    q = qkv.float() if qkv.dtype != F32 else qkv
    S = torch.empty(B, H, N, N, dtype=F32, device=q.device)
    ops.gemm(q, q[:, D:], S, N, N, hd, ld, ld, N, 0, 0, batch=B * H, inner=H, sA=(N * ld, hd),
             sB=(N * ld, hd), sC=(H * N * N, N * N))
    P = torch.empty_like(S)
    Pd = torch.empty_like(S) if p > 0 else None
    ops.softmax_fwd(S, P, Pd, N, scale, p, seed)
    del S
    O = torch.empty(B * N, D, dtype=F32, device=q.device)
    ops.gemm(Pd if p > 0 else P, q[:, 2 * D:], O, N, hd, N, N, ld, D, 0, 1, batch=B * H, inner=H,
             sA=(H * N * N, N * N), sB=(N * ld, hd), sC=(N * D, hd))
    return O, P, Pd


def _attn_mat_bwd(qkv, P, Pd, dO, B, N, H, scale, p, seed):
    D = qkv.shape[1] // 3
    hd = D // H
    ld = 3 * D
    q = qkv.float() if qkv.dtype != F32 else qkv
    dO = as_dtype(dO, F32)
    dPd = torch.empty(B, H, N, N, dtype=F32, device=q.device)
    ops.gemm(dO, q[:, 2 * D:], dPd, N, N, hd, D, ld, N, 0, 0, batch=B * H, inner=H, sA=(N * D, hd),
             sB=(N * ld, hd), sC=(H * N * N, N * N))
    dS = torch.empty_like(dPd)
    ops.softmax_bwd(P, dPd, dS, N, scale, p, seed)
    del dPd
    dqkv = torch.empty(B * N, 3 * D, dtype=F32, device=q.device)
    bat = dict(batch=B * H, inner=H)
    ops.gemm(dS, q[:, D:], dqkv, N, hd, N, N, ld, ld, 0, 1, sA=(H * N * N, N * N), sB=(N * ld, hd),
             sC=(N * ld, hd), **bat)
    ops.gemm(dS, q, dqkv[:, D:], N, hd, N, N, ld, ld, 1, 1, sA=(H * N * N, N * N), sB=(N * ld, hd),
             sC=(N * ld, hd), **bat)
    ops.gemm(Pd if p > 0 else P, dO, dqkv[:, 2 * D:], N, hd, N, N, D, ld, 1, 1, sA=(H * N * N, N * N),
             sB=(N * D, hd), sC=(N * ld, hd), **bat)
    return dqkv


def use_flash(N, hd=64):
    return cdt() == torch.bfloat16 and RT.flash_attention and N % 64 == 0 and hd == 64


# --------------------------------------------------------------------------------------
class BlockFn(torch.autograd.Function):
    """timm Block (pre-LN, MHSA, GELU MLP, 4 dropouts) as one fused forward/backward.
    x: [B*N, D] fp32 residual stream."""

    @staticmethod
    def forward(ctx, x, shape, p_attn, p_proj, hook, premask, n1w, n1b, qkvw, qkvb, projw, projb, n2w, n2b, fc1w,
                fc1b, fc2w, fc2b):
        B, N, H = shape
        M, D = x.shape
        dev = x.device
        c = cdt()
        scale = (D // H) ** -0.5
        seeds = [_seed() for _ in range(4)]
        # is x the previous Block's output (whose fc2 dropout backward this Block's norm1 backward can emit)?
        up = RT._drop_pending.pop(x.data_ptr(), None)
        if up is not None and not (up[0].shape == x.shape and up[0].dtype == x.dtype):
            up = None
        if premask is not None:  # attention keep-mask planes generated ahead on the side stream
            seeds[0] = premask[0]
        h1 = torch.empty(M, D, dtype=c, device=dev)
        m1 = torch.empty(M, dtype=F32, device=dev)
        r1 = torch.empty(M, dtype=F32, device=dev)
        ops.layernorm_fwd(x, n1w.detach(), n1b.detach(), h1, m1, r1)
        qkv = torch.empty(M, 3 * D, dtype=c, device=dev)
        linear_bias(h1, qkvw, qkvb, qkv)
        flash = use_flash(N, D // H)
        if flash:
            o = torch.empty(M, D, dtype=c, device=dev)
            lse = torch.empty(B, H, N, dtype=F32, device=dev)
            pm = premask[1] if premask is not None else None
            if RT.attn_fp8:
                # qkv is rounded in place to the fp8 grid: the saved tensor (and so the bf16 backward)
                # sees exactly what the fp8 forward multiplied
                ws = ops.attn_fp8_workspace(B, N, H, dev)
                ops.attn_quant_fp8(qkv, ws, B, N, H)
                amask = ops.attn_fwd_fp8(ws, o, lse, B, N, H, scale, p_attn, seeds[0], mask=pm)
                del ws
            else:
                amask = ops.attn_fwd(qkv, o, lse, B, N, H, scale, p_attn, seeds[0], mask=pm)
            P, Pd = None, amask
        else:
            o, P, Pd = _attn_mat_fwd(qkv, B, N, H, scale, p_attn, seeds[0])
            o = as_dtype(o, c)
            lse = None
        Hd = fc1w.shape[0]
        planes = (None, None, None)
        if c == torch.bfloat16 and RT.drop_planes and p_proj > 0 and D % 32 == 0 and Hd % 32 == 0:
            # keep-bit planes of the proj / fc1 / fc2 dropouts (seeds 1-3): the fused GEMM epilogues test bits
            # instead of hashing each element; fc1's plane serves the backward's fused GELU' epilogue too
            planes = (ops.dropout_plane(M * D, p_proj, seeds[1], dev), ops.dropout_plane(M * Hd, p_proj, seeds[2], dev),
                      ops.dropout_plane(M * D, p_proj, seeds[3], dev))
        x1 = torch.empty(M, D, dtype=F32, device=dev)
        # attention proj + proj_drop + the residual add: bf16 (autocast) output rounded before the dropout
        # and the fp32 add, in the 8-wave GEMM's epilogue; fp32 parity mode (or an ineligible shape): the
        # fused-epilogue GEMM of gemm.hip
        if not (c == torch.bfloat16 and RT.proj_8w and
                ops.linear_drop_res(o, compute_weight(projw), projb.detach(), x, x1, p_proj, seeds[1], planes[0])):
            ops.linear(o, compute_weight(projw), x1, bias=projb.detach(), residual=x, drop_p=p_proj,
                       seed=seeds[1])
        h2 = torch.empty(M, D, dtype=c, device=dev)
        m2 = torch.empty(M, dtype=F32, device=dev)
        r2 = torch.empty(M, dtype=F32, device=dev)
        ops.layernorm_fwd(x1, n2w.detach(), n2b.detach(), h2, m2, r2)
        a = torch.empty(M, Hd, dtype=c, device=dev)
        pre1 = torch.empty(M, Hd, dtype=c, device=dev)
        x2 = torch.empty(M, D, dtype=F32, device=dev)
        if c == torch.bfloat16:
            # autocast semantics: fc1 / fc2 outputs are bf16 before GELU / dropout / the fp32 residual add.
            # Fused (RT.mlp_split_epilogue False): the 8-wave GEMM finishes GELU + dropout (fc1) and dropout +
            # residual (fc2) in its epilogue (csrc/gemm8w.hip); split: bias-only GEMMs + one elementwise pass
            # each.  Both routes give the same bits (same rounding points, same flat-index dropout masks)
            fused = not RT.mlp_split_epilogue
            if not (fused and ops.linear_gelu_drop(h2, compute_weight(fc1w), fc1b.detach(), pre1, a, p_proj,
                                                   seeds[2], planes[1])):
                linear_bias(h2, fc1w, fc1b, pre1)
                ops.act_drop_fwd(pre1, a, "gelu", drop_p=p_proj, seed=seeds[2])
            if not (fused and ops.linear_drop_res(a, compute_weight(fc2w), fc2b.detach(), x1, x2, p_proj, seeds[3],
                                                  planes[2])):
                t2 = torch.empty(M, D, dtype=c, device=dev)
                linear_bias(a, fc2w, fc2b, t2)
                ops.act_drop_fwd(t2, x2, "none", drop_p=p_proj, seed=seeds[3], residual=x1)
                del t2
        else:
            ops.linear(h2, compute_weight(fc1w), a, bias=fc1b.detach(), act="gelu", aux=pre1, drop_p=p_proj,
                       seed=seeds[2])
            ops.linear(a, compute_weight(fc2w), x2, bias=fc2b.detach(), residual=x1, drop_p=p_proj, seed=seeds[3])
        ctx.save_for_backward(x, h1, m1, r1, qkv, o, lse, P, Pd, x1, h2, m2, r2, pre1, a,
                              n1w, n1b, qkvw, qkvb, projw, projb, n2w, n2b, fc1w, fc1b, fc2w, fc2b)
        ctx.cfg = (B, N, H, p_attn, p_proj, seeds, flash)
        ctx.plane1 = planes[1]
        ctx.up = up[1:] if up is not None else None
        if c == torch.bfloat16 and RT.ln_bwd_drop and any(ctx.needs_input_grad):
            RT._drop_pending[x2.data_ptr()] = (x2, p_proj, seeds[3], fc2b)
        ctx.hook = hook
        return x2

    @staticmethod
    def backward(ctx, g2):
        (x, h1, m1, r1, qkv, o, lse, P, Pd, x1, h2, m2, r2, pre1, a,
         n1w, n1b, qkvw, qkvb, projw, projb, n2w, n2b, fc1w, fc1b, fc2w, fc2b) = ctx.saved_tensors
        B, N, H, p_attn, p_proj, seeds, flash = ctx.cfg
        M, D = x.shape
        dev = x.device
        c = cdt()
        scale = (D // H) ** -0.5
        g2 = as_dtype(g2, F32)
        # fc2 (+drop2, residual): bf16(drop(g2)) and the fc2 bias gradient -- already emitted by the next Block's
        # norm1 backward when g2 is exactly the gradient it produced (hand-off by seed; verified by pointer)
        ready = RT._drop_ready.pop(seeds[3], None)
        if ready is not None and ready[0] == g2.data_ptr() and ready[1].shape == (M, D):
            dpre2 = ready[1]
        else:
            dpre2 = torch.empty(M, D, dtype=c, device=dev)
            ops.act_bwd_bias(None, g2, dpre2, grad_buf(fc2b), "none", drop_p=p_proj, seed=seeds[3])
        ops.linear_dw(dpre2, a, grad_buf(fc2w))
        Hd = fc1w.shape[0]
        # fc1 (gelu + drop1)
        dpre1 = torch.empty(M, Hd, dtype=c, device=dev)
        if c == torch.bfloat16 and RT.act_bwd_in_gemm and ops.linear_dgelu_drop(
                dpre2, compute_weight_t(fc2w), pre1, dpre1, grad_buf(fc1b), p_proj, seeds[2], plane=ctx.plane1):
            # fc2's dX product finishes dropout + GELU' in its epilogue and the fc1 bias gradient as column
            # partials (csrc/gemm8w.hip EPI 3): no [M, 3072] round trip of dA
            pass
        elif RT.act_bwd_in_gemm:
            ops.linear_dx_act(dpre2, compute_weight(fc2w), dpre1, pre1, "gelu", drop_p=p_proj, seed=seeds[2])
            ops.colsum(dpre1, grad_buf(fc1b))
        else:
            da = torch.empty(M, Hd, dtype=c, device=dev)
            linear_dx_w(dpre2, fc2w, da)
            ops.act_bwd_bias(pre1, da, dpre1, grad_buf(fc1b), "gelu", drop_p=p_proj, seed=seeds[2])
            del da
        del dpre2
        ops.linear_dw(dpre1, h2, grad_buf(fc1w))
        # dX of the LN-fed GEMMs in the compute dtype (autocast: the matmul's input grad is half
        # precision before the cast back to the fp32 LayerNorm output); LN backward reads it as is
        dh2 = torch.empty(M, D, dtype=c if RT.ln_dy_lowp else F32, device=dev)
        linear_dx_w(dpre1, fc1w, dh2)
        del dpre1
        g1 = torch.empty(M, D, dtype=F32, device=dev)
        dprep = torch.empty(M, D, dtype=c, device=dev)
        # norm2 backward; with bf16 operands it also emits the proj_drop backward (dprep) and the proj bias
        # gradient in the same pass (ln_bwd DROPO)
        if not (c == torch.bfloat16 and RT.ln_bwd_drop and dh2.dtype == c and
                ops.layernorm_bwd_drop(x1, n2w.detach(), dh2, m2, r2, g1, grad_buf(n2w), grad_buf(n2b), g2, dprep,
                                       p_proj, seeds[1], grad_buf(projb))):
            ops.layernorm_bwd(x1, n2w.detach(), dh2, m2, r2, g1, accum=False, dw=grad_buf(n2w), db=grad_buf(n2b),
                              dx_base=g2)
            # proj (+proj_drop, residual)
            ops.act_bwd_bias(None, g1, dprep, grad_buf(projb), "none", drop_p=p_proj, seed=seeds[1])
        del dh2
        ops.linear_dw(dprep, o, grad_buf(projw))
        do = torch.empty(M, D, dtype=c, device=dev)
        linear_dx_w(dprep, projw, do)
        del dprep
        if flash:
            dqkv = torch.empty(M, 3 * D, dtype=c, device=dev)
            dvec = torch.empty(B, H, N, dtype=F32, device=dev)
            # the qkv bias gradient comes out of the attention backward's epilogues (column partials of dqkv)
            ops.attn_bwd(qkv, o, do, lse, dvec, dqkv, B, N, H, scale, p_attn, seeds[0], mask=Pd,
                         dbias=grad_buf(qkvb) if RT.attn_bias_grad else None)
        else:
            dqkv = as_dtype(_attn_mat_bwd(qkv, P, Pd, do, B, N, H, scale, p_attn, seeds[0]), c)
        del do
        ops.linear_dw(dqkv, h1, grad_buf(qkvw))
        if not (flash and RT.attn_bias_grad):
            ops.colsum(dqkv, grad_buf(qkvb))
        dh1 = torch.empty(M, D, dtype=c if RT.ln_dy_lowp else F32, device=dev)
        linear_dx_w(dqkv, qkvw, dh1)
        del dqkv
        gx = torch.empty(M, D, dtype=F32, device=dev)
        up = ctx.up
        if up is not None and dh1.dtype == c:
            # norm1 backward + the previous Block's fc2 dropout backward and fc2 bias gradient in one pass
            p_up, seed_up, fc2b_up = up
            d_up = torch.empty(M, D, dtype=c, device=dev)
            if ops.layernorm_bwd_drop(x, n1w.detach(), dh1, m1, r1, gx, grad_buf(n1w), grad_buf(n1b), g1, d_up,
                                      p_up, seed_up, grad_buf(fc2b_up)):
                RT._drop_ready[seed_up] = (gx.data_ptr(), d_up)
            else:
                up = None
        if up is None or dh1.dtype != c:
            ops.layernorm_bwd(x, n1w.detach(), dh1, m1, r1, gx, accum=False, dw=grad_buf(n1w), db=grad_buf(n1b),
                              dx_base=g1)
        if ctx.hook is not None:
            ctx.hook()  # every grad of this block is enqueued: launch its DP bucket all-reduce
        return (gx,) + (None,) * 17


def block_forward(blk, x, B, N, p_attn, p_proj):
    """x: [B, N, D] fp32 -> [B, N, D] fp32 through BlockFn."""
    D = x.shape[-1]
    a, m = blk.attn, blk.mlp
    premask = None
    if p_attn > 0 and use_flash(N, D // a.num_heads) and x.is_cuda:
        shape = (B, N, a.num_heads, float(p_attn))
        premask = RT.take_attn_mask(id(blk), shape)
        RT.note_attn_shape(id(blk), shape)  # the next step's masks are generated ahead of time
    y = BlockFn.apply(x.reshape(B * N, D).contiguous(), (B, N, a.num_heads), p_attn, p_proj,
                      getattr(blk, "_uva_bucket_hook", None), premask, blk.norm1.weight, blk.norm1.bias,
                      a.qkv.weight, a.qkv.bias, a.proj.weight, a.proj.bias,
                      blk.norm2.weight, blk.norm2.bias, m.fc1.weight, m.fc1.bias, m.fc2.weight, m.fc2.bias)
    return y.reshape(B, N, D)


# --------------------------------------------------------------------------------------
class AdaLNTrunkFn(torch.autograd.Function):
    """SimpleMLPAdaLN after the embeddings (diffusion_loss.py:261-283):
    sy = SiLU(y); depth x [mod = adaLN(sy); h = LN(x)*(1+scale)+shift; x += gate*fc2(SiLU(fc1(h)))];
    final: LN(x)*(1+scale)+shift -> linear.   x0, y: [R, W] fp32 -> out [R, 2C] fp32."""

    @staticmethod
    def forward(ctx, x0, y, depth, hook, *params):
        R, W = x0.shape
        dev = x0.device
        c = cdt()
        sy = torch.empty(R, W, dtype=c, device=dev)
        ops.act_fwd(y.contiguous(), sy, "silu")
        x = x0.contiguous()
        saved = []
        for i in range(depth):
            modw, modb, w1, b1, w2, b2, lnw, lnb = params[8 * i:8 * i + 8]
            mod = torch.empty(R, 3 * W, dtype=c, device=dev)
            ops.linear(sy, compute_weight(modw), mod, bias=modb.detach())
            h = torch.empty(R, W, dtype=c, device=dev)
            mean = torch.empty(R, dtype=F32, device=dev)
            rstd = torch.empty(R, dtype=F32, device=dev)
            _ln_mod_fwd(x, lnw, lnb, mod, W, h, mean, rstd)
            a = torch.empty(R, W, dtype=c, device=dev)
            pre1 = torch.empty(R, W, dtype=c, device=dev)
            ops.linear(h, compute_weight(w1), a, bias=b1.detach(), act="silu", aux=pre1)
            xn = torch.empty(R, W, dtype=F32, device=dev)
            hm2 = torch.empty(R, W, dtype=F32, device=dev)
            ops.linear(a, compute_weight(w2), xn, bias=b2.detach(), aux=hm2, gate=mod[:, 2 * W:], residual=x)
            saved += [x, mod, h, mean, rstd, a, pre1, hm2]
            x = xn
        fmw, fmb, lw, lb = params[8 * depth:8 * depth + 4]
        fmod = torch.empty(R, 2 * W, dtype=c, device=dev)
        ops.linear(sy, compute_weight(fmw), fmod, bias=fmb.detach())
        hf = torch.empty(R, W, dtype=c, device=dev)
        meanf = torch.empty(R, dtype=F32, device=dev)
        rstdf = torch.empty(R, dtype=F32, device=dev)
        ops.layernorm_fwd(x, None, None, hf, meanf, rstdf, scale=fmod[:, W:], shift=fmod[:, :W], ldm=2 * W)
        out = torch.empty(R, lw.shape[0], dtype=F32, device=dev)
        ops.linear(hf, compute_weight(lw), out, bias=lb.detach())
        saved += [x, fmod, hf, meanf, rstdf]
        ctx.save_for_backward(y, sy, *saved, *params)
        ctx.depth = depth
        ctx.hook = hook
        return out

    @staticmethod
    def backward(ctx, gout):
        depth = ctx.depth
        t = ctx.saved_tensors
        y, sy = t[0], t[1]
        blocks = [t[2 + 8 * i:2 + 8 * i + 8] for i in range(depth)]
        xf, fmod, hf, meanf, rstdf = t[2 + 8 * depth:2 + 8 * depth + 5]
        params = t[2 + 8 * depth + 5:]
        R, W = y.shape
        dev = y.device
        c = cdt()
        fmw, fmb, lw, lb = params[8 * depth:8 * depth + 4]
        dout = as_dtype(gout, c)
        ops.linear_dw(dout, hf, grad_buf(lw))
        ops.colsum(dout, grad_buf(lb))
        dhf = torch.empty(R, W, dtype=F32, device=dev)
        ops.linear_dx(dout, compute_weight(lw), dhf)
        dfmod = torch.empty(R, 2 * W, dtype=c, device=dev)
        dx = torch.empty(R, W, dtype=F32, device=dev)
        ops.layernorm_bwd(xf, None, dhf, meanf, rstdf, dx, accum=False, scale=fmod[:, W:], ldm=2 * W,
                          dscale=dfmod[:, W:], dshift=dfmod[:, :W])
        ops.linear_dw(dfmod, sy, grad_buf(fmw))
        ops.colsum(dfmod, grad_buf(fmb))
        dsy = torch.empty(R, W, dtype=F32, device=dev)
        ops.linear_dx(dfmod, compute_weight(fmw), dsy)
        del dfmod, dhf
        for i in reversed(range(depth)):
            x, mod, h, mean, rstd, a, pre1, hm2 = blocks[i]
            modw, modb, w1, b1, w2, b2, lnw, lnb = params[8 * i:8 * i + 8]
            dmod = torch.empty(R, 3 * W, dtype=c, device=dev)
            dhm2 = torch.empty(R, W, dtype=c, device=dev)
            ops.gate_bwd(dx, hm2, mod[:, 2 * W:], dhm2, dmod[:, 2 * W:])
            ops.linear_dw(dhm2, a, grad_buf(w2))
            ops.colsum(dhm2, grad_buf(b2))
            dpre1 = torch.empty(R, W, dtype=c, device=dev)
            if RT.trunk_act_bwd_in_gemm and pre1.dtype == c:
                ops.linear_dx_act(dhm2, compute_weight(w2), dpre1, pre1, "silu")
                ops.colsum(dpre1, grad_buf(b1))
            else:
                da = torch.empty(R, W, dtype=c, device=dev)
                ops.linear_dx(dhm2, compute_weight(w2), da)
                ops.act_bwd_bias(pre1, da, dpre1, grad_buf(b1), "silu")
            ops.linear_dw(dpre1, h, grad_buf(w1))
            dh = torch.empty(R, W, dtype=F32, device=dev)
            ops.linear_dx(dpre1, compute_weight(w1), dh)
            dxn = torch.empty(R, W, dtype=F32, device=dev)
            _ln_mod_bwd(x, lnw, lnb, mod, W, dh, mean, rstd, dxn, dmod, dx)
            ops.linear_dw(dmod, sy, grad_buf(modw))
            ops.colsum(dmod, grad_buf(modb))
            ops.linear_dx(dmod, compute_weight(modw), dsy, beta=1.0)
            dx = dxn
        dy = torch.empty(R, W, dtype=F32, device=dev)
        ops.act_bwd(y, dsy, dy, "silu")
        if ctx.hook is not None:
            ctx.hook()
        return (dx, dy, None, None) + (None,) * len(params)


def _ln_mod_fwd(x, lnw, lnb, mod, W, h, mean, rstd):
    # ResBlock.in_ln has an affine (weight, bias) AND is modulated: h = (LN(x)*w+b)*(1+scale)+shift.
    ops.layernorm_fwd(x, lnw.detach(), lnb.detach(), h, mean, rstd, scale=mod[:, W:2 * W], shift=mod[:, :W],
                      ldm=3 * W)


def _ln_mod_bwd(x, lnw, lnb, mod, W, dh, mean, rstd, dx_out, dmod, dx_base):
    """backward of h = (LN(x)*w + b)*(1+scale) + shift."""
    R = x.shape[0]
    # d(scale) = dh * (xhat*w+b), d(shift) = dh, d(LN affine out) = dh*(1+scale)
    ops.layernorm_bwd(x, lnw.detach(), dh, mean, rstd, dx_out, accum=False, dw=grad_buf(lnw), db=grad_buf(lnb),
                      scale=mod[:, W:2 * W], ldm=3 * W, dscale=dmod[:, W:2 * W], dshift=dmod[:, :W],
                      dx_base=dx_base, b=lnb.detach())
