"""Thin torch-tensor wrappers over the C ABI (device pointers, strides, current stream).
Shape/dtype checks happen here, before launch (SURVEY §8b C-ABI conventions)."""
import ctypes

import torch

from .lib import lib

F32, BF16 = 0, 1
ACT = {"none": 0, "gelu": 1, "silu": 2, "relu": 3}


def dt(t):
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float32:
        return F32
    raise TypeError(f"unsupported dtype {t.dtype}")


def ptr(t):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


# ---- live kernel tracing (bench.py roofline / per-step accounting): HIP events around launches ----
TRACE = None  # dict tag -> list[(start_event, end_event, flops, side_stream)] when enabled
TRACE_ONLY = None  # optional set of tags: only those launches get events (the roofline pass)


class _traced:
    """events around one library call on the current stream; only the outermost of nested scopes
    records, so every launch is counted once (the explicitly tagged ops carry shapes and FLOPs, every
    other entry point is tagged by its C-ABI name through _call).  Launches on a stream other than the
    device's default stream (the attention keep-mask planes generated ahead on RT's side stream) are
    marked, so per-step accounting can keep their overlapped time apart."""
    __slots__ = ("tag", "flops", "ev")
    depth = 0

    def __init__(self, tag, flops):
        self.tag, self.flops, self.ev = tag, flops, None

    def __enter__(self):
        if TRACE is not None and _traced.depth == 0 and (TRACE_ONLY is None or self.tag in TRACE_ONLY):
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self.ev[0].record()
        _traced.depth += 1
        return self

    def __exit__(self, *a):
        _traced.depth -= 1
        if self.ev is not None:
            self.ev[1].record()
            if TRACE is not None:
                side = torch.cuda.current_stream() != torch.cuda.default_stream()
                TRACE.setdefault(self.tag, []).append((self.ev[0], self.ev[1], self.flops, side))


def _call(name, *args):
    """lib().call under a trace scope tagged by the entry point's name (no FLOP count); with tracing off
    the launch goes straight to the library (no scope object on the hot path)"""
    if TRACE is None:
        return lib().call(name, *args)
    with _traced(name[4:] if name.startswith("uva_") else name, 0.0):
        return lib().call(name, *args)


def _ld(t):
    """leading dimension of a 2-D (row-major, unit inner stride) view."""
    assert t.dim() == 2 and t.stride(1) == 1, (t.shape, t.stride())
    return t.stride(0)


def gemm(A, B, C, M, N, K, lda, ldb, ldc, ta=0, tb=0, batch=1, inner=1, sA=(0, 0), sB=(0, 0), sC=(0, 0),
         bias=None, residual=None, ldr=0, sR=(0, 0), aux=None, act="none", alpha=1.0, beta=0.0,
         drop_p=0.0, seed=0, force_generic=False, splitk=True, gate=None, ldg=0):
    assert A.dtype == B.dtype, (A.dtype, B.dtype)
    ws = workspace(SPLITK_WS_FLOATS, A.device) if (splitk and batch == 1) else None
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous()
    if aux is not None:
        assert aux.dtype == C.dtype
    with _traced(f"gemm[{'NT'[ta]}{'NT'[tb]}] {'bf16' if dt(A) else 'f32'} M{M} N{N} K{K} b{batch}",
                 2.0 * M * N * K * batch):
        _call("uva_gemm", dt(A), dt(C), ta, tb, ptr(A), ptr(B), ptr(C), M, N, K, lda, ldb, ldc, batch, inner,
                   sA[0], sA[1], sB[0], sB[1], sC[0], sC[1], ptr(bias), ptr(residual), ldr, sR[0], sR[1], ptr(aux),
                   ACT[act] if isinstance(act, str) else act, float(alpha), float(beta), float(drop_p),
                   int(seed) & 0xFFFFFFFFFFFFFFFF, dt(residual) if residual is not None else 0, ptr(gate), ldg,
                   dt(gate) if gate is not None else 0, int(force_generic), ptr(ws),
                   ws.numel() if ws is not None else 0, stream())


SPLITK_WS_FLOATS = 1 << 25  # 128 MB fp32 partial slabs


def gemm_plan(M, N, K, ta=0, tb=0, batch=1, splitk=True, gn_prologue=False, dtype=torch.bfloat16):
    """(kernel, BN, splits) the native dispatcher picks for a bf16 GEMM of this shape:
    kernel 0 VALU, 1 MFMA register-staged, 2 MFMA LDS-DMA 128x128, 3 MFMA 8-phase 256-row."""
    code = lib().query("uva_gemm_plan", 1 if dtype == torch.bfloat16 else 0, ta, tb, M, N, K, batch, int(gn_prologue),
                       SPLITK_WS_FLOATS if splitk else 0)
    return code & 15, (code >> 4) & 4095, code >> 16


def gemm_set_persist(on):
    """route eligible full-tile products to the persistent gemm_8pp (True) or gemm_8ph (False);
    returns the previous setting (tests / kernel benchmarks)"""
    return bool(lib().query("uva_gemm_set_persist", int(bool(on))))


def gemm4_set(on=-2, force=-2):
    """measurement switch of the persistent 4-wave kernel (tests / kernel benchmarks): on = 0 routes the
    K-contiguous bias-only products back to gemm_8ph; force = tile configuration (-1 automatic); -2
    leaves a value unchanged.  Returns the previous (on, force)."""
    prev = lib().query("uva_gemm4_set", int(on), int(force))
    return prev & 1, (prev >> 1) - 1


def gemm8w_set(on=-2, mode=-2):
    """measurement switch of the 8-wave GEMM (uva_gemm8w_set) -> previous (on, mode)"""
    prev = lib().query("uva_gemm8w_set", int(on), int(mode))
    return prev & 1, prev >> 1


def linear_gelu_drop(x, w, bias, pre_out, out, drop_p=0.0, seed=0, plane=None):
    """timm Mlp fc1 forward in one launch (uva_linear_gelu_drop): pre_out = bf16(x w^T + b),
    out = bf16(drop(gelu(pre_out))).  -> True if launched, False if the shape is not eligible."""
    M, K = x.shape
    N = w.shape[0]
    assert x.is_contiguous() and w.is_contiguous() and pre_out.is_contiguous() and out.is_contiguous()
    with _traced(f"gemm+gelu+drop bf16 M{M} N{N} K{K}", 2.0 * M * N * K):
        r = lib().query("uva_linear_gelu_drop", ptr(x), ptr(w), ptr(bias), ptr(pre_out), ptr(out), M, N, K,
                        float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(plane), stream())
    if r < 0:
        raise RuntimeError(f"fused Mlp GEMM failed with hipError {-r}")
    return r == 1


def linear_drop_res(x, w, bias, residual, out, drop_p=0.0, seed=0, plane=None):
    """timm Mlp fc2 (or attention proj) forward + dropout + fp32 residual in one launch
    (uva_linear_drop_res): out = residual + drop(bf16(x w^T + b)).  -> True if launched."""
    M, K = x.shape
    N = w.shape[0]
    assert x.is_contiguous() and w.is_contiguous() and residual.is_contiguous() and out.is_contiguous()
    with _traced(f"gemm+drop+res bf16 M{M} N{N} K{K}", 2.0 * M * N * K):
        r = lib().query("uva_linear_drop_res", ptr(x), ptr(w), ptr(bias), ptr(residual), ptr(out), M, N, K,
                        float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(plane), stream())
    if r < 0:
        raise RuntimeError(f"fused Mlp GEMM failed with hipError {-r}")
    return r == 1


def linear_dgelu_drop(dy, wt, pre, dpre, dbias, drop_p=0.0, seed=0, accum_bias=True, plane=None):
    """the timm Mlp backward through fc2 -> dropout -> GELU fused into fc2's dX product
    (uva_linear_dgelu_drop): dpre = bf16(gelu'(pre) * drop(bf16(dy wt^T))), dbias (+)= colsum(dpre).
    wt: fc2's transposed bf16 weight [in, out].  -> True if launched, False if not eligible."""
    M, K = dy.shape
    N = wt.shape[0]
    assert dy.is_contiguous() and wt.is_contiguous() and pre.is_contiguous() and dpre.is_contiguous()
    ws = workspace((M + 255) // 256 * 4 * N, dy.device)
    with _traced(f"gemm+dgelu+drop bf16 M{M} N{N} K{K}", 2.0 * M * N * K):
        r = lib().query("uva_linear_dgelu_drop", ptr(dy), ptr(wt), ptr(pre), ptr(dpre), ptr(dbias), int(accum_bias),
                        ptr(ws), M, N, K, float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(plane), stream())
    if r < 0:
        raise RuntimeError(f"fused Mlp GEMM failed with hipError {-r}")
    return r == 1


def dropout_plane(n, drop_p, seed, device, out=None):
    """keep-bit plane of n flat elements under (drop_p, seed): int32 [ceil(n / 32)] (uva_dropout_plane)"""
    words = lib().query("uva_dropout_plane_words", int(n))
    if out is None:
        out = torch.empty(words, dtype=torch.int32, device=device)
    _call("uva_dropout_plane", ptr(out), int(n), float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, stream())
    return out


def gemm4_plan(M, N, K):
    """(configuration, grid) of the 4-wave kernel for an eligible K-contiguous product, None otherwise"""
    code = lib().query("uva_gemm4_plan", M, N, K)
    return None if code < 0 else (code & 255, code >> 8)


def gemm4_plan_tt(M, N, K, ws_floats=None):
    """(splits, grid) of the 4-wave kernel for an eligible dW (ta = tb = 1, fp32 output) product with the
    default split-K workspace, None otherwise"""
    code = lib().query("uva_gemm4_plan_tt", M, N, K, SPLITK_WS_FLOATS if ws_floats is None else ws_floats)
    return None if code < 0 else (code & 255, code >> 8)


def linear(x, w, out, bias=None, act="none", aux=None, residual=None, drop_p=0.0, seed=0, beta=0.0, gate=None):
    """out[M,N] = epi(x[M,K] @ w[N,K]^T) -- nn.Linear forward."""
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K and out.shape == (M, N)
    gemm(x, w, out, M, N, K, _ld(x), _ld(w), _ld(out), 0, 0, bias=bias, act=act, aux=aux,
         residual=residual, ldr=_ld(residual) if residual is not None else 0, drop_p=drop_p, seed=seed,
         beta=beta, gate=gate, ldg=_ld(gate) if gate is not None else 0)


def linear_dx(dy, w, dx, beta=0.0):
    """dx[M,K] (+)= dy[M,N] @ w[N,K]."""
    M, N = dy.shape
    K = w.shape[1]
    assert dx.shape == (M, K)
    gemm(dy, w, dx, M, K, N, _ld(dy), _ld(w), _ld(dx), 0, 1, beta=beta)


def linear_dx_act(dy, w, dx, pre, act, drop_p=0.0, seed=0):
    """dx[M,K] = act'(pre) * dropout(dy[M,N] @ w[N,K]) -- the dX product of the Linear after an
    activation (+dropout) fused with that activation's backward (epilogue mode act = 16 + kind,
    pre = the saved pre-activation [M,K]); the dropout index is row * K + col, as act_bwd's."""
    M, N = dy.shape
    K = w.shape[1]
    assert dx.shape == (M, K) and pre.shape == (M, K) and pre.is_contiguous() and dx.is_contiguous()
    gemm(dy, w, dx, M, K, N, _ld(dy), _ld(w), _ld(dx), 0, 1, residual=pre, ldr=_ld(pre), act=16 + ACT[act],
         drop_p=drop_p, seed=seed)


def linear_dw(dy, x, dw, beta=1.0):
    """dw[N,K] (+)= dy[M,N]^T @ x[M,K]  (fp32 grad buffer, accumulate by default)."""
    M, N = dy.shape
    K = x.shape[1]
    assert dw.shape == (N, K)
    gemm(dy, x, dw, N, K, M, _ld(dy), _ld(x), _ld(dw), 1, 1, beta=beta)


_WS = {}


def workspace(n_floats, device):
    key = (device, "ws")
    t = _WS.get(key)
    if t is None or t.numel() < n_floats:
        t = torch.empty(max(int(n_floats), 1 << 20), dtype=torch.float32, device=device)
        _WS[key] = t
    return t


def colsum(x, out, accum=True):
    rows, cols = x.shape
    ws = workspace(lib().query("uva_colsum_workspace", rows, cols), x.device)
    _call("uva_colsum", dt(x), ptr(x), _ld(x), ptr(out), rows, cols, int(accum), ptr(ws), stream())


def layernorm_fwd(x, w, b, y, mean, rstd, eps=1e-6, scale=None, shift=None, ldm=0):
    rows, D = x.shape
    assert x.is_contiguous() and y.is_contiguous()
    _call("uva_layernorm_fwd", dt(x), dt(y), ptr(x), ptr(w), ptr(b), ptr(scale), ptr(shift), ldm, ptr(y),
               ptr(mean), ptr(rstd), rows, D, float(eps), stream())


def layernorm_bwd(x, w, dy, mean, rstd, dx, accum, dw=None, db=None, scale=None, ldm=0, dscale=None, dshift=None,
                  out_dtype=None, accum_wb=True, dx_base=None, b=None):
    """dx (= dx_base +) LN backward.  With `scale` (adaLN modulation) the affine (w, b) output is
    modulated: h = (xhat*w + b)*(1+scale) + shift; b is needed for d(scale)."""
    rows, D = x.shape
    assert dy.dtype in (torch.float32, torch.bfloat16) and dx.dtype == torch.float32
    odt = out_dtype if out_dtype is not None else (dt(scale) if scale is not None else dt(x))
    ws = None
    if dw is not None:
        ws = workspace(lib().query("uva_layernorm_bwd_workspace", rows, D), x.device)
    _call("uva_layernorm_bwd", dt(x), odt, ptr(x), ptr(w), ptr(b), ptr(scale), ldm, ptr(dy), dt(dy), ptr(mean),
               ptr(rstd),
               ptr(dx_base), ptr(dx), int(accum), ptr(dscale), ptr(dshift), ptr(dw), ptr(db), int(accum_wb), ptr(ws), rows, D,
               stream())


def layernorm_bwd_drop(x, w, dy, mean, rstd, dx, dw, db, dx_base, drop_out, drop_p, seed, dbias, accum_wb=True,
                       accum_dbias=True):
    """layernorm_bwd (fp32 x / dx, bf16 dy, D 768, affine, dx_base) + drop_out = bf16(drop(dx)) and dbias (+)=
    colsum(drop_out) in one pass (uva_layernorm_bwd_drop).  -> False when the form is not covered."""
    rows, D = x.shape
    if not (D == 768 and x.dtype == torch.float32 and dy.dtype == torch.bfloat16 and dx_base is not None
            and drop_out.dtype == torch.bfloat16 and drop_out.is_contiguous() and dx_base.is_contiguous()):
        return False
    ws = workspace(3 * ((rows + 63) // 64) * D, x.device)
    _call("uva_layernorm_bwd_drop", ptr(x), ptr(w), ptr(dy), ptr(mean), ptr(rstd), ptr(dx_base), ptr(dx), ptr(dw),
          ptr(db), int(accum_wb), ptr(drop_out), float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(dbias),
          int(accum_dbias), ptr(ws), rows, D, stream())
    return True


def softmax_fwd(S, P, Pd, L, scale, drop_p=0.0, seed=0):
    rows = S.numel() // L
    _call("uva_softmax_fwd", dt(S), ptr(S), ptr(P), ptr(Pd), rows, L, float(scale), float(drop_p),
               int(seed) & 0xFFFFFFFFFFFFFFFF, stream())


def softmax_bwd(P, dPd, dS, L, scale, drop_p=0.0, seed=0):
    rows = P.numel() // L
    _call("uva_softmax_bwd", dt(P), ptr(P), ptr(dPd), ptr(dS), rows, L, float(scale), float(drop_p),
               int(seed) & 0xFFFFFFFFFFFFFFFF, stream())


def transpose_bf16(src, dst):
    """dst [C, R] = src [R, C]^T (bf16, contiguous)"""
    R, C = src.shape
    assert src.dtype == dst.dtype == torch.bfloat16 and src.is_contiguous() and dst.is_contiguous()
    assert tuple(dst.shape) == (C, R)
    _call("uva_transpose_bf16", ptr(src), ptr(dst), R, C, stream())


def cast(src, dst):
    if src.dim() == 1 or (src.is_contiguous() and dst.is_contiguous()):
        rows, cols = 1, src.numel()
        lds = ldd = cols
    else:
        rows, cols = src.shape
        lds, ldd = _ld(src), _ld(dst)
    _call("uva_cast", dt(src), ptr(src), lds, dt(dst), ptr(dst), ldd, rows, cols, stream())


def act_fwd(x, y, act):
    _call("uva_act_fwd", dt(x), ptr(x), dt(y), ptr(y), x.numel(), ACT[act], stream())


def act_drop_fwd(x, y, act="none", drop_p=0.0, seed=0, residual=None):
    """y = residual + dropout(act(x)); contiguous, same element count (mask = flat index)."""
    assert x.is_contiguous() and y.is_contiguous() and x.numel() == y.numel()
    if residual is not None:
        assert residual.is_contiguous() and residual.numel() == x.numel()
    _call("uva_act_drop_fwd", dt(x), ptr(x), dt(y), ptr(y), dt(residual) if residual is not None else 0,
               ptr(residual), x.numel(), ACT[act], float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, stream())


def act_bwd(pre, dy, dx, act, drop_p=0.0, seed=0, accum=False):
    """dx (+)= dy * dropout_mask * act'(pre); 2-D views (pre contiguous)."""
    rows, cols = dy.shape
    _call("uva_act_bwd", dt(pre) if pre is not None else F32, ptr(pre), dt(dy), ptr(dy), _ld(dy), dt(dx),
               ptr(dx), _ld(dx), rows, cols, ACT[act], float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, int(accum),
               stream())


def act_bwd_bias(pre, dy, dx, dbias, act, drop_p=0.0, seed=0, accum=False, accum_bias=True):
    """act_bwd + dbias (+)= column sums of dx (one pass: the nn.Linear bias gradient)."""
    rows, cols = dy.shape
    ws = workspace(lib().query("uva_act_bwd_bias_workspace", rows, cols), dy.device)
    _call("uva_act_bwd_bias", dt(pre) if pre is not None else F32, ptr(pre), dt(dy), ptr(dy), _ld(dy), dt(dx),
               ptr(dx), _ld(dx), rows, cols, ACT[act], float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, int(accum),
               ptr(dbias), int(accum_bias), ptr(ws), stream())


def gate_bwd(dout, h, gate, dh, dgate):
    rows, cols = dout.shape
    _call("uva_gate_bwd", ptr(dout), dt(h), ptr(h), dt(gate), ptr(gate), _ld(gate), dt(dh), ptr(dh),
               ptr(dgate), rows, cols, stream())


def fill(t, v):
    _call("uva_fill", ptr(t), t.numel(), float(v), stream())


def _tables_arg(tables):
    arr = (ctypes.c_void_p * 8)(*[t.data_ptr() for t in tables])
    return arr


def q_sample(x0, noise, t, tables, xt):
    rows, C = x0.shape
    arr = _tables_arg(tables)
    _call("uva_q_sample", ptr(x0), ptr(noise), ptr(t), ctypes.cast(arr, ctypes.c_void_p), dt(xt), ptr(xt),
               rows, C, stream())


def timestep_features(t, freqs, out):
    rows = t.numel()
    _call("uva_timestep_features", ptr(t), ptr(freqs), dt(out), ptr(out), rows, freqs.numel(), stream())


def diffusion_loss(x0, noise, t, out, tables, loss_row, dl):
    rows, C = x0.shape
    arr = _tables_arg(tables)
    _call("uva_diffusion_loss", ptr(x0), ptr(noise), ptr(t), dt(out), ptr(out), _ld(out),
               ctypes.cast(arr, ctypes.c_void_p), ptr(loss_row), ptr(dl), rows, C, stream())


def sampler_persistent(pack, mod, coef, noise, x0, x_out, work, clip=True, eps=1e-6):
    """The whole p_sample_loop of the action head in one launch (uva_sampler_persistent).
    pack: dict of the stacked weights (w1, b1, w2, b2, lnw, lnb, win, bin, wf, bfin); mod [S, R, ncol]
    bf16; coef [S, 8] fp32; noise [S, R, C]; x0 / x_out [R, C] fp32; work: uva_sampler_persistent_workspace
    bytes (uint8, 256-B aligned)."""
    S, R, C = noise.shape
    depth, W = pack["b1"].shape
    for t in (coef, noise, x0, x_out, mod):
        if not t.is_contiguous():
            raise ValueError("sampler_persistent: contiguous operands required")
    if mod.shape[:2] != (S, R) or coef.shape != (S, 8) or x0.shape != (R, C) or x_out.shape != (R, C):
        raise ValueError("sampler_persistent: shape mismatch")
    _call("uva_sampler_persistent", R, C, W, depth, S, int(clip), float(eps), ptr(pack["w1"]), ptr(pack["b1"]),
               ptr(pack["w2"]), ptr(pack["b2"]), ptr(pack["lnw"]), ptr(pack["lnb"]), ptr(pack["win"]),
               ptr(pack["bin"]), ptr(pack["wf"]), ptr(pack["bfin"]), ptr(mod), mod.shape[2], ptr(coef), ptr(noise),
               ptr(x0), ptr(x_out), ptr(work), work.numel(), stream())


def sampler_persistent_test_hook(no_publish=True):
    """tests only: the next uva_sampler_persistent launch publishes no phase (forces the give-up path)."""
    _call("uva_sampler_persistent_test_hook", int(bool(no_publish)))


PERSISTENT_SAMPLER_CUS = 64  # workgroups of uva_sampler_persistent, one per CU, all co-resident


def sampler_persistent_fits(device):
    """the persistent sampler's 64 workgroups (96 KB of LDS each: one per CU) can all be resident at
    once on `device` -- False on a partitioned device with fewer CUs, where every hand-off would spin
    into its bound."""
    return torch.cuda.get_device_properties(device).multi_processor_count >= PERSISTENT_SAMPLER_CUS


def sampler_persistent_workspace(W, device):
    return torch.empty(lib().query("uva_sampler_persistent_workspace", W), dtype=torch.uint8, device=device)


def sampler_persistent_status(work):
    """1 if a spin of the last persistent sampler run on `work` gave up (results invalid); syncs."""
    flag = ctypes.c_uint(0)
    _call("uva_sampler_persistent_status", ptr(work), ctypes.cast(ctypes.pointer(flag), ctypes.c_void_p),
               stream())
    return flag.value


def p_sample_step(out, x, noise, coef, x_new, x_net=None, clip=True):
    """One reverse diffusion step (uva_p_sample_step); coef = 8 python floats of the step."""
    rows, C = x.shape
    if out.shape[0] != rows or out.shape[1] != 2 * C or out.stride(1) != 1:
        raise ValueError(f"p_sample_step: out {tuple(out.shape)} vs x {tuple(x.shape)}")
    for t in (x, noise, x_new):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.shape != x.shape:
            raise ValueError("p_sample_step: x / noise / x_new must be contiguous fp32 [rows, C]")
    if x_net is not None and (not x_net.is_contiguous() or x_net.shape != x.shape):
        raise ValueError("p_sample_step: x_net must be contiguous [rows, C]")
    k = (ctypes.c_float * 8)(*coef)
    _call("uva_p_sample_step", dt(out), ptr(out), out.stride(0), ptr(x), ptr(noise),
               ctypes.cast(k, ctypes.c_void_p), ptr(x_new), dt(x_net) if x_net is not None else 0,
               ptr(x_net), int(clip), rows, C, stream())


def sampler_linear(A, W, out, bias=None, act="none", ln=False, lnw=None, lnb=None, shift=None, scale=None,
                   eps=1e-6, gate=None, residual=None):
    """Few-row fused linear (uva_sampler_linear): out = epi(A' @ W^T + bias), A' = A (bf16) or the
    adaLN-modulated LayerNorm of fp32 rows A (ln=True)."""
    R, K = A.shape
    N = W.shape[0]
    if W.shape[1] != K or W.dtype != torch.bfloat16 or W.stride(1) != 1 or W.stride(0) != K:
        raise ValueError(f"sampler_linear: W {tuple(W.shape)} must be contiguous bf16 [N, {K}]")
    if out.shape != (R, N) or out.stride(1) != 1:
        raise ValueError(f"sampler_linear: out {tuple(out.shape)} != {(R, N)}")
    if A.stride(1) != 1 or A.dtype != (torch.float32 if ln else torch.bfloat16):
        raise ValueError("sampler_linear: A must be row-major fp32 (ln) or bf16")
    ldm = 0
    if ln:
        if shift is None or scale is None or shift.stride(0) != scale.stride(0) or shift.dtype != torch.bfloat16:
            raise ValueError("sampler_linear: ln needs bf16 shift/scale views with one row stride")
        ldm = shift.stride(0)
    ldg = gate.stride(0) if gate is not None else 0
    ldr = residual.stride(0) if residual is not None else 0
    _call("uva_sampler_linear", int(ln), ptr(A), A.stride(0), ptr(lnw), ptr(lnb), ptr(shift), ptr(scale), ldm,
               float(eps), ptr(W), ptr(bias), ACT[act], ptr(gate), ldg, ptr(residual), ldr, dt(out), ptr(out),
               out.stride(0), R, N, K, stream())


def weighted_mean(l, w, res):
    _call("uva_weighted_mean", ptr(l), ptr(w), l.numel(), ptr(res), stream())


def loss_grad(dl, w, wsum, g_up, dout):
    rows, C2 = dl.shape
    _call("uva_loss_grad", ptr(dl), ptr(w), ptr(wsum), ptr(g_up), dt(dout), ptr(dout), _ld(dout), rows, C2,
               stream())


def adamw_ema(p, g, m, v, ema, p_bf16, n_decay, lr, b1, b2, eps, wd, step, grad_scale, ema_decay):
    _call("uva_adamw_ema", ptr(p), ptr(g), ptr(m), ptr(v), ptr(ema), ptr(p_bf16), p.numel(), int(n_decay),
               float(lr), float(b1), float(b2), float(eps), float(wd), int(step), float(grad_scale),
               float(ema_decay), stream())


def ema_update(ema, p, decay):
    """ema = decay * ema + (1 - decay) * p over two flat fp32 buffers (uva_ema_update)."""
    if ema.dtype != torch.float32 or p.dtype != torch.float32 or ema.numel() != p.numel():
        raise ValueError("ema_update: two fp32 buffers of equal size")
    _call("uva_ema_update", ptr(ema), ptr(p), ema.numel(), float(decay), stream())


def attn_mask_alloc(B, N, H, device):
    return torch.empty(lib().query("uva_attn_mask_bytes", B, N, H), dtype=torch.uint8, device=device)


def attn_dropmask(B, N, H, drop_p, seed, device, out=None):
    """keep-mask bit planes of attention dropout (counter hash of (seed, element)), shared by
    attn_fwd and attn_bwd of the same step."""
    mask = attn_mask_alloc(B, N, H, device) if out is None else out
    assert mask.numel() == lib().query("uva_attn_mask_bytes", B, N, H) and mask.dtype == torch.uint8
    _call("uva_attn_dropmask", ptr(mask), B, N, H, float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, stream())
    return mask


def attn_fwd(qkv, out, lse2, B, N, H, scale, drop_p=0.0, seed=0, mask=None):
    """-> the dropout mask planes (None when drop_p == 0); pass them to attn_bwd."""
    assert qkv.dtype == torch.bfloat16 and qkv.is_contiguous() and out.is_contiguous()
    assert N % 64 == 0 and qkv.shape[-1] == 3 * H * 64
    assert qkv.numel() == B * N * 3 * H * 64 and out.numel() == B * N * H * 64 and lse2.numel() == B * H * N
    with _traced(f"attn_fwd B{B} N{N} H{H}", 4.0 * B * H * N * N * 64):
        if drop_p > 0 and mask is None:
            mask = attn_dropmask(B, N, H, drop_p, seed, qkv.device)
        _call("uva_attn_fwd", ptr(qkv), ptr(out), ptr(lse2), ptr(mask) if drop_p > 0 else None, B, N, H,
                   float(scale), float(drop_p), stream())
    return mask if drop_p > 0 else None


def attn_fp8_workspace(B, N, H, device):
    return torch.empty(lib().query("uva_attn_fp8_workspace", B, N, H), dtype=torch.uint8, device=device)


def attn_quant_fp8(qkv, ws, B, N, H):
    """round qkv [B,N,3,H,64] bf16 in place to the fp8 grid; fp8 Q/K, V^T and scales -> ws."""
    assert qkv.dtype == torch.bfloat16 and qkv.is_contiguous() and qkv.numel() == B * N * 3 * H * 64
    assert N % 64 == 0 and ws.dtype == torch.uint8 and ws.numel() >= lib().query("uva_attn_fp8_workspace", B, N, H)
    _call("uva_attn_quant_fp8", ptr(qkv), ptr(ws), B, N, H, stream())


def attn_fwd_fp8(ws, out, lse2, B, N, H, scale, drop_p=0.0, seed=0, mask=None, device=None):
    """fp8 forward from attn_quant_fp8's workspace -> the dropout mask planes (None when p == 0)."""
    assert out.dtype == torch.bfloat16 and out.is_contiguous() and out.numel() == B * N * H * 64
    assert lse2.numel() == B * H * N and N % 64 == 0
    with _traced(f"attn_fwd_fp8 B{B} N{N} H{H}", 4.0 * B * H * N * N * 64):
        if drop_p > 0 and mask is None:
            mask = attn_dropmask(B, N, H, drop_p, seed, out.device)
        _call("uva_attn_fwd_fp8", ptr(ws), ptr(out), ptr(lse2), ptr(mask) if drop_p > 0 else None, B, N, H,
                   float(scale), float(drop_p), stream())
    return mask if drop_p > 0 else None


def attn_bwd(qkv, out, dout, lse2, dvec, dqkv, B, N, H, scale, drop_p=0.0, seed=0, mask=None, dbias=None,
             accum_bias=True):
    """flash attention backward -> dqkv; with `dbias` ([3 H 64] fp32) also the qkv bias gradient (column sums of
    dqkv as stored) from the kernels' epilogues (uva_attn_bwd_bias)"""
    assert dout.dtype == torch.bfloat16 and dout.is_contiguous() and dqkv.is_contiguous()
    assert dout.numel() == B * N * H * 64 and dqkv.numel() == B * N * 3 * H * 64 and dvec.numel() == B * H * N
    with _traced(f"attn_bwd B{B} N{N} H{H}", 8.0 * B * H * N * N * 64):
        if drop_p > 0 and mask is None:
            mask = attn_dropmask(B, N, H, drop_p, seed, qkv.device)
        if dbias is not None:
            assert dbias.dtype == torch.float32 and dbias.numel() == 3 * H * 64 and dbias.is_contiguous()
            ws = workspace(B * ((N + 127) // 128) * 3 * H * 64, qkv.device)
            _call("uva_attn_bwd_bias", ptr(qkv), ptr(out), ptr(dout), ptr(lse2), ptr(mask) if drop_p > 0 else None,
                  ptr(dvec), ptr(dqkv), ptr(dbias), int(accum_bias), ptr(ws), B, N, H, float(scale), float(drop_p),
                  stream())
            return
        nb = lib().query("uva_attn_bwd_workspace", B, N, H, float(drop_p))
        ws = torch.empty(nb, dtype=torch.uint8, device=qkv.device) if nb else None
        _call("uva_attn_bwd", ptr(qkv), ptr(out), ptr(dout), ptr(lse2), ptr(mask) if drop_p > 0 else None,
                   ptr(dvec), ptr(dqkv), ptr(ws), B, N, H, float(scale), float(drop_p), stream())


def conv2d(x, w, out, Nimg, Hin, Win, Ci, Co, ks, stride, pad_t, pad_l, Hout, Wout, bias=None, residual=None,
           gn_scale=None, gn_shift=None, gn_silu=True, act="none", force_generic=False, gn_part=None):
    """NHWC implicit-GEMM conv; w stored [Co][ks][ks][Ci]."""
    assert x.dtype == w.dtype == out.dtype
    assert w.numel() == Co * ks * ks * Ci and out.numel() == Nimg * Hout * Wout * Co
    if residual is not None:
        assert residual.dtype == out.dtype and residual.numel() == out.numel()
    with _traced(f"conv{ks}x{ks}/s{stride} {'bf16' if dt(x) else 'f32'} {Hin}x{Win} Ci{Ci} Co{Co} n{Nimg}",
                 2.0 * Nimg * Hout * Wout * Co * ks * ks * Ci):
        _conv_call(x, w, out, Nimg, Hin, Win, Ci, Co, ks, stride, pad_t, pad_l, Hout, Wout, bias, residual, gn_scale,
                   gn_shift, gn_silu, act, force_generic, gn_part)


def _conv_call(x, w, out, Nimg, Hin, Win, Ci, Co, ks, stride, pad_t, pad_l, Hout, Wout, bias, residual, gn_scale,
               gn_shift, gn_silu, act, force_generic, gn_part):
    _call("uva_conv2d", dt(x), ptr(x), ptr(w), ptr(out), ptr(bias), ptr(residual), Nimg, Hin, Win, Ci, Co, ks,
               stride, pad_t, pad_l, Hout, Wout, ptr(gn_scale), ptr(gn_shift), int(gn_silu), ACT[act], ptr(gn_part),
               int(force_generic), stream())


def conv_fuses_gn(Nimg, H, W, Ci, Co, ks, stride, dtype=torch.bfloat16):
    """True when uva_conv2d runs this conv on the halo kernel, which applies a GroupNorm(+SiLU)
    prologue while staging its input tile (no separate GN-apply pass needed)."""
    return (dtype == torch.bfloat16 and ks == 3 and stride == 1 and
            lib().query("uva_conv3x3_halo_bn", Nimg, H, W, Ci, Co) > 0)


def pool4x4_cwh(x, out, n, C):
    """AdaptiveAvgPool2d((4,4)) of NHWC [n,16,16,C] flattened (c w h) -> out [n, 16 C]"""
    assert x.is_contiguous() and out.is_contiguous() and x.dtype == out.dtype
    assert x.numel() == n * 256 * C and out.numel() == n * 16 * C
    _call("uva_pool4x4_cwh", dt(x), ptr(x), ptr(out), n, C, stream())


def pool4x4_relu_bwd(post, gpool, dpre, n, C):
    assert post.is_contiguous() and gpool.is_contiguous() and dpre.is_contiguous() and post.dtype == dpre.dtype
    assert post.numel() == dpre.numel() == n * 256 * C and gpool.numel() == n * 16 * C
    _call("uva_pool4x4_relu_bwd", dt(post), ptr(post), dt(gpool), ptr(gpool), ptr(dpre), n, C, stream())


def im2col3x3(x, cols, n, H, W, Ci):
    assert x.is_contiguous() and cols.is_contiguous() and x.dtype == cols.dtype
    assert x.numel() == n * H * W * Ci and cols.numel() == n * H * W * Ci * 9
    _call("uva_im2col3x3", dt(x), ptr(x), ptr(cols), n, H, W, Ci, stream())


def im2col3x3_tc(x, cols, n, H, W, Ci):
    """tap-major im2col: cols[p][tap*Ci + ci] (uva_im2col3x3_tc)."""
    assert x.is_contiguous() and cols.is_contiguous() and x.dtype == cols.dtype
    assert x.numel() == n * H * W * Ci and cols.numel() == n * H * W * Ci * 9
    _call("uva_im2col3x3_tc", dt(x), ptr(x), ptr(cols), n, H, W, Ci, stream())


def pad_nhwc(x, out, n, H, W, C, G):
    """out[G + (img (H+2) + y) (W+2) + x] = x[img][y-1][x-1] (zero border and G zero guard rows)."""
    assert x.is_contiguous() and out.is_contiguous() and x.dtype == out.dtype
    assert out.numel() == (2 * G + n * (H + 2) * (W + 2)) * C
    _call("uva_pad_nhwc", dt(x), ptr(x), ptr(out), n, H, W, C, G, stream())


def conv3x3_dw_implicit(dy, x, part, n, H, W, Co, Ci):
    """part[co][kh*3 + kw][ci] = sum_p dy[p][co] x[p + tap shift][ci] (fp32, overwritten): the weight
    gradient of a 3x3 / p1 conv over NHWC dy [n,H,W,Co] / x [n,H,W,Ci] as 9 GEMMs on padded copies."""
    G = W + 3
    K = n * (H + 2) * (W + 2)
    dyp = torch.empty(2 * G + K, Co, dtype=dy.dtype, device=dy.device)
    xp = torch.empty(2 * G + K, Ci, dtype=x.dtype, device=x.device)
    pad_nhwc(dy, dyp, n, H, W, Co, G)
    pad_nhwc(x, xp, n, H, W, Ci, G)
    for kh in range(3):
        for kw in range(3):
            tap = kh * 3 + kw
            d = (kh - 1) * (W + 2) + (kw - 1)
            gemm(dyp[G:], xp[G + d:], part[:, tap * Ci:], Co, Ci, K, Co, Ci, 9 * Ci, 1, 1, beta=0.0)


def conv3x3_dw_scatter_add(part, grad):
    """grad[co][ci][kh][kw] += part[co][kh*3 + kw][ci] (fp32)."""
    Co, Ci = grad.shape[0], grad.shape[1]
    assert part.dtype == grad.dtype == torch.float32 and part.is_contiguous() and grad.is_contiguous()
    assert part.numel() == grad.numel() == Co * Ci * 9
    _call("uva_conv3x3_dw_scatter_add", ptr(part), ptr(grad), Co, Ci, stream())


def conv3x3_weight_layout(w, out, mode):
    """fp32 nn.Conv2d weight [Co,Ci,3,3] -> mode 0 [Co,3,3,Ci] / mode 1 flipped [Ci,3,3,Co]"""
    Co, Ci = w.shape[0], w.shape[1]
    assert w.dtype == torch.float32 and w.is_contiguous() and out.is_contiguous() and out.numel() == w.numel()
    _call("uva_conv3x3_weight_layout", ptr(w), dt(out), ptr(out), Co, Ci, int(mode), stream())


def groupnorm_finalize_tiles(part, Nimg, HW, C, gamma, beta, scale, shift, eps=1e-6, tile_rows=128):
    _call("uva_groupnorm_finalize_tiles", ptr(part), Nimg, HW, C, tile_rows, ptr(gamma), ptr(beta), float(eps),
               ptr(scale), ptr(shift), stream())


def groupnorm_apply(x, scale, shift, y, Nimg, HW, C, silu=True):
    _call("uva_groupnorm_apply", ptr(x), ptr(scale), ptr(shift), ptr(y), Nimg, HW, C, int(silu), stream())


def groupnorm_stats(x, Nimg, HW, C, gamma, beta, scale, shift, eps=1e-6):
    ws = workspace(lib().query("uva_groupnorm_workspace", Nimg, HW), x.device)
    _call("uva_groupnorm_stats", dt(x), ptr(x), Nimg, HW, C, ptr(gamma), ptr(beta), float(eps), ptr(scale),
               ptr(shift), ptr(ws), stream())


def resize_select(img, sel, out, Cpad):
    B, T, C, H, W = img.shape
    assert C == 3 and img.dtype == torch.float32 and img.is_contiguous()
    _call("uva_resize_select", ptr(img), B, T, H, W, ptr(sel), sel.numel(), dt(out), ptr(out), Cpad, stream())


def posterior_sample(moments, eps, z, Nimg, scale=0.2325):
    _call("uva_posterior_sample", dt(moments), ptr(moments), ptr(eps), ptr(z), Nimg, float(scale), stream())


def upsample_nearest2x(x, y):
    """NHWC nearest x2 (uva_upsample_nearest2x)."""
    n, H, W, C = x.shape
    if not (x.is_contiguous() and y.is_contiguous() and y.shape == (n, 2 * H, 2 * W, C) and y.dtype == x.dtype):
        raise ValueError(f"upsample_nearest2x: {tuple(x.shape)} -> {tuple(y.shape)}")
    _call("uva_upsample_nearest2x", dt(x), ptr(x), ptr(y), n, H, W, C, stream())
