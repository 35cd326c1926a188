"""Kernel micro-benchmarks at the MAR training shapes (B=32, N=1024, D=768)."""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main(attn_only=False):
    dev = "cuda"
    M = 32 * 1024
    for (N, K) in () if attn_only else ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        dx = torch.empty(M, K, device=dev)
        dw = torch.zeros(N, K, device=dev)
        fl = 2 * M * N * K
        t1 = timeit(lambda: ops.linear(x, w, y))
        t2 = timeit(lambda: ops.linear_dx(dy, w, dx))
        t3 = timeit(lambda: ops.linear_dw(dy, x, dw))
        tt = timeit(lambda: torch.matmul(x, w.t()))
        print(f"gemm M={M} N={N} K={K}: fwd {fl/t1/1e9:.0f} TF  dx {fl/t2/1e9:.0f} TF  dw {fl/t3/1e9:.0f} TF"
              f"   (torch/hipBLASLt fwd {fl/tt/1e9:.0f} TF)")
    B, N, H = 32, 1024, 12
    qkv = torch.randn(B, N, 3 * H * 64, device=dev).to(torch.bfloat16)
    out = torch.empty(B, N, H * 64, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=dev)
    dqkv = torch.empty_like(qkv)
    dvec = torch.empty(B, H, N, device=dev)
    fl = 4 * B * H * N * N * 64
    for p in (0.0, 0.1):
        mask = ops.attn_dropmask(B, N, H, p, 1, dev) if p > 0 else None
        tm = timeit(lambda: ops.attn_dropmask(B, N, H, p, 1, dev)) if p > 0 else 0.0
        t1 = timeit(lambda: ops.attn_fwd(qkv, out, lse, B, N, H, 0.125, p, 1, mask=mask))
        t2 = timeit(lambda: ops.attn_bwd(qkv, out, out, lse, dvec, dqkv, B, N, H, 0.125, p, 1, mask=mask))
        print(f"attn B={B} N={N} H={H} p={p}: mask {tm:.3f} ms, fwd {t1:.3f} ms {fl/t1/1e9:.0f} TF, bwd {t2:.3f} ms "
              f"{2*fl/t2/1e9:.0f} TF(alg 8N^2d)")
    # fp8 forward (UMI config-5 shape: B=56, N=1088) against the bf16 forward of the same shape
    for (B8, N8) in ((32, 1024), (56, 1088)):
        x8 = torch.randn(B8, N8, 3 * H * 64, device=dev).to(torch.bfloat16)
        o8 = torch.empty(B8, N8, H * 64, device=dev, dtype=torch.bfloat16)
        l8 = torch.empty(B8, H, N8, device=dev)
        ws8 = ops.attn_fp8_workspace(B8, N8, H, dev)
        m8 = ops.attn_dropmask(B8, N8, H, 0.1, 1, dev)
        fl8 = 4 * B8 * H * N8 * N8 * 64
        tq = timeit(lambda: ops.attn_quant_fp8(x8, ws8, B8, N8, H))
        tf = timeit(lambda: ops.attn_fwd_fp8(ws8, o8, l8, B8, N8, H, 0.125, 0.1, 1, mask=m8))
        tb = timeit(lambda: ops.attn_fwd(x8, o8, l8, B8, N8, H, 0.125, 0.1, 1, mask=m8))
        print(f"attn B={B8} N={N8} p=0.1: fp8 quant {tq:.3f} ms, fp8 fwd {tf:.3f} ms {fl8/tf/1e9:.0f} TF, "
              f"bf16 fwd {tb:.3f} ms {fl8/tb/1e9:.0f} TF (fp8/bf16 {tf/tb:.2f}, incl. quant {(tf+tq)/tb:.2f})")
    q = qkv.view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    ts = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q[0], q[1], q[2]))
    print(f"torch sdpa fwd {ts:.3f} ms {fl/ts/1e9:.0f} TF")
    x = torch.randn(M, 768, device=dev)
    yb = torch.empty(M, 768, device=dev, dtype=torch.bfloat16)
    w = torch.ones(768, device=dev)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    t = timeit(lambda: ops.layernorm_fwd(x, w, w, yb, mean, rstd))
    print(f"layernorm fwd f32->bf16 [{M},768]: {t*1e3:.1f} us, {M*768*6/t/1e6:.0f} GB/s")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()
if __name__ == "__main__" and sys.argv[1:] == ["attn"]:
    main(attn_only=True)


def conv_bench():
    dev = "cuda"
    x = torch.rand(256, 256, 256, 8, device=dev).to(torch.bfloat16)
    w = (torch.randn(128, 3, 3, 8, device=dev) * 0.05).to(torch.bfloat16)
    out = torch.empty(256, 256, 256, 128, device=dev, dtype=torch.bfloat16)
    part = torch.empty(256 * 256 * 256 // 128, 32, 2, device=dev)
    t = timeit(lambda: ops.conv2d(x, w, out, 256, 256, 256, 8, 128, 3, 1, 1, 1, 256, 256, gn_part=part), iters=5)
    print(f"conv_in n256 256x256 Ci8 Co128: {t:.3f} ms, output stream {out.numel() * 2 / t / 1e6:.0f} GB/s")
    for (n, H, Ci, Co) in ((256, 256, 128, 128), (256, 128, 128, 128), (256, 64, 256, 256), (256, 16, 512, 512)):
        x = torch.randn(n, H, H, Ci, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, 3, 3, Ci, device=dev) * 0.05).to(torch.bfloat16)
        out = torch.empty(n, H, H, Co, device=dev, dtype=torch.bfloat16)
        fl = 2 * n * H * H * Co * 9 * Ci
        t = timeit(lambda: ops.conv2d(x, w, out, n, H, H, Ci, Co, 3, 1, 1, 1, H, H), iters=5)
        sc = torch.rand(n, Ci, device=dev) + 0.5
        sh = torch.randn(n, Ci, device=dev) * 0.3
        res = torch.randn(n, H, H, Co, device=dev).to(torch.bfloat16)
        bias = torch.randn(Co, device=dev)
        part = torch.empty(n * H * H // 128, 32, 2, device=dev)
        tg = timeit(lambda: ops.conv2d(x, w, out, n, H, H, Ci, Co, 3, 1, 1, 1, H, H, gn_scale=sc, gn_shift=sh), iters=5)
        te = timeit(lambda: ops.conv2d(x, w, out, n, H, H, Ci, Co, 3, 1, 1, 1, H, H, bias=bias, residual=res,
                                       gn_part=part), iters=5)
        t2 = timeit(lambda: ops.conv2d(x, w, out, n, H, H, Ci, Co, 3, 1, 1, 1, H, H, bias=bias, residual=res,
                                       gn_scale=sc, gn_shift=sh, gn_part=part), iters=5)
        print(f"conv3x3 n{n} {H}x{H} Ci{Ci} Co{Co}: plain {t:.2f} ms {fl/t/1e9:.0f} TF | GN/SiLU prologue {tg:.2f} | "
              f"bias+res+GN-stats epilogue {te:.2f} | all {t2:.2f} ms {fl/t2/1e9:.0f} TF")


def conv_s2_bench():
    """VAE Downsample convs: F.pad(0,1,0,1) + 3x3 / stride 2 (vaekl.py:36-53) at the encoder shapes."""
    dev = "cuda"
    for (n, H, C) in ((256, 256, 128), (256, 128, 128), (256, 64, 256), (256, 32, 256)):
        x = torch.randn(n, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
        Ho = H // 2
        out = torch.empty(n, Ho, Ho, C, device=dev, dtype=torch.bfloat16)
        bias = torch.randn(C, device=dev)
        part = torch.empty(n * Ho * Ho // 128, 32, 2, device=dev)
        fl = 2 * n * Ho * Ho * C * 9 * C
        t = timeit(lambda: ops.conv2d(x, w, out, n, H, H, C, C, 3, 2, 0, 0, Ho, Ho, bias=bias, gn_part=part), iters=5)
        print(f"conv3x3/s2 n{n} {H}x{H} C{C}: {t:.3f} ms {fl/t/1e9:.0f} TF")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "conv":
    conv_bench()
if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "convs2":
    conv_s2_bench()


def square_bench():
    """Square GEMMs (uniform random bf16) to separate kernel quality from shape effects."""
    dev = "cuda"
    for S in (4096, 8192):
        a = (torch.rand(S, S, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(S, S, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty(S, S, device=dev, dtype=torch.bfloat16)
        fl = 2 * S ** 3
        res = []
        for ta, tb in ((0, 0), (0, 1), (1, 1)):
            t = timeit(lambda: ops.gemm(a, b, c, S, S, S, S, S, S, ta, tb), iters=10)
            res.append(f"({ta},{tb}) {fl/t/1e9:.0f}")
        tt = timeit(lambda: torch.matmul(a, b.t()), iters=10)
        print(f"square {S}^3 plan {ops.gemm_plan(S, S, S)}: " + "  ".join(res) + f" TF   hipBLASLt {fl/tt/1e9:.0f} TF")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "square":
    square_bench()


def rowk_bench():
    """HBM-bound row kernels at the Block shapes: LN fwd / bwd (fp32 residual stream, bf16 dy)."""
    dev = "cuda"
    M, D = 32768, 768
    x = torch.randn(M, D, device=dev)
    w = torch.randn(D, device=dev)
    b = torch.randn(D, device=dev)
    yb = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    t = timeit(lambda: ops.layernorm_fwd(x, w, b, yb, mean, rstd))
    print(f"ln_fwd f32->bf16 [{M},{D}]: {t*1e3:.1f} us, {M*D*6/t/1e6:.0f} GB/s")
    dy = torch.randn(M, D, device=dev).to(torch.bfloat16)
    dxb = torch.randn(M, D, device=dev)
    dx = torch.empty(M, D, device=dev)
    dw = torch.zeros(D, device=dev)
    db = torch.zeros(D, device=dev)
    t = timeit(lambda: ops.layernorm_bwd(x, w, dy, mean, rstd, dx, False, dw=dw, db=db, dx_base=dxb, b=b))
    print(f"ln_bwd x f32 dy bf16 +dx_base [{M},{D}] dw/db: {t*1e3:.1f} us, {M*D*14/t/1e6:.0f} GB/s")
    # DiffLoss res-block adaLN LayerNorm backward: D = 1024, fp32 dy, modulation rows of a [M, 3D] bf16 table
    Wd = 1024
    x1 = torch.randn(M, Wd, device=dev)
    mean1 = x1.mean(-1)
    rstd1 = 1 / x1.var(-1, unbiased=False).add(1e-6).sqrt()
    mod = (torch.randn(M, 3 * Wd, device=dev) * 0.1).to(torch.bfloat16)
    dyf = torch.randn(M, Wd, device=dev)
    dx1 = torch.empty(M, Wd, device=dev)
    dmod = torch.empty(M, 3 * Wd, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.layernorm_bwd(x1, None, dyf, mean1, rstd1, dx1, False, scale=mod[:, Wd:2 * Wd], ldm=3 * Wd,
                                         dscale=dmod[:, Wd:2 * Wd], dshift=dmod[:, :Wd]))
    print(f"ln_bwd adaLN x f32 dy f32 [{M},{Wd}]: {t*1e3:.1f} us, {M*Wd*18/t/1e6:.0f} GB/s")
    # fc1 GELU + dropout backward with the fc1 bias gradient (bf16 pre-activation, bf16 dy / dx)
    F = 3072
    pre = torch.randn(M, F, device=dev).to(torch.bfloat16)
    g = torch.randn(M, F, device=dev).to(torch.bfloat16)
    gx = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    dbias = torch.zeros(F, device=dev)
    t = timeit(lambda: ops.act_bwd_bias(pre, g, gx, dbias, "gelu", drop_p=0.1, seed=3))
    print(f"act_bwd_bias gelu+dropout bf16 [{M},{F}]: {t*1e3:.1f} us, {M*F*6/t/1e6:.0f} GB/s")
    # timm Mlp forward elementwise passes: fc1 GELU + dropout (bf16 -> bf16), fc2 dropout + fp32 residual
    t = timeit(lambda: ops.act_drop_fwd(pre, gx, "gelu", drop_p=0.1, seed=3))
    print(f"act_drop_fwd gelu+dropout bf16 [{M},{F}]: {t*1e3:.1f} us, {M*F*4/t/1e6:.0f} GB/s")
    h = torch.randn(M, D, device=dev).to(torch.bfloat16)
    t = timeit(lambda: ops.act_drop_fwd(h, dx, "none", drop_p=0.1, seed=3, residual=dxb))
    print(f"act_drop_fwd dropout+res bf16/f32 [{M},{D}]: {t*1e3:.1f} us, {M*D*10/t/1e6:.0f} GB/s")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "rowk":
    rowk_bench()


def resgemm_bench():
    """The fp32-residual N = 768 forward products of a timm Block as the training step runs them:
    attention proj (K = 768) and fc2 (K = 3072), bias + dropout 0.1 + fp32 residual, fp32 out."""
    dev = "cuda"
    M, N = 32 * 1024, 768
    for K in (768, 3072):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        res = torch.randn(M, N, device=dev)
        y = torch.empty(M, N, device=dev)
        fl = 2 * M * N * K
        t = timeit(lambda: ops.linear(x, w, y, bias=b, residual=res, drop_p=0.1, seed=5))
        print(f"resgemm M={M} N={N} K={K} bias+drop+f32res: {t:.4f} ms {fl/t/1e9:.0f} TF, "
              f"{(M*K*2 + M*N*8)/t/1e6:.0f} GB/s")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "resgemm":
    resgemm_bench()


def aug_bench():
    """UMI video augmentation (B=56 videos x 8 frames of 224^2, every op on) and Libero ColorJitter
    (B=32 x 8 x 128^2): time per launch and HBM rate on the algorithmic bytes (frames in + out)."""
    from unified_video_action_amd.utils.augment import libero_jitter_params, umi_aug_params, video_augment
    for name, (B, T, S, prm) in {"umi": (56, 8, 224, None), "libero": (32, 8, 128, None)}.items():
        x = torch.rand(B, T, 3, S, S, device="cuda")
        if name == "umi":
            p = umi_aug_params(range(B))
            p[:, 0], p[:, 1], p[:, 2], p[:, 3], p[:, 12], p[:, 13], p[:, 14], p[:, 16] = 1, 8, 8, 1, 1, 1.5, 1, 1
            p[:, 17:22] = torch.tensor([0.05, 0.25, 0.4, 0.25, 0.05])
            p[:, 8:12] = torch.tensor([1.1, 0.9, 1.2, 0.3])
        else:
            p = libero_jitter_params(range(B))
        from unified_video_action_amd.native.lib import lib
        out = torch.empty_like(x)
        from unified_video_action_amd.utils.augment import aug_scratch_floats
        scratch = torch.empty(aug_scratch_floats(B, T, S), device="cuda")
        pd = p.cuda()
        ms_api = timeit(lambda: video_augment(x, p))  # host validation + params H2D included
        ms = timeit(lambda: lib().call("uva_video_augment", ops.ptr(x), ops.ptr(out), ops.ptr(scratch), ops.ptr(pd),
                                       B, T, S, ops.stream()))
        torch.testing.assert_close(out, video_augment(x, p), atol=0, rtol=0)
        print(f"  ({name}: {ms_api:.3f} ms per video_augment() call incl. host-side checks)")
        gb = 2 * x.numel() * 4 / 1e9
        print(f"augment {name:7s} B={B} T={T} S={S}: {ms:.3f} ms  {gb / ms:.2f} TB/s on in+out ({gb:.3f} GB)")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "aug":
    aug_bench()


def conv0_bench():
    """The GN-fused VAE convs as the encoder runs them (GN+SiLU prologue, bias + residual + GN-stats
    epilogue): level 0 (256x256, C128) and level 1 (128x128, C128), n = 256."""
    dev = "cuda"
    for (n, H, Ci, Co) in ((256, 256, 128, 128), (256, 128, 128, 128)):
        x = torch.randn(n, H, H, Ci, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, 3, 3, Ci, device=dev) * 0.05).to(torch.bfloat16)
        out = torch.empty(n, H, H, Co, device=dev, dtype=torch.bfloat16)
        sc = torch.rand(n, Ci, device=dev) + 0.5
        sh = torch.randn(n, Ci, device=dev) * 0.3
        res = torch.randn(n, H, H, Co, device=dev).to(torch.bfloat16)
        bias = torch.randn(Co, device=dev)
        part = torch.empty(n * H * H // 128, 32, 2, device=dev)
        fl = 2 * n * H * H * Co * 9 * Ci
        for r, tag in ((res, ""), (None, " nores")):
            t = timeit(lambda: ops.conv2d(x, w, out, n, H, H, Ci, Co, 3, 1, 1, 1, H, H, bias=bias, residual=r,
                                          gn_scale=sc, gn_shift=sh, gn_part=part), iters=10)
            print(f"gnconv n{n} {H}x{H} C{Ci}{tag}: {t:.3f} ms {fl/t/1e9:.0f} TF")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "conv0":
    conv0_bench()


def blas_bench():
    """This build's products vs hipBLASLt (torch.matmul) at the Block shapes, per transposition:
    fwd x w^T, dX dy w (bf16 out both), dW dy^T x (this build: fp32 accumulate into the grad buffer;
    hipBLASLt: bf16 out, the same FLOPs)."""
    dev = "cuda"
    M = 32 * 1024
    for (N, K) in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(N, K, device=dev)
        fl = 2 * M * N * K
        r = {}
        r["fwd"] = (timeit(lambda: ops.linear(x, w, y), 60), timeit(lambda: torch.matmul(x, w.t()), 60))
        r["dx"] = (timeit(lambda: ops.linear_dx(dy, w, dx), 60), timeit(lambda: torch.matmul(dy, w), 60))
        r["dw"] = (timeit(lambda: ops.linear_dw(dy, x, dw)), timeit(lambda: torch.matmul(dy.t(), x)))
        print(f"M={M} N={N} K={K}: " + "  ".join(f"{k} {fl/a/1e9:.0f}/{fl/b/1e9:.0f}" for k, (a, b) in r.items())
              + "  TF (this build / hipBLASLt)")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "blas":
    blas_bench()
if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "blas_pp":
    ops.gemm_set_persist(True)
    blas_bench()


def skinny_bench():
    """skinny-output dW products (z_proj [768 x 16], DiffLoss input_proj [1024 x 16]) over K = tokens"""
    dev = "cuda"
    for (M, N, K) in ((768, 16, 65536), (1024, 16, 65536), (768, 16, 32768)):
        dy = torch.randn(K, M, device=dev).to(torch.bfloat16)
        x = torch.randn(K, N, device=dev).to(torch.bfloat16)
        dw = torch.zeros(M, N, device=dev)
        t = timeit(lambda: ops.linear_dw(dy, x, dw), 50)
        print(f"skinny dW M={M} N={N} K={K}: {t*1e3:.1f} us  {K*M*2/t/1e6:.0f} GB/s of dY  plan {ops.gemm_plan(M, N, K, 1, 1)}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "skinny":
    skinny_bench()


def cold_bench():
    """the small-N Block products as the step runs them: hot (repeated) vs cold (a 1 GiB write between
    calls evicts L2 and MALL); per-call HIP events around the product only"""
    dev = "cuda"
    M = 32768
    flush = torch.empty(1 << 28, device=dev)
    cases = []
    for (N, K) in ((768, 768), (768, 3072), (3072, 768), (768, 2304)):
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(N, K, device=dev)
        cases.append((f"dx  NN M{M} N{K} K{N}", lambda dy=dy, w=w, dx=dx: ops.linear_dx(dy, w, dx), 2 * M * N * K))
        cases.append((f"dW  TT M{N} N{K} K{M}", lambda dy=dy, x=x, dw=dw: ops.linear_dw(dy, x, dw), 2 * M * N * K))
        cases.append((f"fwd NT M{M} N{N} K{K}", lambda x=x, w=w, dy=dy: ops.linear(x, w, dy), 2 * M * N * K))
    for name, fn, fl in cases:
        res = []
        for cold in (False, True):
            ts = []
            for i in range(12):
                if cold:
                    flush.fill_(float(i))
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn()
                e.record()
                torch.cuda.synchronize()
                if i >= 2:
                    ts.append(s.elapsed_time(e))
            t = sorted(ts)[len(ts) // 2]
            res.append(f"{'cold' if cold else 'hot '} {t*1e3:6.1f} us {fl/t/1e9:5.0f} TF")
        print(f"{name}: " + "  ".join(res))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "cold":
    cold_bench()
