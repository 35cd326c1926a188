"""8-wave GEMM (csrc/gemm8w.hip) vs the 4-wave kernel on the Block's K-contiguous products (B = 32 PushT:
M = 32768), and the fused timm Mlp forwards (fc1 + GELU + dropout, fc2 + dropout + residual) vs the split
route (bias-only gemm_4w + act_drop_fwd); each fused result is compared with the split route's bit for bit
first.  Interleaved rounds in one process.  tools only."""
import sys

import torch

sys.path.insert(0, ".")
from unified_video_action_amd.native import ops  # noqa: E402

SHAPES = [("qkv fwd", 2304, 768), ("fc1 fwd", 3072, 768), ("fc2 fwd", 768, 3072), ("dX N768 K768", 768, 768),
          ("fc1 dX N768 K3072", 768, 3072)]
MODES = {"nw8": 64, "nw4": 32}


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


def diff(a, b):
    a, b = a.float(), b.float()
    return (a != b).sum().item(), (a - b).abs().max().item()


def plain(M, rounds):
    dev = "cuda"
    for r in range(rounds):
        print(f"== plain round {r}", flush=True)
        for name, N, K in SHAPES:
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
            b = torch.rand(N, device=dev)
            y4 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fl = 2.0 * M * N * K
            ops.gemm8w_set(0)
            t4 = timeit(lambda: ops.linear(x, w, y4, bias=b))
            line = f"{name:20s} N{N} K{K}: gemm4 {fl / t4 / 1e9:6.0f}"
            for mname, mode in MODES.items():
                y8 = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
                ops.gemm8w_set(1, mode)
                ops.linear(x, w, y8, bias=b)
                torch.cuda.synchronize()
                nd, md = diff(y8, y4)
                t8 = timeit(lambda: ops.linear(x, w, y8, bias=b))
                line += f" | 8w {mname} {fl / t8 / 1e9:6.0f} (diff {nd}, {md:.2g})"
            ops.gemm8w_set(0, 0)
            print(line + " TF/s", flush=True)


def fused(M, rounds, p=0.1):
    dev = "cuda"
    for r in range(rounds):
        print(f"== fused round {r}", flush=True)
        for mname, mode in MODES.items():
            ops.gemm8w_set(0, mode)
            # fc1: [M, 768] x [3072, 768]^T -> GELU -> dropout
            N, K = 3072, 768
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.1).to(torch.bfloat16)
            b = torch.rand(N, device=dev) * 0.1
            pre_s, a_s = torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            pre_f, a_f = torch.empty_like(pre_s), torch.empty_like(a_s)

            def split1():
                ops.linear(x, w, pre_s, bias=b)
                ops.act_drop_fwd(pre_s, a_s, "gelu", drop_p=p, seed=77)

            def fuse1():
                assert ops.linear_gelu_drop(x, w, b, pre_f, a_f, drop_p=p, seed=77)

            split1()
            fuse1()
            torch.cuda.synchronize()
            d1 = (diff(pre_f, pre_s), diff(a_f, a_s))
            ts, tf = timeit(split1), timeit(fuse1)
            # fc2: [M, 3072] x [768, 3072]^T -> dropout -> + residual (fp32)
            N2, K2 = 768, 3072
            h = (torch.rand(M, K2, device=dev) * 2 - 1).to(torch.bfloat16)
            w2 = ((torch.rand(N2, K2, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
            b2 = torch.rand(N2, device=dev) * 0.1
            res = torch.randn(M, N2, device=dev)
            t2 = torch.empty(M, N2, device=dev, dtype=torch.bfloat16)
            o_s, o_f = torch.empty(M, N2, device=dev), torch.empty(M, N2, device=dev)

            def split2():
                ops.linear(h, w2, t2, bias=b2)
                ops.act_drop_fwd(t2, o_s, "none", drop_p=p, seed=78, residual=res)

            def fuse2():
                assert ops.linear_drop_res(h, w2, b2, res, o_f, drop_p=p, seed=78)

            split2()
            fuse2()
            torch.cuda.synchronize()
            d2 = diff(o_f, o_s)
            ts2, tf2 = timeit(split2), timeit(fuse2)
            # attention proj: [M, 768] x [768, 768]^T -> dropout -> + residual (gemm_8ph fused epilogue today)
            o = (torch.rand(M, 768, device=dev) * 2 - 1).to(torch.bfloat16)
            wp = ((torch.rand(768, 768, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
            x1_s, x1_f = torch.empty(M, 768, device=dev), torch.empty(M, 768, device=dev)

            def split3():
                ops.linear(o, wp, x1_s, bias=b2, residual=res, drop_p=p, seed=79)

            def fuse3():
                assert ops.linear_drop_res(o, wp, b2, res, x1_f, drop_p=p, seed=79)

            split3()
            fuse3()
            torch.cuda.synchronize()
            d3 = diff(x1_f, x1_s)
            ts3, tf3 = timeit(split3), timeit(fuse3)
            # backward: fc2 dX (N 3072, K 768 through the transposed weight) -> dropout -> GELU' (+ fc1 bias grad)
            dy = (torch.randn(M, 768, device=dev) * 0.1).to(torch.bfloat16)
            wt = ((torch.rand(3072, 768, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
            da = torch.empty(M, 3072, device=dev, dtype=torch.bfloat16)
            dp_s, dp_f = torch.empty_like(da), torch.empty_like(da)
            db_s, db_f = torch.zeros(3072, device=dev), torch.zeros(3072, device=dev)

            def split4():
                ops.linear(dy, wt, da)
                ops.act_bwd_bias(pre_s, da, dp_s, db_s, "gelu", drop_p=p, seed=80, accum_bias=False)

            def fuse4():
                assert ops.linear_dgelu_drop(dy, wt, pre_s, dp_f, db_f, drop_p=p, seed=80, accum_bias=False)

            split4()
            fuse4()
            torch.cuda.synchronize()
            d4 = (diff(dp_f, dp_s), ((db_f - db_s).abs().max() / db_s.abs().max()).item())
            ts4, tf4 = timeit(split4), timeit(fuse4)
            print(f"[{mname}] fc2 dX+drop+dgelu+bias: split {ts4 * 1e3:.1f} us, fused {tf4 * 1e3:.1f} us (dpre diff "
                  f"{d4[0]}, dbias rel {d4[1]:.2g})", flush=True)
            # the same with precomputed keep-bit planes (and the plane kernel's own time)
            if p == 0:
                tp1 = tp2 = tp4 = tpl = float("nan")
            else:
                tp1, tp2, tp4, tpl = planes(M, p, x, w, b, pre_f, a_f, h, w2, b2, res, o_f, dy, wt, pre_s, dp_f, db_f)
            print(f"[{mname}] with planes: fc1 {tp1 * 1e3:.1f} us, fc2 {tp2 * 1e3:.1f} us, dgelu {tp4 * 1e3:.1f} us; "
                  f"plane [M, 3072] {tpl * 1e3:.1f} us", flush=True)
            print(f"[{mname}] proj+drop+res: gemm_8ph epilogue {ts3 * 1e3:.1f} us, 8w {tf3 * 1e3:.1f} us (diff {d3})",
                  flush=True)
            print(f"[{mname}] fc1+gelu+drop: split {ts * 1e3:.1f} us, fused {tf * 1e3:.1f} us (pre diff {d1[0]}, "
                  f"out diff {d1[1]}) | fc2+drop+res: split {ts2 * 1e3:.1f} us, fused {tf2 * 1e3:.1f} us (diff {d2})",
                  flush=True)
    ops.gemm8w_set(0, 0)


def planes(M, p, x, w, b, pre_f, a_f, h, w2, b2, res, o_f, dy, wt, pre_s, dp_f, db_f):
    """fused launches reading precomputed keep-bit planes, and the plane kernel's own time"""
    dev = x.device
    pl1 = ops.dropout_plane(M * 3072, p, 77, dev)
    pl2 = ops.dropout_plane(M * 768, p, 78, dev)
    pl4 = ops.dropout_plane(M * 3072, p, 80, dev)
    tp1 = timeit(lambda: ops.linear_gelu_drop(x, w, b, pre_f, a_f, drop_p=p, seed=77, plane=pl1))
    tp2 = timeit(lambda: ops.linear_drop_res(h, w2, b2, res, o_f, drop_p=p, seed=78, plane=pl2))
    tp4 = timeit(lambda: ops.linear_dgelu_drop(dy, wt, pre_s, dp_f, db_f, drop_p=p, seed=80, accum_bias=False,
                                               plane=pl4))
    tpl = timeit(lambda: ops.dropout_plane(M * 3072, p, 81, dev, out=pl1))
    return tp1, tp2, tp4, tpl


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("all", "plain"):
        plain(32768, 2)
    if what in ("all", "fused"):
        fused(32768, 2)
    if what == "fused_p0":  # the same without dropout: the counter hash's share of the epilogues
        fused(32768, 2, p=0.0)
