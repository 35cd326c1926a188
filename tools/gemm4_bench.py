"""Kernel benchmark of the Block's forward / dX products (B = 32 PushT: M = 32768) on this build's
4-wave kernel, on gemm_8ph (the same build with the 4-wave route switched off) and on hipBLASLt
(torch.matmul), interleaved rounds in one process, uniform random bf16 operands.  tools only."""
import sys

import torch

sys.path.insert(0, ".")
from unified_video_action_amd.native import ops  # noqa: E402

SHAPES = [  # (name, N, K): y[M, N] = x[M, K] W[N, K]^T
    ("qkv fwd", 2304, 768), ("fc1 fwd", 3072, 768), ("fc2 fwd", 768, 3072),
    ("proj/qkv dX N768 K768", 768, 768), ("fc2 dX N3072 K768", 3072, 768), ("fc1 dX N768 K3072", 768, 3072),
    ("qkv dX N768 K2304", 768, 2304)]


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


def main(rounds=3, M=32768):
    dev = "cuda"
    for r in range(rounds):
        print(f"== round {r}", flush=True)
        for name, N, K in SHAPES:
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
            b = torch.rand(N, device=dev)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fl = 2.0 * M * N * K
            ops.gemm4_set(1)
            t4 = timeit(lambda: ops.linear(x, w, y, bias=b))
            ops.gemm4_set(0)
            t8 = timeit(lambda: ops.linear(x, w, y, bias=b))
            ops.gemm4_set(1)
            bb = b.to(torch.bfloat16)
            tb = timeit(lambda: torch.addmm(bb, x, w.t(), out=y))
            print(f"{name:24s} M{M} N{N} K{K}: gemm4 {fl/t4/1e9:6.0f}  gemm_8ph {fl/t8/1e9:6.0f}  "
                  f"hipBLASLt {fl/tb/1e9:6.0f} TF/s   ({t4*1e3:.1f} / {t8*1e3:.1f} / {tb*1e3:.1f} us) "
                  f"plan {ops.gemm4_plan(M, N, K)}", flush=True)


def quick(M=32768):
    """gemm4 route only, two shapes (A/B of library builds through tools/ab_run.py)"""
    dev = "cuda"
    for name, N, K in (SHAPES[1], SHAPES[2]):
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        b = torch.rand(N, device=dev)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        t4 = min(timeit(lambda: ops.linear(x, w, y, bias=b)) for _ in range(3))
        print(f"{name:24s} M{M} N{N} K{K}: gemm4 {fl/t4/1e9:6.0f} TF/s {t4*1e3:.1f} us", flush=True)


DW_SHAPES = [  # (name, out, in): dW[out, in] += dY[M, out]^T X[M, in]
    ("qkv dW", 2304, 768), ("proj dW", 768, 768), ("fc1 dW", 3072, 768), ("fc2 dW", 768, 3072)]


def dw(rounds=2, M=32768):
    """the dW products: 4-wave split-K route vs gemm_8ph vs hipBLASLt (bf16 output, no accumulate)"""
    dev = "cuda"
    for r in range(rounds):
        print(f"== dW round {r}", flush=True)
        for name, O, I in DW_SHAPES:
            dy = (torch.rand(M, O, device=dev) * 2 - 1).to(torch.bfloat16)
            x = (torch.rand(M, I, device=dev) * 2 - 1).to(torch.bfloat16)
            g = torch.zeros(O, I, device=dev)
            fl = 2.0 * M * O * I
            ops.gemm4_set(1)
            t4 = timeit(lambda: ops.linear_dw(dy, x, g))
            ops.gemm4_set(0)
            t8 = timeit(lambda: ops.linear_dw(dy, x, g))
            ops.gemm4_set(1)
            gb = torch.empty(O, I, device=dev, dtype=torch.bfloat16)
            tb = timeit(lambda: torch.mm(dy.t(), x, out=gb))
            print(f"{name:10s} {O}x{I} K{M}: gemm4 {fl/t4/1e9:6.0f}  gemm_8ph {fl/t8/1e9:6.0f}  hipBLASLt {fl/tb/1e9:6.0f}"
                  f" TF/s   ({t4*1e3:.1f} / {t8*1e3:.1f} / {tb*1e3:.1f} us) plan {ops.gemm4_plan_tt(O, I, M)}",
                  flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["quick"]:
        quick()
    elif sys.argv[1:2] == ["dw"]:
        dw()
    elif sys.argv[1:2] == ["dwquick"]:  # the 4-wave dW route only (A/B of library builds)
        for name, O, I in DW_SHAPES[2:]:
            dy = (torch.rand(32768, O, device="cuda") * 2 - 1).to(torch.bfloat16)
            x = (torch.rand(32768, I, device="cuda") * 2 - 1).to(torch.bfloat16)
            g = torch.zeros(O, I, device="cuda")
            t4 = min(timeit(lambda: ops.linear_dw(dy, x, g)) for _ in range(3))
            print(f"{name:10s} {O}x{I}: gemm4 {2.0 * 32768 * O * I / t4 / 1e9:6.0f} TF/s {t4 * 1e3:.1f} us", flush=True)
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
