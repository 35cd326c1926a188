"""Block dW products (split-K + slab reduce) timing, tools only: python tools/dw_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
from unified_video_action_amd.native import ops  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


K = 32768
# routes: default (gemm_4w split-K for few-tile shapes, else gemm_8ph), gemm_8ph only, gemm_8w (mode bit 7)
for rnd in range(2):
    for (M, N) in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        dy = torch.randn(K, M, device="cuda").to(torch.bfloat16)
        x = torch.randn(K, N, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(M, N, device="cuda")
        line = f"dW {M}x{N} K{K}:"
        for name, g4, g8 in (("default", 1, 0), ("8ph", 0, 0), ("8w", 1, 128)):
            p4, p8 = ops.gemm4_set(g4), ops.gemm8w_set(-2, g8)
            t = timeit(lambda: ops.linear_dw(dy, x, dw))
            ops.gemm4_set(p4[0]), ops.gemm8w_set(-2, p8[1])
            line += f" | {name} {t * 1e3:6.1f} us {2 * M * N * K / t / 1e9:5.0f} TF/s"
        print(line, flush=True)
