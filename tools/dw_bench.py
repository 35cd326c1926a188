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
for (M, N) in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
    dy = torch.randn(K, M, device="cuda").to(torch.bfloat16)
    x = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    dw = torch.zeros(M, N, device="cuda")
    t = timeit(lambda: ops.linear_dw(dy, x, dw))
    print(f"dW {M}x{N} K{K}: {t * 1e3:.1f} us  {2 * M * N * K / t / 1e9:.0f} TF/s")
