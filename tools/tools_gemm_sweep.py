"""K / N sweep of the bf16 GEMM (NN, bf16 out) vs hipBLASLt: separates per-tile fixed cost from the
per-K-tile main-loop cost.  python tools/tools_gemm_sweep.py"""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops
from tools_kbench import timeit

M = 32768
for N in (3072, 768):
    for K in (256, 512, 768, 1536, 3072, 6144):
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: ops.gemm(a, b, c, M, N, K, K, K, N, 0, 0), iters=10)
        tt = timeit(lambda: torch.matmul(a, b.t()), iters=10)
        fl = 2 * M * N * K
        print(f"N={N} K={K}: ours {t*1e3:7.1f} us {fl/t/1e9:5.0f} TF   hipblaslt {tt*1e3:7.1f} us {fl/tt/1e9:5.0f} TF  "
              f"plan {ops.gemm_plan(M, N, K, 0, 0)}", flush=True)
