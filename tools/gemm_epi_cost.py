"""Epilogue cost of the 8-phase GEMM at training fwd shapes: time the fast path with and without its
output stores (UVA_8PH_VAR=256 / 768, timing-only builds) -- run once per VAR value:
UVA_8PH_VAR=256 python tools/gemm_epi_cost.py"""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from unified_video_action_amd.native import ops

SHAPES = [(32768, 3072, 768), (32768, 2304, 768), (32768, 1024, 1024), (32768, 3072, 1024), (32768, 2048, 1024),
          (8192, 8192, 8192)]
var = os.environ.get("UVA_8PH_VAR", "0")
with ops.gemm_library("kernels"):
    for M, N, K in SHAPES:
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            ops.gemm(a, b, c, M, N, K, K, K, N, 0, 0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        torch.cuda.synchronize()
        e0.record()
        for _ in range(it):
            ops.gemm(a, b, c, M, N, K, K, K, N, 0, 0)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        print(f"VAR={var} {M}x{N}x{K}: {ms * 1e3:8.1f} us  {2 * M * N * K / ms / 1e9:7.0f} TF", flush=True)
