"""Forward-GEMM epilogue cost at the MAR shapes (B=32, N=1024): the same bf16 NN GEMM with
successively heavier fused epilogues (bias, GELU+aux, dropout, fp32 residual)."""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops
from tools_kbench import timeit

dev = "cuda"
M = 32768
for (N, K) in ((3072, 768), (2304, 768), (768, 768), (768, 3072)):
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
    b = torch.randn(N, device=dev) * 0.1
    yb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    yf = torch.empty(M, N, device=dev)
    res = torch.randn(M, N, device=dev)
    fl = 2 * M * N * K
    cases = [
        ("plain bf16", lambda: ops.linear(x, w, yb)),
        ("+bias", lambda: ops.linear(x, w, yb, bias=b)),
        ("+bias gelu aux", lambda: ops.linear(x, w, yb, bias=b, act="gelu", aux=aux)),
        ("+bias gelu aux drop", lambda: ops.linear(x, w, yb, bias=b, act="gelu", aux=aux, drop_p=0.1, seed=3)),
        ("+bias drop", lambda: ops.linear(x, w, yb, bias=b, drop_p=0.1, seed=3)),
        ("f32 out +bias", lambda: ops.linear(x, w, yf, bias=b)),
        ("f32 out +bias drop res", lambda: ops.linear(x, w, yf, bias=b, residual=res, drop_p=0.1, seed=3)),
    ]
    out = []
    for name, fn in cases:
        t = timeit(fn, iters=10)
        out.append(f"{name}: {t*1e3:.0f}us {fl/t/1e9:.0f}TF")
    print(f"M{M} N{N} K{K} plan {ops.gemm_plan(M, N, K)} | " + " | ".join(out))
