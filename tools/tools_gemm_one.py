"""Run one GEMM shape a few times (for rocprofv3 PMC passes): python tools/tools_gemm_one.py M N K ta tb [iters]."""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops

M, N, K, ta, tb = map(int, sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 5
a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
A = a.t().contiguous() if ta else a
B = b.t().contiguous() if tb else b
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    ops.gemm(A, B, c, M, N, K, A.stride(0), B.stride(0), N, ta, tb)
torch.cuda.synchronize()
print("plan", ops.gemm_plan(M, N, K, ta, tb))
