"""One fused fc1 (GELU + dropout) and one fused fc2-dX (dropout + GELU') launch at the Block's B = 32 shape on each
gemm_8w form, for rocprofv3 --pmc passes (tools/jobs/r06_g8w_pmc.sh).  tools only."""
import sys

import torch

sys.path.insert(0, ".")
from unified_video_action_amd.native import ops  # noqa: E402

M, N, K, p = 32768, 3072, 768, 0.1
dev = "cuda"
x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.1).to(torch.bfloat16)
b = torch.rand(N, device=dev) * 0.1
pre, a = torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.empty(M, N, device=dev, dtype=torch.bfloat16)
dy = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
dp, db = torch.empty_like(pre), torch.zeros(N, device=dev)
y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for mode in (0, 32):
    ops.gemm8w_set(0, mode)
    for _ in range(3):
        assert ops.linear_gelu_drop(x, w, b, pre, a, drop_p=p, seed=7)
        assert ops.linear_dgelu_drop(dy, w, pre, dp, db, drop_p=p, seed=8, accum_bias=False)
    ops.gemm8w_set(1, mode)
    for _ in range(3):
        ops.linear(x, w, y, bias=b)
    ops.gemm8w_set(0, 0)
torch.cuda.synchronize()
print("ok")
