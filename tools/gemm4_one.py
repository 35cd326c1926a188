"""One-shot launches of a single product on the current route (for rocprofv3 --pmc passes; tools only).
python tools/gemm4_one.py N K [iters]  (M = 32768, bias, bf16 out)
python tools/gemm4_one.py dw OUT IN [iters]  (dW[OUT, IN] += dY^T X over 32768 tokens, fp32)"""
import sys

import torch

sys.path.insert(0, ".")
from unified_video_action_amd.native import ops  # noqa: E402

if sys.argv[1] == "dw":
    O, I = int(sys.argv[2]), int(sys.argv[3])
    it = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    dy = (torch.rand(32768, O, device="cuda") * 2 - 1).to(torch.bfloat16)
    x = (torch.rand(32768, I, device="cuda") * 2 - 1).to(torch.bfloat16)
    g = torch.zeros(O, I, device="cuda")
    for _ in range(it):
        ops.linear_dw(dy, x, g)
    torch.cuda.synchronize()
    sys.exit(0)
N, K = int(sys.argv[1]), int(sys.argv[2])
it = int(sys.argv[3]) if len(sys.argv) > 3 else 5
M = 32768
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
b = torch.rand(N, device="cuda")
y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(it):
    ops.linear(x, w, y, bias=b)
torch.cuda.synchronize()
