"""One-shot level-0 GN conv (n=256, 256x256, Ci=Co=128, GN+SiLU prologue, bias + residual + GN partials),
3 launches, for PMC passes (tools/pmc_kernel.sh)."""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops

n, H, C = 256, 256, 128
dev = "cuda"
x = torch.randn(n, H, H, C, device=dev).to(torch.bfloat16)
w = (torch.randn(C, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
out = torch.empty(n, H, H, C, device=dev, dtype=torch.bfloat16)
sc = torch.rand(n, C, device=dev) + 0.5
sh = torch.randn(n, C, device=dev) * 0.3
res = None if "nores" in sys.argv else torch.randn(n, H, H, C, device=dev).to(torch.bfloat16)
bias = torch.randn(C, device=dev)
part = torch.empty(n * H * H // 128, 32, 2, device=dev)
for _ in range(3):
    ops.conv2d(x, w, out, n, H, H, C, C, 3, 1, 1, 1, H, H, bias=bias, residual=res, gn_scale=sc, gn_shift=sh,
               gn_part=part)
torch.cuda.synchronize()
print("ok")
