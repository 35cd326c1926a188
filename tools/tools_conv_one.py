"""Run the level-0 VAE conv (GN+SiLU prologue, bias + residual + GN-stats epilogue, n256 256x256
Ci128 Co128) a few times, plus the plain form (for rocprofv3 PMC passes)."""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops

n, H, Ci, Co = 256, 256, 128, 128
dev = "cuda"
x = torch.randn(n, H, H, Ci, device=dev).to(torch.bfloat16)
w = (torch.randn(Co, 3, 3, Ci, device=dev) * 0.05).to(torch.bfloat16)
out = torch.empty(n, H, H, Co, device=dev, dtype=torch.bfloat16)
sc = torch.rand(n, Ci, device=dev) + 0.5
sh = torch.randn(n, Ci, device=dev) * 0.3
res = torch.randn(n, H, H, Co, device=dev).to(torch.bfloat16)
bias = torch.randn(Co, device=dev)
part = torch.empty(n * H * H // 128, 32, 2, device=dev)
for _ in range(3):
    ops.conv2d(x, w, out, n, H, H, Ci, Co, 3, 1, 1, 1, H, H, bias=bias, residual=res, gn_scale=sc, gn_shift=sh,
               gn_part=part)
    if len(sys.argv) > 1 and sys.argv[1] == "plain":
        ops.conv2d(x, w, out, n, H, H, Ci, Co, 3, 1, 1, 1, H, H)
torch.cuda.synchronize()
print("ok")
