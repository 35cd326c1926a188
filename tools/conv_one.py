"""One shape of the GN halo conv (level 0: n256 256x256 Ci128 Co128 + GN prologue + bias/residual/GN
stats), a few launches -- for rocprofv3 --pmc passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from unified_video_action_amd.native import ops  # noqa: E402

dev = "cuda"
n, H, Ci, Co = 256, 256, 128, 128
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
torch.cuda.synchronize()
print("ok")
