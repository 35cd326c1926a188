"""conv_in alone (level-0 shape), for rocprofv3 --pmc passes:  python tools/tools_convin_pmc.py"""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops

dev = "cuda"
x = torch.rand(256, 256, 256, 8, device=dev).to(torch.bfloat16)
w = (torch.randn(128, 3, 3, 8, device=dev) * 0.05).to(torch.bfloat16)
out = torch.empty(256, 256, 256, 128, device=dev, dtype=torch.bfloat16)
part = torch.empty(256 * 256 * 256 // 128, 32, 2, device=dev)
for _ in range(3):
    ops.conv2d(x, w, out, 256, 256, 256, 8, 128, 3, 1, 1, 1, 256, 256, gn_part=part)
torch.cuda.synchronize()
print("ok")
