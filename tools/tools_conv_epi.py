"""Level-0 halo conv epilogue pieces: plain / +bias / +residual / +GN partial stats / all."""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops
from tools_kbench import timeit

dev = "cuda"
n, H, Ci, Co = 256, 256, 128, 128
x = torch.randn(n, H, H, Ci, device=dev).to(torch.bfloat16)
w = (torch.randn(Co, 3, 3, Ci, device=dev) * 0.05).to(torch.bfloat16)
out = torch.empty(n, H, H, Co, device=dev, dtype=torch.bfloat16)
res = torch.randn(n, H, H, Co, device=dev).to(torch.bfloat16)
bias = torch.randn(Co, device=dev)
part = torch.empty(n * H * H // 128, 32, 2, device=dev)
for name, kw in (("plain", {}), ("bias", dict(bias=bias)), ("residual", dict(residual=res)),
                 ("gn stats", dict(gn_part=part)), ("all", dict(bias=bias, residual=res, gn_part=part))):
    t = timeit(lambda: ops.conv2d(x, w, out, n, H, H, Ci, Co, 3, 1, 1, 1, H, H, **kw), iters=5)
    print(f"halo conv level0 {name:10s} {t:.3f} ms")
