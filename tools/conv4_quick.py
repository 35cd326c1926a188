"""conv4 route only, level-0 GN conv with / without residual (A/B of library builds via tools/ab_run.py)"""
import sys

import torch

sys.path.insert(0, ".")
from unified_video_action_amd.native import ops  # noqa: E402
from tools.conv4_bench import timeit  # noqa: E402

n, H = int(sys.argv[1]) if len(sys.argv) > 1 else 128, 256
x = torch.randn(n, H, H, 128, device="cuda").to(torch.bfloat16)
w = (torch.randn(128, 3, 3, 128, device="cuda") * 0.05).to(torch.bfloat16)
b = torch.randn(128, device="cuda") * 0.1
sc = torch.rand(n, 128, device="cuda") + 0.5
sh = torch.randn(n, 128, device="cuda") * 0.3
out = torch.empty_like(x)
part = torch.empty(n * H * H // 128, 32, 2, device="cuda")
fl = 2.0 * n * H * H * 128 * 128 * 9
for res in (None, torch.randn_like(x)):
    f = lambda: ops.conv2d(x, w, out, n, H, H, 128, 128, 3, 1, 1, 1, H, H, bias=b, residual=res,  # noqa: E731
                           gn_scale=sc, gn_shift=sh, gn_silu=True, gn_part=part)
    t = min(timeit(f) for _ in range(3))
    print(f"n{n} {H}x{H} res={res is not None}: {t:.3f} ms {fl / t / 1e9:6.0f} TF/s", flush=True)
