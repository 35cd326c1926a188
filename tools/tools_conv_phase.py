"""Per-tile phase split (prologue / 18-step main loop / epilogue, s_memtime ticks) of the halo conv
at the VAE level-0 shape: UVA_CONV_VAR=1 python tools/tools_conv_phase.py [H Ci Co]
(GN variant: UVA_CONV_GN_VAR=65 UVA_PHASE_GN=1 ...)"""
import ctypes
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops
from unified_video_action_amd.native.lib import lib

H, Ci, Co = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (256, 128, 128)))
n = 256
x = torch.randn(n, H, H, Ci, device="cuda").to(torch.bfloat16)
w = (torch.randn(Co, 3, 3, Ci, device="cuda") * 0.05).to(torch.bfloat16)
out = torch.empty(n, H, H, Co, device="cuda", dtype=torch.bfloat16)
res = torch.randn(n, H, H, Co, device="cuda").to(torch.bfloat16)
bias = torch.randn(Co, device="cuda")
part = torch.empty(n * H * H // 128, 32, 2, device="cuda")
import os
gn = {}
if os.environ.get("UVA_PHASE_GN") == "1":
    gn = dict(gn_scale=torch.rand(n, Ci, device="cuda") + 0.5, gn_shift=torch.randn(n, Ci, device="cuda") * 0.3)
for kw in (dict(gn), dict(gn, bias=bias, residual=res, gn_part=part)):
    for _ in range(3):
        ops.conv2d(x, w, out, n, H, H, Ci, Co, 3, 1, 1, 1, H, H, **kw)
    torch.cuda.synchronize()
    buf = np.zeros(16 * 8 * 4, dtype=np.uint64)
    lib().call("uva_debug_conv_stamps", buf.ctypes.data_as(ctypes.c_void_p))
    st = buf.reshape(16, 8, 4).astype(np.float64)
    print(f"{'plain' if 'bias' not in kw else 'bias+res+gnstats'}{' GN' if gn else ''} {H}x{H} Ci{Ci} Co{Co}: prologue {st[..., 0].mean():.0f}  "
          f"loop {st[..., 1].mean():.0f}  epilogue {st[..., 2].mean():.0f} ticks")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.conv2d(x, w, out, n, H, H, Ci, Co, 3, 1, 1, 1, H, H, **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"   {ms:.3f} ms/launch  {2 * n * H * H * 9 * Ci * Co / ms / 1e9:.0f} TF", flush=True)
