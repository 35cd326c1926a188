"""Time one 8-phase GEMM variant (UVA_8PH_VAR) at S^3 NT bf16; with VAR odd also dump the stamps."""
import os
import sys
import ctypes
import numpy as np
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops
from unified_video_action_amd.native.lib import lib

S = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
var = int(os.environ.get("UVA_8PH_VAR", "0"))
a = (torch.rand(S, S, device="cuda") * 2 - 1).to(torch.bfloat16)
b = (torch.rand(S, S, device="cuda") * 2 - 1).to(torch.bfloat16)
c = torch.empty(S, S, device="cuda", dtype=torch.bfloat16)
f = lambda: ops.gemm(a, b, c, S, S, S, S, S, S, 0, 0)
for _ in range(3):
    f()
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(5):
    ev0.record(); f(); ev1.record(); torch.cuda.synchronize(); ts.append(ev0.elapsed_time(ev1))
t = min(ts)
ref_ok = ""
if not (var & 8):
    r = (a[:256].float() @ b.float().t())
    ref_ok = f" maxrel {((c[:256].float() - r).abs().max() / r.abs().max()).item():.1e}"
print(f"VAR {var}: {t:.3f} ms  {2 * S**3 / t / 1e9:.0f} TF{ref_ok}")
if var & 1:
    buf = np.zeros(16 * 8 * 5, dtype=np.uint64)
    rc = lib().call("uva_debug_gemm8_stamps", buf.ctypes.data_as(ctypes.c_void_p))
    st = buf.reshape(16, 8, 5).astype(np.float64)
    tot = st[..., 4].mean()
    names = ["read+issue+lgkm", "barrier-1 (X)", "mfma issue", "barrier-2 (Y)"]
    for g in (0, 1):
        w = st[:, 4 * g:4 * g + 4]
        print(f"  group {g}: " + "  ".join(f"{n} {w[..., i].mean() / w[..., 4].mean() * 100:.1f}%" for i, n in enumerate(names))
              + f"  loop {w[..., 4].mean():.0f} ticks")
