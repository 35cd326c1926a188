"""Per-tile phase split (prologue / K loop / epilogue, s_memtime ticks) of the 8-phase GEMM at an
M x N x K NN bf16 shape: UVA_8PH_VAR=32 python tools/tools_gemm8_phase.py M N K"""
import ctypes
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops
from unified_video_action_amd.native.lib import lib

M, N, K = (int(x) for x in sys.argv[1:4])
a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    ops.gemm(a, b, c, M, N, K, K, K, N, 0, 0)
torch.cuda.synchronize()
buf = np.zeros(16 * 8 * 5, dtype=np.uint64)
lib().call("uva_debug_gemm8_stamps", buf.ctypes.data_as(ctypes.c_void_p))
st = buf.reshape(16, 8, 5).astype(np.float64)
tot = st[..., 0] + st[..., 1] + st[..., 2]
print(f"{M}x{N}x{K}: prologue {st[..., 0].mean():.0f}  loop {st[..., 1].mean():.0f}  epilogue {st[..., 2].mean():.0f} "
      f"ticks (total {tot.mean():.0f}; block spread of entry {np.ptp(st[:, 0, 3]):.0f})")
if len(sys.argv) > 4:  # VAR & 128: [to loop end, chunk-0 staging, chunk-0 stores, rest]
    print("  epilogue split: to-loop-end %.0f  chunk0 acc->LDS+barrier %.0f  chunk0 read+store %.0f  chunk1 %.0f" %
          tuple(st[..., i].mean() for i in range(4)))
