"""Run the fused attention forward/backward a few times (for rocprofv3 PMC passes)."""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops

B, N, H, p = 32, 1024, 12, 0.1
qkv = torch.randn(B, N, 3 * H * 64, device="cuda").to(torch.bfloat16)
out = torch.empty(B, N, H * 64, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B, H, N, device="cuda")
dqkv = torch.empty_like(qkv)
dvec = torch.empty(B, H, N, device="cuda")
mask = ops.attn_dropmask(B, N, H, p, 1, "cuda")
for _ in range(3):
    ops.attn_fwd(qkv, out, lse, B, N, H, 0.125, p, 1, mask=mask)
    ops.attn_bwd(qkv, out, out, lse, dvec, dqkv, B, N, H, 0.125, p, 1, mask=mask)
torch.cuda.synchronize()
print("ok")
