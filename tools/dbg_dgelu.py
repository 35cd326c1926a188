"""debug: repeat the fused / plain 8-wave products and count mismatches against the split route (tools only)"""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops  # noqa: E402

DEV = "cuda"
M, N, K = 32768, 3072, 768
g = torch.Generator(device=DEV).manual_seed(3 * M + N + K)
dy = (torch.randn(M, K, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
wt = ((torch.rand(N, K, device=DEV, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
pre = (torch.randn(M, N, device=DEV, generator=g) * 1.5).to(torch.bfloat16)
da = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
ops.linear(dy, wt, da)
for p in (0.0, 0.1):
    dp_s = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    db_s = torch.zeros(N, device=DEV)
    ops.act_bwd_bias(pre, da, dp_s, db_s, "gelu", drop_p=p, seed=4321)
    for it in range(8):
        dp_f = torch.full_like(dp_s, float("nan"))
        db_f = torch.zeros(N, device=DEV)
        assert ops.linear_dgelu_drop(dy, wt, pre, dp_f, db_f, drop_p=p, seed=4321)
        torch.cuda.synchronize()
        ne = (dp_f != dp_s).nonzero()
        zero_f = ((dp_f == 0) & (dp_s != 0)).sum().item()
        print(f"dgelu p={p} it={it}: mismatch {len(ne)} (fused 0 where split not: {zero_f})",
              ne[:3].tolist(), flush=True)
# plain products on the 8-wave kernel, repeated
for mode in (0,):
    ops.gemm8w_set(1, mode)
    for it in range(8):
        y8 = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        ops.linear(dy, wt, y8)
        torch.cuda.synchronize()
        ne = (y8 != da).nonzero()
        print(f"plain mode {mode} it={it}: mismatch {len(ne)}", ne[:3].tolist(), flush=True)
    ops.gemm8w_set(0, 0)
# repeated split route itself (is the reference deterministic?)
for it in range(4):
    da2 = torch.empty_like(da)
    ops.linear(dy, wt, da2)
    torch.cuda.synchronize()
    print("gemm4 repeat mismatch", (da2 != da).sum().item(), flush=True)
