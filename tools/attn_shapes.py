"""Attention forward / backward times over (B, N) shapes at p = 0.1 (same-box A/B: tools/ab_run.py)."""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


H, p = 12, 0.1
for B, N in ((32, 1024), (32, 1088), (56, 1024), (56, 1088), (32, 1152)):
    qkv = torch.randn(B, N, 3 * H * 64, device="cuda").to(torch.bfloat16)
    out = torch.empty(B, N, H * 64, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device="cuda")
    dqkv = torch.empty_like(qkv)
    dvec = torch.empty(B, H, N, device="cuda")
    mask = ops.attn_dropmask(B, N, H, p, 1, "cuda")
    tm = timeit(lambda: ops.attn_dropmask(B, N, H, p, 1, "cuda", out=mask))
    tf = timeit(lambda: ops.attn_fwd(qkv, out, lse, B, N, H, 0.125, p, 1, mask=mask))
    tb = timeit(lambda: ops.attn_bwd(qkv, out, out, lse, dvec, dqkv, B, N, H, 0.125, p, 1, mask=mask))
    fl = 4 * B * H * N * N * 64
    print(f"B={B} N={N}: mask {tm:.3f} fwd {tf:.3f} ms ({fl / tf / 1e9:.0f} TF) bwd {tb:.3f} ms ({2 * fl / tb / 1e9:.0f} TF)")
