"""dW products (ta = tb = 1) on the 4-wave route with padded leading dimensions: does the row stride
(L2 / HBM channel mapping) set the DMA rate?  tools only."""
import sys

import torch

sys.path.insert(0, ".")
from unified_video_action_amd.native import ops  # noqa: E402
from tools.gemm4_bench import timeit  # noqa: E402

K = 32768
for O, I in ((3072, 768), (768, 3072)):
    for pad in (0, 64, 128, 256):
        A = (torch.rand(K, O + pad, device="cuda") * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(K, I + pad, device="cuda") * 2 - 1).to(torch.bfloat16)
        C = torch.zeros(O, I, device="cuda")
        t = min(timeit(lambda: ops.gemm(A, B, C, O, I, K, O + pad, I + pad, I, 1, 1, beta=1.0)) for _ in range(3))
        print(f"dW {O}x{I} pad {pad:3d}: {2.0 * K * O * I / t / 1e9:6.0f} TF/s {t * 1e3:.1f} us", flush=True)
