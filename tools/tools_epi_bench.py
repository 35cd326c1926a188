"""GEMM epilogue cost at the MAR fc1 shape (M 32768, N 3072, K 768): plain / +bias / +GELU /
+GELU+pre-activation copy / +GELU+copy+dropout (the training forward of Block.mlp.fc1)."""
import sys
import torch
sys.path.insert(0, ".")
from unified_video_action_amd.native import ops
from tools_kbench import timeit

M, N, K = 32768, 3072, 768
dev = "cuda"
x = torch.randn(M, K, device=dev).to(torch.bfloat16)
w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
b = torch.randn(N, device=dev)
y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
aux = torch.empty_like(y)
fl = 2 * M * N * K
for name, kw in (("plain", {}), ("bias", dict(bias=b)), ("bias+gelu", dict(bias=b, act="gelu")),
                 ("bias+gelu+aux", dict(bias=b, act="gelu", aux=aux)),
                 ("bias+gelu+aux+drop", dict(bias=b, act="gelu", aux=aux, drop_p=0.1, seed=3)),
                 ("bias+drop", dict(bias=b, drop_p=0.1, seed=3))):
    t = timeit(lambda: ops.linear(x, w, y, **kw))
    print(f"fc1 {name:20s} {t*1e3:7.1f} us {fl/t/1e9:6.0f} TF")
