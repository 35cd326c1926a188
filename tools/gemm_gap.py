"""Hand-written GEMM kernels vs the hipBLASLt route on the training-step shapes (M = 32768 tokens):
python tools/gemm_gap.py  -> one line per shape: plan (kernel, BN, splits), own / library TFLOP/s."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from unified_video_action_amd.native import ops  # noqa: E402
from tools_kbench import timeit  # noqa: E402

M = 32768
SHAPES = {  # name: (kind, N_out, K_in)
    "qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072),
    "adaln": (3072, 1024), "mlp": (1024, 1024), "final": (2048, 1024),
}


def run(modes=("kernels", "library", "tuned"), only=None):
    dev = "cuda"
    print(f"{'shape':>8} {'op':>3} {'M':>6} {'N':>6} {'K':>6}  {'plan':>14}  {'own TF':>7} {'lib TF':>7} {'tuned TF':>8}")
    for name, (No, Ki) in SHAPES.items():
        if only and name not in only:
            continue
        x = torch.randn(M, Ki, device=dev).to(torch.bfloat16)
        w = torch.randn(No, Ki, device=dev).to(torch.bfloat16)
        b = torch.randn(No, device=dev)
        y = torch.empty(M, No, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M, No, device=dev).to(torch.bfloat16)
        dx = torch.empty(M, Ki, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(No, Ki, device=dev)
        fl = 2.0 * M * No * Ki
        for op, fn, shp in (("fwd", lambda: ops.linear(x, w, y, bias=b), (M, No, Ki, 0, 0)),
                            ("dx", lambda: ops.linear_dx(dy, w, dx), (M, Ki, No, 0, 1)),
                            ("dw", lambda: ops.linear_dw(dy, x, dw), (No, Ki, M, 1, 1))):
            res = {}
            for mode in modes:
                with ops.gemm_library(mode):
                    res[mode] = fl / timeit(fn) / 1e9
            kern, bn, splits = ops.gemm_plan(shp[0], shp[1], shp[2], shp[3], shp[4])
            print(f"{name:>8} {op:>3} {shp[0]:>6} {shp[1]:>6} {shp[2]:>6}  k{kern} bn{bn:>3} s{splits:>2}     "
                  " ".join(f"{res[m]:7.0f}" for m in modes), flush=True)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="kernels,library,tuned")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    run(tuple(a.modes.split(",")), set(a.only.split(",")) if a.only else None)
