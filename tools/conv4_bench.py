"""Kernel benchmark of the GN+SiLU 3x3 conv (Ci = Co = 128) on the 4-wave route vs the previous
halo kernels (route switched off), level-0 / level-1 shapes, with and without the residual.  tools only.
python tools/conv4_bench.py [n0]   (level-0 image count, default 256 = the bench's)"""
import sys

import torch

sys.path.insert(0, ".")
from unified_video_action_amd.native import ops  # noqa: E402


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main(n0=256):
    for (n, H) in ((n0, 256), (n0, 128)):
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
            ops.conv4_set(1)
            t4 = timeit(f)
            ops.conv4_set(0)
            t0 = timeit(f)
            ops.conv4_set(1)
            print(f"n{n} {H}x{H} res={res is not None}: conv4 {t4:.3f} ms {fl / t4 / 1e9:6.0f} TF/s   "
                  f"previous {t0:.3f} ms {fl / t0 / 1e9:6.0f} TF/s", flush=True)
            del res


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 256)
