"""Probe: does the frozen KL-VAE encode of the NEXT batch overlap with the MAR forward / backward /
optimizer of the current one when they run on two HIP streams?  Times (a) the MAR part alone,
(b) the VAE encode alone, (c) both issued concurrently (VAE on a side stream), PushT video_model
B=32 (bench config).  Prints ms per iteration of each and the overlap saving."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from unified_video_action_amd.runtime import RT  # noqa: E402
from unified_video_action_amd.utils.data_utils import get_trajectory, select_frame_indices, vae_images  # noqa: E402
from unified_video_action_amd import presets  # noqa: E402


def main(iters=10):
    dev = torch.device("cuda:0")
    pol, opt, sched, ema = bench.build("pusht_video", "bf16", dev)
    batch = presets.synthetic_batch("pusht_video", 32, dev, seed=1)
    for _ in range(3):
        bench.step(pol, opt, sched, ema, batch)
    torch.cuda.synchronize()
    img = batch["obs"]["image"]
    B, T = img.shape[:2]
    sel = select_frame_indices(T)
    x = vae_images(img, sel, pol.vae_model.CIN_PAD)
    n_half = B * (len(sel) // 2)
    eps = torch.randn(2 * n_half, pol.vae_model.embed_dim, 16, 16, device=dev)
    with torch.no_grad():
        tok = pol.vae_model.encode_tokens(x, eps)
    z = tok[:n_half].reshape(B, -1, 256, tok.shape[-1]).clone()
    c = tok[n_half:].reshape(B, -1, 256, tok.shape[-1]).clone()
    nact = pol._normalize("action", batch["action"].float())
    _, traj = get_trajectory(nact, T, pol.shift_action, pol.use_history_action)
    side = torch.cuda.Stream(device=dev)

    def mar():
        RT.prefetch_attn_masks(dev)
        loss, _, _ = pol.model(z, c, None, traj, None, task_mode="video_model")
        loss.backward()
        opt.step()
        opt.zero_grad()
        sched.step()
        ema.step(pol)

    def vae():
        with torch.no_grad():
            return pol.vae_model.encode_tokens(x, eps)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / iters

    def both():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            t = vae()
        mar()
        torch.cuda.current_stream().wait_stream(side)
        t.record_stream(side)

    t_mar = timed(mar)
    t_vae = timed(vae)
    t_both = timed(both)
    t_full = timed(lambda: bench.step(pol, opt, sched, ema, batch))
    print(f"mar {t_mar:.2f} ms  vae {t_vae:.2f} ms  sum {t_mar + t_vae:.2f}  concurrent {t_both:.2f}  "
          f"(saving {t_mar + t_vae - t_both:.2f} ms = {100 * (1 - t_both / (t_mar + t_vae)):.1f} %)  full step {t_full:.2f}")


if __name__ == "__main__":
    main()
