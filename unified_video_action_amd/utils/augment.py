"""PushT training augmentation on the device.

Reference: PushTImageDataset._sample_to_data (dataset/pusht_image_dataset.py:93-130), per video
with one seed for every frame:
    RandomApply([RandomCrop(int(96 * 0.95))], p=0.5) -> Resize(96, antialias=True)
    -> RandomApply([GaussianBlur((5, 5), sigma=(0.1, 2.0))], p=0.5)
The reference runs it in CPU dataloader workers; here the per-video parameters are drawn on the
host with torchvision's draw order from that seed (RandomApply: skip when p < rand; RandomCrop:
randint top, randint left; GaussianBlur: uniform sigma) and one HIP kernel (uva_pusht_augment)
produces the augmented frames in HBM.  torchvision is not installed in this image, so the draw
order and the blur follow its published algorithm (parity against torchvision itself: unpinned;
the kernel is pinned to the torch restatement in oracle/uva_oracle.py).
"""
import ctypes

import torch

from ..native import ops
from ..native.lib import lib

FRAME = 96
CROP = int(FRAME * 0.95)  # 91


def gaussian_kernel1d(sigma, ksize=5):
    """torchvision _get_gaussian_kernel1d: exp(-x^2 / (2 sigma^2)) on linspace(-2, 2, 5), normalised."""
    half = (ksize - 1) * 0.5
    x = torch.linspace(-half, half, steps=ksize)
    pdf = torch.exp(-0.5 * (x / sigma).pow(2))
    return pdf / pdf.sum()


def pusht_aug_params(seeds, frame=FRAME, crop=CROP):
    """[B, 9] fp32 {crop, top, left, blur, k0..k4} per video seed."""
    out = torch.zeros(len(seeds), 9)
    for b, seed in enumerate(seeds):
        g = torch.Generator().manual_seed(int(seed))
        if not 0.5 < torch.rand(1, generator=g).item():
            out[b, 0] = 1.0
            out[b, 1] = float(torch.randint(0, frame - crop + 1, (1,), generator=g).item())
            out[b, 2] = float(torch.randint(0, frame - crop + 1, (1,), generator=g).item())
        if not 0.5 < torch.rand(1, generator=g).item():
            sigma = torch.empty(1).uniform_(0.1, 2.0, generator=g).item()
            out[b, 3] = 1.0
            out[b, 4:] = gaussian_kernel1d(sigma)
    return out


def pusht_augment(image, seeds=None, params=None):
    """image [B, T, 3, 96, 96] fp32 in [0, 1] on the GPU -> augmented copy (same layout)."""
    B, T, C, H, W = image.shape
    if H != FRAME or W != FRAME:
        raise ValueError(f"PushT augmentation expects {FRAME}x{FRAME} frames, got {H}x{W}")
    if params is None:
        if seeds is None:
            seeds = torch.randint(0, 10000, (B,)).tolist()  # video_seed (pusht_image_dataset.py:95)
        params = pusht_aug_params(seeds)
    prm = params.to(image.device, torch.float32).contiguous()
    x = image.float().contiguous()
    out = torch.empty_like(x)
    lib().call("uva_pusht_augment", ops.ptr(x), ops.ptr(out), ops.ptr(prm), B, T, C, H, CROP, ops.stream())
    return out
