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
import math

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


# ---- UMI (kornia 0.8) and Libero (torchvision ColorJitter) video augmentation -----------------
# Parameter row per video, AUG_NP floats:
#   0 crop (0/1)  1 top  2 left  3 jitter (0/1)  4-7 op order (0 brightness, 1 contrast,
#   2 saturation, 3 hue)  8-11 factors (hue in radians for kornia, in turns for torchvision)
#   12 sharpness (0/1)  13 sharpness factor  14 autocontrast (0/1)  15 grayscale (0/1)
#   16 blur (0/1)  17-21 normalised 1-D Gaussian taps  22 style (0 kornia, 1 torchvision)
#   23 crop size
AUG_NP = 24
UMI_FRAME, UMI_CROP = 224, 208  # config/task/umi_lazy.yaml:50-56 (RandomCrop 208 -> Resize 224)


def umi_aug_params(seeds, frame=UMI_FRAME, crop=UMI_CROP):
    """[B, AUG_NP] rows with the distributions of the UMI kornia chain (umi_lazy.yaml:50-72):
    RandomCrop(208) p=.5, ColorJitter(0.3, 0.4, 0.5, 0.08) p=.8 (factors U[0.7,1.3], U[0.6,1.4],
    U[0.5,1.5], hue U[-0.08,0.08] turns -> radians, order randperm(4)), RandomSharpness(2) p=.5
    (factor U[0,2]), RandomAutoContrast p=.5, RandomGrayscale p=.2, RandomGaussianBlur((5,5),
    (0.1,2.0)) p=.5.  One draw sequence per video seed; kornia's own RNG stream order is not
    reproduced (kornia absent: unpinned)."""
    if not 0 < crop <= frame:
        raise ValueError(f"crop {crop} must be in (0, {frame}]")
    out = torch.zeros(len(seeds), AUG_NP)
    out[:, 23] = float(crop)
    out[:, 4:8] = torch.arange(4, dtype=torch.float32)
    for b, seed in enumerate(seeds):
        g = torch.Generator().manual_seed(int(seed))
        u = lambda lo, hi: float(torch.empty(1).uniform_(lo, hi, generator=g))  # noqa: E731
        row = out[b]
        if torch.rand(1, generator=g).item() < 0.5:
            row[0] = 1.0
            row[1] = float(torch.randint(0, frame - crop + 1, (1,), generator=g))
            row[2] = float(torch.randint(0, frame - crop + 1, (1,), generator=g))
        if torch.rand(1, generator=g).item() < 0.8:
            row[3] = 1.0
            row[8], row[9], row[10] = u(0.7, 1.3), u(0.6, 1.4), u(0.5, 1.5)
            row[11] = (torch.tensor([u(-0.08, 0.08)]) * 2 * math.pi).item()  # kornia: hue * 2 * pi
            row[4:8] = torch.randperm(4, generator=g).float()
        if torch.rand(1, generator=g).item() < 0.5:
            row[12], row[13] = 1.0, u(0.0, 2.0)
        row[14] = float(torch.rand(1, generator=g).item() < 0.5)
        row[15] = float(torch.rand(1, generator=g).item() < 0.2)
        if torch.rand(1, generator=g).item() < 0.5:
            row[16] = 1.0
            row[17:22] = gaussian_kernel1d(u(0.1, 2.0))
    return out


def libero_jitter_params(seeds, brightness=0.2, contrast=0.2, saturation=0.2, hue=0.05):
    """[B, AUG_NP] torchvision ColorJitter rows (libero_replay_image_dataset.py:229-247): per video,
    torch.manual_seed(video_seed) then ColorJitter.get_params in torchvision's order: randperm(4),
    then brightness, contrast, saturation, hue factors by uniform_ (reproduced from a generator
    seeded the same way)."""
    out = torch.zeros(len(seeds), AUG_NP)
    out[:, 3] = 1.0
    out[:, 22] = 1.0
    for b, seed in enumerate(seeds):
        g = torch.Generator().manual_seed(int(seed))
        out[b, 4:8] = torch.randperm(4, generator=g).float()
        for j, (lo, hi) in enumerate(((1 - brightness, 1 + brightness), (1 - contrast, 1 + contrast),
                                      (1 - saturation, 1 + saturation), (-hue, hue))):
            out[b, 8 + j] = float(torch.empty(1).uniform_(lo, hi, generator=g))
    return out


def aug_scratch_floats(B, T, S):
    """floats of uva_video_augment's scratch: two [B*T, 3, S, S] images + per-band partials."""
    return B * T * (6 * S * S + 7 * ((S + 7) // 8))


def video_augment(video, params):
    """video [B, T, 3, S, S] fp32 in [0, 1] on the GPU, params [B, AUG_NP] -> augmented copy
    (uva_video_augment: one workgroup per frame, whole chain in one launch)."""
    B, T, C, H, W = video.shape
    if C != 3 or H != W or H % 4 or H > 256:
        raise ValueError(f"video augmentation expects [B, T, 3, S, S] with S % 4 == 0 and S <= 256, "
                         f"got {tuple(video.shape)}")
    if tuple(params.shape) != (B, AUG_NP):
        raise ValueError(f"params must be [{B}, {AUG_NP}], got {tuple(params.shape)}")
    crop = params[:, 0] != 0
    if crop.any():
        cs, top, left = params[crop, 23], params[crop, 1], params[crop, 2]
        if (cs < 1).any() or (cs > H).any() or (top < 0).any() or (left < 0).any() or \
                (top + cs > H).any() or (left + cs > W).any():
            raise ValueError("crop window outside the frame")
    if ((params[:, 4:8] < 0) | (params[:, 4:8] > 3)).any():
        raise ValueError("jitter order entries must be 0..3")
    prm = params.to(video.device, torch.float32).contiguous()
    x = video.float().contiguous()
    out = torch.empty_like(x)
    scratch = torch.empty(aug_scratch_floats(B, T, H), device=x.device, dtype=torch.float32)
    lib().call("uva_video_augment", ops.ptr(x), ops.ptr(out), ops.ptr(scratch), ops.ptr(prm), B, T, H, ops.stream())
    return out


# obs image key -> (parameter draw, frame size) of the dataset that owns it
_BATCH_AUG = {
    "image": "pusht",          # dataset/pusht_image_dataset.py:93-130
    "agentview_rgb": "libero",  # dataset/libero_replay_image_dataset.py:229-247
    "camera0_rgb": "umi",      # config/task/umi_lazy.yaml:50-72
}


def augment_batch(batch, seeds=None):
    """Apply the owning dataset's training augmentation to the image entry of a device batch, in
    place of the reference's CPU dataloader augmentation (enable with task.device_augment = True
    and turn the dataset's own data_aug / apply_augmentation_in_cpu off).  One seed per video
    (torch.randint(0, 10000) as the reference's video_seed)."""
    obs = batch["obs"]
    for key, kind in _BATCH_AUG.items():
        if key not in obs:
            continue
        img = obs[key]
        B = img.shape[0]
        if seeds is None:
            seeds = torch.randint(0, 10000, (B,)).tolist()
        if kind == "pusht":
            obs[key] = pusht_augment(img, seeds=seeds)
        elif kind == "libero":
            obs[key] = video_augment(img, libero_jitter_params(seeds))
        else:
            obs[key] = video_augment(img, umi_aug_params(seeds, frame=img.shape[-1],
                                                         crop=min(UMI_CROP, img.shape[-1])))
    return batch
