"""Cosine Gaussian-diffusion schedule as device tables for the fused loss kernel.

Follows create_diffusion(timestep_respacing="", noise_schedule="cosine")
(diffusion/__init__.py:11-47): betas from the cosine alpha-bar with max 0.999
(gaussian_diffusion.py:102-145), re-derived through SpacedDiffusion with every step
kept (respace.py:65-90), tables in float64 (gaussian_diffusion.py:157-202) then
cast to fp32 exactly like _extract_into_tensor (:892-904)."""
import math

import numpy as np
import torch

TABLE_ORDER = ("sqrt_ac", "sqrt_1mac", "coef1", "coef2", "plvc", "log_betas", "sqrt_recip_ac",
               "sqrt_recipm1_ac")


def space_timesteps(num_timesteps, section_counts):
    """Retained steps of the base process (respace.py:14-56): each equal section of the
    T steps is strided to its count, indices rounded from a fractional stride."""
    if isinstance(section_counts, str):
        if section_counts.startswith("ddim"):
            want = int(section_counts[4:])
            for i in range(1, num_timesteps):
                if len(range(0, num_timesteps, i)) == want:
                    return sorted(range(0, num_timesteps, i))
            raise ValueError(f"cannot create exactly {num_timesteps} steps with an integer stride")
        section_counts = [int(x) for x in section_counts.split(",")]
    size_per, extra = divmod(num_timesteps, len(section_counts))
    start, steps = 0, []
    for i, count in enumerate(section_counts):
        size = size_per + (1 if i < extra else 0)
        if size < count:
            raise ValueError(f"cannot divide section of {size} steps into {count}")
        stride = 1 if count <= 1 else (size - 1) / (count - 1)
        cur = 0.0
        for _ in range(count):
            steps.append(start + round(cur))
            cur += stride
        start += size
    return sorted(set(steps))


def cosine_tables(T=1000, respacing=""):
    """Tables of create_diffusion(noise_schedule="cosine", timestep_respacing=respacing).
    The spaced process keeps the base alpha-bars at the retained steps (respace.py:65-90);
    "timestep_map" maps spaced index -> base step fed to the net (_WrappedModel, :118-130)."""
    abar = lambda s: math.cos((s + 0.008) / 1.008 * math.pi / 2) ** 2
    b0 = np.array([min(1 - abar((i + 1) / T) / abar(i / T), 0.999) for i in range(T)], np.float64)
    ac_all = np.cumprod(1.0 - b0)
    keep = space_timesteps(T, respacing) if respacing else list(range(T))
    ac0 = ac_all[keep]
    betas = 1.0 - ac0 / np.concatenate([[1.0], ac0[:-1]])
    ac = np.cumprod(1.0 - betas)
    ac_prev = np.concatenate([[1.0], ac[:-1]])
    pvar = betas * (1.0 - ac_prev) / (1.0 - ac)
    return {
        "timestep_map": np.asarray(keep, np.int64),
        "betas": betas,
        "sqrt_ac": np.sqrt(ac),
        "sqrt_1mac": np.sqrt(1.0 - ac),
        "coef1": betas * np.sqrt(ac_prev) / (1.0 - ac),
        "coef2": (1.0 - ac_prev) * np.sqrt(1.0 - betas) / (1.0 - ac),
        "plvc": np.log(np.concatenate([[pvar[1]], pvar[1:]])),
        "log_betas": np.log(betas),
        "sqrt_recip_ac": np.sqrt(1.0 / ac),
        "sqrt_recipm1_ac": np.sqrt(1.0 / ac - 1.0),
    }


class DiffusionSchedule:
    def __init__(self, T, device):
        self.T = T
        tb = cosine_tables(T)
        self.np = tb
        # fp64 -> fp32 per element, identical to torch.from_numpy(arr)[t].float()
        self.tables = [torch.from_numpy(tb[k]).float().to(device) for k in TABLE_ORDER]


def timestep_freqs(device, dim=256, max_period=10000):
    """fp32 frequencies computed with the same torch CPU ops as diffusion_loss.py:123-127."""
    half = dim // 2
    f = torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
    return f.to(device)


class SamplingSchedule:
    """Per-step fp32 coefficients of the spaced reverse process (gen_diffusion,
    diffusion_action_loss.py:105-107), ordered as the loop visits them (t = S-1 .. 0)."""

    def __init__(self, T=1000, respacing="100"):
        tb = cosine_tables(T, respacing)
        self.np = tb
        self.S = len(tb["timestep_map"])
        f32 = lambda a: [float(v) for v in np.asarray(a, np.float64).astype(np.float32)]
        cols = [f32(tb["sqrt_recip_ac"]), f32(tb["sqrt_recipm1_ac"]), f32(tb["coef1"]), f32(tb["coef2"]),
                f32(tb["plvc"]), f32(tb["log_betas"])]
        self.steps = []  # (spaced t, base timestep, coef[8] without temperature)
        for t in reversed(range(self.S)):
            self.steps.append((t, int(tb["timestep_map"][t]), [c[t] for c in cols] + [1.0 if t != 0 else 0.0]))
