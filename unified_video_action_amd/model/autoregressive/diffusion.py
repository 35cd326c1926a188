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


def cosine_tables(T=1000):
    abar = lambda s: math.cos((s + 0.008) / 1.008 * math.pi / 2) ** 2
    b0 = np.array([min(1 - abar((i + 1) / T) / abar(i / T), 0.999) for i in range(T)], np.float64)
    ac0 = np.cumprod(1.0 - b0)
    betas = 1.0 - ac0 / np.concatenate([[1.0], ac0[:-1]])
    ac = np.cumprod(1.0 - betas)
    ac_prev = np.concatenate([[1.0], ac[:-1]])
    pvar = betas * (1.0 - ac_prev) / (1.0 - ac)
    return {
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
