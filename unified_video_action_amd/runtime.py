"""Process-wide runtime settings of the HIP path: compute precision and the per-call
dropout seeds (counter-based masks need a distinct seed per op per step)."""
import itertools

import torch


class _Runtime:
    def __init__(self):
        self.compute_dtype = torch.bfloat16   # GEMM/attention operand dtype ("bf16" bench mode)
        self.flash_attention = True           # bf16 fused attention; False -> materialised GEMM+softmax
        self._seed_base = 0x5EED
        self._ctr = itertools.count()

    def set_precision(self, name):
        name = str(name).lower()
        if name in ("fp32", "float32", "no"):
            self.compute_dtype = torch.float32
        elif name in ("bf16", "bfloat16", "fp16"):
            # fp16 autocast of the reference maps to bf16 MFMA here (same 16-bit storage,
            # wider exponent; no GradScaler needed)
            self.compute_dtype = torch.bfloat16
        else:
            raise ValueError(f"unknown precision {name}")

    def seed(self, base):
        self._seed_base = int(base)
        self._ctr = itertools.count()

    def next_seed(self):
        return (self._seed_base * 0x9E3779B97F4A7C15 + next(self._ctr) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF


RT = _Runtime()


def cdt():
    return RT.compute_dtype
