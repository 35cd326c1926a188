"""get_scheduler with the reference's signature (model/common/lr_scheduler.py:10-59), which
wraps diffusers 0.18.2 `optimization.TYPE_TO_SCHEDULER_FUNCTION`.  diffusers is not in this
image, so its schedule functions are restated here as torch LambdaLR factors (parity
unpinned against diffusers itself; pinned against this restatement's golden trace,
tests/golden/g6_workspace_trace.npz).  Every schedule is a plain
torch.optim.lr_scheduler.LambdaLR, so it drives any torch.optim.Optimizer -- including the
flat-buffer FusedAdamWEMA that policy.get_optimizer returns.
"""
import math
from functools import partial

from torch.optim.lr_scheduler import LambdaLR


def _warm(step, warm):
    return float(step) / float(max(1, warm))


def _constant(step):
    return 1.0


def _constant_warmup(step, warm):
    return _warm(step, warm) if step < warm else 1.0


def _linear(step, warm, total):
    if step < warm:
        return _warm(step, warm)
    return max(0.0, float(total - step) / float(max(1, total - warm)))


def _cosine(step, warm, total, cycles):
    if step < warm:
        return _warm(step, warm)
    progress = float(step - warm) / float(max(1, total - warm))
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(cycles) * 2.0 * progress)))


def _cosine_restarts(step, warm, total, cycles):
    if step < warm:
        return _warm(step, warm)
    progress = float(step - warm) / float(max(1, total - warm))
    if progress >= 1.0:
        return 0.0
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * ((float(cycles) * progress) % 1.0))))


def _polynomial(step, warm, total, lr_init, lr_end, power):
    if step < warm:
        return _warm(step, warm)
    if step > total:
        return lr_end / lr_init
    decay_steps = total - warm
    remaining = 1 - (step - warm) / decay_steps
    return ((lr_init - lr_end) * remaining ** power + lr_end) / lr_init


SCHEDULES = ("linear", "cosine", "cosine_with_restarts", "polynomial", "constant", "constant_with_warmup")


def get_scheduler(name, optimizer, num_warmup_steps=None, num_training_steps=None, **kwargs):
    """-> LambdaLR.  kwargs: last_epoch (the reference passes global_step - 1), num_cycles
    (cosine: 0.5, cosine_with_restarts: 1), lr_end / power (polynomial)."""
    name = str(getattr(name, "value", name))
    if name not in SCHEDULES:
        raise ValueError(f"unknown lr scheduler {name!r}; one of {SCHEDULES}")
    last_epoch = kwargs.pop("last_epoch", -1)
    if name == "constant":
        return LambdaLR(optimizer, _constant, last_epoch=last_epoch)
    if num_warmup_steps is None:
        raise ValueError(f"{name} requires `num_warmup_steps`, please provide that argument.")
    if name == "constant_with_warmup":
        return LambdaLR(optimizer, partial(_constant_warmup, warm=num_warmup_steps), last_epoch=last_epoch)
    if num_training_steps is None:
        raise ValueError(f"{name} requires `num_training_steps`, please provide that argument.")
    w, t = num_warmup_steps, num_training_steps
    if name == "linear":
        fn = partial(_linear, warm=w, total=t)
    elif name == "cosine":
        fn = partial(_cosine, warm=w, total=t, cycles=kwargs.pop("num_cycles", 0.5))
    elif name == "cosine_with_restarts":
        fn = partial(_cosine_restarts, warm=w, total=t, cycles=kwargs.pop("num_cycles", 1))
    else:
        lr_init = optimizer.defaults["lr"]
        lr_end = kwargs.pop("lr_end", 1e-7)
        if not lr_init > lr_end:
            raise ValueError(f"lr_end ({lr_end}) must be smaller than initial lr ({lr_init})")
        fn = partial(_polynomial, warm=w, total=t, lr_init=lr_init, lr_end=lr_end, power=kwargs.pop("power", 1.0))
    return LambdaLR(optimizer, fn, last_epoch=last_epoch)
