"""Flat parameter store, fused AdamW+EMA optimizer and the data-parallel gradient reducer.

ParamStore: every trainable parameter becomes a view of ONE fp32 buffer (decay group
first, then the no-decay group -- policy:326-341 split), every `.grad` a view of ONE
zero-initialised fp32 gradient buffer, and (bf16 mode) every compute shadow a view of ONE
bf16 buffer.  Parameters of one module (a transformer Block, a diffusion head) stay
contiguous inside each group, so a module = one DP bucket.

FusedAdamWEMA: torch.optim.AdamW semantics (policy:343-360) + EMA (ema_model.py:45-89,
power 0.75) + bf16 shadow refresh + 1/world gradient averaging in one HIP pass
(uva_adamw_ema).  Exposes param_groups/step/zero_grad/state_dict like a torch optimizer
so a diffusers-style LR scheduler drives it.

GradReducer: DP gradient all-reduce over RCCL (torch.distributed "nccl") overlapped with
backward: each fused Block / diffusion-trunk backward ends by launching the async
all-reduce of its own bucket; the rest is reduced once at the end of backward.
"""
import math

import torch
import torch.distributed as dist

from ..native import ops
from ..runtime import cdt


def is_no_decay(name, p):
    return p.ndim == 1 or name.endswith(".bias")


class ParamStore:
    def __init__(self, model):
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        decay = [(n, p) for n, p in named if not is_no_decay(n, p)]
        nodecay = [(n, p) for n, p in named if is_no_decay(n, p)]
        self.order = decay + nodecay
        self.n_decay = sum(p.numel() for _, p in decay)
        total = sum(p.numel() for _, p in self.order)
        dev = named[0][1].device
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.shadow = None
        if cdt() == torch.bfloat16:
            self.shadow = torch.empty(total, dtype=torch.bfloat16, device=dev)
        self.offsets = {}
        off = 0
        for n, p in self.order:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            if self.shadow is not None:
                p._uva_shadow = self.shadow[off:off + k].view_as(p)
                p._uva_shadow_static = True
            self.offsets[id(p)] = (off, k)
            off += k
        self.total = total
        self.refresh_shadow()

    def refresh_shadow(self):
        if self.shadow is not None:
            ops.cast(self.flat, self.shadow)

    def ranges_of(self, module):
        """[(off, len)] covering the module's params, merged per group."""
        rs = sorted(self.offsets[id(p)] for p in module.parameters() if id(p) in self.offsets)
        merged = []
        for o, k in rs:
            if merged and merged[-1][0] + merged[-1][1] == o:
                merged[-1] = (merged[-1][0], merged[-1][1] + k)
            else:
                merged.append((o, k))
        return merged

    def zero_grad(self):
        self.grad.zero_()


def ema_decay(step, update_after_step=0, inv_gamma=1.0, power=0.75, min_value=0.0, max_value=0.9999):
    s = max(0, step - update_after_step - 1)
    if s <= 0:
        return 0.0
    v = 1 - (1 + s / inv_gamma) ** -power
    return max(min_value, min(v, max_value))


class FusedAdamWEMA:
    def __init__(self, model, lr=1e-4, betas=(0.9, 0.95), weight_decay=0.02, eps=1e-8, use_ema=True, ema_cfg=None):
        self.store = ParamStore(model)
        self.param_groups = [{"lr": lr, "initial_lr": lr, "betas": betas, "weight_decay": weight_decay,
                              "eps": eps}]
        self.defaults = dict(self.param_groups[0])
        self.m = torch.zeros_like(self.store.flat)
        self.v = torch.zeros_like(self.store.flat)
        self.ema = self.store.flat.clone() if use_ema else None
        self.ema_cfg = dict(ema_cfg or {})
        self.step_count = 0
        self.ema_step_count = 0
        self.grad_scale = 1.0
        self.state = {}

    def zero_grad(self, set_to_none=False):
        self.store.zero_grad()

    def step(self):
        g = self.param_groups[0]
        self.step_count += 1
        d = ema_decay(self.ema_step_count, **self.ema_cfg) if self.ema is not None else 0.0
        self.ema_step_count += 1
        b1, b2 = g["betas"]
        ops.adamw_ema(self.store.flat, self.store.grad, self.m, self.v, self.ema, self.store.shadow,
                      self.store.n_decay, g["lr"], b1, b2, g["eps"], g["weight_decay"], self.step_count,
                      self.grad_scale, d)

    def state_dict(self):
        return {"step": self.step_count, "ema_step": self.ema_step_count, "m": self.m, "v": self.v,
                "param_groups": [dict(x) for x in self.param_groups]}

    def load_state_dict(self, sd):
        self.step_count = sd["step"]
        self.ema_step_count = sd.get("ema_step", sd["step"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.param_groups = [dict(x) for x in sd["param_groups"]]

    def ema_state(self):
        """EMA weights as a name -> tensor dict (frozen VAE EMA == VAE, not stored)."""
        out = {}
        for n, p in self.store.order:
            o, k = self.store.offsets[id(p)]
            out[n] = self.ema[o:o + k].view_as(p)
        return out


class CosineWithWarmup:
    """diffusers 0.18.2 get_cosine_schedule_with_warmup (restated; lr_scheduler.py:10-59)."""

    def __init__(self, optimizer, num_warmup_steps, num_training_steps, num_cycles=0.5, last_epoch=-1):
        self.opt = optimizer
        self.warm, self.total, self.cycles = num_warmup_steps, num_training_steps, num_cycles
        self.base = [g["initial_lr"] for g in optimizer.param_groups]
        self.last_epoch = last_epoch
        self.step()

    def factor(self, step):
        if step < self.warm:
            return step / max(1, self.warm)
        prog = (step - self.warm) / max(1, self.total - self.warm)
        return max(0.0, 0.5 * (1.0 + math.cos(math.pi * self.cycles * 2.0 * prog)))

    def step(self):
        self.last_epoch += 1
        f = self.factor(self.last_epoch)
        for g, b in zip(self.opt.param_groups, self.base):
            g["lr"] = b * f

    def get_last_lr(self):
        return [g["lr"] for g in self.opt.param_groups]


def default_buckets(model):
    """one bucket per transformer Block and per diffusion-MLP trunk (backward order = reverse)."""
    import torch.nn as nn
    from ..model.autoregressive.diffusion_loss import SimpleMLPAdaLN
    from ..model.autoregressive.mar_con_unified import Block
    out = []
    for m in model.modules():
        if isinstance(m, Block):
            out.append((m, m))
        elif isinstance(m, SimpleMLPAdaLN):
            out.append((nn.ModuleList([m.res_blocks, m.final_layer]), m))
    return out


class GradReducer:
    """Bucketed async all-reduce of the flat gradient buffer, launched from inside backward."""

    def __init__(self, store, buckets, group=None):
        """buckets: [(module whose params form the bucket, module whose fused backward fires the hook)]"""
        self.store = store
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.handles = []
        self.done = set()
        self.buckets = []
        covered = []
        for i, (m, owner) in enumerate(buckets):
            rs = store.ranges_of(m)
            self.buckets.append(rs)
            covered += rs
            if self.world > 1:
                owner._uva_bucket_hook = (lambda i=i: self.launch(i))
        # complement of all hooked ranges -> one tail bucket
        covered.sort()
        tail, pos = [], 0
        for o, k in covered:
            if o > pos:
                tail.append((pos, o - pos))
            pos = max(pos, o + k)
        if pos < store.total:
            tail.append((pos, store.total - pos))
        self.tail = tail

    def launch(self, i):
        if self.world <= 1 or i in self.done:
            return
        self.done.add(i)
        for o, k in self.buckets[i]:
            self.handles.append(dist.all_reduce(self.store.grad[o:o + k], group=self.group, async_op=True))

    def finish(self):
        """after loss.backward(): reduce what is left, then make the compute stream wait."""
        if self.world <= 1:
            return
        for i in range(len(self.buckets)):
            self.launch(i)
        for o, k in self.tail:
            self.handles.append(dist.all_reduce(self.store.grad[o:o + k], group=self.group, async_op=True))
        for h in self.handles:
            h.wait()
        self.handles = []
        self.done = set()
