"""EMAModel with the reference's constructor, decay schedule and step semantics
(model/autoregressive/ema_model.py:6-89; `ema: _target_` in config/uva_*.yaml).

    ema_model = copy.deepcopy(policy)              # workspace:70-72
    ema = EMAModel(ema_model, power=0.75, ...)      # workspace:191-193
    ... optimizer.step(); ...; ema.step(policy)     # workspace:295-302

get_decay(k) = 0 for k - update_after_step <= 1, else clip(1 - (1 + s/inv_gamma)^-power,
min_value, max_value) with s = k - update_after_step - 1 (ema_model.py:45-55).  step():
averaged = d * averaged + (1 - d) * live for every trainable parameter, copy_ of the frozen
ones (ema_model.py:57-89).

MI355X layout: when the live policy trains on the flat-buffer optimizer (get_optimizer ->
FusedAdamWEMA), the averaged model's trainable parameters are re-bound on the first step as
views of ONE fp32 buffer in the optimizer's layout, and the update is one HIP pass over it
(uva_ema_update) -- or no pass at all: the EMA attaches itself to the optimizer, whose fused
AdamW kernel then applies this EMA step's update (same decay, the post-step weights) while it
has the new weights in registers, and step() only advances the counter.  Frozen parameters
(the VAE, normalizer) are copied when their version changes instead of every step (equal
values; the reference copies them unconditionally).  Without a flat optimizer the update is
the reference's per-parameter loop.
"""
import torch
from torch.nn.modules.batchnorm import _BatchNorm

from ...native import ops
from ...runtime import RT


class EMAModel:
    def __init__(self, model, update_after_step=0, inv_gamma=1.0, power=2 / 3, min_value=0.0, max_value=0.9999):
        self.averaged_model = model
        self.averaged_model.eval()
        self.averaged_model.requires_grad_(False)
        self.update_after_step = update_after_step
        self.inv_gamma = inv_gamma
        self.power = power
        self.min_value = min_value
        self.max_value = max_value
        self.decay = 0.0
        self.optimization_step = 0
        self.flat = None          # fp32 EMA buffer in the live optimizer's flat layout
        self._fused_step = None   # optimizer step count whose fused kernel applied our update
        self._opt_step_seen = None
        self._frozen = []         # (live param, ema param, live version at the last copy)

    def get_decay(self, optimization_step):
        step = max(0, optimization_step - self.update_after_step - 1)
        value = 1 - (1 + step / self.inv_gamma) ** -self.power
        if step <= 0:
            return 0.0
        return max(self.min_value, min(value, self.max_value))

    # ---- flat fast path -----------------------------------------------------------------------
    def _bind(self, new_model, opt):
        """averaged trainable params -> views of one buffer laid out like opt.store."""
        st = opt.store
        ema_params = dict(self.averaged_model.named_parameters())
        live = dict(new_model.named_parameters())
        flat = torch.zeros(st.total, dtype=torch.float32, device=st.device)
        for n, p in st.order:
            key = st.prefix + n
            q = ema_params.get(key)
            if q is None or q.shape != p.shape:
                raise ValueError(f"EMA model has no parameter {key} of shape {tuple(p.shape)}")
            o, k = st.offsets[id(p)]
            flat[o:o + k].copy_(q.detach().reshape(-1))
            q.data = flat[o:o + k].view_as(q)
            q._uva_raw_updated = True  # written by HIP kernels: compute shadows keyed by RT generation
        in_store = {st.prefix + n for n, _ in st.order}
        self._frozen = []
        for n, q in ema_params.items():
            p = live.get(n)
            if n in in_store or p is None:
                continue
            q.data = q.data.to(p.device)
            self._frozen.append((p, q, None))
        self.flat = flat
        self._layout = (id(st), st.device)
        opt.attach_ema(self)

    def mark_fused(self, opt_step):
        """called by the optimizer after its kernel applied this EMA's next update."""
        self._fused_step = opt_step

    @torch.no_grad()
    def step(self, new_model):
        self.decay = self.get_decay(self.optimization_step)
        opt = new_model.bound_optimizer() if hasattr(new_model, "bound_optimizer") else None
        if opt is None:
            self._step_generic(new_model)
        else:
            st = opt.store
            if self.flat is None or self._layout != (id(st), st.device):
                self._bind(new_model, opt)
                fused = False
            else:
                fused = self._fused_step is not None and self._fused_step == opt.step_count \
                    and self._opt_step_seen != opt.step_count
            if not fused:
                ops.ema_update(self.flat, st.flat, self.decay)
            self._opt_step_seen = opt.step_count
            self._fused_step = None
            frozen = []
            for p, q, ver in self._frozen:
                if ver != p._version:
                    q.copy_(p.detach().to(q.dtype))
                frozen.append((p, q, p._version))
            self._frozen = frozen
            RT.bump_params()
        self.optimization_step += 1

    def _step_generic(self, new_model):
        """the reference's loop (ema_model.py:62-85)."""
        for module, ema_module in zip(new_model.modules(), self.averaged_model.modules()):
            for param, ema_param in zip(module.parameters(recurse=False), ema_module.parameters(recurse=False)):
                if isinstance(module, _BatchNorm) or not param.requires_grad:
                    ema_param.copy_(param.to(dtype=ema_param.dtype).data)
                else:
                    ema_param.mul_(self.decay)
                    ema_param.add_(param.data.to(dtype=ema_param.dtype), alpha=1 - self.decay)
