"""Flat parameter store, fused AdamW(+EMA) optimizer and the data-parallel gradient reducer.

ParamStore: every trainable parameter becomes a view of ONE fp32 buffer, laid out group by
group in the optimizer's param_groups order (policy.add_weight_decay: no-decay group, then the
decay group -- policy:326-341), each group region 256-B aligned; every `.grad` a view of ONE
zero-initialised fp32 gradient buffer, and (bf16 mode) every compute shadow a view of ONE
bf16 buffer.  Parameters of one module (a transformer Block, a diffusion trunk) stay
contiguous inside each group, so a module = one DP bucket per group.  When the owning module
is moved (`.to(device)`, as accelerate.prepare does after get_optimizer) the store re-binds
the moved tensors into fresh flat buffers on the new device, values and gradients kept.

FusedAdamWEMA: a torch.optim.Optimizer with torch.optim.AdamW semantics (policy:343-360):
torch-format param_groups (dicts holding "params"), state_dict()/load_state_dict() in
torch.optim.AdamW's layout (per-parameter exp_avg / exp_avg_sq / step), so diffusers / torch
LambdaLR schedulers, accelerate's AcceleratedOptimizer + GradScaler.unscale_, and the reference
workspace's checkpoint payloads all work on it.  One HIP pass per param group does AdamW +
1/world gradient averaging + bf16 shadow refresh, and -- when an EMAModel is attached
(model/autoregressive/ema_model.py) -- the EMA update of the same step (ema_model.py:57-89).

GradReducer: DP gradient all-reduce over RCCL (torch.distributed "nccl") overlapped with
backward, the build's replacement of DDP's bucketed reducer (accelerate.prepare,
workspace:208-220): each fused Block / diffusion-trunk backward launches the async
all-reduce of its own bucket the moment its last gradient is enqueued; at the end of the
backward pass (an autograd engine callback, as DDP's) the rest is reduced and the compute
stream waits for every bucket.
"""
import weakref

import torch
import torch.distributed as dist

from ..native import ops
from ..runtime import RT, cdt

GROUP_ALIGN = 64  # elements: 256-B aligned group regions (float4 optimizer body)


def is_no_decay(name, p):
    """policy.add_weight_decay's split (policy:326-341)."""
    return p.ndim == 1 or name.endswith(".bias")


def _align(n, a=GROUP_ALIGN):
    return (n + a - 1) // a * a


class ParamStore:
    def __init__(self, named_groups, prefix=""):
        """named_groups: [[(name, param), ...] per param group]; names relative to the module the
        optimizer was built over, `prefix` its name in the policy (e.g. "model.")."""
        self.groups = [list(g) for g in named_groups]
        self.prefix = prefix
        self.order = [x for g in self.groups for x in g]
        self.offsets = {}
        self.group_ranges = []
        off = 0
        for g in self.groups:
            off = _align(off)
            start = off
            for n, p in g:
                self.offsets[id(p)] = (off, p.numel())
                off += p.numel()
            self.group_ranges.append((start, off - start))
        self.total = _align(off)
        self.n_params = sum(p.numel() for _, p in self.order)
        self.flat = self.grad = self.shadow = None
        self._bind(self.order[0][1].device)

    # ---- binding ------------------------------------------------------------------------
    def _bind(self, dev):
        flat = torch.zeros(self.total, dtype=torch.float32, device=dev)
        grad = torch.zeros(self.total, dtype=torch.float32, device=dev)
        shadow = None
        if cdt() == torch.bfloat16 and dev.type == "cuda":
            shadow = torch.zeros(self.total, dtype=torch.bfloat16, device=dev)
        for n, p in self.order:
            o, k = self.offsets[id(p)]
            flat[o:o + k].copy_(p.detach().reshape(-1))
            if p.grad is not None:
                grad[o:o + k].copy_(p.grad.detach().reshape(-1))
            p.data = flat[o:o + k].view_as(p)
            p.grad = grad[o:o + k].view_as(p)
            # the fused AdamW kernel rewrites p without bumping _version: any compute shadow built
            # outside the store (bf16 switched on after binding) keys on RT.param_gen instead
            p._uva_raw_updated = True
            if shadow is not None:
                p._uva_shadow = shadow[o:o + k].view_as(p)
                p._uva_shadow_owner = id(p)
            else:
                p.__dict__.pop("_uva_shadow", None)
                p.__dict__.pop("_uva_shadow_owner", None)
        self.flat, self.grad, self.shadow = flat, grad, shadow
        self.refresh_shadow()

    @property
    def device(self):
        return self.flat.device

    def is_bound(self):
        """every parameter (checked at both ends of the layout) still a view of the flat buffer."""
        for _, p in (self.order[0], self.order[-1]):
            o, _ = self.offsets[id(p)]
            if p.device != self.flat.device or p.data_ptr() != self.flat.data_ptr() + 4 * o:
                return False
            if p.grad is None or p.grad.data_ptr() != self.grad.data_ptr() + 4 * o:
                return False
        return True

    def rebind(self):
        """re-create the flat buffers on the parameters' current device (after a module move);
        -> True when it re-bound."""
        if self.is_bound():
            return False
        self._bind(self.order[0][1].device)
        return True

    def refresh_shadow(self):
        if self.shadow is not None:
            ops.cast(self.flat, self.shadow)

    def ranges_of(self, module):
        """[(off, len)] covering the params of a module (or of an iterable of parameters), merged."""
        params = module.parameters() if hasattr(module, "parameters") else module
        rs = sorted(self.offsets[id(p)] for p in params if id(p) in self.offsets)
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
    """EMAModel.get_decay (ema_model.py:45-55)."""
    s = max(0, step - update_after_step - 1)
    if s <= 0:
        return 0.0
    v = 1 - (1 + s / inv_gamma) ** -power
    return max(min_value, min(v, max_value))


_ADAMW_GROUP_KEYS = dict(amsgrad=False, foreach=None, maximize=False, capturable=False, differentiable=False,
                         fused=None)


class FusedAdamWEMA(torch.optim.Optimizer):
    """torch.optim.AdamW over flat buffers, one fused HIP pass per param group."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, named=None, prefix=""):
        self._ready = False
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        for g in self.param_groups:
            g.setdefault("initial_lr", g["lr"])
            g["betas"] = tuple(g["betas"])
        names = {id(p): n for n, p in (named or [])}
        groups = [[(names.get(id(p), f"param{gi}.{i}"), p) for i, p in enumerate(g["params"])]
                  for gi, g in enumerate(self.param_groups)]
        self.store = ParamStore(groups, prefix)
        self.m = torch.zeros_like(self.store.flat)
        self.v = torch.zeros_like(self.store.flat)
        self.step_count = 0
        self.grad_scale = 1.0
        self.reducer = None
        self._ema_ref = None
        self._ready = True

    # ---- torch.optim.Optimizer surface ----------------------------------------------------
    def add_param_group(self, param_group):
        if getattr(self, "_ready", False):
            raise NotImplementedError("FusedAdamWEMA: param groups are fixed at construction (flat layout)")
        super().add_param_group(param_group)

    def _sync(self):
        """follow a module move of the parameters (m / v move with them)."""
        if self.store.rebind():
            self.m = self.m.to(self.store.device)
            self.v = self.v.to(self.store.device)

    def zero_grad(self, set_to_none=True):
        """zeroes the flat gradient buffer; gradients stay views of it (set_to_none is ignored:
        a None grad would break the flat layout the fused kernels write into)."""
        self._sync()
        if self.reducer is not None:
            self.reducer.wait_tail()  # never zero under an in-flight all-reduce
        self.store.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._sync()
        if self.reducer is not None:
            self.reducer.finish()
        self.step_count += 1
        ema = self.attached_ema()
        d = ema.get_decay(ema.optimization_step) if ema is not None else 0.0
        st = self.store
        red = self.reducer
        late = red.tail_segments() if (red is not None and red.tail_handles) else []
        # a deferred DP tail (GradReducer.defer_tail): AdamW runs over everything else first, under
        # the tail's all-reduce, then over the tail once it has landed
        for phase in ((0, 1) if late else (None,)):
            if phase == 1:
                red.wait_tail()
            for g, (off, n) in zip(self.param_groups, st.group_ranges):
                if n == 0:
                    continue
                for o, k in _segments(off, n, late, phase):
                    self._adamw(g, o, k, ema, d)
        if ema is not None:
            ema.mark_fused(self.step_count)
        RT.bump_params()
        return loss

    def _adamw(self, g, o, k, ema, d):
        st = self.store
        b1, b2 = g["betas"]
        sl = slice(o, o + k)
        ops.adamw_ema(st.flat[sl], st.grad[sl], self.m[sl], self.v[sl], ema.flat[sl] if ema is not None else None,
                      st.shadow[sl] if st.shadow is not None else None, k if g["weight_decay"] else 0,
                      g["lr"], b1, b2, g["eps"], g["weight_decay"], self.step_count, self.grad_scale, d)

    @property
    def overlap_tail(self):
        return getattr(self, "_overlap_tail", False)

    @overlap_tail.setter
    def overlap_tail(self, on):
        """True: the loop calls step() right after backward with no gradient reader in between (the
        workspace, bench.py), so the DP tail's all-reduce may run under the AdamW of the rest."""
        self._overlap_tail = bool(on)
        if self.reducer is not None:
            self.reducer.defer_tail = self._overlap_tail

    # ---- EMA fusion ------------------------------------------------------------------------
    def attach_ema(self, ema):
        self._ema_ref = weakref.ref(ema) if ema is not None else None

    def attached_ema(self):
        ema = self._ema_ref() if self._ema_ref is not None else None
        if ema is None or ema.flat is None or ema.flat.device != self.store.device:
            return None
        return ema

    # ---- data parallel ---------------------------------------------------------------------
    def maybe_init_reducer(self, model):
        """create the RCCL bucket reducer once a process group of world > 1 exists (accelerate /
        torchrun initialise it after get_optimizer)."""
        if self.reducer is not None or not (dist.is_available() and dist.is_initialized()):
            return self.reducer
        world = dist.get_world_size()
        if world > 1:
            self.reducer = GradReducer(self.store, default_buckets(model))
            self.reducer.defer_tail = self.overlap_tail
            self.grad_scale = 1.0 / world
        return self.reducer

    # ---- torch.optim.AdamW state_dict layout -------------------------------------------------
    def state_dict(self):
        st = self.store
        state, groups, idx = {}, [], 0
        for g, names in zip(self.param_groups, st.groups):
            ids = []
            for n, p in names:
                if self.step_count > 0:
                    o, k = st.offsets[id(p)]
                    state[idx] = {"step": torch.tensor(float(self.step_count)),
                                  "exp_avg": self.m[o:o + k].view_as(p), "exp_avg_sq": self.v[o:o + k].view_as(p)}
                ids.append(idx)
                idx += 1
            d = {k: v for k, v in g.items() if k != "params"}
            for k, v in _ADAMW_GROUP_KEYS.items():
                d.setdefault(k, v)
            d["params"] = ids
            groups.append(d)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        """torch.optim.AdamW.state_dict() with the same groups -> flat m / v / step count."""
        self._sync()
        st = self.store
        groups = sd["param_groups"]
        if len(groups) != len(st.groups) or any(len(a["params"]) != len(b) for a, b in zip(groups, st.groups)):
            raise ValueError("optimizer state does not match this optimizer's param groups "
                             f"({[len(g['params']) for g in groups]} vs {[len(g) for g in st.groups]})")
        steps = set()
        for grp, names in zip(groups, st.groups):
            for (n, p), pid in zip(names, grp["params"]):
                s = sd["state"].get(pid, sd["state"].get(str(pid)))
                if s is None:
                    continue
                o, k = st.offsets[id(p)]
                if s["exp_avg"].numel() != k:
                    raise ValueError(f"optimizer state of {n}: {s['exp_avg'].numel()} values, parameter has {k}")
                self.m[o:o + k].copy_(s["exp_avg"].reshape(-1))
                self.v[o:o + k].copy_(s["exp_avg_sq"].reshape(-1))
                steps.add(int(float(s["step"])))
        if len(steps) > 1:
            raise ValueError(f"per-parameter step counts differ: {sorted(steps)}")
        self.step_count = steps.pop() if steps else 0
        for mine, theirs in zip(self.param_groups, groups):
            for k in ("lr", "betas", "eps", "weight_decay", "initial_lr"):
                if k in theirs:
                    mine[k] = tuple(theirs[k]) if k == "betas" else theirs[k]


def _segments(off, n, late, phase):
    """[off, off + n) split for the two AdamW phases: phase 0 = everything outside the `late`
    segments, phase 1 = inside them, None = all.  `late` is sorted, 16-B aligned (GradReducer.
    tail_segments), so every piece starts 16-B aligned as the AdamW kernel requires."""
    if phase is None:
        return [(off, n)]
    end, out, pos = off + n, [], off
    for o, k in late:
        a, b = max(o, off), min(o + k, end)
        if a >= b:
            continue
        if phase == 0 and a > pos:
            out.append((pos, a - pos))
        if phase == 1:
            out.append((a, b - a))
        pos = b
    if phase == 0 and pos < end:
        out.append((pos, end - pos))
    return out


def _params(*objs):
    out = []
    for o in objs:
        if o is None:
            continue
        if isinstance(o, torch.nn.Parameter):
            out.append(o)
        else:
            out.extend(o.parameters())
    return out


def default_buckets(model):
    """DP buckets in backward order: [(parameters (a module or a list), module whose fused backward
    fires the hook)].

    * one per transformer Block and per diffusion-MLP trunk (their fused backwards fire them);
    * the diffusion heads' remaining parameters (each head's time / cond embeddings and input_proj,
      the conv_fc trunk of every DiffActLoss: conv, fc, interpolate, refine) + the decoder-output
      embeddings + decoder_norm: all of them have had their gradients enqueued before the LAST
      decoder Block's backward starts (its input gradient depends on every head's trunk through
      decoder_norm; the embedding branches are autograd leaves with higher sequence numbers, which
      the engine runs first), so that Block's hook launches them too -- 60-140 MB reduced under the
      remaining 23 Blocks instead of after backward;
    * decoder_embed + the decoder input embeddings + encoder_norm: enqueued before the LAST encoder
      Block's backward, launched by its hook.
    What remains for the tail is the encoder input side (z / action / text projections,
    proj_cond_x_layer, the encoder embeddings: ~2-3 M parameters), whose backward is the last work."""
    import torch.nn as nn
    from ..model.autoregressive.diffusion_action_loss import DiffActLoss
    from ..model.autoregressive.diffusion_loss import DiffLoss, SimpleMLPAdaLN
    from ..model.autoregressive.mar_con_unified import Block
    out = []
    for m in model.modules():
        if isinstance(m, Block):
            out.append((m, m))
        elif isinstance(m, SimpleMLPAdaLN):
            out.append((nn.ModuleList([m.res_blocks, m.final_layer]), m))
    dec = getattr(model, "decoder_blocks", None)
    enc = getattr(model, "encoder_blocks", None)
    if dec is not None and len(dec) and enc is not None and len(enc):
        heads = [h for h in model.modules() if isinstance(h, (DiffLoss, DiffActLoss))]
        extra = []
        for h in heads:
            net = h.net
            extra += _params(net.time_embed, net.cond_embed, net.input_proj)
            if isinstance(h, DiffActLoss):
                extra += _params(h.conv, h.fc, h.interpolate, h.refine)
        extra += _params(getattr(model, "diffusion_temporal_embed", None),
                         getattr(model, "diffusion_spatial_embed", None), getattr(model, "decoder_norm", None))
        out.append((extra, dec[-1]))
        prelude = _params(getattr(model, "decoder_embed", None), getattr(model, "decoder_temporal_pos_embed", None),
                          getattr(model, "decoder_spatial_pos_embed", None),
                          getattr(model, "decoder_text_pos_embed", None), getattr(model, "encoder_norm", None))
        out.append((prelude, enc[-1]))
    return out


class GradReducer:
    """Bucketed async all-reduce (sum; the optimizer applies 1/world) of the flat gradient buffer,
    launched from inside backward.  One reduction per backward pass (gradient accumulation over
    several backward passes is not supported: the reference configs all use
    gradient_accumulate_every = 1)."""

    MIN_BUCKET_ELEMS = 1 << 16  # ranges below 256 KB of fp32 gradients join the tail collective

    def __init__(self, store, buckets, group=None, min_bucket_elems=None):
        """buckets: [(module whose params form the bucket, module whose fused backward fires the hook)]"""
        if min_bucket_elems is not None:
            self.MIN_BUCKET_ELEMS = min_bucket_elems
        self.store = store
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.handles = []
        self.done = set()
        self.buckets = []
        self.pending = False
        self._queued = False
        covered = []
        self.small = []  # per bucket: its ranges below MIN_BUCKET_ELEMS (coalesced across buckets)
        by_owner = {}
        for i, (m, owner) in enumerate(buckets):
            # a module's params sit in two group regions of the flat buffer (weight decay, then
            # none): the large range(s) reduce as one collective each when the hook fires; the small
            # no-decay ranges (LayerNorm / bias, ~40 KB per Block) are held and merged with their
            # neighbours from the buckets that fire next (consecutive Blocks' no-decay ranges are
            # adjacent), then reduced as one collective once the merged run is large enough
            rs = store.ranges_of(m)
            self.buckets.append([r for r in rs if r[1] >= self.MIN_BUCKET_ELEMS])
            self.small.append([r for r in rs if r[1] < self.MIN_BUCKET_ELEMS])
            covered += rs
            by_owner.setdefault(id(owner), (owner, []))[1].append(i)
        if self.world > 1:
            for owner, idx in by_owner.values():
                owner._uva_bucket_hook = (lambda idx=tuple(idx): [self.launch(i) for i in idx])
        self.held = []  # small ranges of launched buckets, not yet reduced
        self.defer_tail = False  # finish() leaves the tail's handles to wait_tail() (the optimizer)
        self.tail_handles = []
        # complement of all hooked ranges -> the tail bucket (reduced at the end of backward)
        covered.sort()
        tail, pos = [], 0
        for o, k in covered:
            if o > pos:
                tail.append((pos, o - pos))
            pos = max(pos, o + k)
        if pos < store.total:
            tail.append((pos, store.total - pos))
        self.tail = tail

    def wait_tail(self):
        for h in self.tail_handles:
            h.wait()
        self.tail_handles = []

    def tail_segments(self):
        """the tail ranges widened to 4-element (16-B) boundaries, merged: the AdamW pieces that must
        wait for the tail's all-reduce (a widened edge only delays a few reduced elements)."""
        segs = []
        for o, k in sorted(self.tail):
            a, b = o // 4 * 4, (o + k + 3) // 4 * 4
            if segs and a <= segs[-1][1]:
                segs[-1][1] = max(segs[-1][1], b)
            else:
                segs.append([a, b])
        return [(a, b - a) for a, b in segs]

    def coverage(self):
        """per flat element: in how many reduced ranges it lies (must be exactly 1 everywhere)."""
        cnt = torch.zeros(self.store.total, dtype=torch.int32)
        for rs in self.buckets + self.small + [self.tail]:
            for o, k in rs:
                cnt[o:o + k] += 1
        return cnt

    def arm(self):
        """a forward pass ran: the next finish() must reduce (even if no bucket hook fires)."""
        self.pending = self.world > 1

    def _launch(self, i, flush=False):
        if i in self.done:
            return
        self.done.add(i)
        grad = self.store.grad
        for o, k in self.buckets[i]:
            self.handles.append(dist.all_reduce(grad[o:o + k], group=self.group, async_op=True))
        self.held += self.small[i]
        self._flush_held(flush)

    def _flush_held(self, force):
        """merge adjacent held small ranges; reduce every merged run that reached MIN_BUCKET_ELEMS
        (all of them when force)."""
        if not self.held:
            return
        runs = []
        for o, k in sorted(self.held):
            if runs and runs[-1][0] + runs[-1][1] == o:
                runs[-1] = (runs[-1][0], runs[-1][1] + k)
            else:
                runs.append((o, k))
        grad = self.store.grad
        keep = []
        for o, k in runs:
            if force or k >= self.MIN_BUCKET_ELEMS:
                self.handles.append(dist.all_reduce(grad[o:o + k], group=self.group, async_op=True))
            else:
                keep.append((o, k))
        self.held = keep

    def launch(self, i):
        """bucket hook, called by a fused backward once all of bucket i's gradients are enqueued."""
        if self.world <= 1:
            return
        if not self._queued:
            # DDP-style: complete the reduction when the autograd engine finishes this backward
            torch.autograd.Variable._execution_engine.queue_callback(self.finish)
            self._queued = True
        self.pending = True
        self._launch(i)

    def finish(self):
        """reduce what is left, then make the compute stream wait (no-op when already done)."""
        self._queued = False
        self.wait_tail()  # a deferred tail nobody stepped on (backward twice without step)
        if not self.pending:
            return
        for i in range(len(self.buckets)):
            self._launch(i)
        self._flush_held(True)
        grad = self.store.grad
        tail = [dist.all_reduce(grad[o:o + k], group=self.group, async_op=True) for o, k in self.tail]
        if self.defer_tail:
            self.tail_handles = tail
        else:
            self.handles += tail
        for h in self.handles:
            h.wait()
        self.handles = []
        self.done = set()
        self.pending = False
