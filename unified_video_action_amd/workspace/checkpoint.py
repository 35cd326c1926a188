"""Training checkpoints in the reference workspace's `.ckpt` payload layout.

Reference: BaseWorkspace.save_checkpoint / load_payload (workspace/base_workspace.py:33-135):
    torch.save({"cfg": cfg, "state_dicts": {"model", "ema_model", "optimizer", "lr_scheduler"},
                "pickles": {"global_step": dill bytes, "epoch": dill bytes}}, path)
with "model" / "ema_model" = UnifiedVideoActionPolicy.state_dict() (vae_model.*, model.*,
normalizer.*), "optimizer" = torch.optim.AdamW.state_dict() over the two groups of
policy.get_optimizer (no-decay first, then decay; policy:326-360) and "lr_scheduler" = the
diffusers LambdaLR state.

The build's optimizer keeps flat fp32 m / v / EMA buffers (workspace/optim.py); this module
converts them to and from that per-parameter layout, so a run can resume from a reference
checkpoint and the reference workspace can resume from ours.  Files are read with
`torch.load(weights_only=True)`; the two `pickles` entries are decoded by an unpickler that
admits no globals at all (plain ints / floats / strings only), so nothing from a checkpoint
executes code.  `cfg` is written as a plain dict (the reference writes an OmegaConf object,
which a weights-only load refuses; it is then skipped).
"""
import io
import pickle

import torch

from .optim import is_no_decay


class _PrimitiveUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"checkpoint pickle references {module}.{name}: refused")


def _loads_primitive(b):
    return _PrimitiveUnpickler(io.BytesIO(b)).load()


def _strip_module(sd):
    """DDP / accelerate prefixes, as load_payload does (base_workspace.py:94-100)."""
    return {k.replace("module.", ""): v for k, v in sd.items()}


def _trainable(model):
    return [(n, p) for n, p in model.named_parameters() if p.requires_grad]


def _groups(model):
    """(no_decay, decay) name lists in named_parameters order (policy.add_weight_decay)."""
    tr = _trainable(model)
    return [n for n, p in tr if is_no_decay(n, p)], [n for n, p in tr if not is_no_decay(n, p)]


def optimizer_state_torch(opt, model):
    """FusedAdamWEMA -> torch.optim.AdamW.state_dict() layout (CPU tensors)."""
    st = opt.store
    params = dict(_trainable(model))
    nod, dec = _groups(model)
    g = opt.param_groups[0]
    state, groups, idx = {}, [], 0
    for names, wd in ((nod, 0.0), (dec, g["weight_decay"])):
        ids = []
        for n in names:
            o, k = st.offsets[id(params[n])]
            if opt.step_count > 0:
                shp = params[n].shape
                state[idx] = {"step": torch.tensor(float(opt.step_count)),
                              "exp_avg": opt.m[o:o + k].detach().reshape(shp).cpu().clone(),
                              "exp_avg_sq": opt.v[o:o + k].detach().reshape(shp).cpu().clone()}
            ids.append(idx)
            idx += 1
        groups.append({"lr": g["lr"], "betas": tuple(g["betas"]), "eps": g["eps"], "weight_decay": wd,
                       "amsgrad": False, "foreach": None, "maximize": False, "capturable": False,
                       "differentiable": False, "fused": None, "initial_lr": g.get("initial_lr", g["lr"]),
                       "params": ids})
    return {"state": state, "param_groups": groups}


def load_optimizer_state_torch(opt, model, sd):
    """torch.optim.AdamW.state_dict() (two groups, policy.get_optimizer order) -> FusedAdamWEMA."""
    st = opt.store
    params = dict(_trainable(model))
    nod, dec = _groups(model)
    groups = sd["param_groups"]
    if len(groups) != 2 or len(groups[0]["params"]) != len(nod) or len(groups[1]["params"]) != len(dec):
        raise ValueError("optimizer state does not match policy.get_optimizer's (no-decay, decay) groups")
    steps = set()
    for names, grp in ((nod, groups[0]), (dec, groups[1])):
        for n, pid in zip(names, grp["params"]):
            s = sd["state"].get(pid, sd["state"].get(str(pid)))
            if s is None:
                continue
            o, k = st.offsets[id(params[n])]
            if s["exp_avg"].numel() != k:
                raise ValueError(f"optimizer state of {n}: {s['exp_avg'].numel()} values, parameter has {k}")
            opt.m[o:o + k].copy_(s["exp_avg"].reshape(-1))
            opt.v[o:o + k].copy_(s["exp_avg_sq"].reshape(-1))
            steps.add(int(float(s["step"])))
    if len(steps) > 1:
        raise ValueError(f"per-parameter step counts differ: {sorted(steps)}")
    opt.step_count = steps.pop() if steps else 0
    g = groups[1]
    opt.param_groups[0].update(lr=g["lr"], betas=tuple(g["betas"]), eps=g["eps"], weight_decay=g["weight_decay"],
                               initial_lr=g.get("initial_lr", g["lr"]))


def lr_scheduler_state(sched):
    """diffusers LambdaLR.state_dict() fields (lr_lambdas are not stored by torch for plain functions)."""
    return {"base_lrs": list(sched.base) * 2, "last_epoch": sched.last_epoch, "_step_count": sched.last_epoch + 1,
            "verbose": False, "_get_lr_called_within_step": False,
            "_last_lr": sched.get_last_lr() * 2, "lr_lambdas": [None, None]}


def load_lr_scheduler_state(sched, sd):
    sched.last_epoch = int(sd["last_epoch"]) - 1
    sched.step()


def ema_policy_state(policy, opt):
    """The EMA copy of the whole policy (the reference EMAs a deepcopy of the policy; frozen VAE and
    normaliser entries equal the live ones)."""
    sd = {k: v.detach().cpu().clone() for k, v in policy.state_dict().items()}
    if opt is not None and opt.ema is not None:
        for n, t in opt.ema_state().items():
            sd["model." + n] = t.detach().cpu().clone()
    return sd


def make_payload(policy, optimizer=None, lr_scheduler=None, global_step=0, epoch=0, cfg=None):
    sds = {"model": {k: v.detach().cpu().clone() for k, v in policy.state_dict().items()}}
    if optimizer is not None:
        if optimizer.ema is not None:
            sds["ema_model"] = ema_policy_state(policy, optimizer)
        sds["optimizer"] = optimizer_state_torch(optimizer, policy.model)
    if lr_scheduler is not None:
        sds["lr_scheduler"] = lr_scheduler_state(lr_scheduler)
    return {"cfg": cfg, "state_dicts": sds,
            "pickles": {"global_step": pickle.dumps(int(global_step)), "epoch": pickle.dumps(int(epoch))}}


def save_checkpoint(path, policy, optimizer=None, lr_scheduler=None, global_step=0, epoch=0, cfg=None):
    torch.save(make_payload(policy, optimizer, lr_scheduler, global_step, epoch, cfg), path)
    return str(path)


def load_checkpoint(path, policy, optimizer=None, lr_scheduler=None, use_ema_weights=False):
    """-> {"global_step", "epoch", "cfg"}.  Restores policy (or its EMA weights), optimizer m/v/step
    and the LR schedule position."""
    payload = torch.load(path, map_location="cpu", weights_only=True)
    sds = payload["state_dicts"]
    key = "ema_model" if (use_ema_weights or "model" not in sds) else "model"
    policy.load_state_dict(_strip_module(sds[key]))
    if optimizer is not None:
        if optimizer.store.shadow is not None:
            optimizer.store.refresh_shadow()
        if "optimizer" in sds:
            load_optimizer_state_torch(optimizer, policy.model, _strip_module(sds["optimizer"]))
        if optimizer.ema is not None and "ema_model" in sds:
            ema = _strip_module(sds["ema_model"])
            st = optimizer.store
            for n, p in st.order:
                o, k = st.offsets[id(p)]
                optimizer.ema[o:o + k].copy_(ema["model." + n].reshape(-1))
            optimizer.ema_step_count = optimizer.step_count
    if lr_scheduler is not None and "lr_scheduler" in sds:
        load_lr_scheduler_state(lr_scheduler, sds["lr_scheduler"])
    pk = payload.get("pickles", {})
    out = {"cfg": payload.get("cfg")}
    for k in ("global_step", "epoch"):
        out[k] = _loads_primitive(pk[k]) if k in pk else 0
    return out
