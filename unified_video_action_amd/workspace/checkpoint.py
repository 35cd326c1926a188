"""Training checkpoints in the reference workspace's `.ckpt` payload layout.

Reference: BaseWorkspace.save_checkpoint / load_payload (workspace/base_workspace.py:33-135):
    torch.save({"cfg": cfg, "state_dicts": {"model", "ema_model", "optimizer", "lr_scheduler"},
                "pickles": {"global_step": dill bytes, "epoch": dill bytes, ...}}, path)
with "model" / "ema_model" = UnifiedVideoActionPolicy.state_dict() (vae_model.*, model.*,
normalizer.*), "optimizer" = torch.optim.AdamW.state_dict() over the two groups of
policy.get_optimizer (no-decay first, then decay; policy:326-360) and "lr_scheduler" = the
LambdaLR state.  The build's FusedAdamWEMA produces / consumes that AdamW layout itself, the
EMA policy is an ordinary module (its parameters are views of the EMA flat buffer), and the
schedulers are torch LambdaLRs, so the payload is built from plain `state_dict()`s both ways.

Loading never executes code from a file (`safe_load`):
  1. torch.load(weights_only=True);
  2. if that refuses the file because of non-tensor globals -- the reference stores its
     OmegaConf `cfg` (base_workspace.py:52), a MAR checkpoint its argparse `args` -- a
     restricted unpickler: torch's own weights-only allowlist, plus inert stand-in classes for
     globals of the configuration modules (omegaconf / hydra / argparse / typing / pathlib),
     which only record the state they are given.  Every other global is refused.  The
     stand-in cfg is converted to plain Python containers where its layout is recognised.
The `pickles` entries (dill / pickle bytes of ints) are decoded with no globals admitted.
"""
import io
import pickle
import types

import torch

STUB_ROOTS = ("omegaconf", "hydra", "argparse", "typing", "pathlib", "enum")
_STUBS = {}


class _Inert:
    """Stand-in for a configuration-module global: records args / state, runs nothing."""

    def __new__(cls, *args, **kwargs):
        obj = object.__new__(cls)
        obj._args = args
        obj._state = None
        return obj

    def __init__(self, *args, **kwargs):
        pass

    def __setstate__(self, state):
        self._state = state

    def __repr__(self):
        return f"<inert {type(self).__module__}.{type(self).__qualname__}>"


def _stub(module, name):
    key = (module, name)
    if key not in _STUBS:
        _STUBS[key] = type(name, (_Inert,), {"__module__": module, "__qualname__": name})
    return _STUBS[key]


def _restricted_pickle_module():
    from torch import _weights_only_unpickler as W
    allowed = W._get_allowed_globals()

    class Unpickler(pickle.Unpickler):
        def find_class(self, module, name):
            key = f"{module}.{name}"
            if key in allowed:
                return allowed[key]
            if module.split(".")[0] in STUB_ROOTS:
                return _stub(module, name)
            raise pickle.UnpicklingError(f"checkpoint global {key} refused (only tensors, containers and "
                                         f"configuration objects are loaded)")

    mod = types.ModuleType("uva_restricted_pickle")
    mod.Unpickler = Unpickler
    mod.load = lambda f, **kw: Unpickler(f, **kw).load()
    mod.__name__ = "uva_restricted_pickle"
    return mod


def to_plain(obj):
    """best-effort: OmegaConf DictConfig / ListConfig / value-node stand-ins -> dict / list / value."""
    if isinstance(obj, _Inert):
        st = obj._state if isinstance(obj._state, dict) else {}
        if "_content" in st:
            return to_plain(st["_content"])
        if "_val" in st:
            return to_plain(st["_val"])
        return None
    if isinstance(obj, dict):
        return {k: to_plain(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [to_plain(v) for v in obj]
    return obj


def safe_load(path, map_location="cpu"):
    try:
        return torch.load(path, map_location=map_location, weights_only=True)
    except pickle.UnpicklingError:
        pass
    return torch.load(path, map_location=map_location, weights_only=False, pickle_module=_restricted_pickle_module())


class _PrimitiveUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"checkpoint pickle references {module}.{name}: refused")


def _loads_primitive(b):
    return _PrimitiveUnpickler(io.BytesIO(b)).load()


def strip_module(sd):
    """DDP / accelerate prefixes, as load_payload does (base_workspace.py:94-100)."""
    return {k.replace("module.", ""): v for k, v in sd.items()}


def _cpu(x):
    """base_workspace._copy_to_cpu."""
    if torch.is_tensor(x):
        return x.detach().to("cpu").clone()
    if isinstance(x, dict):
        return {k: _cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_cpu(v) for v in x)
    return x


def make_payload(model, ema_model=None, optimizer=None, lr_scheduler=None, cfg=None, **pickles):
    sds = {"model": _cpu(model.state_dict())}
    if ema_model is not None:
        sds["ema_model"] = _cpu(ema_model.state_dict())
    if optimizer is not None:
        sds["optimizer"] = _cpu(optimizer.state_dict())
    if lr_scheduler is not None:
        sds["lr_scheduler"] = _cpu(lr_scheduler.state_dict())
    return {"cfg": _plain_cfg(cfg), "state_dicts": sds,
            "pickles": {k: pickle.dumps(v) for k, v in pickles.items()}}


def _plain_cfg(cfg):
    if cfg is None or isinstance(cfg, (int, float, str, bool)):
        return cfg
    if hasattr(cfg, "items"):
        return {k: _plain_cfg(v) for k, v in cfg.items()}
    if isinstance(cfg, (list, tuple)):
        return [_plain_cfg(v) for v in cfg]
    return str(cfg)


def save_checkpoint(path, model, ema_model=None, optimizer=None, lr_scheduler=None, cfg=None, **pickles):
    torch.save(make_payload(model, ema_model, optimizer, lr_scheduler, cfg, **pickles), path)
    return str(path)


def load_payload(payload, model, ema_model=None, optimizer=None, lr_scheduler=None):
    """BaseWorkspace.load_payload (base_workspace.py:86-120): every present state dict into its
    object ("module." stripped), the EMA weights into the model when "model" is absent.
    -> {"cfg", pickles...}."""
    sds = payload["state_dicts"]
    if "model" in sds:
        model.load_state_dict(strip_module(sds["model"]))
    elif "ema_model" in sds:
        model.load_state_dict(strip_module(sds["ema_model"]))
    if ema_model is not None and "ema_model" in sds:
        ema_model.load_state_dict(strip_module(sds["ema_model"]))
    if optimizer is not None and "optimizer" in sds:
        osd = sds["optimizer"]
        if "base_optimizer_state" not in osd:  # DeepSpeed layout is skipped, as the reference does
            optimizer.load_state_dict(osd)
    if lr_scheduler is not None and "lr_scheduler" in sds:
        lr_scheduler.load_state_dict(sds["lr_scheduler"])
    from ..runtime import RT
    RT.bump_params()
    out = {"cfg": to_plain(payload.get("cfg"))}
    for k, b in payload.get("pickles", {}).items():
        out[k] = _loads_primitive(b)
    return out


def load_checkpoint(path, model, ema_model=None, optimizer=None, lr_scheduler=None):
    return load_payload(safe_load(path), model, ema_model, optimizer, lr_scheduler)
