"""BaseWorkspace with the reference's checkpoint surface (workspace/base_workspace.py:10-165):
save_checkpoint(path|tag) writes the `.ckpt` payload {cfg, state_dicts, pickles} of every
attribute that has state_dict/load_state_dict (model, ema_model, optimizer, lr_scheduler) plus
the include_keys pickles (global_step, epoch), optionally on a background thread from CPU
copies; load_checkpoint / load_payload restore them ("module." prefixes stripped, EMA weights
into the model when "model" is absent).  Files are read with checkpoint.safe_load (no code
from a checkpoint ever executes); snapshots (whole-workspace pickles) are not offered for the
same reason.
"""
import os
import pathlib
import pickle
import threading

import torch

from .checkpoint import _cpu, _loads_primitive, _plain_cfg, safe_load, strip_module


_SKIP = object()


def _primitive(v):
    """v as plain Python data (paths as str), or _SKIP when it has no such form."""
    if v is None or isinstance(v, (bool, int, float, str, bytes)):
        return v
    if isinstance(v, os.PathLike):
        return os.fspath(v)
    if isinstance(v, (list, tuple)):
        out = [_primitive(x) for x in v]
        return _SKIP if any(x is _SKIP for x in out) else type(v)(out)
    if isinstance(v, dict):
        out = {k: _primitive(x) for k, x in v.items()}
        ok = all(isinstance(k, (str, int)) for k in out) and not any(x is _SKIP for x in out.values())
        return out if ok else _SKIP
    return _SKIP


class BaseWorkspace:
    include_keys = tuple()
    exclude_keys = tuple()

    def __init__(self, cfg, output_dir=None):
        self.cfg = cfg
        self._output_dir = output_dir
        self._saving_thread = None

    @property
    def output_dir(self):
        out = self._output_dir
        if out is None:
            run_dir = None
            try:
                run_dir = self.cfg["multi_run"]["run_dir"]
            except (KeyError, TypeError):
                pass
            out = run_dir or os.path.join("outputs", "uva")
        return out

    def run(self):
        raise NotImplementedError

    def get_checkpoint_path(self, tag="latest"):
        return pathlib.Path(self.output_dir).joinpath("checkpoints", f"{tag}.ckpt")

    def _state_objects(self, exclude_keys):
        for key, value in self.__dict__.items():
            if key not in exclude_keys and hasattr(value, "state_dict") and hasattr(value, "load_state_dict"):
                yield key, value

    def save_checkpoint(self, path=None, tag="latest", exclude_keys=None, include_keys=None, use_thread=True):
        path = self.get_checkpoint_path(tag) if path is None else pathlib.Path(path)
        exclude_keys = tuple(self.exclude_keys) if exclude_keys is None else exclude_keys
        include_keys = (tuple(self.include_keys) + ("_output_dir",)) if include_keys is None else include_keys
        path.parent.mkdir(parents=True, exist_ok=True)
        payload = {"cfg": _plain_cfg(self.cfg), "state_dicts": {}, "pickles": {}}
        for key, value in self._state_objects(exclude_keys):
            payload["state_dicts"][key] = _cpu(value.state_dict())
        for key in include_keys:
            if key in self.__dict__:
                value = _primitive(self.__dict__[key])
                if value is not _SKIP:  # only what load_payload's global-free unpickler can read back
                    payload["pickles"][key] = pickle.dumps(value)
        self.wait_for_save()
        if use_thread:
            self._saving_thread = threading.Thread(target=torch.save, args=(payload, str(path)))
            self._saving_thread.start()
        else:
            torch.save(payload, str(path))
        return str(path.absolute())

    def wait_for_save(self):
        if self._saving_thread is not None:
            self._saving_thread.join()
            self._saving_thread = None

    def load_payload(self, payload, exclude_keys=None, include_keys=None, **kwargs):
        exclude_keys = tuple() if exclude_keys is None else exclude_keys
        pickles = payload.get("pickles", {})
        include_keys = pickles.keys() if include_keys is None else include_keys
        sds = dict(payload["state_dicts"])
        if "lr_scheduler" not in self.__dict__:
            sds.pop("lr_scheduler", None)
        for key, value in sds.items():
            if key in exclude_keys or key not in self.__dict__:
                continue
            value = strip_module(value) if key != "optimizer" else value
            if key == "optimizer" and "base_optimizer_state" in value:
                continue  # DeepSpeed layout, skipped as the reference does (base_workspace.py:103-105)
            self.__dict__[key].load_state_dict(value, **kwargs)
        if "model" not in sds and "ema_model" in sds:
            self.__dict__["model"].load_state_dict(strip_module(sds["ema_model"]), **kwargs)
        for key in include_keys:
            if key in pickles:
                self.__dict__[key] = _loads_primitive(pickles[key])
        from ..runtime import RT
        RT.bump_params()

    def load_checkpoint(self, path=None, tag="latest", exclude_keys=None, include_keys=None, **kwargs):
        path = self.get_checkpoint_path(tag) if path is None else pathlib.Path(path)
        payload = safe_load(str(path))
        self.load_payload(payload, exclude_keys=exclude_keys, include_keys=include_keys)
        return payload
