"""LinearNormalizer / SingleFieldLinearNormalizer with the reference's semantics, API and
state-dict layout (model/common/normalizer.py:12-297, dict_of_tensor_mixin.py):

  * fit: per key, statistics over all leading dims with the trailing `last_n_dims` flattened into
    one feature axis; "limits" maps [min, max] to [output_min, output_max] (constant dims centred
    at the output midpoint), or with fit_offset=False scales by the largest |value| only;
    "gaussian" standardises;
  * normalize(x) = x * scale + offset over that feature axis (unnormalize inverts it), for a dict
    of fields or a single tensor (the "_default" field), numpy or torch input;
  * stored as nn.ParameterDict params_dict.<key>.{scale, offset, input_stats.{min,max,mean,std}}.

Pinned by the reference's own normalizer.pkl (tests/golden/ref_fixtures.npz: fit arithmetic and
normalize / unnormalize on its action / agent_pos / image fields) and by the normalizer.py:300
test() known-answer checks restated in tests/test_ref_fixtures_cpu.py."""
import numpy as np
import torch
import torch.nn as nn


def _fit(data, last_n_dims=1, dtype=torch.float32, mode="limits", output_max=1.0, output_min=-1.0,
         range_eps=1e-4, fit_offset=True):
    """normalizer.py:195-280"""
    if mode not in ("limits", "gaussian"):
        raise ValueError(mode)
    assert last_n_dims >= 0 and output_max > output_min
    data = torch.as_tensor(np.asarray(data) if not torch.is_tensor(data) else data)
    if dtype is not None:
        data = data.to(dtype)
    dim = int(np.prod(data.shape[-last_n_dims:])) if last_n_dims > 0 else 1
    data = data.reshape(-1, dim)
    lo, hi = data.min(dim=0).values, data.max(dim=0).values
    mean, std = data.mean(dim=0), data.std(dim=0)
    if mode == "limits":
        if fit_offset:
            rng = hi - lo
            const = rng < range_eps
            rng[const] = output_max - output_min
            scale = (output_max - output_min) / rng
            offset = output_min - scale * lo
            offset[const] = (output_max + output_min) / 2 - lo[const]
        else:
            assert output_max > 0 and output_min < 0
            out_abs = min(abs(output_min), abs(output_max))
            in_abs = torch.maximum(lo.abs(), hi.abs())
            const = in_abs < range_eps
            in_abs[const] = out_abs
            scale = out_abs / in_abs
            offset = torch.zeros_like(mean)
    else:
        const = std < range_eps
        scale = std.clone()
        scale[const] = 1
        scale = 1 / scale
        offset = -mean * scale if fit_offset else torch.zeros_like(mean)
    p = nn.ParameterDict({"scale": scale, "offset": offset,
                          "input_stats": nn.ParameterDict({"min": lo, "max": hi, "mean": mean, "std": std})})
    p.requires_grad_(False)
    return p


def _normalize(x, params, forward=True):
    """normalizer.py:283-297: over the last scale.numel() features, shape preserved"""
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(x)
    scale, offset = params["scale"], params["offset"]
    # (the reference moves x to the parameters' device; here the parameters follow x, so a
    # normalizer loaded after the policy moved to the GPU normalises device batches in place)
    scale, offset = scale.to(x.device), offset.to(x.device)
    x = x.to(dtype=scale.dtype)
    shape = x.shape
    x = x.reshape(-1, scale.shape[0])
    x = x * scale + offset if forward else (x - offset) / scale
    return x.reshape(shape)


class _ParamsModule(nn.Module):
    """dict_of_tensor_mixin.DictOfTensorMixin: params_dict, and a state-dict loader that rebuilds
    the nested ParameterDict from flat keys params_dict.<key>.<field>[.<stat>]"""

    def __init__(self, params_dict=None):
        super().__init__()
        self.params_dict = nn.ParameterDict() if params_dict is None else params_dict

    @property
    def device(self):
        return next(iter(self.parameters())).device

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        root = prefix + "params_dict."
        out = nn.ParameterDict()
        for k, v in state_dict.items():
            if not k.startswith(root):
                continue
            node, parts = out, k[len(root):].split(".")
            for p in parts[:-1]:
                if p not in node:
                    node[p] = nn.ParameterDict()
                node = node[p]
            node[parts[-1]] = nn.Parameter(v.clone(), requires_grad=False)
        self.params_dict = out
        self.params_dict.requires_grad_(False)


class SingleFieldLinearNormalizer(_ParamsModule):
    @torch.no_grad()
    def fit(self, data, **kw):
        self.params_dict = _fit(data, **kw)

    @classmethod
    def create_fit(cls, data, **kw):
        obj = cls()
        obj.fit(data, **kw)
        return obj

    @classmethod
    def create_manual(cls, scale, offset, input_stats_dict):
        def flat(x):
            return (x if torch.is_tensor(x) else torch.from_numpy(np.asarray(x))).flatten()

        for x in [offset] + list(input_stats_dict.values()):
            assert x.shape == scale.shape and x.dtype == scale.dtype
        p = nn.ParameterDict({"scale": flat(scale), "offset": flat(offset),
                              "input_stats": nn.ParameterDict({k: flat(v) for k, v in input_stats_dict.items()})})
        p.requires_grad_(False)
        return cls(p)

    @classmethod
    def create_identity(cls, dtype=torch.float32):
        t = lambda v: torch.tensor([v], dtype=dtype)  # noqa: E731
        return cls.create_manual(t(1), t(0), {"min": t(-1), "max": t(1), "mean": t(0), "std": t(1)})

    # the policy's earlier name for the parameter dict
    @property
    def params(self):
        return self.params_dict

    def normalize(self, x):
        return _normalize(x, self.params_dict, forward=True)

    def unnormalize(self, x):
        return _normalize(x, self.params_dict, forward=False)

    def get_input_stats(self):
        return self.params_dict["input_stats"]

    def get_output_stats(self):
        return {k: self.normalize(v) for k, v in self.params_dict["input_stats"].items()}

    def __call__(self, x):
        return self.normalize(x)


class LinearNormalizer(_ParamsModule):
    @torch.no_grad()
    def fit(self, data, **kw):
        if isinstance(data, dict):
            for k, v in data.items():
                self.params_dict[k] = _fit(v, **kw)
        else:
            self.params_dict["_default"] = _fit(data, **kw)

    def __call__(self, x):
        return self.normalize(x)

    def __getitem__(self, key):
        return SingleFieldLinearNormalizer(self.params_dict[key])

    def __setitem__(self, key, value):
        self.params_dict[key] = value.params_dict

    def __contains__(self, key):
        return key in self.params_dict

    def _apply_norm(self, x, forward):
        if isinstance(x, dict):
            return {k: _normalize(v, self.params_dict[k], forward) for k, v in x.items()}
        if "_default" not in self.params_dict:
            raise RuntimeError("Not initialized")
        return _normalize(x, self.params_dict["_default"], forward)

    def normalize(self, x):
        return self._apply_norm(x, True)

    def unnormalize(self, x):
        return self._apply_norm(x, False)

    def get_input_stats(self):
        if len(self.params_dict) == 0:
            raise RuntimeError("Not initialized")
        if len(self.params_dict) == 1 and "_default" in self.params_dict:
            return self.params_dict["_default"]["input_stats"]
        return {k: v["input_stats"] for k, v in self.params_dict.items() if k != "_default"}

    def get_output_stats(self):
        stats = self.get_input_stats()
        if "min" in stats:
            return {k: self.normalize(v) for k, v in stats.items()}
        return {key: {n: self.normalize({key: v})[key] for n, v in group.items()} for key, group in stats.items()}
