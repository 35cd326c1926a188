"""LinearNormalizer with the reference's semantics and state-dict layout
(model/common/normalizer.py:12-297): per-key scale/offset fitted in "limits" mode
(map [min, max] to [-1, 1], constant dims centred) or "gaussian" mode; normalize is
x * scale + offset over the last dim.  Stored as nn.ParameterDict(params_dict.<key>.*)."""
import torch
import torch.nn as nn


def _fit(data, mode="limits", output_max=1.0, output_min=-1.0, range_eps=1e-4, fit_offset=True):
    data = torch.as_tensor(data).float()
    data = data.reshape(-1, data.shape[-1])
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
            out_abs = min(abs(output_min), abs(output_max))
            in_abs = torch.maximum(lo.abs(), hi.abs())
            const = in_abs < range_eps
            in_abs[const] = out_abs
            scale = out_abs / in_abs
            offset = torch.zeros_like(mean)
    elif mode == "gaussian":
        const = std < range_eps
        scale = std.clone()
        scale[const] = 1
        scale = 1 / scale
        offset = -mean * scale if fit_offset else torch.zeros_like(mean)
    else:
        raise ValueError(mode)
    p = nn.ParameterDict({"scale": scale, "offset": offset,
                          "input_stats": nn.ParameterDict({"min": lo, "max": hi, "mean": mean, "std": std})})
    for q in p.parameters():
        q.requires_grad_(False)
    return p


class SingleFieldLinearNormalizer:
    def __init__(self, params):
        self.params = params

    def normalize(self, x):
        s, o = self.params["scale"], self.params["offset"]
        return x * s.to(x.device) + o.to(x.device)

    def unnormalize(self, x):
        s, o = self.params["scale"], self.params["offset"]
        return (x - o.to(x.device)) / s.to(x.device)


class LinearNormalizer(nn.Module):
    def __init__(self):
        super().__init__()
        self.params_dict = nn.ParameterDict()

    def fit(self, data, mode="limits", **kw):
        for k, v in data.items():
            self.params_dict[k] = _fit(v, mode=mode, **kw)

    def __getitem__(self, key):
        return SingleFieldLinearNormalizer(self.params_dict[key])

    def __contains__(self, key):
        return key in self.params_dict

    def normalize(self, x):
        return {k: (self[k].normalize(v) if k in self.params_dict else v) for k, v in x.items()}

    def load_state_dict(self, state_dict, strict=True):
        # rebuild the nested ParameterDict from flat keys params_dict.<key>.<field>[.<stat>]
        tree = {}
        for k, v in state_dict.items():
            parts = k.split(".")
            if parts[0] != "params_dict":
                continue
            node = tree
            for p in parts[1:-1]:
                node = node.setdefault(p, {})
            node[parts[-1]] = v

        def build(d):
            return nn.ParameterDict({k: (build(v) if isinstance(v, dict)
                                         else nn.Parameter(v.clone(), requires_grad=False)) for k, v in d.items()})

        self.params_dict = build(tree)
