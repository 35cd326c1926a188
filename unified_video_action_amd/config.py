"""Hydra-compatible configuration composition without hydra / omegaconf (neither is in this
image), for the reference's config surface (train.py:26-60, config/uva_*.yaml,
config/{model,task}/*.yaml):

  * `defaults:` lists (`_self_`, `group: option`, `optional group: option`, plain names), each
    group's file merged under the group's key, `_self_` placed where it is listed;
  * command-line overrides `a.b=v` (value parsed as YAML), `+a.b=v` (add), `~a.b` (delete) and
    group selections `task=libero10`;
  * `${a.b}` interpolation (absolute, or relative with leading dots), nested interpolation
    inside strings, `${now:<strftime>}`, and the reference's `${eval:'...'}` resolver --
    evaluated by a restricted arithmetic evaluator (literals, + - * / // % **, comparisons,
    list / range / tuple / int / float / len / min / max / abs / round / ListConfig), never
    Python's eval;
  * `instantiate(node, **kw)` of `_target_` nodes (recursive, like hydra.utils.instantiate),
    with `unified_video_action.*` targets that are not importable mapped onto this package's
    classes of the same module path (the policy, workspace, EMAModel, lr scheduler) -- so the
    reference's own YAML files run unchanged on the MI355X path.
"""
import ast
import copy
import datetime
import importlib
import operator
import os
import re

import yaml


class Node(dict):
    """dict with attribute access (OmegaConf DictConfig reading surface)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    def __delattr__(self, k):
        del self[k]

    def __deepcopy__(self, memo):
        return Node({k: copy.deepcopy(v, memo) for k, v in self.items()})


def to_node(x):
    if isinstance(x, dict):
        return Node({k: to_node(v) for k, v in x.items()})
    if isinstance(x, list):
        return [to_node(v) for v in x]
    return x


def to_container(x):
    if isinstance(x, dict):
        return {k: to_container(v) for k, v in x.items()}
    if isinstance(x, list):
        return [to_container(v) for v in x]
    return x


def _merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _load_yaml(path):
    with open(path) as f:
        d = yaml.safe_load(f)
    return d or {}


def _find(config_dir, name):
    for cand in (name, name + ".yaml"):
        p = os.path.join(config_dir, cand)
        if os.path.isfile(p):
            return p
    raise FileNotFoundError(f"config {name!r} not found in {config_dir}")


def _compose_file(config_dir, rel, group_choice):
    raw = _load_yaml(_find(config_dir, rel))
    defaults = raw.pop("defaults", None) or []
    # `override group: option` entries re-select a group inside the configs this one inherits
    # (command-line selections win: they are already in group_choice)
    group_choice = dict(group_choice)
    plain = []
    for d in defaults:
        if isinstance(d, dict) and next(iter(d)).startswith("override "):
            (gk, opt), = d.items()
            group_choice.setdefault(gk.split(" ")[-1].lstrip("/"), opt)
        else:
            plain.append(d)
    defaults = plain
    out = {}
    placed_self = False
    for d in defaults:
        if d == "_self_":
            _merge(out, raw)
            placed_self = True
            continue
        if isinstance(d, str):  # `name` or `name@package`, relative to this file's group directory
            name, _, pkg = d.partition("@")
            path = name.lstrip("/") if name.startswith("/") else os.path.join(os.path.dirname(rel), name)
            sub = _compose_file(config_dir, path, group_choice)
            node = out
            for part in [x for x in pkg.split(".") if x]:
                node = node.setdefault(part, {})
            _merge(node, sub)
            continue
        (gk, opt), = d.items()
        optional = gk.startswith("optional ")
        group = gk.split(" ")[-1].lstrip("/")
        opt = group_choice.get(group, opt)
        if opt is None:
            continue
        path = os.path.join(group, str(opt))
        try:
            sub = _compose_file(config_dir, path, group_choice)
        except FileNotFoundError:
            if optional:
                continue
            raise
        pkg = group.replace("/", ".")
        node = out
        for part in pkg.split(".")[:-1]:
            node = node.setdefault(part, {})
        node[pkg.split(".")[-1]] = _merge(node.get(pkg.split(".")[-1], {}) or {}, sub)
    if not placed_self:  # Hydra 1.1+: the primary config is applied last by default
        _merge(out, raw)
    return out


def _set(cfg, dotted, value, add=False):
    parts = dotted.split(".")
    node = cfg
    for p in parts[:-1]:
        if p not in node or not isinstance(node[p], dict):
            if not add:
                raise KeyError(f"override {dotted}: no key {p!r}")
            node[p] = {}
        node = node[p]
    if parts[-1] not in node and not add:
        raise KeyError(f"override {dotted}: key does not exist (use +{dotted}=...)")
    node[parts[-1]] = value


def _delete(cfg, dotted):
    parts = dotted.split(".")
    node = cfg
    for p in parts[:-1]:
        node = node[p]
    node.pop(parts[-1], None)


def compose(config_dir, config_name, overrides=()):
    """-> Node of the resolved configuration."""
    group_choice, values = {}, []
    groups = {d for d in os.listdir(config_dir) if os.path.isdir(os.path.join(config_dir, d))}
    for ov in overrides:
        if ov.startswith("~"):
            values.append(("del", ov[1:], None))
            continue
        key, _, val = ov.partition("=")
        add = key.startswith("+") or key.startswith("++")
        key = key.lstrip("+")
        if key in groups and not add:
            group_choice[key] = val
            continue
        values.append(("add" if add else "set", key, yaml.safe_load(val) if val != "" else None))
    cfg = _compose_file(config_dir, config_name, group_choice)
    for kind, key, val in values:
        if kind == "del":
            _delete(cfg, key)
        else:
            _set(cfg, key, val, add=(kind == "add"))
    return to_node(resolve(cfg))


# ---- interpolation ----------------------------------------------------------------------------
_INTERP = re.compile(r"\$\{([^${}]*)\}")


class _ListConfig(list):
    pass


_EVAL_FUNCS = {"list": list, "range": range, "tuple": tuple, "int": int, "float": float, "len": len, "min": min,
               "max": max, "abs": abs, "round": round, "ListConfig": _ListConfig, "str": str, "bool": bool}
_BINOPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul, ast.Div: operator.truediv,
           ast.FloorDiv: operator.floordiv, ast.Mod: operator.mod, ast.Pow: operator.pow}
_CMPOPS = {ast.Eq: operator.eq, ast.NotEq: operator.ne, ast.Lt: operator.lt, ast.LtE: operator.le,
           ast.Gt: operator.gt, ast.GtE: operator.ge}


def safe_eval(expr):
    """the `${eval:...}` resolver over a restricted expression grammar (no attribute access, no
    names beyond a few pure builtins)."""
    def ev(n):
        if isinstance(n, ast.Expression):
            return ev(n.body)
        if isinstance(n, ast.Constant):
            return n.value
        if isinstance(n, (ast.List, ast.Tuple)):
            vals = [ev(e) for e in n.elts]
            return vals if isinstance(n, ast.List) else tuple(vals)
        if isinstance(n, ast.BinOp) and type(n.op) in _BINOPS:
            a, b = ev(n.left), ev(n.right)
            if isinstance(n.op, ast.Pow) and abs(b) > 64:
                raise ValueError("exponent too large")
            return _BINOPS[type(n.op)](a, b)
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, (ast.USub, ast.UAdd, ast.Not)):
            v = ev(n.operand)
            return -v if isinstance(n.op, ast.USub) else (+v if isinstance(n.op, ast.UAdd) else not v)
        if isinstance(n, ast.Compare) and len(n.ops) == 1 and type(n.ops[0]) in _CMPOPS:
            return _CMPOPS[type(n.ops[0])](ev(n.left), ev(n.comparators[0]))
        if isinstance(n, ast.IfExp):
            return ev(n.body) if ev(n.test) else ev(n.orelse)
        if isinstance(n, ast.Call) and isinstance(n.func, ast.Name) and n.func.id in _EVAL_FUNCS and not n.keywords:
            args = [ev(a) for a in n.args]
            if n.func.id == "range" and len(range(*args)) > 1_000_000:
                raise ValueError("range too long")
            out = _EVAL_FUNCS[n.func.id](*args)
            return list(out) if isinstance(out, (range, _ListConfig)) else out
        raise ValueError(f"${{eval:}} expression not allowed: {ast.dump(n)[:80]}")
    return ev(ast.parse(expr.strip(), mode="eval"))


def _lookup(root, path, here):
    if path.startswith("."):
        up = len(path) - len(path.lstrip("."))
        node_path = here[:len(here) - up] if up <= len(here) else []
        path = ".".join(node_path + [path.lstrip(".")])
    node = root
    for p in path.split("."):
        if isinstance(node, list):
            node = node[int(p)]
        else:
            node = node[p]
    return node


def resolve(cfg):
    """resolve every interpolation in place (OmegaConf.resolve)."""
    root = cfg
    busy = set()

    def res_str(s, here, depth):
        if depth > 32:
            raise ValueError(f"interpolation too deep: {s}")
        full = re.fullmatch(r"\$\{([^${}]*)\}", s)
        while True:
            m = _INTERP.search(s)
            if m is None:
                return s
            inner = m.group(1)
            val = res_expr(inner, here, depth)
            if full is not None and m.span() == (0, len(s)):
                return val  # whole-string interpolation keeps the value's type
            s = s[:m.start()] + str(val) + s[m.end():]
            full = re.fullmatch(r"\$\{([^${}]*)\}", s)

    def res_expr(inner, here, depth):
        if inner.startswith("eval:"):
            arg = inner[5:].strip()
            if len(arg) >= 2 and arg[0] == arg[-1] and arg[0] in "'\"":
                arg = arg[1:-1]
            return safe_eval(arg)
        if inner.startswith("now:"):
            return datetime.datetime.now().strftime(inner[4:])
        key = inner.strip()
        if key in busy:
            raise ValueError(f"interpolation cycle at ${{{key}}}")
        busy.add(key)
        try:
            v = _lookup(root, key, here)
            if isinstance(v, str):
                v = res_str(v, key.split("."), depth + 1)
            elif isinstance(v, (dict, list)):
                v = walk(v, key.split("."), depth + 1)
        finally:
            busy.discard(key)
        return v

    def walk(node, here, depth=0):
        items = node.items() if isinstance(node, dict) else enumerate(node)
        for k, v in list(items):
            if isinstance(v, str) and "${" in v:
                # nested ${...${...}...} (e.g. eval of interpolations): resolve innermost first
                node[k] = res_str(v, here, depth)
            elif isinstance(v, (dict, list)):
                walk(v, here + [str(k)], depth)
        return node

    return walk(cfg, [])


# ---- instantiation ---------------------------------------------------------------------------
REF_PKG = "unified_video_action."
OWN_PKG = "unified_video_action_amd."


def get_class(path):
    mod, _, name = path.rpartition(".")
    try:
        return getattr(importlib.import_module(mod), name)
    except (ImportError, AttributeError):
        if path.startswith(REF_PKG):
            own = OWN_PKG + path[len(REF_PKG):]
            mod, _, name = own.rpartition(".")
            try:
                return getattr(importlib.import_module(mod), name)
            except (ImportError, AttributeError):
                pass
        raise ImportError(f"_target_ {path} is not importable here (and has no {OWN_PKG} counterpart)")


def instantiate(node, **kwargs):
    if isinstance(node, list):
        return [instantiate(v) for v in node]
    if not isinstance(node, dict):
        return node
    if "_target_" not in node:
        return Node({k: instantiate(v) if isinstance(v, dict) and "_target_" in v else v for k, v in node.items()})
    args = {k: v for k, v in node.items() if not k.startswith("_")}
    args = {k: (instantiate(v) if isinstance(v, dict) and "_target_" in v else v) for k, v in args.items()}
    args.update(kwargs)
    return get_class(node["_target_"])(**args)
