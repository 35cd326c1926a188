"""Reference-layout `.ckpt` payloads (workspace/checkpoint.py, workspace/base_workspace.py;
reference base_workspace.py:33-135): round trip, optimizer state exchanged with a real
torch.optim.AdamW built like the reference policy.get_optimizer (policy:326-360), loading a
payload whose cfg pickles as OmegaConf objects through the restricted loader (nothing from the
file executes), refusal of any other global, and the pretrained warm start
(policy:113-118,140-218) from MAR `model_ema` and UVA `state_dicts.ema_model` payloads."""
import copy
import pickle
import sys
import types

import pytest
import torch

import replay


@pytest.fixture
def fp32():
    from unified_video_action_amd.runtime import RT
    RT.set_precision("fp32")
    yield
    RT.set_precision("bf16")


def _packed(opt, buf):
    """the parameter regions of a flat optimizer buffer (group padding dropped)."""
    return torch.cat([buf[o:o + k] for o, k in (opt.store.offsets[id(p)] for _, p in opt.store.order)])


def _opt_with_state(pol):
    opt = pol.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    g = torch.Generator().manual_seed(0)
    opt.m.copy_(torch.randn(opt.m.shape, generator=g))
    opt.v.copy_(torch.rand(opt.v.shape, generator=g))
    opt.step_count = 7
    return opt


def test_payload_round_trip(tmp_path, fp32):
    from unified_video_action_amd.model.common.lr_scheduler import get_scheduler
    from unified_video_action_amd.workspace.checkpoint import load_checkpoint, safe_load, save_checkpoint
    pol = replay.golden_policy()
    ema = copy.deepcopy(pol)
    with torch.no_grad():
        for p in ema.model.parameters():
            p.mul_(0.5)
    opt = _opt_with_state(pol)
    sch = get_scheduler("cosine", opt, num_warmup_steps=10, num_training_steps=100)
    for _ in range(12):
        sch.step()
    path = tmp_path / "latest.ckpt"
    save_checkpoint(path, pol, ema, opt, sch, cfg={"name": "uva_pusht"}, global_step=12, epoch=3)
    payload = torch.load(path, weights_only=True)  # plain tensors / containers only
    assert set(payload["state_dicts"]) == {"model", "ema_model", "optimizer", "lr_scheduler"}
    assert "ddp_anchor" not in payload["state_dicts"]["model"]
    assert payload["state_dicts"]["optimizer"]["param_groups"][0]["weight_decay"] == 0.0
    assert payload["state_dicts"]["optimizer"]["param_groups"][1]["weight_decay"] == 0.02

    pol2 = replay.golden_policy()
    with torch.no_grad():
        for p in pol2.model.parameters():
            p.zero_()
    ema2 = copy.deepcopy(pol2)
    opt2 = pol2.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    sch2 = get_scheduler("cosine", opt2, num_warmup_steps=10, num_training_steps=100)
    meta = load_checkpoint(path, pol2, ema2, opt2, sch2)
    assert meta["global_step"] == 12 and meta["epoch"] == 3 and meta["cfg"] == {"name": "uva_pusht"}
    for (n, a), (_, b) in zip(pol.state_dict().items(), pol2.state_dict().items()):
        assert torch.equal(a, b), n
    for (n, a), (_, b) in zip(ema.state_dict().items(), ema2.state_dict().items()):
        assert torch.equal(a, b), n
    assert torch.equal(_packed(opt2, opt2.m), _packed(opt, opt.m)) and torch.equal(_packed(opt2, opt2.v), _packed(opt, opt.v))
    assert opt2.step_count == 7
    assert sch2.last_epoch == sch.last_epoch and sch2.get_last_lr() == sch.get_last_lr()
    assert safe_load(path)["state_dicts"]["optimizer"]["state"][0]["step"].item() == 7.0


def test_optimizer_state_exchanges_with_torch_adamw(fp32):
    pol = replay.golden_policy()
    opt = _opt_with_state(pol)
    sd = opt.state_dict()
    ref = torch.optim.AdamW(pol.add_weight_decay(pol.model, 0.02), lr=1e-4, betas=(0.9, 0.95))
    ref.load_state_dict(copy.deepcopy(sd))  # the reference workspace resumes from our optimizer state
    for (n, p) in pol.model.named_parameters():
        o, k = opt.store.offsets[id(p)]
        assert torch.equal(ref.state[p]["exp_avg"].reshape(-1), opt.m[o:o + k]), n
    opt2 = pol.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    opt2.load_state_dict(ref.state_dict())  # and we resume from the reference's
    assert torch.equal(_packed(opt2, opt2.m), _packed(opt, opt.m)) and torch.equal(_packed(opt2, opt2.v), _packed(opt, opt.v))
    assert opt2.step_count == 7


def _fake_omegaconf():
    """stand-ins for omegaconf's container classes (omegaconf is not installed), pickled as
    module "omegaconf.dictconfig" like the reference's cfg."""
    mod = types.ModuleType("omegaconf")
    sub = types.ModuleType("omegaconf.dictconfig")

    class DictConfig:
        def __init__(self, content):
            self._content = content

        def __getstate__(self):
            return {"_content": self._content, "_metadata": None, "_parent": None}

        def __setstate__(self, s):
            self.__dict__.update(s)

    DictConfig.__module__ = "omegaconf.dictconfig"
    DictConfig.__qualname__ = "DictConfig"
    sub.DictConfig = DictConfig
    mod.dictconfig = sub
    return mod, sub, DictConfig


def test_reference_style_cfg_loads_without_executing(tmp_path, fp32):
    from unified_video_action_amd.workspace.checkpoint import load_checkpoint, make_payload
    pol = replay.golden_policy()
    mod, sub, DictConfig = _fake_omegaconf()
    sys.modules["omegaconf"], sys.modules["omegaconf.dictconfig"] = mod, sub
    try:
        payload = make_payload(pol, global_step=5, epoch=1)
        payload["cfg"] = DictConfig({"name": "uva", "training": DictConfig({"seed": 42})})
        path = tmp_path / "ref.ckpt"
        torch.save(payload, path)
    finally:
        del sys.modules["omegaconf"], sys.modules["omegaconf.dictconfig"]
    with pytest.raises(pickle.UnpicklingError):
        torch.load(path, weights_only=True)  # what the previous loader did: the whole file refused
    pol2 = replay.golden_policy()
    meta = load_checkpoint(path, pol2)
    assert meta["cfg"] == {"name": "uva", "training": {"seed": 42}} and meta["global_step"] == 5
    assert "omegaconf" not in sys.modules


class _Evil:
    def __reduce__(self):
        return (print, ("executed from a checkpoint",))


def test_restricted_loader_refuses_other_globals(tmp_path):
    from unified_video_action_amd.workspace.checkpoint import safe_load
    path = tmp_path / "evil.ckpt"
    torch.save({"state_dicts": {}, "cfg": _Evil()}, path)
    with pytest.raises(pickle.UnpicklingError, match="refused"):
        safe_load(path)


@pytest.mark.parametrize("layout", ["mar", "uva"])
def test_pretrained_warm_start(tmp_path, layout, fp32):
    from unified_video_action_amd.model.autoregressive import mar_con_unified as pmar  # noqa: F401
    src = replay.golden_policy()
    with torch.no_grad():
        for p in src.model.parameters():
            p.add_(1.0)
    sd = src.model.state_dict()
    sd["z_proj.weight"] = torch.zeros(3, 3)  # shape mismatch: must keep its own init
    sd["not_a_param"] = torch.ones(2)
    path = tmp_path / f"{layout}.pth"
    if layout == "mar":
        torch.save({"model_ema": sd, "epoch": 3}, path)
    else:
        torch.save({"state_dicts": {"ema_model": {"model." + k: v for k, v in sd.items()}}}, path)
    pol = replay.golden_policy()
    init = {k: v.clone() for k, v in pol.model.state_dict().items()}
    pol.pretrained_model_path = str(path)
    rep = pol.load_pretrained_model()
    got = pol.model.state_dict()
    assert torch.equal(got["z_proj.weight"], init["z_proj.weight"])
    assert "z_proj.weight" in rep["kept_init"]
    for k in got:
        if k != "z_proj.weight":
            assert torch.equal(got[k], sd[k]), k
