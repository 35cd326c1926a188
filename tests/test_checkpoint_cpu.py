"""Reference-layout `.ckpt` payloads (workspace/checkpoint.py; base_workspace.py:33-135): round
trip through torch.save / torch.load(weights_only=True), and the optimizer state exchanged with
torch.optim.AdamW built the way policy.get_optimizer builds it (policy:326-360)."""
import pickle
from functools import partial

import pytest
import torch
import torch.nn as nn

import cases
from hashinit import hash_init_


@pytest.fixture
def fp32():
    from unified_video_action_amd.runtime import RT
    RT.set_precision("fp32")
    yield
    RT.set_precision("bf16")


def _policy():
    from unified_video_action_amd.model.autoregressive import mar_con_unified as pmar
    from unified_video_action_amd.policy.unified_video_action_policy import UnifiedVideoActionPolicy
    pmar.mar_golden = lambda **kw: pmar.MAR(norm_layer=partial(nn.LayerNorm, eps=1e-6), **cases.MAR_GOLDEN, **kw)
    amp = dict(pretrained_model_path=None, model_size="mar_golden")
    for k in cases.POLICY_AMP_KEYS:
        amp[k] = cases.MAR_KW[k]
    pol = UnifiedVideoActionPolicy(
        vae_model_params=dict(autoencoder_path=None, ddconfig=dict(vae_embed_dim=16, ch_mult=[1, 1, 2, 2, 4])),
        autoregressive_model_params=amp, action_model_params=dict(predict_action=True, act_model_type="conv_fc"),
        shape_meta={"action": {"shape": [2]}}, n_action_steps=8, shift_action=True, language_emb_model=None,
        task_name="pusht", task_modes=[], normalizer_type="all", selected_training_mode=None,
        use_history_action=False, use_proprioception=False, action_mask_ratio=0.5, different_history_freq=False,
        predict_wrist_img=False, predict_proprioception=False)
    hash_init_(pol.model, "mar.")
    return pol


def _opt(pol):
    opt = pol.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    g = torch.Generator().manual_seed(0)
    opt.m.copy_(torch.randn(opt.m.shape, generator=g))
    opt.v.copy_(torch.rand(opt.v.shape, generator=g))
    opt.ema.copy_(torch.randn(opt.ema.shape, generator=g))
    opt.step_count = opt.ema_step_count = 7
    return opt


def test_checkpoint_round_trip(tmp_path, fp32):
    from unified_video_action_amd.workspace.checkpoint import load_checkpoint, save_checkpoint
    from unified_video_action_amd.workspace.optim import CosineWithWarmup
    pol = _policy()
    opt = _opt(pol)
    sch = CosineWithWarmup(opt, 10, 100)
    for _ in range(12):
        sch.step()
    path = tmp_path / "latest.ckpt"
    save_checkpoint(path, pol, opt, sch, global_step=12, epoch=3, cfg={"name": "uva_pusht"})
    payload = torch.load(path, weights_only=True)  # loadable with the safe loader
    assert set(payload) == {"cfg", "state_dicts", "pickles"}
    assert set(payload["state_dicts"]) == {"model", "ema_model", "optimizer", "lr_scheduler"}
    assert pickle.loads(payload["pickles"]["global_step"]) == 12

    pol2 = _policy()
    with torch.no_grad():
        for p in pol2.model.parameters():
            p.zero_()
    opt2 = pol2.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    sch2 = CosineWithWarmup(opt2, 10, 100)
    meta = load_checkpoint(path, pol2, opt2, sch2)
    assert meta == {"cfg": {"name": "uva_pusht"}, "global_step": 12, "epoch": 3}
    assert torch.equal(opt2.store.flat, opt.store.flat)
    assert torch.equal(opt2.m, opt.m) and torch.equal(opt2.v, opt.v) and torch.equal(opt2.ema, opt.ema)
    assert opt2.step_count == 7
    assert sch2.last_epoch == sch.last_epoch and opt2.param_groups[0]["lr"] == opt.param_groups[0]["lr"]
    for k, v in pol.state_dict().items():
        assert torch.equal(pol2.state_dict()[k], v), k
    # EMA weights can be loaded as the model (load_payload without "model", base_workspace.py:115-124)
    pol3 = _policy()
    load_checkpoint(path, pol3, use_ema_weights=True)
    ema = opt.ema_state()
    for n, p in pol3.model.named_parameters():
        assert torch.equal(p.detach(), ema[n]), n


def test_optimizer_state_exchanges_with_torch_adamw(fp32):
    """ours -> torch AdamW.load_state_dict -> its state_dict -> ours: identical, and the layout
    (groups, ids, per-param state) is the one torch produces for policy.get_optimizer's groups."""
    from unified_video_action_amd.workspace.checkpoint import load_optimizer_state_torch, optimizer_state_torch
    pol = _policy()
    opt = _opt(pol)
    sd = optimizer_state_torch(opt, pol.model)
    ref_model = _policy().model
    groups = pol.add_weight_decay(ref_model, 0.02)  # same grouping rule as the reference (policy:326-342)
    topt = torch.optim.AdamW(groups, lr=1e-4, betas=(0.9, 0.95))
    for g in topt.param_groups:
        g["initial_lr"] = g["lr"]
    topt.load_state_dict(sd)
    tsd = topt.state_dict()
    assert [len(g["params"]) for g in tsd["param_groups"]] == [len(g["params"]) for g in sd["param_groups"]]
    assert [g["weight_decay"] for g in tsd["param_groups"]] == [0.0, 0.02]
    for i, s in sd["state"].items():
        assert torch.equal(tsd["state"][i]["exp_avg"], s["exp_avg"])
        assert float(tsd["state"][i]["step"]) == 7.0
    # a state produced by torch itself (one real AdamW step) loads into ours
    for p in ref_model.parameters():
        p.grad = torch.randn_like(p)
    topt.step()
    opt2 = pol.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    load_optimizer_state_torch(opt2, pol.model, topt.state_dict())
    assert opt2.step_count == 8
    back = optimizer_state_torch(opt2, pol.model)
    for i, s in topt.state_dict()["state"].items():
        assert torch.equal(back["state"][i]["exp_avg_sq"], s["exp_avg_sq"])


def test_checkpoint_pickles_refuse_globals(tmp_path, fp32):
    from unified_video_action_amd.workspace.checkpoint import _loads_primitive
    assert _loads_primitive(pickle.dumps(5)) == 5
    with pytest.raises(pickle.UnpicklingError):
        _loads_primitive(pickle.dumps(torch.float32))
