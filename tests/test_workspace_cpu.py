"""The drop-in training surface on the CPU (no kernels run): policy.get_optimizer returns a real
torch.optim.Optimizer (FusedAdamWEMA) that torch's LambdaLR / this build's get_scheduler drive,
GradScaler.unscale_ reaches through accelerate-style param_groups, zero_grad(set_to_none) and
module moves keep the flat-buffer binding, a deepcopy (the reference's EMA policy,
workspace:70-72) does not inherit it, DDP sees only the anchor parameter, and the workspace
(configs -> instantiate -> setup) reproduces the reference's LR trace (tests/golden/g6)."""
import copy

import numpy as np
import pytest
import torch

import cases
import replay


@pytest.fixture
def fp32():
    from unified_video_action_amd.runtime import RT
    RT.set_precision("fp32")
    yield
    RT.set_precision("bf16")


def test_optimizer_is_torch_optimizer_with_reference_groups(fp32):
    pol = replay.golden_policy()
    opt = pol.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=[0.9, 0.95])
    assert isinstance(opt, torch.optim.Optimizer)
    ref_groups = pol.add_weight_decay(pol.model, 0.02)
    assert [g["weight_decay"] for g in opt.param_groups] == [0.0, 0.02]
    for g, r in zip(opt.param_groups, ref_groups):
        assert [id(p) for p in g["params"]] == [id(p) for p in r["params"]]
        assert g["initial_lr"] == 1e-4 and g["betas"] == (0.9, 0.95)
    assert opt.store.is_bound() and pol.bound_optimizer() is opt
    with pytest.raises(NotImplementedError):
        opt.add_param_group({"params": [torch.nn.Parameter(torch.zeros(2))]})


def test_scheduler_trace_matches_reference_workspace(fp32):
    from unified_video_action_amd.model.common.lr_scheduler import get_scheduler
    pol = replay.golden_policy()
    L = cases.TRACE_LR
    opt = pol.get_optimizer(weight_decay=L["weight_decay"], learning_rate=L["lr"], betas=L["betas"])
    sch = get_scheduler(L["name"], opt, num_warmup_steps=L["warmup"], num_training_steps=L["total"])
    g = replay.load("g6_workspace_trace.npz")
    got = []
    for _ in range(cases.TRACE_STEPS):
        opt._opt_called = True  # silence torch's order warning (no kernels on the CPU)
        sch.step()
        got.append(sch.get_last_lr()[0])
    np.testing.assert_allclose(got, g["rows"][:, 3], rtol=0, atol=1e-15)
    # also torch's own LambdaLR over it, and every diffusers schedule shape
    for name in ("linear", "cosine_with_restarts", "polynomial", "constant", "constant_with_warmup"):
        s = get_scheduler(name, opt, num_warmup_steps=2, num_training_steps=10)
        assert len(s.get_last_lr()) == 2


def test_grad_scaler_and_zero_grad_keep_flat_binding(fp32):
    pol = replay.golden_policy()
    opt = pol.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    opt.store.grad.fill_(1.0)
    scaler = torch.amp.GradScaler("cpu", init_scale=1024.0)
    scaler.scale(torch.ones(()))
    scaler.unscale_(opt)  # accelerate's fp16 path: foreach unscale over param_groups' grads
    assert opt.store.is_bound()
    p = opt.param_groups[1]["params"][0]
    assert torch.allclose(p.grad, torch.full_like(p.grad, 1 / 1024.0))
    opt.zero_grad(set_to_none=True)
    assert opt.store.is_bound() and float(opt.store.grad.abs().sum()) == 0.0


def test_module_move_rebinds_and_deepcopy_does_not_inherit(fp32):
    pol = replay.golden_policy()
    opt = pol.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    opt.m.fill_(3.0)
    before = {n: p.detach().clone() for n, p in pol.model.named_parameters()}
    pol._apply(lambda t: t.clone())  # what .to(device) does to every parameter tensor
    assert opt.store.is_bound()
    for n, p in pol.model.named_parameters():
        assert torch.equal(p, before[n]), n
    assert float(opt.m[:10].sum()) == 30.0
    ema = copy.deepcopy(pol)
    assert ema.bound_optimizer() is None
    q = dict(ema.model.named_parameters())["z_proj.weight"]
    assert q.untyped_storage().data_ptr() != opt.store.flat.untyped_storage().data_ptr()


def test_ddp_sees_only_the_anchor_and_state_dicts_exclude_it(fp32):
    pol = replay.golden_policy()
    ignored = set(pol._ddp_params_and_buffers_to_ignore)
    names = {n for n, _ in pol.named_parameters()}
    assert names - ignored == {"ddp_anchor"}
    sd = pol.state_dict()
    assert "ddp_anchor" not in sd
    pol2 = replay.golden_policy()
    pol2.load_state_dict(sd, strict=True)  # a reference state dict (no anchor) loads strictly


def test_workspace_setup_from_config(tmp_path, fp32):
    from unified_video_action_amd import config as C
    from unified_video_action_amd.model.autoregressive import mar_con_unified as pmar
    import train
    replay.golden_policy(normalizer=False)  # registers mar_golden
    assert hasattr(pmar, "mar_golden")
    L = cases.TRACE_LR
    cfg = train.build_cfg([
        "--config-name=uva_pusht", "model.policy.autoregressive_model_params.model_size=mar_golden",
        "model.policy.action_model_params.predict_action=true", f"training.lr_warmup_steps={L['warmup']}",
        "training.num_epochs=1", "dataloader.batch_size=1", "dataloader.num_workers=0",
        f"task.dataset.n_samples={L['total']}", "training.resume=false", "training.mixed_precision=no",
        f"multi_run.run_dir={tmp_path}"])
    cls = C.get_class(cfg.model._target_)
    ws = cls(cfg)
    assert isinstance(ws.optimizer, torch.optim.Optimizer) and ws.ema_model is not None
    ws.setup(device="cpu")
    assert len(ws.train_dataloader) == L["total"]
    batch = next(iter(ws.train_dataloader))
    assert batch["obs"]["image"].shape == (1, 32, 3, 96, 96) and batch["action"].shape == (1, 32, 2)
    assert ws.lr_scheduler.get_last_lr()[0] == 0.0  # warmup step 0
    assert ws.model.normalizer["action"].params["scale"][0].item() == pytest.approx(2 / 512)
    from unified_video_action_amd.model.autoregressive.ema_model import EMAModel
    assert isinstance(ws.ema, EMAModel) and ws.ema.power == 0.75


def test_topk_fallback_keeps_configured_monitor_key(tmp_path):
    """a call without the configured monitor key ranks by train_loss in a ranking
    of its own and leaves monitor_key / mode / format_str alone, so the configured key is used
    again once it is logged."""
    from unified_video_action_amd.workspace.train_unified_video_action_workspace import TopKCheckpointManager
    m = TopKCheckpointManager(str(tmp_path), "test_mean_score", mode="max", k=2)
    p1 = m.get_ckpt_path({"epoch": 1, "train_loss": 1.0})
    p2 = m.get_ckpt_path({"epoch": 2, "train_loss": 0.5})
    assert p1 and p2 and "train_loss" in p1
    assert m.get_ckpt_path({"epoch": 3, "train_loss": 2.0}) is None  # worse than both kept
    assert (m.monitor_key, m.mode, m.format_str) == ("test_mean_score", "max", "epoch={epoch:03d}.ckpt")
    q = m.get_ckpt_path({"epoch": 4, "train_loss": 0.1, "test_mean_score": 0.3})
    assert q.endswith("epoch=004.ckpt") and m.path_value_map == {q: 0.3}
