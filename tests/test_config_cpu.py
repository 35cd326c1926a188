"""Hydra-style composition without hydra (unified_video_action_amd/config.py): this build's
config tree, command-line overrides, interpolation, the restricted ${eval:} resolver, target
mapping -- and, when the reference checkout is present in this container, the reference's own
config tree (train.py --config-dir=<reference>/unified_video_action/config)."""
import os

import pytest

from unified_video_action_amd import config as C

OWN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "unified_video_action_amd", "config")
REF = "/root/reference/unified_video_action/config"


def test_own_configs_compose():
    c = C.compose(OWN, "uva_pusht", [])
    assert c.task.name == "pusht" and c.model.policy.shape_meta == c.task.shape_meta
    assert c.model.policy.action_model_params.predict_action is False
    c = C.compose(OWN, "uva_libero10", [])
    assert c.task.name == "libero_10" and c.task.dataset.language_emb_model == "clip"
    assert c.model.policy.action_model_params == {"predict_action": True, "act_model_type": "conv_fc"}
    c = C.compose(OWN, "uva_umi_multi", ["task.dataset.n_samples=8"])
    assert c.task.task_modes == ["policy_model", "full_dynamic_model"] and c.dataloader.batch_size == 56
    assert c.model.policy.different_history_freq is True and c.task.dataset.n_samples == 8


def test_overrides_and_group_selection():
    c = C.compose(OWN, "uva_pusht", ["task=libero10", "training.seed=7", "+training.extra=[1, 2]",
                                     "~checkpoint.topk"])
    assert c.task.name == "libero_10" and c.training.seed == 7 and c.training.extra == [1, 2]
    assert "topk" not in c.checkpoint
    with pytest.raises(KeyError):
        C.compose(OWN, "uva_pusht", ["training.no_such_key=1"])


def test_interpolation_and_restricted_eval():
    cfg = {"a": {"b": 3, "c": "${a.b}", "d": "x${a.b}y"}, "e": "${eval:'(${a.b} - 1) * 2'}",
           "f": "${eval:\"ListConfig(list(range(-12, 17, 4)))\"}", "g": "${a}"}
    r = C.to_node(C.resolve(cfg))
    assert r.a.c == 3 and r.a.d == "x3y" and r.e == 4 and r.f == list(range(-12, 17, 4)) and r.g.b == 3
    for bad in ("__import__('os').system('true')", "().__class__", "open('x')", "10 ** 1000"):
        with pytest.raises(ValueError):
            C.safe_eval(bad)


def test_targets_map_to_this_build():
    ema = C.get_class("unified_video_action.model.autoregressive.ema_model.EMAModel")
    assert ema.__module__ == "unified_video_action_amd.model.autoregressive.ema_model"
    ws = C.get_class("unified_video_action.workspace.train_unified_video_action_workspace."
                     "TrainUnifiedVideoActionWorkspace")
    assert ws.__module__.startswith("unified_video_action_amd.")
    with pytest.raises(ImportError):
        C.get_class("unified_video_action.dataset.pusht_image_dataset.PushTImageDataset")


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
@pytest.mark.parametrize("name", ["uva_pusht.yaml", "uva_libero10.yaml", "uva_umi_multi.yaml", "uva_umi.yaml",
                                  "uva_toolhang.yaml", "uva_human_pp.yaml"])
def test_reference_config_tree_composes(name):
    c = C.compose(REF, name, ["training.debug=true"])
    assert C.get_class(c.model.policy._target_).__module__ == \
        "unified_video_action_amd.policy.unified_video_action_policy"
    assert C.get_class(c.model._target_).__name__ == "TrainUnifiedVideoActionWorkspace"
    assert c.model.policy.shape_meta == c.task.shape_meta
    if name == "uva_umi_multi.yaml":  # umi_lazy@dataset package default + ${eval:...} resolvers
        ds = c.task.dataset
        assert isinstance(ds.dataset_configs, dict) and len(ds.dataset_configs) == 3
