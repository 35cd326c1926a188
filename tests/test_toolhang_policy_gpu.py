"""Toolhang with the second camera (use_proprioception, predict_proprioception, predict_wrist_img; no
shipped config turns them on -- config/task/toolhang.yaml + uva.yaml nulls) end to end through
UnifiedVideoActionPolicy.  The MAR streams and losses themselves are pinned against the reference's runs
by the toolhang_prop / toolhang_wrist cases of test_parity_gpu.py (fp32 1e-4 / grads 3e-3, bf16); here
the policy plumbing of data_utils.py:228-285 / 395-410: the wrist frames at the selected indices through
the KL-VAE (history half -> second_image_z, future half -> the wrist video target), the eef / gripper
states split into history / future halves, every head receiving gradient, and predict_action with the
whole eval window."""
import pytest
import torch

import cases
import replay
from hashinit import hash_init_, hash_tensor

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _toolhang_policy():
    from unified_video_action_amd.policy.unified_video_action_policy import UnifiedVideoActionPolicy
    replay.golden_policy(normalizer=False)  # registers model_size "mar_golden"
    amp = dict(pretrained_model_path=None, model_size="mar_golden")
    for k in cases.POLICY_AMP_KEYS:
        amp[k] = cases.MAR_KW[k]
    pol = UnifiedVideoActionPolicy(
        vae_model_params=dict(autoencoder_path=None, ddconfig=dict(vae_embed_dim=16, ch_mult=[1, 1, 2, 2, 4])),
        autoregressive_model_params=amp,
        action_model_params=dict(predict_action=True, act_model_type="conv_fc"),
        shape_meta={"action": {"shape": [10]}}, n_action_steps=8, shift_action=False, language_emb_model=None,
        task_name="toolhang", task_modes=["full_dynamic_model"], normalizer_type="none",
        selected_training_mode=None, use_history_action=False, use_proprioception=True, action_mask_ratio=0.5,
        different_history_freq=False, predict_wrist_img=True, predict_proprioception=True)
    hash_init_(pol.vae_model, "vae.")
    hash_init_(pol.model, "mar.")
    return pol.to(DEV)


def _obs(B, T, tag):
    o = {"image": (torch.from_numpy(hash_tensor(f"{tag}/img", (B, T, 3, 96, 96))) + 1.0) * 0.5,
         "wrist_image": (torch.from_numpy(hash_tensor(f"{tag}/wrist", (B, T, 3, 96, 96))) + 1.0) * 0.5}
    for k, n in (("robot0_eef_pos", 3), ("robot0_eef_quat", 4), ("robot0_gripper_qpos", 2)):
        o[k] = torch.from_numpy(hash_tensor(f"{tag}/{k}", (B, T, n)))
    return {k: v.to(DEV) for k, v in o.items()}


def test_toolhang_second_camera_policy_compute_loss_and_predict():
    from unified_video_action_amd.runtime import RT
    RT.set_precision("bf16")
    pol = _toolhang_policy().train()
    B = 2
    batch = {"obs": _obs(B, 32, "th"), "action": torch.from_numpy(hash_tensor("th/action", (B, 32, 10))).to(DEV)}
    for p in pol.model.parameters():
        p.grad = torch.zeros_like(p)
    loss, (lv, la) = pol.compute_loss(batch, rng={"task_mode": "full_dynamic_model"})
    assert torch.isfinite(loss) and float(lv) > 0 and float(la) > 0
    loss.backward()
    m = pol.model
    for p in (m.proprioception_image_proj_cond.weight, m.proprioception_proj_cond.weight, m.z_proj_wrist.weight,
              m.diffloss_wrist.net.input_proj.weight, m.diffproploss.net.input_proj.weight):
        assert torch.isfinite(p.grad).all() and p.grad.abs().sum() > 0
    pol.eval()
    out = pol.predict_action(_obs(B, 16, "th_eval"))
    assert out["action_pred"].shape == (B, 16, 10) and torch.isfinite(out["action_pred"]).all()
