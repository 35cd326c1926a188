"""use_history_action end to end through UnifiedVideoActionPolicy (no shipped config selects it:
uva.yaml use_history_action null).  The MAR's history-action stream itself is pinned against the
reference's run by the pusht_hist cases of test_parity_gpu.py (cases.EXTRA_VARIANTS, fp32 1e-4 /
grads 3e-3 and bf16); here the policy plumbing: every observation drops its first step
(policy:395-396), the trajectory splits nactions[:, 1:] into history / future halves
(data_utils.get_trajectory), the history reaches the encoder (its projection receives gradient), and
predict_action takes obs["past_action"] (normalize_past_action, policy:256-264)."""
import pytest
import torch

import cases
import replay
from hashinit import hash_init_, hash_tensor

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _history_policy():
    from unified_video_action_amd.model.common.normalizer import LinearNormalizer
    from unified_video_action_amd.policy.unified_video_action_policy import UnifiedVideoActionPolicy
    replay.golden_policy(normalizer=False)  # registers model_size "mar_golden"
    amp = dict(pretrained_model_path=None, model_size="mar_golden")
    for k in cases.POLICY_AMP_KEYS:
        amp[k] = cases.MAR_KW[k]
    pol = UnifiedVideoActionPolicy(
        vae_model_params=dict(autoencoder_path=None, ddconfig=dict(vae_embed_dim=16, ch_mult=[1, 1, 2, 2, 4])),
        autoregressive_model_params=amp,
        action_model_params=dict(predict_action=True, act_model_type="conv_fc"),
        shape_meta={"action": {"shape": [2]}}, n_action_steps=8, shift_action=False, language_emb_model=None,
        task_name="pusht", task_modes=["full_dynamic_model"], normalizer_type="all", selected_training_mode=None,
        use_history_action=True, use_proprioception=False, action_mask_ratio=0.5, different_history_freq=False,
        predict_wrist_img=False, predict_proprioception=False)
    hash_init_(pol.vae_model, "vae.")
    hash_init_(pol.model, "mar.")
    norm = LinearNormalizer()
    lim = torch.zeros(2, 2)
    lim[1] = 512.0
    norm.fit({"action": lim, "agent_pos": lim})
    pol.set_normalizer(norm)
    return pol.to(DEV)


def test_history_action_policy_compute_loss_and_predict():
    from unified_video_action_amd.runtime import RT
    RT.set_precision("bf16")
    pol = _history_policy().train()
    B, T = 2, 33  # the history-action loader's horizon: one step more than the 32 of the plain one
    img = (torch.from_numpy(hash_tensor("hist/image", (B, T, 3, 96, 96))) + 1.0) * 0.5
    pos = (torch.from_numpy(hash_tensor("hist/pos", (B, T, 2))) + 1.0) * 256.0
    act = (torch.from_numpy(hash_tensor("hist/action", (B, T, 2))) + 1.0) * 256.0
    batch = {"obs": {"image": img.to(DEV), "agent_pos": pos.to(DEV)}, "action": act.to(DEV)}
    for p in pol.model.parameters():
        p.grad = torch.zeros_like(p)
    loss, (lv, la) = pol.compute_loss(batch, rng={"task_mode": "full_dynamic_model"})
    assert torch.isfinite(loss) and float(la) > 0 and float(lv) > 0
    loss.backward()
    gw = pol.model.history_action_proj_cond.weight.grad
    assert gw is not None and torch.isfinite(gw).all() and gw.abs().sum() > 0
    pol.eval()
    g = torch.Generator().manual_seed(5)
    rng = {"vae_eps": torch.randn(B * 4, 16, 16, 16, generator=g), "noise": torch.randn(B * 16, 2, generator=g).to(DEV),
           "step_noise": torch.randn(100, B * 16, 2, generator=g).to(DEV)}
    obs = {"image": img[:, 1:].to(DEV), "agent_pos": pos[:, 1:].to(DEV)}
    out = pol.predict_action(dict(obs, past_action=act[:, :16].to(DEV)), rng=rng)
    assert out["action_pred"].shape == (B, 16, 2) and torch.isfinite(out["action_pred"]).all()
    # without past actions the encoder takes the fake history latent: same draws, other actions
    out2 = pol.predict_action(dict(obs), rng=rng)
    assert out2["action_pred"].shape == (B, 16, 2) and torch.isfinite(out2["action_pred"]).all()
    assert (out["action_pred"] - out2["action_pred"]).abs().max() > 0
    out3 = pol.predict_action(dict(obs, past_action=act[:, :16].to(DEV)), rng=rng)
    assert torch.equal(out3["action_pred"], out["action_pred"])  # the history path is deterministic
