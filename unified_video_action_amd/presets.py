"""Policy constructor kwargs of the BASELINE.json configs, mirroring the reference YAML
(config/model/uva.yaml:3-62, config/uva_pusht.yaml, config/task/{pusht,libero10,umi_multi}.yaml)
plus synthetic device-resident batches of the same shapes."""
import copy

import torch

MODEL_UVA = dict(
    selected_training_mode=None, n_action_steps=8, use_proprioception=False, use_history_action=False,
    action_mask_ratio=0.5, different_history_freq=False, predict_wrist_img=False, predict_proprioception=False,
    vae_model_params=dict(autoencoder_path=None, ddconfig=dict(vae_embed_dim=16, ch_mult=[1, 1, 2, 2, 4])),
    autoregressive_model_params=dict(
        pretrained_model_path=None, model_size="mar_base", img_size=256, vae_stride=16, patch_size=1,
        vae_embed_dim=16, mask_ratio_min=0.7, label_drop_prob=0.1, attn_dropout=0.1, proj_dropout=0.1,
        diffloss_d=6, diffloss_w=1024, diffloss_act_d=6, diffloss_act_w=1024, num_sampling_steps="100",
        diffusion_batch_mul=1, grad_checkpointing=False, num_iter=1, cfg=1, cfg_schedule="linear",
        temperature=0.95, predict_video=True, act_diff_training_steps=1000, act_diff_testing_steps="100"),
    action_model_params=dict(predict_action=False, act_model_type="conv_fc"),
    shift_action=True,
    optimizer=dict(learning_rate=1e-4, weight_decay=0.02, betas=[0.9, 0.95]),
)

TASKS = {
    "pusht": dict(name="pusht", task_modes=[], action_dim=2, image=(32, 96), normalizer_type="all",
                  language_emb_model=None),
    "libero10": dict(name="libero_10", task_modes=[], action_dim=10, image=(32, 128), normalizer_type="all",
                     language_emb_model="clip"),
    "umi_multi": dict(name="umi", task_modes=["policy_model", "full_dynamic_model"], action_dim=10,
                      image=(8, 224), normalizer_type="none", language_emb_model="clip"),
}

# BASELINE.json configs -> (task, overrides)
CONFIGS = {
    "pusht_video": ("pusht", dict(selected_training_mode="video_model")),
    "pusht_joint": ("pusht", dict(action_model_params=dict(predict_action=True, act_model_type="conv_fc"))),
    "libero10_joint": ("libero10", dict(action_model_params=dict(predict_action=True, act_model_type="conv_fc"))),
    "umi_multi": ("umi_multi", dict(action_model_params=dict(predict_action=True, act_model_type="conv_fc"),
                                    use_proprioception=True, predict_proprioception=True,
                                    different_history_freq=True, shift_action=False)),
}


def policy_kwargs(config, **over):
    task, ov = CONFIGS[config]
    t = TASKS[task]
    kw = copy.deepcopy(MODEL_UVA)
    for k, v in ov.items():
        kw[k] = copy.deepcopy(v)
    for k, v in over.items():
        if isinstance(v, dict) and isinstance(kw.get(k), dict):
            kw[k].update(v)
        else:
            kw[k] = v
    kw.pop("optimizer")
    kw.update(task_name=t["name"], task_modes=t["task_modes"], normalizer_type=t["normalizer_type"],
              language_emb_model=t["language_emb_model"], shape_meta={"action": {"shape": [t["action_dim"]]}})
    return kw


def synthetic_batch(config, B, device, seed=0):
    """U[0,1] frames at the dataset resolution, U[0,512] agent_pos/actions (PushT) or N(0,1)
    proprio (UMI), language latents ~0.1 N(0,1)."""
    task, _ = CONFIGS[config]
    t = TASKS[task]
    T, H = t["image"]
    g = torch.Generator(device="cpu").manual_seed(seed)
    obs = {}
    key = {"pusht": "image", "libero10": "agentview_rgb", "umi_multi": "camera0_rgb"}[task]
    obs[key] = torch.rand(B, T, 3, H, H, generator=g)
    batch = {"obs": obs}
    if task == "pusht":
        obs["agent_pos"] = torch.rand(B, 32, 2, generator=g) * 512
        batch["action"] = torch.rand(B, 32, 2, generator=g) * 512
    elif task == "libero10":
        batch["action"] = torch.rand(B, 32, 10, generator=g) * 2 - 1
        batch["language_latents"] = torch.randn(B, 512, generator=g) * 0.1
    else:
        for k, d in (("robot0_eef_pos", 3), ("robot0_eef_rot_axis_angle", 6), ("robot0_gripper_width", 1),
                     ("robot0_eef_rot_axis_angle_wrt_start", 6)):
            obs[k] = torch.randn(B, 32, d, generator=g)
        hist = torch.stack([torch.sort(torch.randperm(16, generator=g)[:4]).values for _ in range(B)])
        idx = torch.cat([hist, torch.tensor([19, 23, 27, 31]).expand(B, 4)], dim=1)
        obs["img_indices"] = idx[..., None].float()
        batch["action"] = torch.randn(B, 32, 10, generator=g)
        batch["language_latents"] = torch.randn(B, 512, generator=g) * 0.1

    def mv(x):
        return {k: mv(v) for k, v in x.items()} if isinstance(x, dict) else x.to(device)

    return mv(batch)


def fit_normalizer(config, policy):
    from .model.common.normalizer import LinearNormalizer
    task, _ = CONFIGS[config]
    t = TASKS[task]
    n = LinearNormalizer()
    if t["normalizer_type"] == "all":
        lim = torch.zeros(2, t["action_dim"])
        if task == "pusht":
            lim[1] = 512.0
            n.fit({"action": lim, "agent_pos": lim[:, :2].clone()})
        else:
            lim[0], lim[1] = -1.0, 1.0
            n.fit({"action": lim})
    policy.set_normalizer(n)
    return n
