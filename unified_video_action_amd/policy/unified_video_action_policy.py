"""Drop-in policy for `model.policy._target_` (reference:
policy/unified_video_action_policy.py:33-428).

Same constructor kwargs (vae_model_params, autoregressive_model_params, action_model_params,
shape_meta, n_action_steps, shift_action, language_emb_model, task_name, task_modes,
**kwargs incl. normalizer_type, selected_training_mode, use_proprioception, ...) and the
same training surface: forward(batch) -> (loss, (video_loss, action_loss)),
compute_loss, get_optimizer(weight_decay, learning_rate, betas), set_normalizer,
add_weight_decay.  The step runs on libuva_hip.so end to end (frame select+resize,
VAE encoder, MAR, diffusion heads, backward).  Inference: predict_action(obs_dict) ->
{"action", "action_pred"} on the same kernels plus the HIP-graph reverse-diffusion sampler
(policy:221-320).

Differences that do not change results: frames are selected before the bilinear resize
(per-frame op), and the "loss += 0*p.sum()" DDP workaround (policy:421-423) is replaced
by the zero-initialised flat gradient buffer that the DP reducer all-reduces whole.

Data parallel under the reference's launcher (`accelerate launch`, workspace:208-220): the
fused backward writes parameter gradients straight into the optimizer's flat buffer, which
DDP's autograd hooks never see.  The policy therefore lists every parameter in
`_ddp_params_and_buffers_to_ignore` (DDP skips them: no broadcast hooks, no reducer buckets)
except one zero-valued `ddp_anchor` scalar that DDP reduces instead (it enters the loss as
0 * anchor, and is dropped from state dicts), and the optimizer's own RCCL bucket reducer
(workspace/optim.GradReducer, created on the first forward after the process group exists)
all-reduces the flat gradients from inside backward.
"""
import os
import random
import weakref

import numpy as np
import torch
import torch.nn as nn

from ..model.autoregressive import mar_con_unified as mar
from ..model.common.normalizer import LinearNormalizer
from ..utils.data_utils import (get_trajectory, image_key, select_frame_indices, umi_proprioception,
                                vae_images)
from ..runtime import RT
from ..vae.vaekl import AutoencoderKL

ALL_TASK_MODES = ["video_model", "dynamic_model", "policy_model", "inverse_model", "full_dynamic_model"]


def _get(cfg, key, default=None):
    if cfg is None:
        return default
    if isinstance(cfg, dict):
        return cfg.get(key, default)
    return getattr(cfg, key, default)


def _plain(cfg):
    if isinstance(cfg, dict):
        return {k: _plain(v) for k, v in cfg.items()}
    if hasattr(cfg, "items"):
        return {k: _plain(v) for k, v in cfg.items()}
    return cfg


def _drop_anchor(module, state_dict, prefix, local_metadata):
    state_dict.pop(prefix + "ddp_anchor", None)
    return state_dict


def _add_anchor(module, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys, error_msgs):
    state_dict.setdefault(prefix + "ddp_anchor", torch.zeros((), device=module.ddp_anchor.device))


def _after_load(module, incompatible_keys):
    """loaded weights went into the flat fp32 buffer in place: refresh its bf16 compute shadow."""
    opt = module.bound_optimizer()
    if opt is not None:
        opt.store.refresh_shadow()
    from ..runtime import RT
    RT.bump_params()


def _ddp_active():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


class UnifiedVideoActionPolicy(nn.Module):
    def __init__(self, vae_model_params, autoregressive_model_params, action_model_params, shape_meta,
                 n_action_steps, shift_action=True, language_emb_model=None, task_name=None, task_modes=[],
                 **kwargs):
        super().__init__()
        self.task_name = task_name or ""
        self.task_modes = list(task_modes or [])
        self.autoregressive_model_params = autoregressive_model_params
        self.n_action_steps = n_action_steps
        self.shift_action = shift_action
        self.language_emb_model = language_emb_model
        shape_meta = _plain(shape_meta)
        self.action_dim = shape_meta["action"]["shape"][0]
        self.kwargs = kwargs
        self.normalizer_type = kwargs.get("normalizer_type", "all")
        self.selected_training_mode = kwargs.get("selected_training_mode")
        self.use_history_action = kwargs.get("use_history_action") or False
        self.use_proprioception = kwargs.get("use_proprioception") or False
        self.different_history_freq = kwargs.get("different_history_freq") or False

        self.vae_model = AutoencoderKL(**_plain(vae_model_params))
        self.vae_model.eval()
        for p in self.vae_model.parameters():
            p.requires_grad = False

        ap = autoregressive_model_params
        self.sample_params = dict(num_iter=_get(ap, "num_iter", 1), cfg=_get(ap, "cfg", 1.0),
                                  cfg_schedule=_get(ap, "cfg_schedule", "linear"),
                                  temperature=_get(ap, "temperature", 0.95))
        self.model = getattr(mar, _get(ap, "model_size", "mar_base"))(
            img_size=_get(ap, "img_size", 256), vae_stride=_get(ap, "vae_stride", 16),
            patch_size=_get(ap, "patch_size", 1), vae_embed_dim=_get(ap, "vae_embed_dim", 16),
            mask_ratio_min=_get(ap, "mask_ratio_min", 0.7), label_drop_prob=_get(ap, "label_drop_prob", 0.1),
            attn_dropout=_get(ap, "attn_dropout", 0.1), proj_dropout=_get(ap, "proj_dropout", 0.1),
            diffloss_d=_get(ap, "diffloss_d", 6), diffloss_w=_get(ap, "diffloss_w", 1024),
            diffloss_act_d=_get(ap, "diffloss_act_d", 6), diffloss_act_w=_get(ap, "diffloss_act_w", 1024),
            num_sampling_steps=_get(ap, "num_sampling_steps", "100"),
            diffusion_batch_mul=_get(ap, "diffusion_batch_mul", 1),
            grad_checkpointing=_get(ap, "grad_checkpointing", False), predict_video=_get(ap, "predict_video", True),
            act_diff_training_steps=_get(ap, "act_diff_training_steps", 1000),
            act_diff_testing_steps=_get(ap, "act_diff_testing_steps", "100"),
            action_model_params=_plain(action_model_params), use_history_action=self.use_history_action,
            action_mask_ratio=kwargs.get("action_mask_ratio", 0.5), use_proprioception=self.use_proprioception,
            predict_wrist_img=kwargs.get("predict_wrist_img") or False,
            different_history_freq=self.different_history_freq,
            predict_proprioception=kwargs.get("predict_proprioception") or False, task_name=self.task_name,
            language_emb_model=language_emb_model, shape_meta=shape_meta)
        self.normalizer = LinearNormalizer()
        # DDP anchor (see module docstring); not part of state dicts
        self.ddp_anchor = nn.Parameter(torch.zeros(()))
        self._register_state_dict_hook(_drop_anchor)
        self._register_load_state_dict_pre_hook(_add_anchor, with_module=True)
        self.register_load_state_dict_post_hook(_after_load)
        self._uva_opt = None
        # warm start (policy:112-118): a MAR checkpoint's model_ema or a UVA .ckpt's ema_model
        self.pretrained_model_path = _get(ap, "pretrained_model_path", None)
        if self.pretrained_model_path is not None:
            if os.path.exists(self.pretrained_model_path):
                self.load_pretrained_model()
            else:
                print("pretrained model not found: ", self.pretrained_model_path)
        if self.selected_training_mode is None:
            if len(self.task_modes) == 0:
                self.task_modes = list(ALL_TASK_MODES)
        elif self.selected_training_mode == "policy_model_full_dynamics_model":
            self.task_modes = ["policy_model", "full_dynamic_model"]
        else:
            self.task_modes = [self.selected_training_mode]

    @property
    def device(self):
        return next(self.model.parameters()).device

    # ---- training surface ------------------------------------------------------------------
    def set_normalizer(self, normalizer):
        self.normalizer.load_state_dict(normalizer.state_dict())

    def add_weight_decay(self, model, weight_decay=1e-5, skip_list=()):
        decay, no_decay = [], []
        for name, p in model.named_parameters():
            if not p.requires_grad:
                continue
            (no_decay if (p.ndim == 1 or name.endswith(".bias") or name in skip_list) else decay).append(p)
        return [{"params": no_decay, "weight_decay": 0.0}, {"params": decay, "weight_decay": weight_decay}]

    def get_optimizer(self, weight_decay, learning_rate, betas):
        """policy:343-360: AdamW over (no-decay, decay) groups of self.model, initial_lr set --
        as the flat-buffer FusedAdamWEMA (a torch.optim.Optimizer)."""
        from ..workspace.optim import FusedAdamWEMA
        groups = self.add_weight_decay(self.model, weight_decay=weight_decay)
        opt = FusedAdamWEMA(groups, lr=learning_rate, betas=tuple(betas), named=list(self.model.named_parameters()),
                            prefix="model.")
        for g in opt.param_groups:
            g.setdefault("initial_lr", g["lr"])
        self._uva_opt = (weakref.ref(opt), id(self))  # a deepcopy (the EMA policy) does not inherit it
        return opt

    def bound_optimizer(self):
        """the flat-buffer optimizer built by this policy's get_optimizer (None otherwise)."""
        if self._uva_opt is None or self._uva_opt[1] != id(self):
            return None
        return self._uva_opt[0]()

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        opt = self.bound_optimizer()
        if opt is not None:
            opt._sync()  # .to(device) replaced the parameter tensors: re-bind the flat buffers
        return out

    @property
    def _ddp_params_and_buffers_to_ignore(self):
        return [n for n, _ in self.named_parameters() if n != "ddp_anchor"] + [n for n, _ in self.named_buffers()]

    def load_pretrained_model(self):
        """policy:140-218: name- and shape-filtered load into self.model from a UVA checkpoint's
        state_dicts.ema_model ("model." prefix stripped) or a MAR checkpoint's model_ema.  Read with
        the checkpoint module's safe loader (no code executes from the file)."""
        from ..workspace.checkpoint import safe_load
        ck = safe_load(self.pretrained_model_path)
        if "state_dicts" in ck:
            if "ema_model" not in ck["state_dicts"]:
                raise NotImplementedError("UVA checkpoint without state_dicts.ema_model")
            src = {k[6:]: v for k, v in ck["state_dicts"]["ema_model"].items() if k.startswith("model.")}
        elif "model_ema" in ck:
            src = ck["model_ema"]
        else:
            raise NotImplementedError("pretrained checkpoint has neither state_dicts.ema_model nor model_ema")
        sd = self.model.state_dict()
        take = {k: v for k, v in src.items() if k in sd and sd[k].size() == v.size()}
        skipped = [k for k, v in sd.items() if k not in src or src[k].size() != v.size()]
        if not sd or not take:
            raise ValueError(f"pretrained checkpoint {self.pretrained_model_path}: no matching parameters")
        sd.update(take)
        missing, unexpected = self.model.load_state_dict(sd, strict=False)
        _after_load(self, None)
        self.pretrained_report = {"loaded": sorted(take), "kept_init": skipped, "missing": list(missing),
                                  "unexpected": list(unexpected)}
        return self.pretrained_report

    def _normalize(self, key, x):
        if self.normalizer_type == "all" and key in self.normalizer:
            return self.normalizer[key].normalize(x)
        return x

    def compute_loss(self, batch, rng=None):
        """batch: {"obs": {<image key>: [B,T,3,H,W] in [0,1] (any H), low-dim keys...},
        "action": [B,T,Da], optional "language_latents": [B,512]}.  `rng` injects the step's
        random draws (cases.py semantics) for parity runs."""
        rng = rng or {}
        obs = batch["obs"]
        img = obs.get("image", obs.get(image_key(self.task_name)))
        B, T = img.shape[:2]
        dev = img.device
        text_latents = None
        if self.language_emb_model == "clip":
            if "language_latents" not in batch:
                raise NotImplementedError("CLIP text encoding needs network weights; pass language_latents")
            text_latents = batch["language_latents"]
        nactions = self._normalize("action", batch["action"].float())
        if self.normalizer_type == "all":  # normalize_obs: every non-image key (policy:389-393)
            obs = dict(obs)
            for k in list(obs):
                if "image" not in k and k in self.normalizer:
                    obs[k] = self.normalizer[k].normalize(obs[k])
        T_traj = T
        if self.use_history_action:
            # (policy:395-396) every observation drops its first step; the trajectory split keeps the
            # loaded horizon T (get_trajectory: history = nactions[:, 1:] first half)
            obs = {k: (v[:, 1:] if torch.is_tensor(v) and v.dim() >= 2 else v) for k, v in obs.items()}
            img = obs.get("image", obs.get(image_key(self.task_name)))
            T = img.shape[1]
        opt = self.bound_optimizer()
        if opt is not None and self.training:
            red = opt.maybe_init_reducer(self.model)
            if red is not None:
                red.arm()
        indices, prop = None, {}
        if "umi" in self.task_name:
            sel = np.arange(T)
            if "img_indices" in obs:
                indices = obs["img_indices"].int().squeeze(2)
            T = T * 4  # 8 loaded frames stand for a 32-step horizon (data_utils.py:215-219)
            if self.use_proprioception:
                prop = umi_proprioception(obs, indices, self.different_history_freq)
        else:
            sel = select_frame_indices(T, different_history_freq=self.different_history_freq,
                                       rng_choice=rng.get("history_combination"))
            if self.use_proprioception:
                prop = self._second_camera_prop(obs, sel, train=True, eps=rng.get("vae_eps_wrist"))
        if self.training and dev.type == "cuda":
            if getattr(self, "_wt_params", None) is None:
                from ..model.autoregressive.mar_con_unified import Block
                self._wt_params = [w for m in self.model.modules() if isinstance(m, Block)
                                   for w in (m.attn.qkv.weight, m.attn.proj.weight, m.mlp.fc1.weight, m.mlp.fc2.weight)]
            RT._weight_t_params = self._wt_params  # their transposed bf16 copies are built on the side stream too
            RT.arm_attn_prefetch(dev)  # attention dropout planes under the VAE encode (side stream)
        x = vae_images(img, sel, self.vae_model.CIN_PAD)
        n_half = B * (len(sel) // 2)
        eps = rng.get("vae_eps_x")
        if eps is not None:
            eps = torch.cat([torch.as_tensor(rng["vae_eps_x"]), torch.as_tensor(rng["vae_eps_c"])]).to(dev)
        else:
            eps = torch.randn(2 * n_half, self.vae_model.embed_dim, 16, 16, device=dev)
        tokens = self.vae_model.encode_tokens(x, eps)
        RT.fire_attn_prefetch()  # (an encode that did not fire it)
        z = tokens[:n_half].reshape(B, -1, 256, tokens.shape[-1])
        c = tokens[n_half:].reshape(B, -1, 256, tokens.shape[-1])
        history, trajectory = get_trajectory(nactions, T_traj, self.shift_action, self.use_history_action)
        mode = rng.get("task_mode") or random.choice(self.task_modes)
        loss, video_loss, act_loss = self.model(z, c, history if self.use_history_action else None, trajectory,
                                                text_latents, task_mode=mode, proprioception_input=prop, rng=rng)
        if torch.is_grad_enabled() and _ddp_active():
            loss = loss + 0.0 * self.ddp_anchor  # the one parameter DDP reduces (see module docstring)
        return loss, (video_loss, act_loss)

    def forward(self, batch, **kwargs):
        return self.compute_loss(batch, **kwargs)

    def _second_camera_prop(self, obs, sel, train, eps=None):
        """process_data's second-camera branch (toolhang, data_utils.py:228-285) + get_vae_latent's
        second-image encodes (:395-410): the wrist frames at the selected indices through the KL-VAE
        (history half -> second_image_z, future half -> pred_second_image_z when training), the
        eef pos / quat / gripper states split into history / future halves (train) or whole (eval)."""
        wk = "wrist_image" if "wrist_image" in obs else "robot0_eye_in_hand_image"
        wrist = obs[wk]
        B = wrist.shape[0]
        h = len(sel) // 2
        xw = vae_images(wrist, sel, self.vae_model.CIN_PAD)  # [future half | history half]
        # eps: the wrist posterior draws [future half | history half] (rng key 'vae_eps_wrist', as vae_eps_x / _c)
        if eps is None:
            eps = torch.randn(xw.shape[0], self.vae_model.embed_dim, 16, 16, device=wrist.device)
        else:
            eps = torch.as_tensor(eps).to(wrist.device)
            assert tuple(eps.shape) == (xw.shape[0], self.vae_model.embed_dim, 16, 16), eps.shape
        tok = self.vae_model.encode_tokens(xw, eps).reshape(2, B, h, 256, -1)
        prop = {}
        keys = ("robot0_eef_pos", "robot0_eef_quat", "robot0_gripper_qpos")
        if train:
            prop["second_image_z"], prop["pred_second_image_z"] = tok[1], tok[0]
            for k in keys:
                prop[k], prop[k + "_pred"] = torch.chunk(obs[k].float(), 2, dim=1)
                if self.different_history_freq:
                    prop[k] = prop[k][:, torch.as_tensor(np.asarray(sel[:h]), device=wrist.device)]
        else:
            prop["second_image_z"] = torch.cat([tok[1], tok[0]], dim=1)  # all selected frames, in order
            for k in keys:
                v = obs[k].float()
                prop[k] = v[:, torch.as_tensor(np.asarray(sel), device=wrist.device)] if self.different_history_freq else v
        return prop

    _EVAL_IMAGE_KEYS = (("libero", "agentview_image"), ("toolhang", "sideview_image"), ("umi", "camera0_rgb"))

    @torch.no_grad()
    def predict_action(self, obs_dict, language_goal=None, rng=None):
        """obs_dict: {"image" (or the task's camera key): [B,T,3,H,W] in [0,1], low-dim keys}
        -> {"action": [B, n_action_steps, Da], "action_pred": [B, 16, Da]}  (policy:221-320).
        language_goal: precomputed text latents [B, 512] (CLIP needs network weights).
        rng injects {"vae_eps": [B*4,16,16,16] (posterior.sample, reference (b t) order),
        "noise", "step_noise"} for parity runs."""
        rng = rng or {}
        obs = dict(obs_dict)
        history = None
        if self.use_history_action and "past_action" in obs:  # normalize_past_action (policy:256-264)
            history = self._normalize("action", obs.pop("past_action").float())
        for task, key in self._EVAL_IMAGE_KEYS:  # resize_image_eval key mapping (data_utils.py:86-104)
            if task in self.task_name and key in obs:
                obs["image"] = obs.pop(key)
        img = obs["image"]
        B, T = img.shape[:2]
        dev = img.device
        text_latents = None
        if self.language_emb_model == "clip":
            if not torch.is_tensor(language_goal):
                raise NotImplementedError("CLIP text encoding needs network weights; pass text latents [B, 512]")
            text_latents = language_goal.to(dev).float()
        if self.normalizer_type == "all":  # normalize_obs: every non-image key (data_utils.py:185-203)
            for k in list(obs):
                if "image" not in k and k in self.normalizer:
                    obs[k] = self.normalizer[k].normalize(obs[k])
        prop = {}
        if "umi" in self.task_name:
            sel = np.arange(T)
            if self.use_proprioception:
                idx = obs["img_indices"].int().squeeze(2) if "img_indices" in obs else None
                prop = umi_proprioception(obs, idx, self.different_history_freq, train=False)
        else:
            sel = select_frame_indices(T, eval=True)
            if self.use_proprioception:
                prop = self._second_camera_prop(obs, sel, train=False)
        if len(sel) % 2:
            raise ValueError(f"eval frame selection {sel.tolist()} must hold an even number of frames")
        x = vae_images(img, sel, self.vae_model.CIN_PAD)  # [sel[h:] per sample | sel[:h] per sample]
        h = len(sel) // 2
        eps = rng.get("vae_eps")
        if eps is not None:
            e = torch.as_tensor(eps).to(dev).reshape(B, 2, h, *eps.shape[1:])
            eps = torch.cat([e[:, 1].reshape(B * h, *eps.shape[1:]), e[:, 0].reshape(B * h, *eps.shape[1:])])
        else:
            eps = torch.randn(B * len(sel), self.vae_model.embed_dim, 16, 16, device=dev)
        tok = self.vae_model.encode_tokens(x, eps).reshape(2, B, h, 256, -1)
        c = torch.cat([tok[1], tok[0]], dim=1)  # [B, len(sel), 256, 16] in selection order
        sp = self.sample_params
        _, act = self.model.sample_tokens(bsz=B, cond=c, text_latents=text_latents, num_iter=sp["num_iter"],
                                          cfg=sp["cfg"], cfg_schedule=sp["cfg_schedule"],
                                          temperature=sp["temperature"], proprioception_input=prop,
                                          history_nactions=history, task_mode="policy_model",
                                          vae_model=self.vae_model, rng=rng)
        action_pred = act[..., :self.action_dim]
        if self.normalizer_type == "all":
            action_pred = self.normalizer["action"].unnormalize(action_pred)
        return {"action": action_pred[:, :self.n_action_steps], "action_pred": action_pred}
