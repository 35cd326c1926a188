"""MAR video+action transformer on the HIP path (reference:
model/autoregressive/mar_con_unified.py:28-943; size presets :1162-1234).

Same constructor surface and parameter names (timm Block names norm1/attn.qkv/attn.proj/
norm2/mlp.fc1/mlp.fc2) as the reference, so `model.policy.autoregressive_model_params.*`
configs and checkpoints carry over.  Training forward only (the sampler is §8f "next").

Token layout: latents arrive either in the reference layout [B, T, C, H, W] or already
patchified as tokens [B, T, 256, C] (the VAE path writes tokens directly); token index
t*256 + h*16 + w, channels last.  Every random draw can be injected through `rng`
(orders, mask_rate, text_drop_u, randint/randn_like queues) for bit-exact token indexing
against the reference; otherwise they are drawn like the reference (numpy shuffle,
scipy truncnorm, torch RNG).
"""
from functools import partial

import math

import numpy as np
import scipy.stats as stats
import torch
import torch.nn as nn

from ...runtime import RT, cdt
from .diffusion_action_loss import DiffActLoss
from .diffusion_loss import DiffLoss
from .functional import F32, block_forward, layer_norm, linear


class Attention(nn.Module):
    def __init__(self, dim, num_heads, qkv_bias=True):
        super().__init__()
        assert dim % num_heads == 0
        self.num_heads = num_heads
        self.qkv = nn.Linear(dim, 3 * dim, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)


class Block(nn.Module):
    """timm 0.9.7 Block (pre-LN); forward = functional.BlockFn (one fused autograd node)."""

    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=True, norm_layer=nn.LayerNorm, proj_drop=0.0,
                 attn_drop=0.0):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = Attention(dim, num_heads, qkv_bias)
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))
        self.attn_drop = attn_drop
        self.proj_drop = proj_drop

    def forward(self, x):
        B, N, _ = x.shape
        pa = self.attn_drop if self.training else 0.0
        pp = self.proj_drop if self.training else 0.0
        return block_forward(self, x, B, N, pa, pp)


class MAR(nn.Module):
    def __init__(self, img_size=256, vae_stride=16, patch_size=1, encoder_embed_dim=1024, encoder_depth=16,
                 encoder_num_heads=16, decoder_embed_dim=1024, decoder_depth=16, decoder_num_heads=16,
                 mlp_ratio=4.0, norm_layer=nn.LayerNorm, vae_embed_dim=16, mask_ratio_min=0.7, label_drop_prob=0.1,
                 attn_dropout=0.1, proj_dropout=0.1, diffloss_d=3, diffloss_w=1024, diffloss_act_d=3,
                 diffloss_act_w=1024, num_sampling_steps="100", diffusion_batch_mul=4, grad_checkpointing=False,
                 predict_video=True, act_diff_training_steps=1000, act_diff_testing_steps="100",
                 action_model_params={}, **kwargs):
        super().__init__()
        self.task_name = kwargs["task_name"]
        self.different_history_freq = kwargs.get("different_history_freq") or False
        self.use_history_action = kwargs.get("use_history_action") or False
        self.use_proprioception = kwargs.get("use_proprioception") or False
        self.predict_wrist_img = kwargs.get("predict_wrist_img") or False
        self.predict_proprioception = kwargs.get("predict_proprioception") or False
        self.umi = self.task_name == "umi"
        if self.predict_wrist_img and self.umi:
            # the reference's wrist branch reads proprioception_image_cond, which its UMI branch never
            # builds (mar_con_unified.py:579-587): unrunnable there too
            raise NotImplementedError("predict_wrist_img with the UMI proprioception streams")
        self.n_frames = 4
        self.seq_h = self.seq_w = img_size // vae_stride // patch_size
        self.seq_len = self.seq_h * self.seq_w
        self.token_embed_dim = vae_embed_dim * patch_size ** 2
        self.vae_embed_dim = vae_embed_dim
        self.label_drop_prob = label_drop_prob
        self.attn_dropout, self.proj_dropout = attn_dropout, proj_dropout
        self.mask_ratio_generator = stats.truncnorm((mask_ratio_min - 1.0) / 0.25, 0, loc=1.0, scale=0.25)
        D, Dd = encoder_embed_dim, decoder_embed_dim
        self.z_proj_cond = nn.Linear(self.token_embed_dim, D)
        self.z_proj = nn.Linear(self.token_embed_dim, D)
        self.predict_action = action_model_params["predict_action"]
        act_dim = kwargs["shape_meta"]["action"]["shape"][0]
        self.action_proj_cond = nn.Linear(act_dim, D)
        self.buffer_size_action = 64
        self.fake_latent_x = nn.Parameter(torch.zeros(1, D))
        self.fake_action_latent = nn.Parameter(torch.zeros(1, D))
        n_streams = 3
        if self.predict_wrist_img:  # (:97-114, 465-498): the wrist camera's latents as one more stream
            self.z_proj_wrist = nn.Linear(self.token_embed_dim, D)
            self.fake_latent_wrist_x = nn.Parameter(torch.zeros(1, D))
            n_streams += 1
        if self.use_history_action:  # (:115-124, 504-522): one more conditioning stream
            self.action_mask_ratio = kwargs["action_mask_ratio"]
            self.fake_latent_history_action = nn.Parameter(torch.zeros(1, D))
            self.history_action_proj_cond = nn.Linear(act_dim, D)
            n_streams += 1
        if self.use_proprioception:
            if not self.umi and ("pusht" in self.task_name or "block_push" in self.task_name):
                # the reference builds a 2-d state projection there but its encoder reads the
                # second camera and the robot0_* states (:545-566): unrunnable in the reference
                raise NotImplementedError("use_proprioception for pusht / block_push")
            self.buffer_size_properception = 64 * 4 if self.different_history_freq else 64
            # (:126-147) UMI: 16-d state stream; toolhang & co: the second camera's latents + 9-d state
            self.proprioception_proj_cond = nn.Linear(16 if self.umi else 9, D)
            self.proprioception_image_proj_cond = nn.Linear(self.token_embed_dim, D)
            n_streams += 1 if self.umi else 2
        self.language_emb_model = kwargs.get("language_emb_model")
        self.clip = self.language_emb_model == "clip"
        if self.clip:
            self.fake_latent = nn.Parameter(torch.zeros(1, D))
            self.text_proj_cond = nn.Linear(512, D)
            self.buffer_size_text = 64
            self.text_pos_embed = nn.Parameter(torch.zeros(1, self.buffer_size_text, D))
        self.proj_cond_x_layer = nn.Linear(n_streams * D, D)
        self.temporal_pos_embed = nn.Parameter(torch.zeros(1, self.n_frames, D))
        self.spatial_pos_embed = nn.Parameter(torch.zeros(1, self.seq_len, D))
        self.z_proj_ln = nn.LayerNorm(D, eps=1e-6)
        blk = partial(Block, mlp_ratio=mlp_ratio, qkv_bias=True, norm_layer=norm_layer, proj_drop=proj_dropout,
                      attn_drop=attn_dropout)
        self.encoder_blocks = nn.ModuleList([blk(D, encoder_num_heads) for _ in range(encoder_depth)])
        self.encoder_norm = norm_layer(D)
        self.decoder_embed = nn.Linear(D, Dd)
        self.decoder_temporal_pos_embed = nn.Parameter(torch.zeros(1, self.n_frames, Dd))
        self.decoder_spatial_pos_embed = nn.Parameter(torch.zeros(1, self.seq_len, Dd))
        if self.clip:
            self.decoder_text_pos_embed = nn.Parameter(torch.zeros(1, self.buffer_size_text, Dd))
        self.decoder_blocks = nn.ModuleList([blk(Dd, decoder_num_heads) for _ in range(decoder_depth)])
        self.decoder_norm = norm_layer(Dd)
        self.diffusion_temporal_embed = nn.Parameter(torch.zeros(1, self.n_frames, Dd))
        self.diffusion_spatial_embed = nn.Parameter(torch.zeros(1, self.seq_len, Dd))
        self.initialize_weights()
        self.predict_video = predict_video
        if predict_video:
            self.diffloss = DiffLoss(self.token_embed_dim, Dd, diffloss_d, diffloss_w, num_sampling_steps,
                                     grad_checkpointing, n_frames=self.n_frames)
            if self.predict_wrist_img:  # (:281-294)
                self.diffloss_wrist = DiffLoss(self.token_embed_dim, Dd, diffloss_d, diffloss_w, num_sampling_steps,
                                               grad_checkpointing, n_frames=self.n_frames)
        if self.predict_action:
            self.diffactloss = DiffActLoss(act_dim, Dd, diffloss_act_d, diffloss_act_w, num_sampling_steps,
                                           grad_checkpointing, n_frames=self.n_frames,
                                           act_model_type=action_model_params.get("act_model_type", "conv_fc"),
                                           act_diff_training_steps=act_diff_training_steps)
        if self.predict_proprioception:
            # (:313-344) UMI: 6-d rotation targets; toolhang: eef pos + quat + gripper (9-d)
            if not (self.umi or self.task_name == "toolhang"):
                raise NotImplementedError(f"predict_proprioception for task {self.task_name}")
            self.diffproploss = DiffActLoss(6 if self.umi else 9, Dd, diffloss_act_d, diffloss_act_w,
                                            num_sampling_steps, grad_checkpointing, n_frames=self.n_frames,
                                            act_model_type=action_model_params.get("act_model_type", "conv_fc"),
                                            act_diff_training_steps=act_diff_training_steps)

    # ---- init (mar_con_unified.py:349-391) ----------------------------------------------
    def initialize_weights(self):
        for p in (self.fake_latent_x, self.fake_action_latent, self.temporal_pos_embed, self.spatial_pos_embed,
                  self.decoder_temporal_pos_embed, self.decoder_spatial_pos_embed, self.diffusion_temporal_embed,
                  self.diffusion_spatial_embed):
            nn.init.normal_(p, std=0.02)
        if self.clip:
            for p in (self.fake_latent, self.text_pos_embed, self.decoder_text_pos_embed):
                nn.init.normal_(p, std=0.02)
        if self.use_history_action:
            nn.init.normal_(self.fake_latent_history_action, std=0.02)
        if self.predict_wrist_img:
            nn.init.normal_(self.fake_latent_wrist_x, std=0.02)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.LayerNorm) and m.weight is not None:
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    # ---- token bookkeeping (bit-exact index semantics of :393-443) ------------------------
    @staticmethod
    def to_tokens(z):
        """[B,T,C,H,W] -> [B,T,H*W,C]  or pass-through [B,T,S,C]."""
        if z.dim() == 5:
            B, T, C, H, W = z.shape
            return z.permute(0, 1, 3, 4, 2).reshape(B, T, H * W, C)
        return z

    def sample_orders(self, bsz):
        orders = []
        for _ in range(bsz):
            order = np.arange(self.seq_len)
            np.random.shuffle(order)
            orders.append(order)
        return np.stack(orders)

    def token_mask(self, orders, mask_rate, device):
        """[B, T*S] float mask: 1 for the first ceil(S*rate) tokens of each order, every frame."""
        B = orders.shape[0]
        n = int(np.ceil(self.seq_len * mask_rate))
        sm = np.zeros((B, self.seq_len), np.float32)
        np.put_along_axis(sm, np.asarray(orders)[:, :n], 1.0, axis=1)
        m = np.repeat(sm[:, None, :], self.n_frames, axis=1).reshape(B, -1)
        return torch.from_numpy(m).to(device)

    def _pos(self, temporal, spatial):
        return (temporal[:, :, None, :] + spatial[:, None, :, :]).reshape(1, -1, temporal.shape[-1])

    # ---- encoder (:445-659) -------------------------------------------------------------
    def forward_mae_encoder(self, x, mask, cond, text_latents, nactions, task_mode, prop, text_drop_u,
                            history_nactions=None, hist_u=None):
        B, T, S, _ = x.shape
        D = self.fake_latent_x.shape[1]
        c = cdt()
        fake = self.fake_latent_x.to(c)
        wrist = None
        if self.predict_wrist_img:
            fw = self.fake_latent_wrist_x.to(c)
        if task_mode == "policy_model":
            cond_e = linear(cond, self.z_proj_cond, out_dtype=c).reshape(B, T * S, D)
            x_e = fake.expand(B, T * S, D)
            if self.predict_wrist_img:
                wrist = fw.expand(B, T * S, D)
        elif task_mode == "inverse_model":
            x_e = linear(x, self.z_proj, out_dtype=c).reshape(B, T * S, D)
            cond_e = fake.expand(B, T * S, D)
            if self.predict_wrist_img:
                wrist = linear(prop["pred_second_image_z"], self.z_proj_wrist, out_dtype=c).reshape(B, T * S, D)
        else:
            cond_e = linear(cond, self.z_proj_cond, out_dtype=c).reshape(B, T * S, D)
            x_e = linear(x, self.z_proj, out_dtype=c).reshape(B, T * S, D)
            x_e = torch.where(mask[..., None] == 1, fake.expand(B, T * S, D), x_e)
            if self.predict_wrist_img:
                wrist = linear(prop["pred_second_image_z"], self.z_proj_wrist, out_dtype=c).reshape(B, T * S, D)
                wrist = torch.where(mask[..., None] == 1, fw.expand(B, T * S, D), wrist)
        if task_mode == "dynamic_model":
            act = linear(nactions, self.action_proj_cond, out_dtype=c)
        else:
            act = self.fake_action_latent.to(c)[None].expand(B, 16, D)
        # stream order of :579-603: x (, wrist), cond (, history), action (, proprioception)
        streams = [x_e] + ([wrist] if wrist is not None else []) + [cond_e]
        if self.use_history_action:
            # history actions [B, T*4, Da] -> latents, training drops each to the fake latent with
            # probability 1 - action_mask_ratio (torch.rand(B, T*4) > ratio, :512-518)
            fh = self.fake_latent_history_action.to(c)
            if history_nactions is None:
                ha = fh[None].expand(B, T * self.n_frames, D)
            else:
                ha = linear(history_nactions.float(), self.history_action_proj_cond, out_dtype=c)
                if self.training:
                    u = hist_u if hist_u is not None else torch.rand(B, T * self.n_frames)
                    drop = (torch.as_tensor(u).to(ha.device) > self.action_mask_ratio)[..., None]
                    ha = torch.where(drop, fh[None].expand_as(ha), ha)
            streams.append(ha.repeat_interleave(self.buffer_size_action, dim=1))
        streams.append(act.repeat_interleave(self.buffer_size_action, dim=1))
        if self.use_proprioception:
            if self.umi:
                ps = torch.cat([prop["robot0_eef_pos"], prop["robot0_eef_rot_axis_angle"], prop["robot0_gripper_width"],
                                prop["robot0_eef_rot_axis_angle_wrt_start"]], dim=-1).float()
            else:  # (:545-566): the second camera's latents, then eef pos + quat + gripper
                pi = linear(prop["second_image_z"], self.proprioception_image_proj_cond, out_dtype=c)
                streams.append(pi.reshape(B, -1, D))
                ps = torch.cat([prop["robot0_eef_pos"], prop["robot0_eef_quat"], prop["robot0_gripper_qpos"]],
                               dim=-1).float()
            pe = linear(ps, self.proprioception_proj_cond, out_dtype=c)
            streams.append(pe.repeat_interleave(self.buffer_size_properception, dim=1))
        h = linear(torch.cat(streams, dim=-1), self.proj_cond_x_layer, out_dtype=F32)
        h = h + self._pos(self.temporal_pos_embed, self.spatial_pos_embed)
        if self.clip:
            txt = text_latents[:, None, :].expand(B, self.buffer_size_text, D)
            if self.training:
                drop = (text_drop_u < self.label_drop_prob).to(F32).to(h.device)[:, None, None]
                txt = drop * self.fake_latent[:, None, :] + (1 - drop) * txt
            h = torch.cat([txt + self.text_pos_embed, h], dim=1)
        h = layer_norm(h, self.z_proj_ln, out_dtype=F32)
        for blk in self.encoder_blocks:
            h = blk(h)
        return layer_norm(h, self.encoder_norm, out_dtype=c)

    # ---- decoder (:661-726) -------------------------------------------------------------
    def forward_mae_decoder(self, x):
        h = linear(x, self.decoder_embed, out_dtype=F32)
        pos = self._pos(self.decoder_temporal_pos_embed, self.decoder_spatial_pos_embed)
        if self.clip:
            pos = torch.cat([self.decoder_text_pos_embed, pos], dim=1)
        h = h + pos
        for blk in self.decoder_blocks:
            h = blk(h)
        h = layer_norm(h, self.decoder_norm, out_dtype=F32)
        if self.clip:
            h = h[:, self.buffer_size_text:]
        return h + self._pos(self.diffusion_temporal_embed, self.diffusion_spatial_embed)

    # ---- losses (:728-787) --------------------------------------------------------------
    def forward_loss(self, z, target, mask, nactions, task_mode, prop, draws, gt_wrist=None):
        zero = torch.zeros((), device=z.device)
        video_loss = act_loss = zero

        def nxt():
            t = draws["randint"].pop(0) if draws["randint"] else None
            nz = draws["randn_like"].pop(0) if draws["randn_like"] else None
            return t, nz

        if task_mode in ("video_model", "dynamic_model", "full_dynamic_model"):
            t, nz = nxt()
            video_loss = self.diffloss(target, z, mask, t=t, noise=nz)
            if self.predict_wrist_img:  # (:738-776) the wrist video loss is part of the video loss
                t, nz = nxt()
                video_loss = video_loss + self.diffloss_wrist(gt_wrist, z, mask, t=t, noise=nz)
        if task_mode in ("policy_model", "inverse_model", "full_dynamic_model"):
            t, nz = nxt()
            act_loss = self.diffactloss(nactions, z, task_mode, t=t, noise=nz)
        if task_mode == "full_dynamic_model":
            loss = video_loss + act_loss
        elif task_mode in ("video_model", "dynamic_model"):
            loss = video_loss
        else:
            loss = act_loss
        if self.predict_proprioception:
            t, nz = nxt()
            if self.umi:
                gt_prop = prop["robot0_eef_rot_axis_angle_wrt_start_pred"]
            else:  # toolhang (:891-897)
                gt_prop = torch.cat([prop["robot0_eef_pos_pred"], prop["robot0_eef_quat_pred"],
                                     prop["robot0_gripper_qpos_pred"]], dim=-1)
            loss = loss + self.diffproploss(gt_prop, z, t=t, noise=nz)
        return loss, video_loss, act_loss

    def forward(self, imgs, cond, history_nactions=None, nactions=None, text_latents=None, task_mode=None,
                proprioception_input={}, rng=None):
        RT.begin_forward()
        dev = cond.device
        x = self.to_tokens(imgs).to(F32)
        cnd = self.to_tokens(cond).to(F32)
        B = x.shape[0]
        if text_latents is not None and self.clip:
            text_latents = linear(text_latents.to(dev).float(), self.text_proj_cond, out_dtype=F32)
        gt = x.reshape(B, -1, x.shape[-1])
        rng = rng or {}
        orders = rng["orders"] if "orders" in rng else self.sample_orders(B)
        rate = rng["mask_rate"] if "mask_rate" in rng else self.mask_ratio_generator.rvs(1)[0]
        mask = self.token_mask(orders, rate, dev)
        tdu = rng.get("text_drop_u")
        tdu = torch.as_tensor(tdu) if tdu is not None else torch.rand(B)
        draws = {"randint": [torch.as_tensor(a).to(dev) for a in rng.get("randint", [])],
                 "randn_like": [torch.as_tensor(a).to(dev) for a in rng.get("randn_like", [])]}
        prop = self._prop_tokens(proprioception_input)
        h = self.forward_mae_encoder(x, mask, cnd, text_latents, nactions, task_mode, prop, tdu,
                                     history_nactions, rng.get("hist_u"))
        z = self.forward_mae_decoder(h)
        gt_wrist = prop["pred_second_image_z"].reshape(B, -1, x.shape[-1]) if self.predict_wrist_img else None
        return self.forward_loss(z, gt, mask, nactions, task_mode, prop, draws, gt_wrist)

    def _prop_tokens(self, prop):
        """second-camera latents [B, T, C, H, W] (or token-major [B, T, S, C]) -> fp32 tokens (:816-845)"""
        prop = dict(prop)
        for k in ("second_image_z", "pred_second_image_z"):
            if k in prop and prop[k] is not None:
                prop[k] = self.to_tokens(prop[k]).to(F32)
        return prop


    # ---- inference (:945-1151) ----------------------------------------------------------
    @torch.no_grad()
    def sample_tokens(self, bsz, cond, text_latents=None, num_iter=64, cfg=1.0, cfg_schedule="linear",
                      temperature=1.0, progress=False, history_nactions=None, nactions=None,
                      proprioception_input={}, task_mode=None, vae_model=None, x=None, rng=None):
        """policy_model / inverse_model: one encoder+decoder pass over the fully masked (policy) or
        fully visible (inverse) grid, then the action head's reverse diffusion (act_cfg = 1.0)
        -> (None, actions [B, 16, Da]) -- the reference returns on the first iteration (:1040-1041).
        Video modes (video_model, dynamic_model, full_dynamic_model): the MaskGIT loop (:1043-1115)
        -- each iteration re-encodes the grid, samples the action head (when present), picks the
        tokens to predict from the cosine mask schedule over the generation order, and samples
        them with the video diffusion head -> (latents [(B*4), C, 16, 16], actions or None).
        `rng` injects {"orders", and per iteration i: "act_noise"/"act_step_noise"[i],
        "video_noise"/"video_step_noise"[i]} (or "noise"/"step_noise" for the action-only modes)."""
        if cfg != 1.0:
            raise NotImplementedError("classifier-free guidance (forward_with_cfg) is not on the built path")
        rng = rng or {}
        dev = cond.device
        cnd = self.to_tokens(cond).to(F32)
        B = cnd.shape[0]
        T, L = self.n_frames, self.seq_len
        if text_latents is not None and self.clip:
            text_latents = linear(text_latents.to(dev).float(), self.text_proj_cond, out_dtype=F32)
        proprioception_input = self._prop_tokens(proprioception_input)
        wrist = self.predict_wrist_img and task_mode != "inverse_model"
        if wrist:
            # (:1003-1006) the wrist stream starts from zero latents; the video modes sample it every
            # iteration with diffloss_wrist on the rows the video head samples (:1118-1140)
            proprioception_input["pred_second_image_z"] = torch.zeros(B, T, L, self.token_embed_dim, device=dev)
        if task_mode == "inverse_model":
            tokens = self.to_tokens(x).to(F32)
            mask = np.zeros((B, L), np.float32)
        else:
            tokens = torch.zeros(B, T, L, self.token_embed_dim, device=dev)
            mask = np.ones((B, L), np.float32)
        orders = np.asarray(rng["orders"]) if "orders" in rng else self.sample_orders(bsz)
        act_modes = ("policy_model", "inverse_model")
        if task_mode not in act_modes + ("video_model", "dynamic_model", "full_dynamic_model"):
            raise NotImplementedError(f"sample_tokens task_mode={task_mode}")
        if task_mode in act_modes and not self.predict_action:
            raise NotImplementedError("sample_tokens without an action head returns nothing on this path")
        if task_mode != "policy_model" and task_mode != "inverse_model" and not self.predict_video:
            raise NotImplementedError("video sampling without predict_video")

        def pick(key, i):
            v = rng.get(key)
            return None if v is None else v[i]

        act = None
        for step in range(num_iter if task_mode not in act_modes else 1):
            m_full = torch.from_numpy(np.repeat(mask[:, None, :], T, axis=1).reshape(B, T * L)).to(dev)
            h = self.forward_mae_encoder(tokens, m_full, cnd, text_latents, nactions, task_mode,
                                         proprioception_input, torch.ones(B), history_nactions)
            z = self.forward_mae_decoder(h)
            if self.predict_action:
                if task_mode in act_modes:
                    an, asn = rng.get("noise"), rng.get("step_noise")
                else:
                    an, asn = pick("act_noise", step), pick("act_step_noise", step)
                act = self.diffactloss.sample(z, temperature, cfg=1.0, text_latents=text_latents, noise=an,
                                              step_noise=asn)
            if task_mode in act_modes:
                return None, act
            # mask schedule (:1049-1086), bit-exact on the host: float32 as the reference's tensors
            ratio = np.cos(math.pi / 2.0 * (step + 1) / num_iter)
            mask_len = np.float32(np.floor(L * ratio))
            mask_len = max(np.float32(1.0), min(np.float32(mask[0].sum() - 1), mask_len))
            nxt = np.zeros((B, L), np.float32)
            np.put_along_axis(nxt, orders[:, :int(mask_len)], 1.0, axis=1)
            cur = mask.astype(bool)
            to_pred = cur if step >= num_iter - 1 else np.logical_xor(cur, nxt.astype(bool))
            mask = nxt
            sel = torch.from_numpy(np.repeat(to_pred[:, None, :], T, axis=1).reshape(-1).nonzero()[0]).to(dev)
            zr = z.reshape(B * T * L, -1).index_select(0, sel)
            lat = self.diffloss.sample(zr, temperature, 1.0, text_latents=text_latents,
                                       noise=pick("video_noise", step), step_noise=pick("video_step_noise", step))
            flat = tokens.reshape(B * T * L, -1).clone()
            flat.index_copy_(0, sel, lat.to(flat.dtype))
            tokens = flat.reshape(B, T, L, -1)
            if wrist:  # (:1118-1140) the wrist head on the same decoder rows, after the video head
                wlat = self.diffloss_wrist.sample(zr, temperature, 1.0, text_latents=text_latents,
                                                  noise=pick("wrist_noise", step),
                                                  step_noise=pick("wrist_step_noise", step))
                wflat = proprioception_input["pred_second_image_z"].reshape(B * T * L, -1).clone()
                wflat.index_copy_(0, sel, wlat.to(wflat.dtype))
                proprioception_input["pred_second_image_z"] = wflat.reshape(B, T, L, -1)
        # unpatchify (patch_size 1): [(b t), s, c] -> [(b t), c, h, w]; with the wrist stream the
        # reference returns the wrist tokens in place of the main ones (:1143-1157)
        res = proprioception_input["pred_second_image_z"] if wrist else tokens
        out = res.reshape(B * T, self.seq_h, self.seq_w, -1).permute(0, 3, 1, 2).contiguous()
        return out, act


def _mar(D, depth, heads, **kwargs):
    return MAR(encoder_embed_dim=D, encoder_depth=depth, encoder_num_heads=heads, decoder_embed_dim=D,
               decoder_depth=depth, decoder_num_heads=heads, mlp_ratio=4,
               norm_layer=partial(nn.LayerNorm, eps=1e-6), **kwargs)


def mar_tiny(**kw):
    return _mar(768, 3, 6, **kw)


def mar_small(**kw):
    return _mar(768, 6, 6, **kw)


def mar_base(**kw):
    return _mar(768, 12, 12, **kw)


def mar_large(**kw):
    return _mar(1024, 16, 16, **kw)


def mar_huge(**kw):
    return _mar(1280, 20, 16, **kw)
