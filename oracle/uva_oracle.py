"""ORACLE -- test infrastructure, never shipped, never on the product path.

PyTorch-CPU fp32 restatement of the reference UVA training step (SURVEY §8a rows
a1-a14).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import it.  It is pinned against the golden fixtures in tests/golden/, which
were produced by running the reference itself (tests/golden/make_golden.py), so
parity of the HIP path is transitively parity with the reference.

Parameter names follow the reference (timm Block names, MAR/DiffLoss/VAE
attribute names) so that hash-initialised weights and checkpoints line up.
Every random draw of the step is taken from an explicit `rng` dict (see
tests/golden/cases.py) instead of global generators.

The MAR restatement also covers the variants no shipped config turns on (use_history_action,
the toolhang second camera + 9-d state streams and proprioception head, predict_wrist_img),
pinned by the reference-run goldens of cases.EXTRA_VARIANTS (test_oracle_golden.py).
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

LN_EPS = 1e-6
LATENT_SCALE = 0.2325  # data_utils.py:396


# --------------------------------------------------------------------------------------
# Gaussian diffusion tables (gaussian_diffusion.py:102-202, respace.py:65-90)
# --------------------------------------------------------------------------------------
class DiffusionTables:
    """float64 tables of the cosine schedule, spaced over all T steps like SpacedDiffusion."""

    def __init__(self, T=1000, use_timesteps=None):
        abar = lambda s: math.cos((s + 0.008) / 1.008 * math.pi / 2) ** 2
        b0 = np.array([min(1 - abar((i + 1) / T) / abar(i / T), 0.999) for i in range(T)])
        ac0 = np.cumprod(1.0 - b0)
        # respacing (respace.py:65-90): betas re-derived from consecutive retained alpha-bars
        keep = set(range(T)) if use_timesteps is None else set(use_timesteps)
        prev, nb, tmap = 1.0, [], []
        for i, a in enumerate(ac0):
            if i in keep:
                nb.append(1.0 - a / prev)
                prev = a
                tmap.append(i)
        self.timestep_map = np.array(tmap, np.int64)
        T = len(nb)
        betas = np.array(nb, dtype=np.float64)
        ac = np.cumprod(1.0 - betas)
        ac_prev = np.concatenate([[1.0], ac[:-1]])
        pvar = betas * (1.0 - ac_prev) / (1.0 - ac)
        self.T = T
        self.betas = betas
        self.log_betas = np.log(betas)
        self.alphas_cumprod = ac
        self.sqrt_ac = np.sqrt(ac)
        self.sqrt_1mac = np.sqrt(1.0 - ac)
        self.sqrt_recip_ac = np.sqrt(1.0 / ac)
        self.sqrt_recipm1_ac = np.sqrt(1.0 / ac - 1.0)
        self.plvc = np.log(np.concatenate([[pvar[1]], pvar[1:]]))
        self.coef1 = betas * np.sqrt(ac_prev) / (1.0 - ac)
        self.coef2 = (1.0 - ac_prev) * np.sqrt(1.0 - betas) / (1.0 - ac)

    def gather(self, name, t):
        """float64 table lookup then cast to fp32 (gaussian_diffusion.py:892-904)."""
        return torch.from_numpy(getattr(self, name))[t].float()[:, None]


def space_timesteps(num_timesteps, section_counts):
    """respace.py:14-56 for comma-separated section counts (e.g. "100")."""
    counts = [int(x) for x in str(section_counts).split(",")]
    size_per, extra = num_timesteps // len(counts), num_timesteps % len(counts)
    start, steps = 0, set()
    for i, n in enumerate(counts):
        size = size_per + (1 if i < extra else 0)
        stride = 1 if n <= 1 else (size - 1) / (n - 1)
        cur = 0.0
        for _ in range(n):
            steps.add(start + round(cur))
            cur += stride
        start += size
    return steps


def p_sample_loop(tb, model_fn, noise, step_noise, temperature=1.0, clip=True):
    """gaussian_diffusion.py:260-346 (p_mean_variance, learned-range variance, eps model,
    clip_denoised) + :395-492 (p_sample / p_sample_loop_progressive); the wrapped model gets
    the base timestep (respace.py:118-130).  step_noise[k] is the k-th randn_like draw."""
    x = noise
    C = x.shape[1]
    for k, i in enumerate(reversed(range(tb.T))):
        t = torch.full((x.shape[0],), i, dtype=torch.long)
        out = model_fn(x, torch.from_numpy(tb.timestep_map)[t])
        eps, v = out[:, :C], out[:, C:]
        frac = (v + 1) / 2
        log_var = frac * tb.gather("log_betas", t) + (1 - frac) * tb.gather("plvc", t)
        x0 = tb.gather("sqrt_recip_ac", t) * x - tb.gather("sqrt_recipm1_ac", t) * eps
        if clip:
            x0 = x0.clamp(-1, 1)
        mean = tb.gather("coef1", t) * x0 + tb.gather("coef2", t) * x
        nonzero = (t != 0).float()[:, None]
        x = mean + nonzero * torch.exp(0.5 * log_var) * step_noise[k] * temperature
    return x


def _approx_cdf(x):
    return 0.5 * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x.pow(3))))


def diffusion_training_loss(tables, model_fn, x0, t, noise):
    """Per-row loss = eps-MSE + VB(learned range) -- gaussian_diffusion.py:746-818."""
    x_t = tables.gather("sqrt_ac", t) * x0 + tables.gather("sqrt_1mac", t) * noise
    out = model_fn(x_t, t)
    C = x0.shape[1]
    eps, v = out[:, :C], out[:, C:]
    eps_d = eps.detach()
    # posterior q(x_{t-1}|x_t,x_0)
    c1, c2 = tables.gather("coef1", t), tables.gather("coef2", t)
    true_mean = c1 * x0 + c2 * x_t
    true_lv = tables.gather("plvc", t)
    # model p(x_{t-1}|x_t) with frozen eps
    frac = (v + 1) / 2
    model_lv = frac * tables.gather("log_betas", t) + (1 - frac) * tables.gather("plvc", t)
    x0_hat = tables.gather("sqrt_recip_ac", t) * x_t - tables.gather("sqrt_recipm1_ac", t) * eps_d
    model_mean = c1 * x0_hat + c2 * x_t
    kl = 0.5 * (-1.0 + model_lv - true_lv + torch.exp(true_lv - model_lv)
                + (true_mean - model_mean) ** 2 * torch.exp(-model_lv))
    kl = kl.mean(dim=1) / math.log(2.0)
    # discretized gaussian NLL at t == 0 (diffusion_utils.py:47-73)
    inv_std = torch.exp(-0.5 * model_lv)
    cen = x0 - model_mean
    cdf_p = _approx_cdf(inv_std * (cen + 1.0 / 255.0))
    cdf_m = _approx_cdf(inv_std * (cen - 1.0 / 255.0))
    lp = torch.where(x0 < -0.999, torch.log(cdf_p.clamp(min=1e-12)),
                     torch.where(x0 > 0.999, torch.log((1.0 - cdf_m).clamp(min=1e-12)),
                                 torch.log((cdf_p - cdf_m).clamp(min=1e-12))))
    nll = -lp.mean(dim=1) / math.log(2.0)
    vb = torch.where(t == 0, nll, kl)
    mse = ((noise - eps) ** 2).mean(dim=1)
    return mse + vb, mse, vb


# --------------------------------------------------------------------------------------
# Transformer block (timm 0.9.7 Block as used by mar_con_unified.py:201-249)
# --------------------------------------------------------------------------------------
class _Attn(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.heads = heads
        self.qkv = nn.Linear(dim, 3 * dim)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x, p_drop=0.0):
        B, N, D = x.shape
        hd = D // self.heads
        q, k, v = self.qkv(x).view(B, N, 3, self.heads, hd).permute(2, 0, 3, 1, 4)
        s = (q @ k.transpose(-1, -2)) * (hd ** -0.5)
        a = s.softmax(dim=-1)
        if p_drop > 0:
            a = F.dropout(a, p_drop)
        o = (a @ v).transpose(1, 2).reshape(B, N, D)
        return self.proj(o)


class _Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x)))


class Block(nn.Module):
    def __init__(self, dim, heads, mlp_ratio=4.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=LN_EPS)
        self.attn = _Attn(dim, heads)
        self.norm2 = nn.LayerNorm(dim, eps=LN_EPS)
        self.mlp = _Mlp(dim, int(dim * mlp_ratio))
        self.p_drop = 0.0  # attn_dropout = proj_dropout (uva.yaml:31-32); 0 for parity runs

    def forward(self, x):
        p = self.p_drop if self.training else 0.0
        x = x + F.dropout(self.attn(self.norm1(x), p), p, self.training)
        h = F.dropout(F.gelu(self.mlp.fc1(self.norm2(x))), p, self.training)
        return x + F.dropout(self.mlp.fc2(h), p, self.training)


def set_dropout(model, p):
    """configure the 4 timm Block dropouts (only for CPU-baseline timing; parity uses 0)."""
    for m in model.modules():
        if isinstance(m, Block):
            m.p_drop = p


# --------------------------------------------------------------------------------------
# Diffusion MLP head (diffusion_loss.py:97-283)
# --------------------------------------------------------------------------------------
def timestep_features(t, dim=256, max_period=10000):
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / half)
    a = t[:, None].float() * freqs[None]
    return torch.cat([torch.cos(a), torch.sin(a)], dim=-1)


class _TimeEmbed(nn.Module):
    def __init__(self, width):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(256, width), nn.SiLU(), nn.Linear(width, width))

    def forward(self, t):
        return self.mlp(timestep_features(t))


class _ResBlock(nn.Module):
    def __init__(self, w):
        super().__init__()
        self.in_ln = nn.LayerNorm(w, eps=LN_EPS)
        self.mlp = nn.Sequential(nn.Linear(w, w), nn.SiLU(), nn.Linear(w, w))
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(w, 3 * w))

    def forward(self, x, y):
        shift, scale, gate = self.adaLN_modulation(y).chunk(3, dim=-1)
        return x + gate * self.mlp(self.in_ln(x) * (1 + scale) + shift)


class _Final(nn.Module):
    def __init__(self, w, out):
        super().__init__()
        self.linear = nn.Linear(w, out)
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(w, 2 * w))

    def forward(self, x, y):
        shift, scale = self.adaLN_modulation(y).chunk(2, dim=-1)
        h = F.layer_norm(x, x.shape[-1:], eps=LN_EPS)
        return self.linear(h * (1 + scale) + shift)


class SimpleMLPAdaLN(nn.Module):
    def __init__(self, in_ch, width, out_ch, z_ch, depth):
        super().__init__()
        self.time_embed = _TimeEmbed(width)
        self.cond_embed = nn.Linear(z_ch, width)
        self.input_proj = nn.Linear(in_ch, width)
        self.res_blocks = nn.ModuleList([_ResBlock(width) for _ in range(depth)])
        self.final_layer = _Final(width, out_ch)

    def forward(self, x, t, c):
        h = self.input_proj(x)
        y = self.time_embed(t) + self.cond_embed(c)
        for blk in self.res_blocks:
            h = blk(h, y)
        return self.final_layer(h, y)


class DiffLoss(nn.Module):
    """Video diffusion loss (diffusion_loss.py:8-66)."""

    def __init__(self, target_ch, z_ch, width, depth):
        super().__init__()
        self.net = SimpleMLPAdaLN(target_ch, width, 2 * target_ch, z_ch, depth)
        self.tables = DiffusionTables(1000)

    def forward(self, target, z, mask, t, noise):
        rows = target.shape[0] * target.shape[1]
        tgt = target.reshape(rows, -1)
        c = z.reshape(rows, -1)
        m = mask.reshape(rows)
        loss, _, _ = diffusion_training_loss(self.tables, lambda xt, tt: self.net(xt, tt, c),
                                             tgt, t, noise)
        return (loss * m).sum() / m.sum()

    def sample(self, z, noise, step_noise, temperature=1.0, respacing="100"):
        """diffusion_loss.py:68-90 with cfg = 1.0, clip_denoised=False -> [R, C]."""
        tb = DiffusionTables(1000, space_timesteps(1000, respacing))
        return p_sample_loop(tb, lambda xt, tt: self.net(xt, tt, z), noise, step_noise, temperature, clip=False)


class DiffActLoss(nn.Module):
    """conv_fc action/proprio diffusion loss (diffusion_action_loss.py:35-61,109-166)."""

    def __init__(self, target_ch, z_ch, width, depth, T=1000):
        super().__init__()
        self.conv = nn.Sequential(nn.Conv2d(z_ch, z_ch, 3, padding=1), nn.ReLU(),
                                  nn.AdaptiveAvgPool2d((4, 4)))
        self.fc = nn.Sequential(nn.Linear(z_ch * 16, z_ch), nn.ReLU(), nn.Linear(z_ch, z_ch))
        self.interpolate = nn.Linear(4, 16)
        self.refine = nn.Sequential(nn.Linear(z_ch, z_ch), nn.ReLU(), nn.Linear(z_ch, z_ch))
        self.net = SimpleMLPAdaLN(target_ch, width, 2 * target_ch, z_ch, depth)
        self.tables = DiffusionTables(T)

    def trunk(self, z):
        B, N, D = z.shape
        f = z.reshape(B * 4, 16, 16, D).permute(0, 3, 1, 2)  # (b t) c w h, s = w*16 + h
        f = self.conv(f).reshape(B * 4, D * 16)
        f = self.fc(f).reshape(B, 4, D)
        f = self.interpolate(f.transpose(1, 2)).transpose(1, 2)  # B,16,D
        return self.refine(f)

    def forward(self, target, z, t, noise):
        B, S, _ = target.shape
        c = self.trunk(z).reshape(B * S, -1)
        loss, _, _ = diffusion_training_loss(self.tables, lambda xt, tt: self.net(xt, tt, c),
                                             target.reshape(B * S, -1), t, noise)
        return loss.reshape(B, S).mean()

    def sample(self, z, noise, step_noise, temperature=1.0, respacing="100"):
        """diffusion_action_loss.py:168-232 with cfg = 1.0 -> [B, 16, C]."""
        B = z.shape[0]
        c = self.trunk(z).reshape(B * 16, -1)
        tb = DiffusionTables(1000, space_timesteps(1000, respacing))
        x = p_sample_loop(tb, lambda xt, tt: self.net(xt, tt, c), noise, step_noise, temperature)
        return x.reshape(B, 16, -1)


# --------------------------------------------------------------------------------------
# MAR (mar_con_unified.py:28-943), training forward only
# --------------------------------------------------------------------------------------
class MAR(nn.Module):
    def __init__(self, encoder_embed_dim=768, encoder_depth=12, encoder_num_heads=12,
                 decoder_embed_dim=768, decoder_depth=12, decoder_num_heads=12, mlp_ratio=4,
                 vae_embed_dim=16, diffloss_d=6, diffloss_w=1024, diffloss_act_d=6,
                 diffloss_act_w=1024, task_name="pusht", act_dim=2, predict_action=True,
                 use_proprioception=False, predict_proprioception=False,
                 different_history_freq=False, language_emb_model=None, use_history_action=False,
                 predict_wrist_img=False, action_mask_ratio=0.5, **unused):
        super().__init__()
        D, Dd = encoder_embed_dim, decoder_embed_dim
        self.task_name = task_name
        self.umi = task_name == "umi"
        self.n_frames, self.seq_len, self.C = 4, 256, vae_embed_dim
        self.use_proprioception = use_proprioception
        self.predict_proprioception = predict_proprioception
        self.use_history_action = use_history_action
        self.predict_wrist_img = predict_wrist_img
        self.action_mask_ratio = action_mask_ratio
        self.clip = language_emb_model == "clip"
        self.z_proj_cond = nn.Linear(self.C, D)
        self.z_proj = nn.Linear(self.C, D)
        if predict_wrist_img:  # mar_con_unified.py:97-114
            self.z_proj_wrist = nn.Linear(self.C, D)
            self.fake_latent_wrist_x = nn.Parameter(torch.zeros(1, D))
        self.action_proj_cond = nn.Linear(act_dim, D)
        self.fake_latent_x = nn.Parameter(torch.zeros(1, D))
        self.fake_action_latent = nn.Parameter(torch.zeros(1, D))
        n_streams = 3 + int(predict_wrist_img)
        if use_history_action:  # :115-124
            self.fake_latent_history_action = nn.Parameter(torch.zeros(1, D))
            self.history_action_proj_cond = nn.Linear(act_dim, D)
            n_streams += 1
        if use_proprioception:  # :126-147 (umi: 16-d state; toolhang: second camera + 9-d state)
            self.prop_repeat = 256 if different_history_freq else 64
            self.proprioception_proj_cond = nn.Linear(16 if self.umi else 9, D)
            self.proprioception_image_proj_cond = nn.Linear(self.C, D)  # unused on UMI
            n_streams += 1 if self.umi else 2
        if self.clip:
            self.fake_latent = nn.Parameter(torch.zeros(1, D))
            self.text_proj_cond = nn.Linear(512, D)
            self.text_pos_embed = nn.Parameter(torch.zeros(1, 64, D))
        self.proj_cond_x_layer = nn.Linear(n_streams * D, D)
        self.temporal_pos_embed = nn.Parameter(torch.zeros(1, 4, D))
        self.spatial_pos_embed = nn.Parameter(torch.zeros(1, 256, D))
        self.z_proj_ln = nn.LayerNorm(D, eps=LN_EPS)
        self.encoder_blocks = nn.ModuleList([Block(D, encoder_num_heads, mlp_ratio)
                                             for _ in range(encoder_depth)])
        self.encoder_norm = nn.LayerNorm(D, eps=LN_EPS)
        self.decoder_embed = nn.Linear(D, Dd)
        self.decoder_temporal_pos_embed = nn.Parameter(torch.zeros(1, 4, Dd))
        self.decoder_spatial_pos_embed = nn.Parameter(torch.zeros(1, 256, Dd))
        if self.clip:
            self.decoder_text_pos_embed = nn.Parameter(torch.zeros(1, 64, Dd))
        self.decoder_blocks = nn.ModuleList([Block(Dd, decoder_num_heads, mlp_ratio)
                                             for _ in range(decoder_depth)])
        self.decoder_norm = nn.LayerNorm(Dd, eps=LN_EPS)
        self.diffusion_temporal_embed = nn.Parameter(torch.zeros(1, 4, Dd))
        self.diffusion_spatial_embed = nn.Parameter(torch.zeros(1, 256, Dd))
        self.diffloss = DiffLoss(self.C, Dd, diffloss_w, diffloss_d)
        if predict_wrist_img:  # :281-294
            self.diffloss_wrist = DiffLoss(self.C, Dd, diffloss_w, diffloss_d)
        self.predict_action = predict_action
        if predict_action:
            self.diffactloss = DiffActLoss(act_dim, Dd, diffloss_act_w, diffloss_act_d)
        if predict_proprioception:  # :313-344
            self.diffproploss = DiffActLoss(6 if self.umi else 9, Dd, diffloss_act_w, diffloss_act_d)

    @staticmethod
    def patchify(z):
        """[n, c, h, w] -> [n, h*w, c] (p=1; mar_con_unified.py:393-401)."""
        n, c, h, w = z.shape
        return z.permute(0, 2, 3, 1).reshape(n, h * w, c)

    @staticmethod
    def token_mask(orders, rate, T=4, L=256):
        """mask[b,t,s] = 1 for the first ceil(L*rate) tokens of orders[b] (:424-443)."""
        n = int(np.ceil(L * rate))
        m = torch.zeros(orders.shape[0], L)
        m.scatter_(1, orders[:, :n], 1.0)
        return m[:, None, :].expand(-1, T, -1)

    def _pos(self, temporal, spatial):
        return (temporal[:, :, None, :] + spatial[:, None, :, :]).reshape(1, -1, temporal.shape[-1])

    def encode(self, x, cond, mask, nactions, text, mode, prop, text_drop_u, hist=None, hist_u=None):
        B = x.shape[0]
        D = self.fake_latent_x.shape[1]
        m = mask.reshape(B, -1)
        wrist = None
        if mode == "policy_model":
            cond = self.z_proj_cond(cond).reshape(B, -1, D)
            x = self.fake_latent_x.expand(B, cond.shape[1], -1)
            if self.predict_wrist_img:
                wrist = self.fake_latent_wrist_x.expand(B, cond.shape[1], -1)
        elif mode == "inverse_model":
            x = self.z_proj(x).reshape(B, -1, D)
            cond = self.fake_latent_x.expand(B, x.shape[1], -1)
            if self.predict_wrist_img:
                wrist = self.z_proj_wrist(prop["pred_second_image_z"]).reshape(B, -1, D)
        else:
            cond = self.z_proj_cond(cond).reshape(B, -1, D)
            x = self.z_proj(x).reshape(B, -1, D)
            x = torch.where(m[..., None] == 1, self.fake_latent_x.expand_as(x), x)
            if self.predict_wrist_img:
                wrist = self.z_proj_wrist(prop["pred_second_image_z"]).reshape(B, -1, D)
                wrist = torch.where(m[..., None] == 1, self.fake_latent_wrist_x.expand_as(wrist), wrist)
        if mode == "dynamic_model":
            act = self.action_proj_cond(nactions)
        else:
            act = self.fake_action_latent[None].expand(B, 16, -1)
        # stream order :579-603: x (, wrist), cond (, history), action (, proprioception)
        streams = [x] + ([wrist] if wrist is not None else []) + [cond]
        if self.use_history_action:  # :504-522
            if hist is None:
                ha = self.fake_latent_history_action[None].expand(B, 16, -1)
            else:
                ha = self.history_action_proj_cond(hist)
                if self.training:
                    drop = (torch.as_tensor(hist_u) > self.action_mask_ratio)[..., None]
                    ha = torch.where(drop, self.fake_latent_history_action[None].expand_as(ha), ha)
            streams.append(ha.repeat_interleave(64, dim=1))
        streams.append(act.repeat_interleave(64, dim=1))
        if self.use_proprioception:
            if self.umi:
                ps = torch.cat([prop["robot0_eef_pos"], prop["robot0_eef_rot_axis_angle"],
                                prop["robot0_gripper_width"],
                                prop["robot0_eef_rot_axis_angle_wrt_start"]], dim=-1)
            else:  # :545-566
                streams.append(self.proprioception_image_proj_cond(prop["second_image_z"]).reshape(B, -1, D))
                ps = torch.cat([prop["robot0_eef_pos"], prop["robot0_eef_quat"], prop["robot0_gripper_qpos"]],
                               dim=-1)
            streams.append(self.proprioception_proj_cond(ps.float())
                           .repeat_interleave(self.prop_repeat, dim=1))
        h = self.proj_cond_x_layer(torch.cat(streams, dim=-1))
        h = h + self._pos(self.temporal_pos_embed, self.spatial_pos_embed)
        if self.clip:
            txt = text[:, None, :].expand(B, 64, -1)
            drop = (text_drop_u < 0.1).float()[:, None, None]
            txt = drop * self.fake_latent[:, None, :] + (1 - drop) * txt
            h = torch.cat([txt + self.text_pos_embed, h], dim=1)
        h = self.z_proj_ln(h)
        for blk in self.encoder_blocks:
            h = blk(h)
        return self.encoder_norm(h)

    def decode(self, h):
        h = self.decoder_embed(h)
        pos = self._pos(self.decoder_temporal_pos_embed, self.decoder_spatial_pos_embed)
        if self.clip:
            pos = torch.cat([self.decoder_text_pos_embed, pos], dim=1)
        h = h + pos
        for blk in self.decoder_blocks:
            h = blk(h)
        h = self.decoder_norm(h)
        if self.clip:
            h = h[:, 64:]
        return h + self._pos(self.diffusion_temporal_embed, self.diffusion_spatial_embed)

    @torch.no_grad()
    def sample_policy(self, c, text_latents, noise, step_noise, temperature=1.0, prop=None, mode="policy_model",
                      x=None):
        """sample_tokens, task_mode policy_model / inverse_model (mar_con_unified.py:945-1041): one
        pass over the fully masked (policy) or fully visible (inverse, tokens = x) grid, eval mode
        (no text drop), then the action head's sampler."""
        B = c.shape[0]
        cond = self.patchify(c.reshape(B * 4, *c.shape[2:])).reshape(B, 4, 256, -1)
        if mode == "inverse_model":
            x = self.patchify(x.reshape(B * 4, *x.shape[2:])).reshape(B, 4, 256, -1)
            mask = torch.zeros(B, 4 * 256)
        else:
            x = torch.zeros_like(cond)
            mask = torch.ones(B, 4 * 256)
        text = self.text_proj_cond(text_latents) if self.clip else None
        h = self.encode(x, cond, mask, None, text, mode, prop, torch.ones(B))
        return self.diffactloss.sample(self.decode(h), noise, step_noise, temperature)

    @torch.no_grad()
    def sample_video(self, c, text_latents, mode, num_iter, rng, temperature=1.0, nactions=None, prop=None):
        """sample_tokens video modes (mar_con_unified.py:1000-1151): MaskGIT loop with the cosine
        schedule over the generation orders (mask_by_order :17-25), action head sampled every
        iteration, video head on the tokens predicted in that iteration."""
        B = c.shape[0]
        cond = self.patchify(c.reshape(B * 4, *c.shape[2:])).reshape(B, 4, 256, -1)
        tokens = torch.zeros_like(cond)
        text = self.text_proj_cond(text_latents) if self.clip else None
        orders = torch.as_tensor(rng["orders"])
        mask = torch.ones(B, 4, 256)
        act = None
        for step in range(num_iter):
            h = self.encode(tokens, cond, mask.reshape(B, -1), nactions, text, mode, prop, torch.ones(B))
            z = self.decode(h)
            if hasattr(self, "diffactloss"):
                act = self.diffactloss.sample(z, torch.as_tensor(rng["act_noise"][step]),
                                              torch.as_tensor(rng["act_step_noise"][step]), temperature)
            ratio = np.cos(math.pi / 2.0 * (step + 1) / num_iter)
            mask_len = torch.Tensor([np.floor(256 * ratio)])
            mask_len = torch.maximum(torch.Tensor([1]), torch.minimum(mask[:, 0].sum(-1, keepdim=True) - 1, mask_len))
            nxt = torch.zeros(B, 256).scatter(-1, orders[:, :int(mask_len[0].item())], torch.ones(B, 256)).bool()
            nxt = nxt[:, None, :].expand(-1, 4, -1).reshape(B, -1)
            cur = mask.reshape(B, -1).bool()
            to_pred = cur if step >= num_iter - 1 else torch.logical_xor(cur, nxt)
            mask = nxt.reshape(B, 4, 256).float()
            idx = to_pred.nonzero(as_tuple=True)
            lat = self.diffloss.sample(z[idx], torch.as_tensor(rng["video_noise"][step]),
                                       torch.as_tensor(rng["video_step_noise"][step]), temperature)
            flat = tokens.reshape(B, 1024, -1).clone()
            flat[idx] = lat
            tokens = flat.reshape(B, 4, 256, -1)
        out = tokens.reshape(B * 4, 16, 16, -1).permute(0, 3, 1, 2)
        return out, act

    def forward(self, z, c, nactions, text_latents, mode, rng, prop=None, hist=None):
        """Training forward -> (loss, video_loss, act_loss) with injected draws `rng`."""
        B = z.shape[0]
        x = self.patchify(z.reshape(B * 4, *z.shape[2:])).reshape(B, 4, 256, -1)
        cond = self.patchify(c.reshape(B * 4, *c.shape[2:])).reshape(B, 4, 256, -1)
        prop = dict(prop or {})
        for k in ("second_image_z", "pred_second_image_z"):  # :816-845
            if k in prop:
                v = prop[k]
                prop[k] = self.patchify(v.reshape(B * 4, *v.shape[2:])).reshape(B, 4, 256, -1)
        text = self.text_proj_cond(text_latents) if self.clip else None
        mask = self.token_mask(torch.as_tensor(rng["orders"]), rng["mask_rate"])
        h = self.encode(x, cond, mask, nactions, text, mode, prop,
                        torch.as_tensor(rng.get("text_drop_u", np.ones(B, np.float32))), hist, rng.get("hist_u"))
        zdec = self.decode(h)
        gt = x.reshape(B, 1024, -1)
        ti = iter(torch.as_tensor(a) for a in rng["randint"])
        ni = iter(torch.as_tensor(a) for a in rng["randn_like"])
        zero = torch.tensor(0.0)
        lv = la = zero
        if mode in ("video_model", "dynamic_model", "full_dynamic_model"):
            lv = self.diffloss(gt, zdec, mask.reshape(B, -1), next(ti), next(ni))
            if self.predict_wrist_img:  # :738-776
                lv = lv + self.diffloss_wrist(prop["pred_second_image_z"].reshape(B, 1024, -1), zdec,
                                              mask.reshape(B, -1), next(ti), next(ni))
        if mode in ("policy_model", "inverse_model", "full_dynamic_model"):
            la = self.diffactloss(nactions, zdec, next(ti), next(ni))
        loss = lv + la if mode == "full_dynamic_model" else (lv if la is zero else la)
        if self.predict_proprioception:
            if self.umi:
                gt_prop = prop["robot0_eef_rot_axis_angle_wrt_start_pred"]
            else:  # toolhang :891-897
                gt_prop = torch.cat([prop["robot0_eef_pos_pred"], prop["robot0_eef_quat_pred"],
                                     prop["robot0_gripper_qpos_pred"]], dim=-1)
            loss = loss + self.diffproploss(gt_prop, zdec, next(ti), next(ni))
        return loss, lv, la


def mar_base(**kw):
    return MAR(encoder_embed_dim=768, encoder_depth=12, encoder_num_heads=12,
               decoder_embed_dim=768, decoder_depth=12, decoder_num_heads=12, **kw)


# --------------------------------------------------------------------------------------
# KL-VAE encoder (vaekl.py:9-273, 400-493), forward only
# --------------------------------------------------------------------------------------
def _gn(c):
    return nn.GroupNorm(32, c, eps=1e-6)


class _ResnetBlock(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.norm1, self.conv1 = _gn(cin), nn.Conv2d(cin, cout, 3, padding=1)
        self.norm2, self.conv2 = _gn(cout), nn.Conv2d(cout, cout, 3, padding=1)
        if cin != cout:
            self.nin_shortcut = nn.Conv2d(cin, cout, 1)

    def forward(self, x):
        h = self.conv1(F.silu(self.norm1(x)))
        h = self.conv2(F.silu(self.norm2(h)))
        if hasattr(self, "nin_shortcut"):
            x = self.nin_shortcut(x)
        return x + h


class _AttnBlock(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.norm = _gn(c)
        self.q, self.k, self.v = (nn.Conv2d(c, c, 1) for _ in range(3))
        self.proj_out = nn.Conv2d(c, c, 1)

    def forward(self, x):
        n, c, hh, ww = x.shape
        h = self.norm(x)
        q = self.q(h).reshape(n, c, -1)
        k = self.k(h).reshape(n, c, -1)
        v = self.v(h).reshape(n, c, -1)
        a = torch.softmax((q.transpose(1, 2) @ k) * (int(c) ** -0.5), dim=2)
        o = (v @ a.transpose(1, 2)).reshape(n, c, hh, ww)
        return x + self.proj_out(o)


class _Down(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, stride=2)

    def forward(self, x):
        return self.conv(F.pad(x, (0, 1, 0, 1)))


class Encoder(nn.Module):
    def __init__(self, ch=128, ch_mult=(1, 1, 2, 2, 4), num_res_blocks=2, z_channels=16,
                 resolution=256, attn_resolutions=(16,)):
        super().__init__()
        self.conv_in = nn.Conv2d(3, ch, 3, padding=1)
        self.down = nn.ModuleList()
        cin, res = ch, resolution
        for lvl, mult in enumerate(ch_mult):
            d = nn.Module()
            d.block = nn.ModuleList()
            d.attn = nn.ModuleList()
            for _ in range(num_res_blocks):
                d.block.append(_ResnetBlock(cin, ch * mult))
                cin = ch * mult
                if res in attn_resolutions:
                    d.attn.append(_AttnBlock(cin))
            if lvl != len(ch_mult) - 1:
                d.downsample = _Down(cin)
                res //= 2
            self.down.append(d)
        self.mid = nn.Module()
        self.mid.block_1, self.mid.attn_1, self.mid.block_2 = (
            _ResnetBlock(cin, cin), _AttnBlock(cin), _ResnetBlock(cin, cin))
        self.norm_out = _gn(cin)
        self.conv_out = nn.Conv2d(cin, 2 * z_channels, 3, padding=1)

    def forward(self, x):
        h = self.conv_in(x)
        for d in self.down:
            for i, blk in enumerate(d.block):
                h = blk(h)
                if len(d.attn):
                    h = d.attn[i](h)
            if hasattr(d, "downsample"):
                h = d.downsample(h)
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(h)))
        return self.conv_out(F.silu(self.norm_out(h)))


class _Up(nn.Module):
    """Upsample (vaekl.py:20-33): nearest x2 then conv3x3."""

    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, padding=1)

    def forward(self, x):
        return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))


class Decoder(nn.Module):
    """vaekl.py:276-397 with attn_resolutions=() (AutoencoderKL's construction)."""

    def __init__(self, ch=128, out_ch=3, ch_mult=(1, 1, 2, 2, 4), num_res_blocks=2, z_channels=16):
        super().__init__()
        block_in = ch * ch_mult[-1]
        self.conv_in = nn.Conv2d(z_channels, block_in, 3, padding=1)
        self.mid = nn.Module()
        self.mid.block_1 = _ResnetBlock(block_in, block_in)
        self.mid.attn_1 = _AttnBlock(block_in)
        self.mid.block_2 = _ResnetBlock(block_in, block_in)
        ups = []
        for lvl in reversed(range(len(ch_mult))):
            u = nn.Module()
            u.block = nn.ModuleList()
            for _ in range(num_res_blocks + 1):
                u.block.append(_ResnetBlock(block_in, ch * ch_mult[lvl]))
                block_in = ch * ch_mult[lvl]
            if lvl != 0:
                u.upsample = _Up(block_in)
            ups.insert(0, u)
        self.up = nn.ModuleList(ups)
        self.norm_out = _gn(block_in)
        self.conv_out = nn.Conv2d(block_in, out_ch, 3, padding=1)

    def forward(self, z):
        h = self.conv_in(z)
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(h)))
        for lvl in reversed(range(len(self.up))):
            for blk in self.up[lvl].block:
                h = blk(h)
            if hasattr(self.up[lvl], "upsample"):
                h = self.up[lvl].upsample(h)
        return self.conv_out(F.silu(self.norm_out(h)))


class AutoencoderKLDecoder(nn.Module):
    """AutoencoderKL.decode (vaekl.py:56-58): post_quant_conv -> Decoder."""

    def __init__(self, embed_dim=16, ch_mult=(1, 1, 2, 2, 4)):
        super().__init__()
        self.decoder = Decoder(ch_mult=ch_mult, z_channels=embed_dim)
        self.post_quant_conv = nn.Conv2d(embed_dim, embed_dim, 1)

    def decode(self, z):
        return self.decoder(self.post_quant_conv(z))


class AutoencoderKLEncoder(nn.Module):
    """Encoder half of AutoencoderKL (vaekl.py:449-493); the decoder is out of scope."""

    def __init__(self, embed_dim=16, ch_mult=(1, 1, 2, 2, 4), ch=128):
        super().__init__()
        self.encoder = Encoder(ch=ch, ch_mult=tuple(ch_mult), z_channels=embed_dim)
        self.quant_conv = nn.Conv2d(2 * embed_dim, 2 * embed_dim, 1)

    def moments(self, x):
        return self.quant_conv(self.encoder(x))

    def sample(self, x, eps):
        mean, logvar = self.moments(x).chunk(2, dim=1)
        logvar = logvar.clamp(-30.0, 20.0)
        return (mean + torch.exp(0.5 * logvar) * eps) * LATENT_SCALE


# --------------------------------------------------------------------------------------
# Batch plumbing (data_utils.py:19-426) and policy loss (policy:362-425)
# --------------------------------------------------------------------------------------
def resize_256(img):
    """[B,T,3,H,W] -> [B,T,3,256,256], bilinear, align_corners=False (data_utils.py:72-81)."""
    B, T, C, H, W = img.shape
    if H == 256:
        return img
    y = F.interpolate(img.reshape(B * T, C, H, W), size=(256, 256), mode="bilinear",
                      align_corners=False)
    return y.reshape(B, T, C, 256, 256)


def train_frame_indices(T=32, k=4):
    """[3, 7, ..., 31] for T=32 (data_utils.py:140-158)."""
    return torch.arange(0, T, T // (2 * k)) + k - 1


def pusht_augment(image, params, crop=91):
    """PushT dataset augmentation (pusht_image_dataset.py:93-130) with drawn parameters
    {crop, top, left, blur, k0..k4} per video: crop -> Resize(96, antialias) -> reflect-padded
    5x5 Gaussian (torchvision gaussian_blur restated; torchvision absent: parity unpinned)."""
    B, T, C, S, _ = image.shape
    out = []
    for b in range(B):
        x = image[b]
        p = params[b]
        if p[0] != 0:
            t, l = int(p[1]), int(p[2])
            x = F.interpolate(x[..., t:t + crop, l:l + crop], size=(S, S), mode="bilinear", align_corners=False,
                              antialias=True)
        if p[3] != 0:
            k = p[4:9].float()
            k2 = (k[:, None] * k[None, :]).expand(C, 1, 5, 5)
            x = F.conv2d(F.pad(x, (2, 2, 2, 2), mode="reflect"), k2, groups=C)
        out.append(x)
    return torch.stack(out)


# ---- §8f-3: UMI (kornia 0.8 VideoSequential) and Libero (torchvision 0.16 ColorJitter) ----------
# Parameter row per video (utils/augment.py AUG_NP = 24): 0 crop, 1 top, 2 left, 3 jitter,
# 4-7 op order (0 brightness, 1 contrast, 2 saturation, 3 hue), 8-11 factors (hue already in the
# style's unit: radians for kornia, turns for torchvision), 12 sharpness, 13 its factor,
# 14 autocontrast, 15 grayscale, 16 blur, 17-21 1-D Gaussian taps, 22 style (0 kornia,
# 1 torchvision), 23 crop size.  kornia and torchvision are absent here: these are restatements
# of their published algorithms (parity against the libraries themselves: unpinned).

def _gray_k(x):
    """kornia.color.rgb_to_grayscale (0.299, 0.587, 0.114)."""
    return 0.299 * x[..., 0:1, :, :] + 0.587 * x[..., 1:2, :, :] + 0.114 * x[..., 2:3, :, :]


def _gray_tv(x):
    """torchvision F_t.rgb_to_grayscale (0.2989, 0.587, 0.114)."""
    r, g, b = x.unbind(dim=-3)
    return (0.2989 * r + 0.587 * g + 0.114 * b).unsqueeze(-3)


def _k_rgb2hsv(img, eps=1e-8):
    """kornia.color.rgb_to_hsv: h in [0, 2pi), first channel wins a tie for the max."""
    max_rgb, argmax_rgb = img.max(-3)
    min_rgb = img.min(-3).values
    deltac = max_rgb - min_rgb
    v = max_rgb
    s = deltac / (max_rgb + eps)
    deltac = torch.where(deltac == 0, torch.ones_like(deltac), deltac)
    rc, gc, bc = torch.unbind(max_rgb.unsqueeze(-3) - img, dim=-3)
    h = torch.stack((bc - gc, (rc - bc) + 2.0 * deltac, (gc - rc) + 4.0 * deltac), dim=-3) / deltac.unsqueeze(-3)
    h = torch.gather(h, -3, argmax_rgb.unsqueeze(-3)).squeeze(-3)
    h = (h / 6.0) % 1.0
    return torch.stack((2.0 * math.pi * h, s, v), dim=-3)


def _k_hsv2rgb(img):
    """kornia.color.hsv_to_rgb (sector gather over (v,q,p,p,t,v | t,v,v,q,p,p | p,p,t,v,v,q))."""
    h = img[..., 0, :, :] / (2 * math.pi)
    s, v = img[..., 1, :, :], img[..., 2, :, :]
    hi = torch.floor(h * 6) % 6
    f = ((h * 6) % 6) - hi
    p, q, t = v * (1 - s), v * (1 - f * s), v * (1 - (1 - f) * s)
    hi = hi.long()
    idx = torch.stack([hi, hi + 6, hi + 12], dim=-3)
    out = torch.stack((v, q, p, p, t, v, t, v, v, q, p, p, p, p, t, v, v, q), dim=-3)
    return torch.gather(out, -3, idx)


def _tv_rgb2hsv(img):
    """torchvision F_t._rgb2hsv (h in turns)."""
    r, g, b = img.unbind(dim=-3)
    maxc, minc = img.max(dim=-3).values, img.min(dim=-3).values
    eqc = maxc == minc
    cr = maxc - minc
    ones = torch.ones_like(maxc)
    s = cr / torch.where(eqc, ones, maxc)
    crd = torch.where(eqc, ones, cr)
    rc, gc, bc = (maxc - r) / crd, (maxc - g) / crd, (maxc - b) / crd
    hr = (maxc == r) * (bc - gc)
    hg = ((maxc == g) & (maxc != r)) * (2.0 + rc - bc)
    hb = ((maxc != g) & (maxc != r)) * (4.0 + gc - rc)
    h = torch.fmod((hr + hg + hb) / 6.0 + 1.0, 1.0)
    return torch.stack((h, s, maxc), dim=-3)


def _tv_hsv2rgb(img):
    """torchvision F_t._hsv2rgb (clamped p / q / t, sector select)."""
    h, s, v = img.unbind(dim=-3)
    i = torch.floor(h * 6.0)
    f = h * 6.0 - i
    i = i.to(torch.int32) % 6
    p = torch.clamp(v * (1.0 - s), 0.0, 1.0)
    q = torch.clamp(v * (1.0 - s * f), 0.0, 1.0)
    t = torch.clamp(v * (1.0 - s * (1.0 - f)), 0.0, 1.0)
    mask = (i.unsqueeze(-3) == torch.arange(6).view(-1, 1, 1)).to(img.dtype)
    a4 = torch.stack((torch.stack((v, q, p, p, t, v), -3), torch.stack((t, v, v, q, p, p), -3),
                      torch.stack((p, p, t, v, v, q), -3)), -4)
    return torch.einsum("...ijk,...xijk->...xjk", mask, a4)


def _jitter_op(x, op, fac, tv):
    """One ColorJitter op on frames [T, 3, H, W]: kornia 0.8 ColorJitter (brightness_accumulative,
    contrast_with_mean_subtraction, saturation_with_gray_subtraction, adjust_hue) or torchvision
    0.16 ColorJitter (_blend forms, adjust_hue)."""
    gray = _gray_tv if tv else _gray_k
    if op == 0:
        return (fac * x).clamp(0.0, 1.0)
    if op == 1:
        m = gray(x).mean(dim=(-3, -2, -1), keepdim=True)
        return (fac * x + (1.0 - fac) * m).clamp(0.0, 1.0)
    if op == 2:
        return (fac * x + (1.0 - fac) * gray(x)).clamp(0.0, 1.0)
    if fac == 0.0:
        return x  # both libraries skip a zero hue shift
    if tv:
        h, s, v = _tv_rgb2hsv(x).unbind(-3)
        return _tv_hsv2rgb(torch.stack(((h + fac) % 1.0, s, v), -3))
    h, s, v = _k_rgb2hsv(x).unbind(-3)
    return _k_hsv2rgb(torch.stack((torch.fmod(h + fac, 2 * math.pi), s, v), -3))


def _sharpness_k(x, fac):
    """kornia.enhance.sharpness: 3x3 (1,1,1;1,5,1;1,1,1)/13 smoothing on the valid interior,
    clamped, border pixels kept, then blended back: deg + fac * (x - deg), clamped."""
    C = x.shape[-3]
    k = torch.tensor([[1.0, 1.0, 1.0], [1.0, 5.0, 1.0], [1.0, 1.0, 1.0]]) / 13
    deg = F.conv2d(x, k.view(1, 1, 3, 3).repeat(C, 1, 1, 1), groups=C).clamp(0.0, 1.0)
    res = x.clone()
    res[..., 1:-1, 1:-1] = deg
    return (res + (x - res) * fac).clamp(0.0, 1.0)


def video_augment(video, params):
    """video [B, T, 3, S, S] in [0, 1] -> augmented copy, one parameter row per video.
    kornia style (UMI, base_lazy_dataset.py:365-411 + config/task/umi_lazy.yaml:50-72):
    RandomCrop(cs) -> Resize(S) (bilinear, upscaling: antialias inert) -> ColorJitter ->
    RandomSharpness -> RandomAutoContrast (normalize_min_max per frame and channel, eps 1e-6,
    clipped) -> RandomGrayscale -> RandomGaussianBlur (separable, reflect, x then y).
    torchvision style (Libero, libero_replay_image_dataset.py:229-247): ColorJitter only."""
    B, T, C, S, _ = video.shape
    out = []
    for b in range(B):
        x = video[b].float()
        p = params[b].tolist()
        tv = p[22] != 0
        cs = int(p[23])
        if p[0]:
            t, l = int(p[1]), int(p[2])
            x = F.interpolate(x[..., t:t + cs, l:l + cs], size=(S, S), mode="bilinear", align_corners=False)
        if p[3]:
            for k in range(4):
                op = int(p[4 + k])
                x = _jitter_op(x, op, torch.tensor(p[8 + op], dtype=torch.float32).item(), tv)
        if p[12]:
            x = _sharpness_k(x, p[13])
        if p[14]:
            mn = x.amin(dim=(-2, -1), keepdim=True)
            mx = x.amax(dim=(-2, -1), keepdim=True)
            x = ((x - mn) / (mx - mn + 1e-6)).clamp(0.0, 1.0)
        if p[15]:
            x = _gray_k(x).expand(-1, C, -1, -1).contiguous()
        if p[16]:
            k = torch.tensor(p[17:22], dtype=torch.float32)
            x = F.conv2d(F.pad(x, (2, 2, 0, 0), mode="reflect"), k.view(1, 1, 1, 5).repeat(C, 1, 1, 1), groups=C)
            x = F.conv2d(F.pad(x, (0, 0, 2, 2), mode="reflect"), k.view(1, 1, 5, 1).repeat(C, 1, 1, 1), groups=C)
        out.append(x)
    return torch.stack(out)


def eval_frame_indices(T=32, k=4):
    """[3, 11, 19, 27] for T=32 (select_frames eval=True, data_utils.py:141-142)."""
    return torch.arange(0, T, T // k) + k - 1


def vae_input(img, eval=False):
    """x*255 -> frame select -> /127.5-1 -> b c t h w (data_utils.py:206-226)."""
    x = img * 255.0
    x = x[:, (eval_frame_indices if eval else train_frame_indices)(img.shape[1])]
    return (x / 127.5 - 1).permute(0, 2, 1, 3, 4)


def trajectory(nactions, T=32, shift_action=True):
    """data_utils.py:368-388 (no history action)."""
    if shift_action:
        return nactions[:, T // 2 - 1:-1]
    return torch.chunk(nactions, 2, dim=1)[1]


class PolicyOracle(nn.Module):
    """compute_loss of UnifiedVideoActionPolicy for the PushT-style path (policy:362-425)."""

    def __init__(self, mar, vae, action_scale, action_offset):
        super().__init__()
        self.model = mar
        self.vae_model = vae
        self.register_buffer("a_scale", torch.as_tensor(action_scale, dtype=torch.float32))
        self.register_buffer("a_offset", torch.as_tensor(action_offset, dtype=torch.float32))

    def compute_loss(self, image, action, mode, rng):
        B = image.shape[0]
        nact = action * self.a_scale + self.a_offset
        x = vae_input(resize_256(image))
        c_frames, x_frames = torch.chunk(x, 2, dim=2)
        with torch.no_grad():
            def enc(fr, eps):
                f = fr.permute(0, 2, 1, 3, 4).reshape(-1, *fr.shape[1:2], *fr.shape[3:])
                zz = self.vae_model.sample(f, torch.as_tensor(eps))
                return zz.reshape(B, 4, *zz.shape[1:])
            z = enc(x_frames, rng["vae_eps_x"])
            c = enc(c_frames, rng["vae_eps_c"])
        loss, lv, la = self.model(z, c, trajectory(nact), None, mode, rng)
        for p in self.model.parameters():  # policy:421-423 (adds exact zeros)
            loss = loss + 0 * p.sum()
        return loss, (lv, la)

    @torch.no_grad()
    def predict_action(self, image, rng, temperature=0.95, n_action_steps=8):
        """predict_action (policy:221-320), PushT: resize_image_eval -> eval frame select ->
        VAE posterior sample (eps in (b t) order) -> sample_tokens(policy_model) -> unnormalize."""
        B = image.shape[0]
        x = vae_input(resize_256(image), eval=True)
        f = x.permute(0, 2, 1, 3, 4).reshape(-1, 3, 256, 256)
        c = self.vae_model.sample(f, torch.as_tensor(rng["vae_eps"]))
        c = c.reshape(B, 4, *c.shape[1:])
        act = self.model.sample_policy(c, None, torch.as_tensor(rng["noise"]), torch.as_tensor(rng["step_noise"]),
                                       temperature)
        pred = (act[..., :self.a_scale.numel()] - self.a_offset) / self.a_scale
        return pred[:, :n_action_steps], pred


# --------------------------------------------------------------------------------------
# Optimizer groups, EMA decay, LR schedule (policy:326-360, ema_model.py:45-55,
# diffusers 0.18.2 get_cosine_schedule_with_warmup -- restated, parity unpinned)
# --------------------------------------------------------------------------------------
def weight_decay_split(named_params):
    decay, no_decay = [], []
    for n, p in named_params:
        if not p.requires_grad:
            continue
        (no_decay if (p.ndim == 1 or n.endswith(".bias")) else decay).append(n)
    return decay, no_decay


def ema_decay(step, update_after_step=0, inv_gamma=1.0, power=0.75, min_value=0.0,
              max_value=0.9999):
    s = max(0, step - update_after_step - 1)
    if s <= 0:
        return 0.0
    v = 1 - (1 + s / inv_gamma) ** -power
    return max(min_value, min(v, max_value))


def cosine_lr_factor(step, warmup, total, num_cycles=0.5):
    if step < warmup:
        return step / max(1, warmup)
    prog = (step - warmup) / max(1, total - warmup)
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * num_cycles * 2.0 * prog)))
