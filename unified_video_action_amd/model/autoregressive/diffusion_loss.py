"""Video diffusion-loss head on the HIP path (reference: model/autoregressive/diffusion_loss.py).

DiffLoss.forward = q_sample -> SimpleMLPAdaLN -> fused eps-MSE + learned-range VB loss ->
masked mean (diffusion_loss.py:44-66).  Module/parameter names match the reference.
"""
import torch
import torch.nn as nn

from ...native import ops
from ...runtime import cdt
from .diffusion import DiffusionSchedule, timestep_freqs
from .functional import F32, AdaLNTrunkFn, linear

_SCHED = {}


def schedule(T, device):
    key = (T, str(device))
    if key not in _SCHED:
        _SCHED[key] = DiffusionSchedule(T, device)
    return _SCHED[key]


_FREQS = {}


def freqs(device):
    key = str(device)
    if key not in _FREQS:
        _FREQS[key] = timestep_freqs(device)
    return _FREQS[key]


class TimestepEmbedder(nn.Module):
    def __init__(self, hidden_size, frequency_embedding_size=256):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(frequency_embedding_size, hidden_size), nn.SiLU(),
                                 nn.Linear(hidden_size, hidden_size))
        self.frequency_embedding_size = frequency_embedding_size

    def forward(self, t):
        f = torch.empty(t.numel(), self.frequency_embedding_size, dtype=cdt(), device=t.device)
        ops.timestep_features(t, freqs(t.device), f)
        h = linear(f, self.mlp[0], act="silu", out_dtype=cdt())
        return linear(h, self.mlp[2], out_dtype=F32)


class ResBlock(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.channels = channels
        self.in_ln = nn.LayerNorm(channels, eps=1e-6)
        self.mlp = nn.Sequential(nn.Linear(channels, channels), nn.SiLU(), nn.Linear(channels, channels))
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(channels, 3 * channels))

    def trunk_params(self):
        return [self.adaLN_modulation[1].weight, self.adaLN_modulation[1].bias, self.mlp[0].weight,
                self.mlp[0].bias, self.mlp[2].weight, self.mlp[2].bias, self.in_ln.weight, self.in_ln.bias]


class FinalLayer(nn.Module):
    def __init__(self, model_channels, out_channels):
        super().__init__()
        self.norm_final = nn.LayerNorm(model_channels, elementwise_affine=False, eps=1e-6)
        self.linear = nn.Linear(model_channels, out_channels)
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(model_channels, 2 * model_channels))

    def trunk_params(self):
        return [self.adaLN_modulation[1].weight, self.adaLN_modulation[1].bias, self.linear.weight,
                self.linear.bias]


class SimpleMLPAdaLN(nn.Module):
    def __init__(self, in_channels, model_channels, out_channels, z_channels, num_res_blocks,
                 grad_checkpointing=False):
        super().__init__()
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_res_blocks = num_res_blocks
        self.time_embed = TimestepEmbedder(model_channels)
        self.cond_embed = nn.Linear(z_channels, model_channels)
        self.input_proj = nn.Linear(in_channels, model_channels)
        self.res_blocks = nn.ModuleList([ResBlock(model_channels) for _ in range(num_res_blocks)])
        self.final_layer = FinalLayer(model_channels, out_channels)
        self.initialize_weights()

    def initialize_weights(self):
        # same init recipe as the reference (diffusion_loss.py:237-259)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                nn.init.zeros_(m.bias)
        nn.init.normal_(self.time_embed.mlp[0].weight, std=0.02)
        nn.init.normal_(self.time_embed.mlp[2].weight, std=0.02)
        for blk in self.res_blocks:
            nn.init.zeros_(blk.adaLN_modulation[-1].weight)
            nn.init.zeros_(blk.adaLN_modulation[-1].bias)
        nn.init.zeros_(self.final_layer.adaLN_modulation[-1].weight)
        nn.init.zeros_(self.final_layer.adaLN_modulation[-1].bias)
        nn.init.zeros_(self.final_layer.linear.weight)
        nn.init.zeros_(self.final_layer.linear.bias)

    def forward(self, x, t, c):
        """x: [R, C_in] (x_t), t: [R] int64, c: [R, z] -> [R, C_out] fp32."""
        t_emb = self.time_embed(t)
        y = linear(c, self.cond_embed, out_dtype=F32, residual=t_emb)
        x0 = linear(x, self.input_proj, out_dtype=F32)
        params = []
        for blk in self.res_blocks:
            params += blk.trunk_params()
        params += self.final_layer.trunk_params()
        return AdaLNTrunkFn.apply(x0, y, len(self.res_blocks), getattr(self, "_uva_bucket_hook", None), *params)


class DiffusionLossFn(torch.autograd.Function):
    """sum_r w_r * (mse_r + vb_r) / sum_r w_r with w = mask (video) or 1 (actions)."""

    @staticmethod
    def forward(ctx, out, x0, noise, t, w, sched):
        rows, C = x0.shape
        lrow = torch.empty(rows, dtype=F32, device=out.device)
        dl = torch.empty(rows, 2 * C, dtype=F32, device=out.device)
        ops.diffusion_loss(x0, noise, t, out.contiguous(), sched.tables, lrow, dl)
        res = torch.empty(2, dtype=F32, device=out.device)
        ops.weighted_mean(lrow, w, res)
        ctx.save_for_backward(dl, w, res)
        ctx.lrow = lrow
        return res[0].clone()

    @staticmethod
    def backward(ctx, g):
        dl, w, res = ctx.saved_tensors
        dout = torch.empty(dl.shape, dtype=F32, device=dl.device)
        ops.loss_grad(dl, w, res[1:2], g.reshape(1).contiguous().float(), dout)
        return dout, None, None, None, None, None


def diffusion_head_loss(net, sched, target, cond, weights, t=None, noise=None):
    """q_sample -> net -> fused loss.  target [R, C] fp32, cond [R, z]."""
    rows, C = target.shape
    dev = target.device
    if t is None:
        t = torch.randint(0, sched.T, (rows,), device=dev)
    if noise is None:
        noise = torch.randn(rows, C, device=dev)
    t = t.to(dev, torch.int64).contiguous()
    noise = noise.to(dev, F32).contiguous()
    x0 = target.to(F32).contiguous()
    xt = torch.empty(rows, C, dtype=cdt(), device=dev)
    ops.q_sample(x0, noise, t, sched.tables, xt)
    out = net(xt, t, cond)
    return DiffusionLossFn.apply(out, x0, noise, t, weights, sched)


class DiffLoss(nn.Module):
    """Diffusion Loss (diffusion_loss.py:8-66)."""

    def __init__(self, target_channels, z_channels, depth, width, num_sampling_steps, grad_checkpointing=False,
                 **kwargs):
        super().__init__()
        self.in_channels = target_channels
        self.n_frames = kwargs.get("n_frames", 4)
        self.net = SimpleMLPAdaLN(target_channels, width, target_channels * 2, z_channels, depth, grad_checkpointing)
        self.num_timesteps = 1000
        self.num_sampling_steps = str(num_sampling_steps)
        self._sampler = None

    @torch.no_grad()
    def sample(self, z, temperature=1.0, cfg=1.0, text_latents=None, noise=None, step_noise=None):
        """z [R, D] decoder rows of the tokens to predict -> token latents [R, C]
        (diffusion_loss.py:68-90: p_sample_loop over create_diffusion(num_sampling_steps), no clipping).
        noise [R, C] / step_noise [S, R, C] may be injected."""
        if cfg != 1.0:
            raise NotImplementedError("classifier-free guidance (forward_with_cfg) is not on the built path")
        from .sampler import ActionSampler
        if self._sampler is None:
            self._sampler = ActionSampler(self.net, self.num_sampling_steps, clip_denoised=False)
        R = z.shape[0]
        S = self._sampler.sched.S
        dev = z.device
        if noise is None:
            noise = torch.randn(R, self.in_channels, device=dev)
        if step_noise is None:
            step_noise = torch.randn(S, R, self.in_channels, device=dev)
        return self._sampler(z.float().contiguous(), noise.to(dev, torch.float32),
                             step_noise.to(dev, torch.float32), temperature)

    def forward(self, target, z, mask=None, conf_score=None, text_latents=None, t=None, noise=None):
        bsz, seq_len, _ = target.shape
        rows = bsz * seq_len
        w = None if mask is None else mask.reshape(rows).to(F32).contiguous()
        return diffusion_head_loss(self.net, schedule(self.num_timesteps, target.device),
                                   target.reshape(rows, -1), z.reshape(rows, -1), w, t, noise)
