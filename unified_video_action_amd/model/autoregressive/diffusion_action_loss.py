"""Action / proprioception diffusion-loss head on the HIP path
(reference: model/autoregressive/diffusion_action_loss.py, act_model_type="conv_fc").

Trunk: z [B, 4*256, D] -> per-frame NHWC 16x16 -> conv3x3+ReLU (implicit-GEMM HIP conv,
fused ReLU epilogue) -> AdaptiveAvgPool(4,4) + flatten (HIP) -> fc(ReLU) -> fc -> Linear(4->16 frames)
-> refine MLP -> SimpleMLPAdaLN diffusion loss over B*16 rows (plain mean).
sample(): the same trunk, then the spaced reverse-diffusion loop (sampler.ActionSampler).
"""
import torch
import torch.nn as nn

from ...native import ops
from ...runtime import cdt
from .diffusion_loss import SimpleMLPAdaLN, diffusion_head_loss, schedule
from .functional import F32, as_dtype, grad_buf, linear
from .sampler import ActionSampler


class ConvReluPoolFn(torch.autograd.Function):
    """Conv2d(D, D, 3, p=1) + bias + ReLU + AdaptiveAvgPool2d((4, 4)) + flatten (c w h) of NHWC
    [n, 16, 16, D] (diffusion_action_loss.py:42-47, 113-124); weight in nn.Conv2d layout [Co, Ci, 3, 3].
    No ATen kernels: the weight changes layout in one HIP pass, the pool writes (c w h) directly,
    the backward fuses the pool's broadcast with the ReLU mask, and dW is 9 GEMMs over zero-padded
    copies of dpre / x (a tap = a constant row shift: no im2col), added into the Conv2d-layout gradient
    by a scatter-add pass."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        n, H, W, Ci = x.shape
        Co = weight.shape[0]
        cd = cdt()
        xc = as_dtype(x, cd)
        wk = torch.empty(Co, 3, 3, Ci, dtype=cd, device=x.device)
        ops.conv3x3_weight_layout(weight.detach(), wk, 0)
        post = torch.empty(n, H, W, Co, dtype=cd, device=x.device)
        ops.conv2d(xc, wk, post, n, H, W, Ci, Co, 3, 1, 1, 1, H, W, bias=bias.detach(), act="relu")
        pooled = torch.empty(n, Co * 16, dtype=cd, device=x.device)
        ops.pool4x4_cwh(post, pooled, n, Co)
        ctx.save_for_backward(xc, weight, bias, post)
        ctx.xdt = x.dtype
        return pooled

    @staticmethod
    def backward(ctx, g):
        xc, weight, bias, post = ctx.saved_tensors
        n, H, W, Ci = xc.shape
        Co = weight.shape[0]
        cd = cdt()
        dpre = torch.empty(n, H, W, Co, dtype=cd, device=g.device)
        ops.pool4x4_relu_bwd(post, g.contiguous(), dpre, n, Co)
        # dX = conv(dpre, W flipped & transposed)
        wt = torch.empty(Ci, 3, 3, Co, dtype=cd, device=g.device)
        ops.conv3x3_weight_layout(weight.detach(), wt, 1)
        dx = torch.empty(n, H, W, Ci, dtype=cd, device=g.device)
        ops.conv2d(dpre, wt, dx, n, H, W, Co, Ci, 3, 1, 1, 1, H, W)
        # dW[co][(kh, kw, ci)] as an implicit GEMM: dpre and x zero-padded to 18 x 18 (plus guard rows),
        # so tap (kh, kw) is a constant row shift of x -- 9 GEMMs over the padded pixels, no im2col --
        # then added into the nn.Conv2d-layout gradient [co][ci][kh][kw]
        part = torch.empty(Co, 9 * Ci, dtype=F32, device=g.device)
        ops.conv3x3_dw_implicit(dpre, xc, part, n, H, W, Co, Ci)
        ops.conv3x3_dw_scatter_add(part, grad_buf(weight))
        ops.colsum(dpre.reshape(-1, Co), grad_buf(bias))
        return as_dtype(dx, ctx.xdt), None, None


class DiffActLoss(nn.Module):
    def __init__(self, target_channels, z_channels, depth, width, num_sampling_steps, grad_checkpointing=False,
                 n_frames=4, act_diff_training_steps=1000, act_diff_testing_steps="100", act_model_type="conv_fc",
                 **kwargs):
        super().__init__()
        if act_model_type != "conv_fc":
            raise NotImplementedError("only act_model_type=conv_fc is on the accelerated path")
        self.in_channels = target_channels
        self.n_frames = n_frames
        self.act_model_type = act_model_type
        self.w = self.h = 16
        self.num_frames, self.num_actions = 4, 16
        self.conv = nn.Sequential(nn.Conv2d(z_channels, z_channels, 3, 1, 1), nn.ReLU(), nn.AdaptiveAvgPool2d((4, 4)))
        self.fc = nn.Sequential(nn.Linear(z_channels * 16, z_channels), nn.ReLU(), nn.Linear(z_channels, z_channels))
        self.interpolate = nn.Linear(self.num_frames, self.num_actions)
        self.refine = nn.Sequential(nn.Linear(z_channels, z_channels), nn.ReLU(), nn.Linear(z_channels, z_channels))
        self.net = SimpleMLPAdaLN(target_channels, width, target_channels * 2, z_channels, depth, grad_checkpointing)
        self.num_timesteps = act_diff_training_steps
        self.act_diff_testing_steps = act_diff_testing_steps
        self._sampler = None

    def trunk(self, z):
        B, N, D = z.shape
        f = z.reshape(B * 4, 16, 16, D)  # (b t), w, h, c   with s = w*16 + h
        f = ConvReluPoolFn.apply(f, self.conv[0].weight, self.conv[0].bias)  # [B*4, D*16] in (c w h) order
        f = linear(f, self.fc[0], act="relu", out_dtype=cdt())
        f = linear(f, self.fc[2], out_dtype=F32).reshape(B, 4, D)
        f = linear(f.transpose(1, 2), self.interpolate, out_dtype=F32).transpose(1, 2)  # B,16,D
        f = linear(f, self.refine[0], act="relu", out_dtype=cdt())
        return linear(f, self.refine[2], out_dtype=F32)

    def forward(self, target, z, task_mode=None, text_latents=None, t=None, noise=None):
        bsz, seq_len, _ = target.shape
        c = self.trunk(z).reshape(bsz * seq_len, -1)
        return diffusion_head_loss(self.net, schedule(self.num_timesteps, target.device),
                                   target.reshape(bsz * seq_len, -1), c, None, t, noise)

    @torch.no_grad()
    def sample(self, z, temperature=1.0, cfg=1.0, text_latents=None, noise=None, step_noise=None):
        """z [B, 4*256, D] decoder tokens -> sampled action latents [B, 16, C]
        (diffusion_action_loss.py:168-232).  noise [B*16, C] (x_T) and step_noise [S, B*16, C]
        (the per-step randn_like of p_sample, gaussian_diffusion.py:431) may be injected."""
        if cfg != 1.0:
            # forward_with_cfg needs a doubled (cond, uncond) batch; the policy/inverse paths
            # always sample the action head with act_cfg = 1.0 (mar_con_unified.py:1031-1036).
            raise NotImplementedError("classifier-free guidance on the action head is not on the policy path")
        c = self.trunk(z)
        bsz, seq_len, _ = c.shape
        rows = bsz * seq_len
        if self._sampler is None:
            self._sampler = ActionSampler(self.net, self.act_diff_testing_steps)
        S = self._sampler.sched.S
        dev = z.device
        if noise is None:
            noise = torch.randn(rows, self.in_channels, device=dev)
        if step_noise is None:
            step_noise = torch.randn(S, rows, self.in_channels, device=dev)
        x = self._sampler(c.reshape(rows, -1).float().contiguous(), noise.to(dev, F32).reshape(rows, -1),
                          step_noise.to(dev, F32).reshape(S, rows, -1), temperature)
        return x.reshape(bsz, seq_len, -1)
