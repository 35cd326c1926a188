"""Action / proprioception diffusion-loss head on the HIP path
(reference: model/autoregressive/diffusion_action_loss.py, act_model_type="conv_fc").

Trunk: z [B, 4*256, D] -> per-frame NHWC 16x16 -> conv3x3+ReLU (implicit-GEMM HIP conv,
fused ReLU epilogue) -> AdaptiveAvgPool(4,4) -> fc(ReLU) -> fc -> Linear(4->16 frames)
-> refine MLP -> SimpleMLPAdaLN diffusion loss over B*16 rows (plain mean).
sample(): the same trunk, then the spaced reverse-diffusion loop (sampler.ActionSampler).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ...native import ops
from ...runtime import cdt
from .diffusion_loss import SimpleMLPAdaLN, diffusion_head_loss, schedule
from .functional import F32, as_dtype, grad_buf, linear
from .sampler import ActionSampler


class Conv3x3ReluFn(torch.autograd.Function):
    """NHWC conv3x3 (stride 1, pad 1) + bias + ReLU; weight in nn.Conv2d layout [Co, Ci, 3, 3]."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        n, H, W, Ci = x.shape
        Co = weight.shape[0]
        xc = as_dtype(x, cdt())
        wk = as_dtype(weight.detach().permute(0, 2, 3, 1), cdt())
        out = torch.empty(n, H, W, Co, dtype=cdt(), device=x.device)
        ops.conv2d(xc, wk, out, n, H, W, Ci, Co, 3, 1, 1, 1, H, W, bias=bias.detach(), act="relu")
        ctx.save_for_backward(xc, weight, bias, out)
        ctx.xdt = x.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        xc, weight, bias, out = ctx.saved_tensors
        n, H, W, Ci = xc.shape
        Co = weight.shape[0]
        dpre = torch.empty(n * H * W, Co, dtype=cdt(), device=g.device)
        ops.act_bwd(out.reshape(-1, Co), g.contiguous().reshape(-1, Co), dpre, "relu")
        # dX = conv(dpre, W flipped & transposed)
        wt = as_dtype(weight.detach().flip(2, 3).permute(1, 2, 3, 0), cdt())
        dx = torch.empty(n, H, W, Ci, dtype=cdt(), device=g.device)
        ops.conv2d(dpre, wt, dx, n, H, W, Co, Ci, 3, 1, 1, 1, H, W)
        # dW[co][(kh,kw,ci)] = dpre^T im2col(x)
        cols = F.pad(xc, (0, 0, 1, 1, 1, 1)).unfold(1, 3, 1).unfold(2, 3, 1)  # n,H,W,Ci,3,3
        cols = cols.permute(0, 1, 2, 4, 5, 3).reshape(n * H * W, 9 * Ci).contiguous()
        dwk = torch.zeros(Co, 9 * Ci, dtype=F32, device=g.device)
        ops.linear_dw(dpre, cols, dwk, beta=0.0)
        grad_buf(weight).add_(dwk.reshape(Co, 3, 3, Ci).permute(0, 3, 1, 2))
        ops.colsum(dpre, grad_buf(bias))
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
        f = Conv3x3ReluFn.apply(f, self.conv[0].weight, self.conv[0].bias)
        f = f.reshape(B * 4, 4, 4, 4, 4, D).mean(dim=(2, 4))  # AdaptiveAvgPool2d((4,4)) 16 -> 4
        f = f.permute(0, 3, 1, 2).reshape(B * 4, D * 16)  # (c w h)
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
