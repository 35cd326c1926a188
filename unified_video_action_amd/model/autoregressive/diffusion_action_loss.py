"""Action / proprioception diffusion-loss head on the HIP path
(reference: model/autoregressive/diffusion_action_loss.py).

Trunk (act_model_type, diffusion_action_loss.py:35-89, 109-141):
  conv_fc (every config): z [B, 4*256, D] -> per-frame NHWC 16x16 -> conv3x3+ReLU (halo HIP conv, fused
    ReLU epilogue) -> AdaptiveAvgPool(4,4) + flatten (HIP) -> fc(ReLU) -> fc -> Linear(4->16 frames) ->
    refine MLP;
  conv_ori: ConvTranspose3d((4,1,1), stride 4) + AvgPool3d((1,16,16)) as frame means + one GEMM;
  conv2: Conv1d(1024 -> 256, k7) + ReLU + Conv1d(256 -> 16, k7) over the feature axis (the 1024 tokens
    are the channels) as im2col columns + GEMMs;
  fc2: Linear(1024 -> 256) + ReLU + Linear(256 -> 16) over the token axis;
then the SimpleMLPAdaLN diffusion loss over B*16 rows (plain mean).
sample(): the same trunk, then the spaced reverse-diffusion loop (sampler.ActionSampler).
Every contraction is a HIP GEMM; the off-config trunks' reshapes / im2col / frame means are torch
glue (conv_fc is the only trunk any reference config uses).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ...native import ops
from ...runtime import cdt
from .diffusion_loss import SimpleMLPAdaLN, diffusion_head_loss, schedule
from .functional import F32, as_dtype, compute_weight, grad_buf, linear
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


class FrameMeanConvTFn(torch.autograd.Function):
    """ConvTranspose3d(D, D, (4,1,1), stride (4,1,1)) + AvgPool3d((1,16,16)) of z [B, T*256, D]
    (act_model_type="conv_ori", diffusion_action_loss.py:63-71, 125-134).  The pool commutes with the
    per-pixel transposed conv, so each frame's 256 tokens are averaged first and ONE GEMM maps the frame
    mean to its 4 output steps: out[b, 4t + k, co] = bias[co] + sum_ci mean_s z[b, 256t + s, ci] W[ci, co, k]
    (W [ci, co, 4] read as the [ci, co*4] matrix of its layout)."""

    @staticmethod
    def forward(ctx, z, weight, bias):
        B, N, D = z.shape
        T = N // 256
        mc = as_dtype(z.detach().reshape(B * T, 256, D).float().mean(1), cdt())
        wm = compute_weight(weight).reshape(D, D * 4)
        out = torch.empty(B * T, D * 4, dtype=F32, device=z.device)
        ops.gemm(mc, wm, out, B * T, D * 4, D, D, D * 4, D * 4, 0, 1,
                 bias=bias.detach().repeat_interleave(4).contiguous())
        ctx.save_for_backward(mc, weight, bias)
        ctx.dims = (B, T, D, z.dtype)
        return out.view(B, T, D, 4).permute(0, 1, 3, 2).reshape(B, T * 4, D)

    @staticmethod
    def backward(ctx, g):
        mc, weight, bias = ctx.saved_tensors
        B, T, D, zdt = ctx.dims
        gk = g.reshape(B, T, 4, D).permute(0, 1, 3, 2).reshape(B * T, D * 4).contiguous()
        gkc = as_dtype(gk, cdt())
        ops.linear_dw(mc, gkc, grad_buf(weight).view(D, D * 4))     # dW[ci, (co,k)] += mean^T g
        grad_buf(bias).add_(gk.sum(0).view(D, 4).sum(1))
        dm = torch.empty(B * T, D, dtype=F32, device=g.device)
        ops.linear(gkc, compute_weight(weight).reshape(D, D * 4), dm)  # g [BT, co*4] @ W^T
        dz = (dm / 256.0).unsqueeze(1).expand(B * T, 256, D).reshape(B, T * 256, D)
        return dz.to(zdt), None, None


def _cols_k7(x):
    """im2col of a channels-first [B, C, L] sequence for a k=7 / pad-3 Conv1d: [B*L, C*7] with column
    c*7 + j = x[b, c, l + j - 3] (the Conv1d weight [out, C, 7] order)."""
    B, C, L = x.shape
    return F.pad(x, (3, 3)).unfold(2, 7, 1).permute(0, 2, 1, 3).reshape(B * L, C * 7)


class DiffActLoss(nn.Module):
    def __init__(self, target_channels, z_channels, depth, width, num_sampling_steps, grad_checkpointing=False,
                 n_frames=4, act_diff_training_steps=1000, act_diff_testing_steps="100", act_model_type="conv_fc",
                 **kwargs):
        super().__init__()
        self.in_channels = target_channels
        self.n_frames = n_frames
        self.act_model_type = act_model_type
        if act_model_type == "conv_fc":
            self.w = self.h = 16
            self.num_frames, self.num_actions = 4, 16
            self.conv = nn.Sequential(nn.Conv2d(z_channels, z_channels, 3, 1, 1), nn.ReLU(),
                                      nn.AdaptiveAvgPool2d((4, 4)))
            self.fc = nn.Sequential(nn.Linear(z_channels * 16, z_channels), nn.ReLU(),
                                    nn.Linear(z_channels, z_channels))
            self.interpolate = nn.Linear(self.num_frames, self.num_actions)
            self.refine = nn.Sequential(nn.Linear(z_channels, z_channels), nn.ReLU(),
                                        nn.Linear(z_channels, z_channels))
        elif act_model_type == "conv_ori":
            self.w = self.h = 16
            self.conv_transpose3d = nn.ConvTranspose3d(z_channels, z_channels, kernel_size=(4, 1, 1), stride=(4, 1, 1))
            self.avg_pool = nn.AvgPool3d(kernel_size=(1, self.w, self.h))
        elif act_model_type == "conv2":
            self.conv = nn.Sequential(nn.Conv1d(1024, 256, kernel_size=7, padding=3), nn.ReLU(),
                                      nn.Conv1d(256, 16, kernel_size=7, padding=3))
        elif act_model_type == "fc2":
            self.fc = nn.Sequential(nn.Linear(1024, 256), nn.ReLU(), nn.Linear(256, 16))
        else:
            raise NotImplementedError(act_model_type)  # the reference raises the same (:88-89)
        self.net = SimpleMLPAdaLN(target_channels, width, target_channels * 2, z_channels, depth, grad_checkpointing)
        self.num_timesteps = act_diff_training_steps
        self.act_diff_testing_steps = act_diff_testing_steps
        self._sampler = None

    def trunk(self, z):
        B, N, D = z.shape
        if self.act_model_type == "conv_ori":
            return FrameMeanConvTFn.apply(z, self.conv_transpose3d.weight, self.conv_transpose3d.bias)
        if self.act_model_type == "conv2":
            f = linear(_cols_k7(z.to(cdt())), self.conv[0], act="relu", out_dtype=cdt())  # [B*D, 256]
            f = F.pad(f.reshape(B, D, 256), (0, 0, 3, 3)).unfold(1, 7, 1).reshape(B * D, 256 * 7)
            return linear(f, self.conv[2], out_dtype=F32).reshape(B, D, 16).transpose(1, 2)
        if self.act_model_type == "fc2":
            f = linear(z.transpose(1, 2), self.fc[0], act="relu", out_dtype=cdt())  # [B, D, 256]
            return linear(f, self.fc[2], out_dtype=F32).transpose(1, 2)
        f = z.reshape(B * 4, 16, 16, D)  # (b t), w, h, c   with s = w*16 + h
        f = ConvReluPoolFn.apply(f, self.conv[0].weight, self.conv[0].bias)  # [B*4, D*16] in (c w h) order
        f = linear(f, self.fc[0], act="relu", out_dtype=cdt())
        f = linear(f, self.fc[2], out_dtype=F32).reshape(B, 4, D)
        f = linear(f.transpose(1, 2), self.interpolate, out_dtype=F32).transpose(1, 2)  # B,16,D
        f = linear(f, self.refine[0], act="relu", out_dtype=cdt())
        return linear(f, self.refine[2], out_dtype=F32)

    def forward(self, target, z, task_mode=None, text_latents=None, t=None, noise=None):
        bsz, seq_len, _ = target.shape
        c = self.trunk(z).reshape(bsz * seq_len, -1).contiguous()
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
