"""Frozen KL-VAE encoder on the HIP path (reference: unified_video_action/vae/vaekl.py).

Parameters keep the reference module tree (encoder.conv_in, encoder.down.{i}.block.{j}.
{norm1,conv1,norm2,conv2,nin_shortcut}, encoder.down.{i}.attn.{j}.{norm,q,k,v,proj_out},
encoder.down.{i}.downsample.conv, encoder.mid.*, encoder.norm_out, encoder.conv_out,
quant_conv, post_quant_conv, decoder.conv_in, decoder.mid.*, decoder.up.{i}.block.{j},
decoder.up.{i}.upsample.conv, decoder.norm_out, decoder.conv_out) so reference checkpoints
(kl16.ckpt "model" dict) load unchanged.  decode() (vaekl.py:56-58, Decoder :276-397; the
consumer of generated latents: video sampling and the FVD eval) reuses the encoder's
resblock / attention / conv pieces plus a nearest-x2 upsample kernel.

Forward runs entirely in NHWC on libuva_hip.so:
  * every conv = implicit-GEMM MFMA kernel with the residual add in its epilogue; the
    epilogue also emits deterministic per-tile GroupNorm partial sums of its output, so the
    next GroupNorm needs no statistics pass: finalize (tiny) + one vectorised GN-apply+SiLU
    pass (once per element, not once per 3x3 tap); fp32 parity path: separate stats pass and
    GN+SiLU in the conv A-loader;
  * AttnBlock = fused qkv 1x1 conv (GN prologue, no SiLU) -> batched QK^T GEMM -> row
    softmax -> PV GEMM -> proj_out 1x1 conv + residual;
  * quant_conv 1x1, then the posterior sample kernel writes MAR tokens directly.
"""
import os

import torch
import torch.nn as nn

from ..native import ops
from ..runtime import RT, cdt

F32 = torch.float32


def _gn(c):
    return nn.GroupNorm(32, c, eps=1e-6, affine=True)


class ResnetBlock(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.norm1 = _gn(in_channels)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, 1, 1)
        self.norm2 = _gn(out_channels)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, 1, 1)
        if in_channels != out_channels:
            self.nin_shortcut = nn.Conv2d(in_channels, out_channels, 1)


class AttnBlock(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.norm = _gn(c)
        self.q = nn.Conv2d(c, c, 1)
        self.k = nn.Conv2d(c, c, 1)
        self.v = nn.Conv2d(c, c, 1)
        self.proj_out = nn.Conv2d(c, c, 1)


class Downsample(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 2, 0)


class Upsample(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 1, 1)


class Decoder(nn.Module):
    """vaekl.py:276-397 (attn_resolutions=(), as AutoencoderKL builds it)."""

    def __init__(self, ch=128, out_ch=3, ch_mult=(1, 1, 2, 2, 4), num_res_blocks=2, resolution=256, z_channels=16,
                 **ignore):
        super().__init__()
        self.num_resolutions = len(ch_mult)
        self.num_res_blocks = num_res_blocks
        block_in = ch * ch_mult[-1]
        self.conv_in = nn.Conv2d(z_channels, block_in, 3, 1, 1)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(block_in, block_in)
        self.mid.attn_1 = AttnBlock(block_in)
        self.mid.block_2 = ResnetBlock(block_in, block_in)
        ups = []
        for lvl in reversed(range(self.num_resolutions)):
            u = nn.Module()
            u.block, u.attn = nn.ModuleList(), nn.ModuleList()
            for _ in range(num_res_blocks + 1):
                u.block.append(ResnetBlock(block_in, ch * ch_mult[lvl]))
                block_in = ch * ch_mult[lvl]
            if lvl != 0:
                u.upsample = Upsample(block_in)
            ups.insert(0, u)
        self.up = nn.ModuleList(ups)
        self.norm_out = _gn(block_in)
        self.conv_out = nn.Conv2d(block_in, out_ch, 3, 1, 1)


class Encoder(nn.Module):
    def __init__(self, ch=128, ch_mult=(1, 1, 2, 2, 4), num_res_blocks=2, attn_resolutions=(16,), in_channels=3,
                 resolution=256, z_channels=16, double_z=True, **ignore):
        super().__init__()
        self.ch = ch
        self.num_resolutions = len(ch_mult)
        self.num_res_blocks = num_res_blocks
        self.conv_in = nn.Conv2d(in_channels, ch, 3, 1, 1)
        in_mult = (1,) + tuple(ch_mult)
        res = resolution
        self.down = nn.ModuleList()
        for lvl in range(self.num_resolutions):
            d = nn.Module()
            d.block, d.attn = nn.ModuleList(), nn.ModuleList()
            cin = ch * in_mult[lvl]
            for _ in range(num_res_blocks):
                d.block.append(ResnetBlock(cin, ch * ch_mult[lvl]))
                cin = ch * ch_mult[lvl]
                if res in attn_resolutions:
                    d.attn.append(AttnBlock(cin))
            if lvl != self.num_resolutions - 1:
                d.downsample = Downsample(cin)
                res //= 2
            self.down.append(d)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(cin, cin)
        self.mid.attn_1 = AttnBlock(cin)
        self.mid.block_2 = ResnetBlock(cin, cin)
        self.norm_out = _gn(cin)
        self.conv_out = nn.Conv2d(cin, 2 * z_channels if double_z else z_channels, 3, 1, 1)


class _Prepared:
    """compute-dtype NHWC copies of the frozen weights ([Co][kh][kw][Ci])."""

    def __init__(self, vae, dtype, device, cin_pad):
        self.w, self.b = {}, {}
        for name, m in vae.named_modules():
            if isinstance(m, nn.Conv2d):
                w = m.weight.detach().to(device)
                b = m.bias.detach().to(device, F32)
                if name.endswith("conv_in") and w.shape[1] < cin_pad:
                    w = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, cin_pad - w.shape[1]))
                if w.shape[0] < cin_pad:  # decoder.conv_out: 3 output channels padded to 8 (sliced after)
                    w = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, 0, 0, cin_pad - w.shape[0]))
                    b = torch.nn.functional.pad(b, (0, cin_pad - b.shape[0]))
                self.w[name] = w.permute(0, 2, 3, 1).contiguous().to(dtype)
                self.b[name] = b.contiguous()
        for name, m in vae.named_modules():
            if isinstance(m, AttnBlock):
                self.w[name + ".qkv"] = torch.cat([self.w[name + ".q"], self.w[name + ".k"], self.w[name + ".v"]])
                self.b[name + ".qkv"] = torch.cat([self.b[name + ".q"], self.b[name + ".k"], self.b[name + ".v"]])


class AutoencoderKL(nn.Module):
    CIN_PAD = 8  # RGB padded to 8 channels so every conv has 16-B channel chunks

    def __init__(self, autoencoder_path=None, ddconfig=None, use_variational=True, output_dir=None, **kwargs):
        super().__init__()
        get = (lambda k, d: getattr(ddconfig, k, d) if not isinstance(ddconfig, dict) else ddconfig.get(k, d))
        embed_dim = get("vae_embed_dim", 16)
        ch_mult = tuple(get("ch_mult", (1, 1, 2, 2, 4)))
        self.encoder = Encoder(ch_mult=ch_mult, z_channels=embed_dim)
        self.use_variational = use_variational
        self.quant_conv = nn.Conv2d(2 * embed_dim, (2 if use_variational else 1) * embed_dim, 1)
        self.decoder = Decoder(ch_mult=ch_mult, z_channels=embed_dim)
        self.post_quant_conv = nn.Conv2d(embed_dim, embed_dim, 1)
        self.embed_dim = embed_dim
        self._prep = None
        if autoencoder_path is not None and os.path.exists(autoencoder_path):
            self.init_from_ckpt(autoencoder_path)

    def init_from_ckpt(self, path):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        sd = sd.get("model", sd)
        self.load_state_dict(sd, strict=False)
        self._prep = None

    def _prepared(self, device):
        key = (cdt(), str(device))
        if self._prep is None or self._prep[0] != key:
            self._prep = (key, _Prepared(self, cdt(), device, self.CIN_PAD))
        return self._prep[1]

    # ---- HIP forward pieces --------------------------------------------------------------
    # A GroupNorm'd tensor travels as (tensor, stats) where stats are the fused per-tile partial
    # sums written by the producing conv's epilogue (bf16 MFMA path) or None (computed by a
    # separate pass: fp32 parity path).
    def _fused(self):
        return cdt() == torch.bfloat16

    def _gn_in_conv(self, n, H, W, ci, co):
        return (self._fused() and RT.vae_gn_in_conv and
                ops.conv_fuses_gn(n, H, W, ci, co, 3, 1, torch.bfloat16))

    def _gn(self, x, stats, norm, n, hw, c):
        sc = torch.empty(n, c, dtype=F32, device=x.device)
        sh = torch.empty(n, c, dtype=F32, device=x.device)
        if stats is not None:
            ops.groupnorm_finalize_tiles(stats, n, hw, c, norm.weight.detach(), norm.bias.detach(), sc, sh,
                                         eps=norm.eps)
        else:
            ops.groupnorm_stats(x, n, hw, c, norm.weight.detach(), norm.bias.detach(), sc, sh, eps=norm.eps)
        return sc, sh

    def _norm_act(self, x, stats, norm, n, hw, c, silu=True, in_conv=False):
        """GN(+SiLU) applied ONCE per element (fused path) -> (input for the next conv, prologue or None).
        in_conv: the consuming conv applies the prologue while staging its input tile (halo kernel)."""
        g = self._gn(x, stats, norm, n, hw, c)
        if not self._fused() or in_conv:
            return x, g  # fp32 path: apply inside the conv A-loader; halo path: inside the halo staging
        y = torch.empty_like(x)
        ops.groupnorm_apply(x, g[0], g[1], y, n, hw, c, silu)
        return y, None

    def _conv(self, P, name, x, n, H, W, stride=1, gn=None, gn_silu=True, residual=None, stats=False):
        w = P.w[name]
        Co, ks, Ci = w.shape[0], w.shape[1], w.shape[3]
        if ks == 3 and stride == 1:
            pad, Ho, Wo = 1, H, W
        elif ks == 3:
            pad, Ho, Wo = 0, H // 2, W // 2  # F.pad(0,1,0,1) then stride-2 conv (vaekl.py:47-50)
        else:
            pad, Ho, Wo = 0, H, W
        out = torch.empty(n, Ho, Wo, Co, dtype=x.dtype, device=x.device)
        if ks == 1 and gn is None and residual is None and not stats and self._fused():
            # plain 1x1 conv (nin_shortcut): a bias-only GEMM -> the tuned library/kernel route
            ops.linear(x.reshape(-1, Ci), w.reshape(Co, Ci), out.reshape(-1, Co), bias=P.b[name])
            return out, Ho, Wo, None
        part = None
        if stats and self._fused() and (Ho * Wo) % 128 == 0 and Co % 32 == 0:
            part = torch.empty(n * Ho * Wo // 128, 32, 2, dtype=F32, device=x.device)
        ops.conv2d(x, w, out, n, H, W, Ci, Co, ks, stride, pad, pad, Ho, Wo, bias=P.b[name], residual=residual,
                   gn_scale=None if gn is None else gn[0], gn_shift=None if gn is None else gn[1], gn_silu=gn_silu,
                   gn_part=part)
        return out, Ho, Wo, part

    def _resblock(self, P, name, blk, x, xs_stats, n, H, W):
        c_in, c_out = blk.in_channels, blk.out_channels
        # GN+SiLU either inside the halo conv's input staging (in_conv: no separate apply pass; with
        # two co-resident workgroups per CU that VALU work runs under the other tile's MFMAs) or as
        # one vectorised apply pass per element (RT.vae_gn_in_conv = False)
        f1 = self._gn_in_conv(n, H, W, c_in, c_out)
        a, g1 = self._norm_act(x, xs_stats, blk.norm1, n, H * W, c_in, in_conv=f1)
        h, _, _, hs = self._conv(P, name + ".conv1", a, n, H, W, gn=g1, stats=True)
        f2 = self._gn_in_conv(n, H, W, c_out, c_out)
        a2, g2 = self._norm_act(h, hs, blk.norm2, n, H * W, c_out, in_conv=f2)
        xs = self._conv(P, name + ".nin_shortcut", x, n, H, W)[0] if c_in != c_out else x
        out, _, _, os_ = self._conv(P, name + ".conv2", a2, n, H, W, gn=g2, residual=xs, stats=True)
        return out, os_

    def _attn(self, P, name, blk, x, xs_stats, n, H, W):
        C = x.shape[-1]
        L = H * W
        g = self._gn(x, xs_stats, blk.norm, n, L, C)
        if self._fused():
            # one GN-apply pass, then the 1x1 conv as a plain LDS-DMA GEMM (a GN prologue forces the
            # register-staged kernel: 235 TFLOP/s at this shape)
            xn = torch.empty_like(x)
            ops.groupnorm_apply(x, g[0], g[1], xn, n, L, C, False)
            qkv = self._conv(P, name + ".qkv", xn, n, H, W)[0]  # [n, H, W, 3C]
        else:
            qkv = self._conv(P, name + ".qkv", x, n, H, W, gn=g, gn_silu=False)[0]
        q = qkv.reshape(n * L, 3 * C)
        S = torch.empty(n, L, L, dtype=x.dtype, device=x.device)
        ops.gemm(q, q[:, C:], S, L, L, C, 3 * C, 3 * C, L, 0, 0, batch=n, sA=(L * 3 * C, 0), sB=(L * 3 * C, 0),
                 sC=(L * L, 0))
        Pm = torch.empty_like(S)
        ops.softmax_fwd(S, Pm, None, L, float(C) ** -0.5)
        O = torch.empty(n * L, C, dtype=x.dtype, device=x.device)
        ops.gemm(Pm, q[:, 2 * C:], O, L, C, L, L, 3 * C, C, 0, 1, batch=n, sA=(L * L, 0), sB=(L * 3 * C, 0),
                 sC=(L * C, 0))
        out, _, _, os_ = self._conv(P, name + ".proj_out", O.reshape(n, H, W, C), n, H, W, residual=x, stats=True)
        return out, os_

    @torch.no_grad()
    def moments_nhwc(self, x):
        """x: NHWC [n, 256, 256, CIN_PAD] in the compute dtype -> moments NHWC [n, 16, 16, 2*embed]."""
        P = self._prepared(x.device)
        e = self.encoder
        n, H, W, _ = x.shape
        h, H, W, hs = self._conv(P, "encoder.conv_in", x, n, H, W, stats=True)
        for lvl, d in enumerate(e.down):
            RT.fire_attn_prefetch(lvl)  # the MAR's attention keep-mask planes, armed by the policy
            for j, blk in enumerate(d.block):
                h, hs = self._resblock(P, f"encoder.down.{lvl}.block.{j}", blk, h, hs, n, H, W)
                if len(d.attn):
                    h, hs = self._attn(P, f"encoder.down.{lvl}.attn.{j}", d.attn[j], h, hs, n, H, W)
            if hasattr(d, "downsample"):
                h, H, W, hs = self._conv(P, f"encoder.down.{lvl}.downsample.conv", h, n, H, W, stride=2, stats=True)
        RT.fire_attn_prefetch()
        h, hs = self._resblock(P, "encoder.mid.block_1", e.mid.block_1, h, hs, n, H, W)
        h, hs = self._attn(P, "encoder.mid.attn_1", e.mid.attn_1, h, hs, n, H, W)
        h, hs = self._resblock(P, "encoder.mid.block_2", e.mid.block_2, h, hs, n, H, W)
        a, g = self._norm_act(h, hs, e.norm_out, n, H * W, h.shape[-1])
        h, H, W, _ = self._conv(P, "encoder.conv_out", a, n, H, W, gn=g)
        return self._conv(P, "quant_conv", h, n, H, W)[0]

    @torch.no_grad()
    def encode_tokens(self, x, eps, scale=0.2325):
        """NHWC images -> latent tokens [n, 256, embed] fp32 = (mean + std*eps)*scale
        (DiagonalGaussianDistribution.sample + data_utils.py:396).  eps: NCHW [n, embed, 16, 16]."""
        mom = self.moments_nhwc(x)
        n = x.shape[0]
        z = torch.empty(n, 256, self.embed_dim, dtype=F32, device=x.device)
        ops.posterior_sample(mom, eps.contiguous().float(), z, n, scale)
        return z

    @torch.no_grad()
    def decode_nhwc(self, z):
        """z NHWC [n, 16, 16, embed] (compute dtype) -> images NHWC [n, 256, 256, CIN_PAD] (3 used)."""
        P = self._prepared(z.device)
        d = self.decoder
        n, H, W, _ = z.shape
        h = self._conv(P, "post_quant_conv", z, n, H, W)[0]
        h, H, W, hs = self._conv(P, "decoder.conv_in", h, n, H, W, stats=True)
        h, hs = self._resblock(P, "decoder.mid.block_1", d.mid.block_1, h, hs, n, H, W)
        h, hs = self._attn(P, "decoder.mid.attn_1", d.mid.attn_1, h, hs, n, H, W)
        h, hs = self._resblock(P, "decoder.mid.block_2", d.mid.block_2, h, hs, n, H, W)
        for lvl in reversed(range(d.num_resolutions)):
            u = d.up[lvl]
            for j, blk in enumerate(u.block):
                h, hs = self._resblock(P, f"decoder.up.{lvl}.block.{j}", blk, h, hs, n, H, W)
            if hasattr(u, "upsample"):
                hu = torch.empty(n, 2 * H, 2 * W, h.shape[-1], dtype=h.dtype, device=h.device)
                ops.upsample_nearest2x(h, hu)
                H, W = 2 * H, 2 * W
                h, _, _, hs = self._conv(P, f"decoder.up.{lvl}.upsample.conv", hu, n, H, W, stats=True)
        a, g = self._norm_act(h, hs, d.norm_out, n, H * W, h.shape[-1])
        return self._conv(P, "decoder.conv_out", a, n, H, W, gn=g)[0]

    @torch.no_grad()
    def decode(self, z):
        """AutoencoderKL.decode (vaekl.py:56-58): z NCHW [n, embed, 16, 16] -> images NCHW fp32 [n, 3, 256, 256]."""
        zz = z.permute(0, 2, 3, 1).contiguous().to(cdt())
        out = self.decode_nhwc(zz)
        return out[..., :3].permute(0, 3, 1, 2).float().contiguous()
