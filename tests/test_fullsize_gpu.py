"""The benched kernels pinned at production size (VERDICT r2 "What's weak" 1):

  * the KL-VAE encoder at the full per-GPU batch (config 2: n = 256 images = 32 samples x 8
    frames; UMI B = 56: n = 448), where the level-0 activation is 256 x 256 x 256 x 128 bf16 =
    2^32 bytes (7.5 GB at n = 448) -- the reference golden image g3_vae at slots {0, n/2, n-1} of a
    batch whose other slots hold distinct images: those slots' posterior moments match the
    reference within the bf16 tolerance of test_parity_gpu (5e-2 of max) and equal each other
    bit for bit (64-bit offsets / per-image descriptors of the halo conv, GN statistics per image);
  * the full-width model end to end: mar_base (D 768, 12 + 12 Blocks, DiffLoss 1024 x 6) with the
    full VAE through UnifiedVideoActionPolicy.compute_loss at BASELINE configs[0]'s workload (PushT,
    B = 2, video_model) and the joint model's full_dynamic_model mode, fp32 (exact-f32 VALU GEMMs,
    materialised attention), against the oracle's CPU restatement of the same weights and draws:
    loss within 1e-4 relative, every parameter gradient checksum within 3e-3 (reference:
    policy/unified_video_action_policy.py:362-425, vae/vaekl.py:246-273)."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
HERE = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(HERE, "golden"), os.path.join(os.path.dirname(HERE), "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import cases  # noqa: E402
import replay  # noqa: E402
from hashinit import hash_init_, hash_tensor  # noqa: E402


def _precision(name):
    from unified_video_action_amd.runtime import RT
    RT.set_precision(name)


def _nhwc8(x):
    """[n, 3, H, W] in [-1, 1] -> the VAE's NHWC input padded to 8 channels"""
    n, c, h, w = x.shape
    out = torch.zeros(n, h, w, 8, device=x.device, dtype=x.dtype)
    out[..., :c] = x.permute(0, 2, 3, 1)
    return out


@pytest.mark.parametrize("n", [256, 448])
def test_vae_encoder_full_batch_production_grid(n):
    from unified_video_action_amd.vae.vaekl import AutoencoderKL
    _precision("bf16")
    g = replay.load("g3_vae.npz")
    vae = AutoencoderKL(ddconfig=dict(vae_embed_dim=16, ch_mult=[1, 1, 2, 2, 4]))
    hash_init_(vae, "vae.")
    vae = vae.to(DEV)
    ref_img = torch.from_numpy(hash_tensor("vae/x", (1, 3, 256, 256))).to(DEV)
    gen = torch.Generator(device=DEV).manual_seed(1234)
    x = torch.rand(n, 3, 256, 256, device=DEV, generator=gen) * 2 - 1
    slots = (0, n // 2, n - 1)
    for s in slots:
        x[s] = ref_img[0]
    xin = _nhwc8(x).to(torch.bfloat16)
    del x
    with torch.no_grad():
        mom = vae.moments_nhwc(xin)  # [n, 16, 16, 32]
    torch.cuda.synchronize()
    assert torch.isfinite(mom).all()
    got = mom[list(slots)].float().permute(0, 3, 1, 2).cpu().numpy()
    ref = g["moments"][0]
    for i, s in enumerate(slots):
        err = np.abs(got[i] - ref).max()
        assert err <= 5e-2 * np.abs(ref).max(), (s, err)
        assert np.array_equal(got[i], got[0]), f"slot {s} differs from slot 0"
    # the other slots are different images: their moments differ from the reference image's
    assert not torch.equal(mom[1], mom[0])


def _full_policy(config, mode):
    from unified_video_action_amd import presets
    from unified_video_action_amd.policy.unified_video_action_policy import UnifiedVideoActionPolicy
    kw = presets.policy_kwargs(config, autoregressive_model_params=dict(attn_dropout=0.0, proj_dropout=0.0),
                               selected_training_mode=mode)
    pol = UnifiedVideoActionPolicy(**kw)
    hash_init_(pol.vae_model, "vae.")
    hash_init_(pol.model, "mar.")
    pol = pol.to(DEV).train()
    presets.fit_normalizer(config, pol)
    return pol


@pytest.mark.timeout(600)
@pytest.mark.parametrize("config,mode", [("pusht_video", "video_model"), ("pusht_joint", "full_dynamic_model")])
def test_mar_base_full_vae_fp32_vs_oracle(config, mode):
    import uva_oracle as O
    _precision("fp32")
    try:
        B = 2
        pol = _full_policy(config, mode)
        predict_action = config == "pusht_joint"
        b = cases.policy_batch(B)
        rng = cases.policy_rng(mode, B)
        rng["task_mode"] = mode
        batch = replay.device_batch(b, DEV)
        for p in pol.model.parameters():
            p.grad = torch.zeros_like(p)
        loss, (lv, la) = pol.compute_loss(batch, rng=rng)
        loss.backward()
        torch.cuda.synchronize()

        torch.set_num_threads(min(16, os.cpu_count() or 1))
        mar = O.mar_base(vae_embed_dim=16, diffloss_d=6, diffloss_w=1024, diffloss_act_d=6, diffloss_act_w=1024,
                         task_name="pusht", act_dim=2, predict_action=predict_action)
        hash_init_(mar, "mar.")
        vae = O.AutoencoderKLEncoder()
        hash_init_(vae, "vae.")
        opol = O.PolicyOracle(mar, vae, [2 / 512, 2 / 512], [-1.0, -1.0])
        oloss, (olv, ola) = opol.compute_loss(torch.from_numpy(b["image"]), torch.from_numpy(b["action"]), mode, rng)
        oloss.backward()
        for got, want in zip((loss.item(), float(lv), float(la)), (oloss.item(), float(olv), float(ola))):
            assert abs(got - want) <= 1e-4 * max(abs(want), 1e-6), (got, want)
        ours = dict(pol.model.named_parameters())
        worst = (None, 0.0)
        n_cmp = 0
        for name, p in mar.named_parameters():
            if p.grad is None:
                continue
            assert name in ours, name
            a = ours[name].grad.detach().double().cpu().reshape(-1)
            r = p.grad.detach().double().reshape(-1)
            scale = max(r.pow(2).mean().sqrt().item(), 1e-12)
            e_sum = abs(a.sum().item() - r.sum().item()) / (scale * np.sqrt(r.numel()))
            e_sq = abs(a.pow(2).sum().item() - r.pow(2).sum().item()) / (r.pow(2).sum().item() + 1e-30)
            e = max(e_sum, e_sq)
            n_cmp += 1
            if e > worst[1]:
                worst = (name, e)
        assert n_cmp > 300, n_cmp
        assert worst[1] < 3e-3, worst
    finally:
        _precision("bf16")
