"""PushT device augmentation (utils/augment.py, dataset/pusht_image_dataset.py:93-130): parameter
draws, the torch restatement's own invariants (CPU) and the HIP kernel against it (GPU).
torchvision is absent here: parity with torchvision itself is unpinned (documented)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import uva_oracle as O


def test_aug_params_draws():
    from unified_video_action_amd.utils.augment import CROP, FRAME, gaussian_kernel1d, pusht_aug_params
    p = pusht_aug_params(range(400))
    assert p.shape == (400, 9)
    crop, blur = p[:, 0] == 1, p[:, 3] == 1
    assert 0.4 < crop.float().mean() < 0.6 and 0.4 < blur.float().mean() < 0.6  # p = 0.5 each
    assert (p[crop, 1:3] >= 0).all() and (p[crop, 1:3] <= FRAME - CROP).all()
    torch.testing.assert_close(p[blur, 4:].sum(1), torch.ones(int(blur.sum())))
    assert torch.equal(pusht_aug_params([7]), pusht_aug_params([7]))  # one seed -> one draw sequence
    k = gaussian_kernel1d(1.0)
    assert torch.allclose(k, k.flip(0)) and k.argmax() == 2


def test_oracle_augment_identity_and_upscale():
    """no crop / no blur is the identity; antialiased 91->96 upscaling equals plain bilinear (the
    kernel's formulation)."""
    x = torch.rand(2, 3, 3, 96, 96)
    assert torch.equal(O.pusht_augment(x, torch.zeros(2, 9)), x)
    c = torch.rand(3, 3, 91, 91)
    a = F.interpolate(c, size=(96, 96), mode="bilinear", align_corners=False, antialias=True)
    b = F.interpolate(c, size=(96, 96), mode="bilinear", align_corners=False)
    assert (a - b).abs().max().item() < 1e-6


@pytest.mark.gpu
def test_pusht_augment_kernel_vs_oracle():
    from unified_video_action_amd.utils.augment import pusht_aug_params, pusht_augment
    g = torch.Generator().manual_seed(0)
    x = torch.rand(12, 4, 3, 96, 96, generator=g)
    params = pusht_aug_params(range(100, 112))
    params[0, :4] = torch.tensor([1.0, 0.0, 5.0, 1.0])  # crop at the window limits + blur
    params[0, 4:] = torch.tensor([0.1, 0.2, 0.4, 0.2, 0.1])
    params[1, :4] = torch.tensor([1.0, 5.0, 0.0, 0.0])
    params[2, :4] = torch.tensor([0.0, 0.0, 0.0, 1.0])
    params[2, 4:] = torch.tensor([0.0, 0.0, 1.0, 0.0, 0.0])
    got = pusht_augment(x.cuda(), params=params).cpu()
    want = O.pusht_augment(x, params)
    torch.testing.assert_close(got, want, rtol=0, atol=2e-6)
    assert torch.equal(got[2], x[2])  # delta blur kernel, no crop


# ---- UMI (kornia 0.8 chain, umi_lazy.yaml:50-72) and Libero (torchvision ColorJitter) ----------

def _umi_cases(B, seed0=300):
    """drawn rows plus forced rows: every op on, contrast at each jitter position, crop at the
    window limits, each op alone."""
    from unified_video_action_amd.utils.augment import gaussian_kernel1d, umi_aug_params
    p = umi_aug_params(range(seed0, seed0 + B))
    allon = torch.tensor([1, 16, 0, 1, 2, 1, 3, 0, 1.2, 0.7, 1.4, 0.4, 1, 1.7, 1, 1, 1] + [0] * 5 + [0, 208.0])
    allon[17:22] = gaussian_kernel1d(1.3)
    p[0] = allon
    for k in range(1, min(B, 5)):
        p[k] = allon.clone()
        order = [0, 2, 3]
        order.insert(k - 1, 1)  # contrast at position k-1
        p[k, 4:8] = torch.tensor(order, dtype=torch.float32)
        p[k, 11] = -0.45
        p[k, 15] = 0.0
    if B > 5:
        p[5, :3] = torch.tensor([1.0, 0.0, 16.0])
        p[5, 3] = 0.0
    return p


def test_umi_params_draws():
    from unified_video_action_amd.utils.augment import AUG_NP, UMI_CROP, UMI_FRAME, umi_aug_params
    p = umi_aug_params(range(2000))
    assert p.shape == (2000, AUG_NP)
    rate = lambda col: (p[:, col] != 0).float().mean().item()  # noqa: E731
    assert abs(rate(0) - 0.5) < 0.05 and abs(rate(3) - 0.8) < 0.05 and abs(rate(12) - 0.5) < 0.05
    assert abs(rate(14) - 0.5) < 0.05 and abs(rate(15) - 0.2) < 0.05 and abs(rate(16) - 0.5) < 0.05
    crop = p[:, 0] == 1
    assert (p[crop, 1:3] >= 0).all() and (p[crop, 1:3] <= UMI_FRAME - UMI_CROP).all()
    jit = p[:, 3] == 1
    assert torch.equal(p[jit, 4:8].sort(1).values, torch.arange(4.0).expand(int(jit.sum()), 4))
    for col, lo, hi in ((8, 0.7, 1.3), (9, 0.6, 1.4), (10, 0.5, 1.5), (11, -0.08 * 2 * np.pi, 0.08 * 2 * np.pi)):
        assert p[jit, col].min() >= lo - 1e-6 and p[jit, col].max() <= hi + 1e-6
    sh = p[:, 12] == 1
    assert p[sh, 13].min() >= 0 and p[sh, 13].max() <= 2
    bl = p[:, 16] == 1
    torch.testing.assert_close(p[bl, 17:22].sum(1), torch.ones(int(bl.sum())))
    assert torch.equal(umi_aug_params([5, 6]), umi_aug_params([5, 6]))


def test_libero_params_follow_torch_global_rng():
    """torch.manual_seed(video_seed) + ColorJitter.get_params draw order (randperm, b, c, s, h)."""
    from unified_video_action_amd.utils.augment import libero_jitter_params
    for seed in (0, 7, 9999):
        torch.manual_seed(seed)
        order = torch.randperm(4).float()
        f = [float(torch.empty(1).uniform_(0.8, 1.2)) for _ in range(3)] + [float(torch.empty(1).uniform_(-0.05, 0.05))]
        row = libero_jitter_params([seed])[0]
        assert torch.equal(row[4:8], order) and row[8:12].tolist() == pytest.approx(f, abs=0)
        assert row[22] == 1 and row[3] == 1 and row[0] == 0


def test_oracle_video_augment_invariants():
    from unified_video_action_amd.utils.augment import AUG_NP
    g = torch.Generator().manual_seed(1)
    x = torch.rand(2, 3, 3, 32, 32, generator=g)
    p = torch.zeros(2, AUG_NP)
    assert torch.equal(O.video_augment(x, p), x)  # nothing applied
    # the two HSV restatements round-trip and agree on a hue rotation (radians vs turns)
    f = x[0]
    torch.testing.assert_close(O._k_hsv2rgb(O._k_rgb2hsv(f)), f, atol=2e-6, rtol=0)
    torch.testing.assert_close(O._tv_hsv2rgb(O._tv_rgb2hsv(f)), f, atol=2e-6, rtol=0)
    a = O._jitter_op(f, 3, 0.3 * 2 * np.pi, tv=False)
    b = O._jitter_op(f, 3, 0.3, tv=True)
    torch.testing.assert_close(a, b, atol=1e-5, rtol=0)
    # grayscale: equal channels; autocontrast: each frame / channel spans [0, 1]
    p[0, 15] = 1
    p[1, 14] = 1
    y = O.video_augment(x, p)
    assert torch.equal(y[0, :, 0], y[0, :, 1]) and torch.equal(y[0, :, 1], y[0, :, 2])
    assert y[1].amin(dim=(-2, -1)).abs().max() < 1e-6 and (y[1].amax(dim=(-2, -1)) - 1).abs().max() < 1e-5
    # sharpness with factor 1 is the identity; blur with a delta kernel is the identity
    p.zero_()
    p[:, 12], p[:, 13] = 1, 1.0
    torch.testing.assert_close(O.video_augment(x, p), x, atol=0, rtol=0)
    p.zero_()
    p[:, 16], p[:, 19] = 1, 1.0
    torch.testing.assert_close(O.video_augment(x, p), x, atol=0, rtol=0)


def test_video_augment_rejects_bad_windows():
    from unified_video_action_amd.utils.augment import AUG_NP, video_augment
    x = torch.rand(1, 1, 3, 16, 16)
    p = torch.zeros(1, AUG_NP)
    p[0, :3] = torch.tensor([1.0, 4.0, 0.0])
    p[0, 23] = 14.0
    with pytest.raises(ValueError):
        video_augment(x, p)
    with pytest.raises(ValueError):
        video_augment(x, torch.zeros(2, AUG_NP))


@pytest.mark.gpu
def test_umi_video_augment_kernel_vs_oracle():
    from unified_video_action_amd.utils.augment import video_augment
    g = torch.Generator().manual_seed(2)
    x = torch.rand(10, 2, 3, 224, 224, generator=g)
    x[1, :, :, :40] = 1.0  # saturated rows: channel ties in the HSV sector choice
    params = _umi_cases(10)
    got = video_augment(x.cuda(), params).cpu()
    want = O.video_augment(x, params)
    err = (got - want).abs().amax(dim=(1, 2, 3, 4))
    assert err.max() < 2e-5, err


@pytest.mark.gpu
def test_libero_color_jitter_kernel_vs_oracle():
    from unified_video_action_amd.utils.augment import libero_jitter_params, video_augment
    g = torch.Generator().manual_seed(3)
    x = torch.rand(6, 3, 3, 128, 128, generator=g)
    x[0, :, :, :16, :16] = 0.5  # gray pixels: the r == g == b branch
    params = libero_jitter_params(range(40, 46))
    params[1, 11] = 0.0  # zero hue shift is skipped
    got = video_augment(x.cuda(), params).cpu()
    want = O.video_augment(x, params)
    err = (got - want).abs().amax(dim=(1, 2, 3, 4))
    assert err.max() < 2e-5, err


@pytest.mark.gpu
def test_augment_batch_dispatch_umi_libero():
    """augment_batch picks the owning dataset's chain from the obs image key."""
    from unified_video_action_amd.utils.augment import (augment_batch, libero_jitter_params, umi_aug_params,
                                                        video_augment)
    g = torch.Generator().manual_seed(4)
    umi = torch.rand(2, 8, 3, 224, 224, generator=g).cuda()
    lib = torch.rand(2, 4, 3, 128, 128, generator=g).cuda()
    out = augment_batch({"obs": {"camera0_rgb": umi.clone(), "robot0_eef_pos": torch.zeros(2, 8, 3)}}, seeds=[1, 2])
    torch.testing.assert_close(out["obs"]["camera0_rgb"], video_augment(umi, umi_aug_params([1, 2])), atol=0, rtol=0)
    out = augment_batch({"obs": {"agentview_rgb": lib.clone()}}, seeds=[3, 4])
    torch.testing.assert_close(out["obs"]["agentview_rgb"], video_augment(lib, libero_jitter_params([3, 4])),
                               atol=0, rtol=0)


def test_oracle_hue_matches_python_colorsys():
    """Both restated hue paths (kornia radians, torchvision turns) against an independent
    implementation of the same HSV model: Python's colorsys, per pixel in double precision."""
    import colorsys
    g = torch.Generator().manual_seed(5)
    x = torch.rand(1, 3, 8, 25, generator=g)
    x[0, :, 0, :5] = 0.25  # gray pixels (undefined hue: s = 0)
    x[0, 0, 1, :5] = x[0, 1, 1, :5]  # r == g ties
    for shift in (0.07, -0.31, 0.5):
        want = torch.empty_like(x)
        for i in range(8):
            for j in range(25):
                h, s, v = colorsys.rgb_to_hsv(*x[0, :, i, j].double().tolist())
                want[0, :, i, j] = torch.tensor(colorsys.hsv_to_rgb((h + shift) % 1.0, s, v))
        tv = O._jitter_op(x, 3, shift, tv=True)
        kn = O._jitter_op(x, 3, float(torch.tensor(shift) * 2 * np.pi), tv=False)
        torch.testing.assert_close(tv, want, atol=2e-6, rtol=0)
        torch.testing.assert_close(kn, want, atol=2e-6, rtol=0)


def test_oracle_sharpness_matches_pil_enhance():
    """kornia.enhance.sharpness follows PIL's ImageEnhance.Sharpness (SMOOTH 3x3 kernel
    (1,1,1;1,5,1;1,1,1)/13 on the interior, border pixels kept, then blended with the image);
    the restatement against PIL itself on 8-bit images.  PIL rounds the smoothed image to 8 bits
    and truncates the blend: (1 + |1 - f| / 2) / 255 tolerance; border pixels must match exactly
    (a wrong kernel or border rule is off by many 8-bit steps)."""
    from PIL import Image, ImageEnhance
    g = torch.Generator().manual_seed(6)
    u8 = (torch.rand(3, 20, 24, generator=g) * 255).round().to(torch.uint8)
    img = Image.fromarray(u8.permute(1, 2, 0).numpy(), "RGB")
    x = u8.float().unsqueeze(0) / 255.0
    for f in (0.0, 0.4, 1.0, 1.7):
        want = torch.from_numpy(np.array(ImageEnhance.Sharpness(img).enhance(f))).permute(2, 0, 1).float() / 255
        got = O._sharpness_k(x, f)[0]
        assert (got - want).abs().max().item() <= (1.0 + 0.5 * abs(1 - f)) / 255 + 1e-6, f
        for edge in (got[:, 0] - want[:, 0], got[:, -1] - want[:, -1], got[:, :, 0] - want[:, :, 0]):
            assert edge.abs().max().item() < 1e-6
