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
