"""The off-config action trunks of DiffActLoss (act_model_type conv_ori / conv2 / fc2,
diffusion_action_loss.py:63-89, 125-141 of the reference; no shipped config selects them) against the
reference's own run (tests/golden/make_golden.py gen_act_trunks -> g3_act_trunks.npz): hash-initialised
weights, z [2, 1024, 64], target [2, 16, 2], injected t / noise.

fp32 mode: loss within 1e-4 relative, dL/dz rows within 1e-3 of their max, every parameter-gradient
checksum within 3e-3 (replay.grad_rel_errors, as the MAR parity cases).  bf16 mode (bf16 GEMM
operands): loss within 3e-2 relative, dL/dz rows within 6e-2 of their max (conv2's dL/dz crosses two
bf16 contractions of 7168 / 1792 terms and a ReLU whose mask bf16 rounding flips: 4.7e-2 measured)."""
import numpy as np
import pytest
import torch

import cases
import replay
from hashinit import hash_init_, hash_normal

pytestmark = pytest.mark.gpu
DEV = "cuda"
KINDS = ("conv_ori", "conv2", "fc2")


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("kind", KINDS)
def test_action_trunk_vs_reference(kind, prec):
    from unified_video_action_amd.model.autoregressive.diffusion_action_loss import DiffActLoss
    from unified_video_action_amd.runtime import RT
    RT.set_precision(prec)
    try:
        g = replay.load("g3_act_trunks.npz")
        m = DiffActLoss(2, 64, 2, 64, "100", n_frames=4, act_model_type=kind)
        hash_init_(m, f"act_{kind}.")
        m = m.to(DEV).train()
        z = torch.from_numpy(hash_normal(f"act_{kind}/z", (2, 1024, 64))).to(DEV).requires_grad_(True)
        target = torch.from_numpy(hash_normal(f"act_{kind}/target", (2, 16, 2))).to(DEV)
        t = torch.from_numpy(cases.t_steps(f"act_{kind}", 32)).to(DEV)
        noise = torch.from_numpy(hash_normal(f"act_{kind}/noise", (32, 2))).to(DEV)
        loss = m(target, z, t=t, noise=noise)
        loss.backward()
        want = float(g[f"{kind}_loss"][0])
        tol = 1e-4 if prec == "fp32" else 3e-2
        assert abs(loss.item() - want) <= tol * abs(want), (loss.item(), want)
        gz = z.grad[:, ::64].detach().cpu().numpy()
        ref = g[f"{kind}_gz_rows"]
        assert np.abs(gz - ref).max() <= (1e-3 if prec == "fp32" else 6e-2) * np.abs(ref).max()
        if prec == "fp32":
            errs = replay.grad_rel_errors(m.named_parameters(), g, f"{kind}_gnames", f"{kind}_gsums",
                                          f"{kind}_gheads")
            assert max(errs.values()) < 3e-3, max(errs.items(), key=lambda kv: kv[1])
    finally:
        RT.set_precision("bf16")


@pytest.mark.parametrize("kind", KINDS)
def test_action_trunk_sample_shapes(kind):
    """sample() runs the same trunk, then the spaced reverse loop: [B, 16, C] action latents."""
    from unified_video_action_amd.model.autoregressive.diffusion_action_loss import DiffActLoss
    m = DiffActLoss(2, 64, 2, 64, "10", n_frames=4, act_model_type=kind, act_diff_testing_steps="10")
    hash_init_(m, f"act_{kind}.")
    m = m.to(DEV).eval()
    z = torch.from_numpy(hash_normal(f"act_{kind}/z", (2, 1024, 64))).to(DEV)
    x = m.sample(z)
    assert x.shape == (2, 16, 2) and torch.isfinite(x).all()
