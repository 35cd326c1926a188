"""The reference's own shipped fixtures, extracted WITHOUT unpickling by
tests/golden/extract_ref_fixtures.py into tests/golden/ref_fixtures.npz:

  G5  uva_human_pp_video_act_model/normalizer.pkl -- a LinearNormalizer fitted by the reference
      (normalizer.py:195-280, "limits" mode) on real robot data: the stored (input_stats -> scale,
      offset) pairs pin this build's fit arithmetic, and normalize / unnormalize are checked on
      its stats; plus the normalizer.py:300 test() known-answer checks, restated.
  G6  prepared_data/language_latents.pkl -- the cup / towel / mouse CLIP latents; they are the
      text latents of the Libero / UMI policy goldens (cases.policy_variant_batch, g2_policy_variants)
      and are checked here for shape, dtype and the regeneration of those goldens' inputs."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.dirname(HERE))

from unified_video_action_amd.model.common.normalizer import (LinearNormalizer,  # noqa: E402
                                                              SingleFieldLinearNormalizer)

FIX = np.load(os.path.join(HERE, "golden", "ref_fixtures.npz"))
FIELDS = ("action", "agent_pos", "image")


def _field(name):
    g = lambda k: torch.from_numpy(FIX[f"normalizer/{name}/{k}"])  # noqa: E731
    return {"scale": g("scale"), "offset": g("offset"),
            "stats": {s: g(f"input_stats/{s}") for s in ("min", "max", "mean", "std")}}


@pytest.mark.parametrize("name", FIELDS)
def test_normalizer_pkl_fit_arithmetic(name):
    """The reference stored scale / offset as its "limits" fit of input_stats min / max: this build's
    fit of data with exactly those per-dimension extremes reproduces them (float32, 2 ulp)."""
    f = _field(name)
    lo, hi = f["stats"]["min"], f["stats"]["max"]
    data = torch.stack([lo, hi, 0.5 * (lo + hi)])  # the extremes (and an interior row)
    n = LinearNormalizer()
    n.fit({name: data}, mode="limits")
    p = n.params_dict[name]
    torch.testing.assert_close(p["scale"], f["scale"], rtol=2.5e-7, atol=0)
    torch.testing.assert_close(p["offset"], f["offset"], rtol=2.5e-7, atol=2.5e-7)
    torch.testing.assert_close(p["input_stats"]["min"], lo, rtol=0, atol=0)
    torch.testing.assert_close(p["input_stats"]["max"], hi, rtol=0, atol=0)


@pytest.mark.parametrize("name", FIELDS)
def test_normalizer_pkl_normalize_roundtrip(name):
    """normalize maps the reference's recorded min / max to -1 / +1 per dimension (constant dims to
    0), unnormalize inverts it; the policy's state-dict path (params_dict.<key>.*) loads it."""
    f = _field(name)
    sd = {f"params_dict.{name}.scale": f["scale"], f"params_dict.{name}.offset": f["offset"]}
    sd.update({f"params_dict.{name}.input_stats.{k}": v for k, v in f["stats"].items()})
    n = LinearNormalizer()
    n.load_state_dict(sd)
    lo, hi = f["stats"]["min"], f["stats"]["max"]
    const = (hi - lo) < 1e-4
    x = torch.stack([lo, hi])
    y = n.normalize({name: x})[name]
    want_lo = torch.where(const, torch.zeros_like(lo), -torch.ones_like(lo))
    want_hi = torch.where(const, torch.zeros_like(hi), torch.ones_like(hi))
    torch.testing.assert_close(y[0], want_lo, rtol=0, atol=2e-6)
    torch.testing.assert_close(y[1], want_hi, rtol=0, atol=2e-6)
    g = torch.Generator().manual_seed(7)
    xs = lo + (hi - lo) * torch.rand(64, lo.numel(), generator=g)
    back = n[name].unnormalize(n[name].normalize(xs))
    torch.testing.assert_close(back, xs, rtol=0, atol=2e-6)
    # reference's recorded output range of its own stats (get_output_stats of min / max)
    out = n.get_output_stats()
    assert set(out) == {name} and set(out[name]) == {"min", "max", "mean", "std"}


def test_normalizer_reference_test_kat():
    """normalizer.py:300 test(), restated: SingleField limits (last_n_dims 2), limits without
    offset (last_n_dims 1), gaussian (last_n_dims 0), dict fit + state-dict round trip."""
    torch.manual_seed(0)
    data = torch.zeros((100, 10, 9, 2)).uniform_()
    data[..., 0, 0] = 0
    n = SingleFieldLinearNormalizer()
    n.fit(data, mode="limits", last_n_dims=2)
    dn = n.normalize(data)
    assert dn.shape == data.shape
    assert np.allclose(dn.max(), 1.0) and np.allclose(dn.min(), -1.0)
    assert torch.allclose(data, n.unnormalize(dn), atol=1e-7)
    n.get_input_stats()
    n.get_output_stats()

    n = SingleFieldLinearNormalizer()
    n.fit(data, mode="limits", last_n_dims=1, fit_offset=False)
    dn = n.normalize(data)
    assert dn.shape == data.shape
    assert np.allclose(dn.max(), 1.0, atol=1e-3) and np.allclose(dn.min(), 0.0, atol=1e-3)
    assert torch.allclose(data, n.unnormalize(dn), atol=1e-7)

    data = torch.zeros((100, 10, 9, 2)).uniform_()
    n = SingleFieldLinearNormalizer()
    n.fit(data, mode="gaussian", last_n_dims=0)
    dn = n.normalize(data)
    assert dn.shape == data.shape
    assert np.allclose(dn.mean(), 0.0, atol=1e-3) and np.allclose(dn.std(), 1.0, atol=1e-3)
    assert torch.allclose(data, n.unnormalize(dn), atol=1e-7)

    data = torch.zeros((100, 10, 9, 2)).uniform_()
    data[..., 0, 0] = 0
    n = LinearNormalizer()
    n.fit(data, mode="limits", last_n_dims=2)
    dn = n.normalize(data)
    assert dn.shape == data.shape
    assert np.allclose(dn.max(), 1.0) and np.allclose(dn.min(), -1.0)
    assert torch.allclose(data, n.unnormalize(dn), atol=1e-7)
    n.get_input_stats()
    n.get_output_stats()

    data = {"obs": torch.zeros((1000, 128, 9, 2)).uniform_() * 512,
            "action": torch.zeros((1000, 128, 2)).uniform_() * 512}
    n = LinearNormalizer()
    n.fit(data)
    back = n.unnormalize(n.normalize(data))
    for k in data:
        assert torch.allclose(data[k], back[k], atol=1e-4)
    n.get_input_stats()
    n.get_output_stats()
    m = LinearNormalizer()
    m.load_state_dict(n.state_dict())
    back = m.unnormalize(m.normalize(data))
    for k in data:
        assert torch.allclose(data[k], back[k], atol=1e-4)


def test_language_latents_fixture():
    """G6: three float32[512] CLIP latents, finite and distinct; they are the policy goldens' text."""
    import cases
    lat = {k: FIX[f"language_latents/{k}"] for k in ("cup", "towel", "mouse")}
    for k, v in lat.items():
        assert v.dtype == np.float32 and v.shape == (512,) and np.isfinite(v).all(), k
    assert not np.allclose(lat["cup"], lat["towel"]) and not np.allclose(lat["towel"], lat["mouse"])
    b = cases.policy_variant_batch("libero")
    np.testing.assert_array_equal(b["language_latents"][0], lat["cup"])
    b = cases.policy_variant_batch("umi")
    np.testing.assert_array_equal(b["language_latents"][0], lat["towel"])
