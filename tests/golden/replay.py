"""Helpers that rebuild golden cases (weights + inputs + injected RNG) for the oracle
and for the HIP path, and compare results with the committed fixtures."""
import os

import numpy as np
import torch

import cases
from hashinit import hash_init_, hash_normal, hash_tensor

GOLDEN = os.path.dirname(os.path.abspath(__file__))


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def checksum(t):
    a = t.detach().double().reshape(-1).cpu()
    return np.array([a.sum().item(), (a * a).sum().item(), a.abs().max().item()], np.float64)


def mar_ctor_kwargs(variant):
    v = cases.variant_def(variant)
    m = cases.MAR_GOLDEN
    return dict(
        encoder_embed_dim=m["encoder_embed_dim"], encoder_depth=m["encoder_depth"],
        encoder_num_heads=m["encoder_num_heads"], decoder_embed_dim=m["decoder_embed_dim"],
        decoder_depth=m["decoder_depth"], decoder_num_heads=m["decoder_num_heads"],
        mlp_ratio=m["mlp_ratio"], vae_embed_dim=16, diffloss_d=cases.MAR_KW["diffloss_d"],
        diffloss_w=cases.MAR_KW["diffloss_w"], diffloss_act_d=cases.MAR_KW["diffloss_act_d"],
        diffloss_act_w=cases.MAR_KW["diffloss_act_w"], task_name=v["task_name"],
        act_dim=v["Da"], predict_action=True, use_proprioception=v["use_proprioception"],
        predict_proprioception=v["predict_proprioception"],
        different_history_freq=v["different_history_freq"],
        use_history_action=v.get("use_history_action", False), predict_wrist_img=v.get("predict_wrist_img", False),
        action_mask_ratio=cases.MAR_KW["action_mask_ratio"],
        language_emb_model="clip" if v["clip"] else None)


def mar_case(variant, mode, device="cpu", dtype=torch.float32):
    """(inputs dict of tensors, rng dict) for one golden MAR case."""
    inp = {k: torch.from_numpy(x).to(device) for k, x in cases.mar_inputs(variant).items()}
    rng = cases.mar_rng(variant, mode)
    return inp, rng


def grad_rel_errors(named_params, fixture, names_key, sums_key, heads_key):
    """max relative error of (sum, sumsq) and head values per parameter grad."""
    ref_names = [str(n) for n in fixture[names_key]]
    sums, heads = fixture[sums_key], fixture[heads_key]
    got = {n: p.grad for n, p in named_params if p.grad is not None}
    errs = {}
    for i, n in enumerate(ref_names):
        assert n in got, f"missing grad for {n}"
        g = got[n].detach().double().cpu().reshape(-1)
        scale = max(np.sqrt(sums[i][1] / max(g.numel(), 1)), 1e-12)
        e_sum = abs(g.sum().item() - sums[i][0]) / (scale * np.sqrt(g.numel()) + 1e-30)
        e_sq = abs((g * g).sum().item() - sums[i][1]) / (sums[i][1] + 1e-30)
        h = g[:4].numpy()
        e_head = np.max(np.abs(h - heads[i][: len(h)])) / scale
        errs[n] = max(e_sum, e_sq, e_head)
    return errs


def golden_policy(predict_action=True, normalizer=True):
    """This build's UnifiedVideoActionPolicy configured like make_golden._ref_policy: full KL-VAE,
    reduced MAR (cases.MAR_GOLDEN) as model_size "mar_golden", hash-initialised, PushT limits
    normalizer; on the CPU, train mode."""
    from functools import partial

    import torch.nn as nn
    from unified_video_action_amd.model.autoregressive import mar_con_unified as pmar
    from unified_video_action_amd.model.common.normalizer import LinearNormalizer
    from unified_video_action_amd.policy.unified_video_action_policy import UnifiedVideoActionPolicy
    pmar.mar_golden = lambda **kw: pmar.MAR(norm_layer=partial(nn.LayerNorm, eps=1e-6), **cases.MAR_GOLDEN, **kw)
    amp = dict(pretrained_model_path=None, model_size="mar_golden")
    for k in cases.POLICY_AMP_KEYS:
        amp[k] = cases.MAR_KW[k]
    pol = UnifiedVideoActionPolicy(
        vae_model_params=dict(autoencoder_path=None, ddconfig=dict(vae_embed_dim=16, ch_mult=[1, 1, 2, 2, 4])),
        autoregressive_model_params=amp,
        action_model_params=dict(predict_action=predict_action, act_model_type="conv_fc"),
        shape_meta={"action": {"shape": [2]}}, n_action_steps=8, shift_action=True, language_emb_model=None,
        task_name="pusht", task_modes=[], normalizer_type="all", selected_training_mode=None,
        use_history_action=False, use_proprioception=False, action_mask_ratio=0.5, different_history_freq=False,
        predict_wrist_img=False, predict_proprioception=False)
    hash_init_(pol.vae_model, "vae.")
    hash_init_(pol.model, "mar.")
    if normalizer:
        norm = LinearNormalizer()
        lim = torch.zeros(2, 2)
        lim[1] = 512.0
        norm.fit({"action": lim, "agent_pos": lim})
        pol.set_normalizer(norm)
    return pol.train()


def device_batch(b, device):
    return {"obs": {"image": torch.from_numpy(b["image"]).to(device),
                    "agent_pos": torch.from_numpy(b["agent_pos"]).to(device)},
            "action": torch.from_numpy(b["action"]).to(device)}
