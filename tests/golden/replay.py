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
    v = cases.VARIANTS[variant]
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
