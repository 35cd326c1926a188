"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
(/root/reference, imported read-only with ref_shims) on hash-initialised weights
and hash-generated inputs with injected RNG (cases.py).

Run in the build container only:   python tests/golden/make_golden.py
The outputs are small .npz files of inputs-free data (the inputs are
regenerated from cases.py by name) holding expected outputs / checksums.
"""
import contextlib
import os
import random
import sys
from functools import partial

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_shims  # noqa: E402

ref_shims.install()
from hashinit import hash_init_, hash_normal, hash_tensor  # noqa: E402
import cases  # noqa: E402

import unified_video_action.model.autoregressive.mar_con_unified as ref_mar  # noqa: E402
from unified_video_action.model.autoregressive.diffusion import create_diffusion  # noqa: E402
from unified_video_action.model.autoregressive.diffusion_loss import SimpleMLPAdaLN  # noqa: E402
from unified_video_action.model.autoregressive.ema_model import EMAModel  # noqa: E402
from unified_video_action.vae import vaekl  # noqa: E402
from unified_video_action.utils import data_utils  # noqa: E402

torch.set_num_threads(8)
OUT = HERE


def checksum(t):
    a = t.detach().double().reshape(-1)
    return np.array([a.sum().item(), (a * a).sum().item(), a.abs().max().item()], np.float64)


_CAPTURE = None    # gen_bf16_extras: collect the arrays a generator would save instead of writing
_AUTOCAST = False  # gen_bf16_extras: run the reference's loss under CPU bf16 autocast


def _save(path, **d):
    if _CAPTURE is not None:
        _CAPTURE[path] = d
    else:
        np.savez(path, **d)


def _amp():
    return torch.autocast("cpu", dtype=torch.bfloat16) if _AUTOCAST else contextlib.nullcontext()


def sketch_table(module):
    """cases.grad_sketch of every parameter gradient, in grad_table's order."""
    return np.stack([cases.grad_sketch(n, p.grad.detach().double().reshape(-1).numpy())
                     for n, p in module.named_parameters() if p.grad is not None])


def grad_table(module):
    names, sums, heads = [], [], []
    for n, p in module.named_parameters():
        if p.grad is None:
            continue
        names.append(n)
        sums.append(checksum(p.grad))
        h = np.zeros(4, np.float64)
        g = p.grad.detach().double().reshape(-1)[:4].numpy()
        h[: len(g)] = g
        heads.append(h)
    return np.array(names), np.stack(sums), np.stack(heads)


@contextlib.contextmanager
def injected(rng):
    """Replace the reference's RNG call sites by queues of pre-drawn values."""
    q_int = [torch.from_numpy(x) for x in rng.get("randint", [])]
    q_nrm = [torch.from_numpy(x) for x in rng.get("randn_like", [])]
    q_eps = [torch.from_numpy(rng[k]) for k in ("vae_eps_x", "vae_eps_c") if k in rng]
    if "vae_eps_wrist" in rng:  # second camera: history half (second_image) first, then the future half
        w = torch.from_numpy(rng["vae_eps_wrist"])
        q_eps = [w[len(w) // 2:], w[: len(w) // 2]] + q_eps
    saved = (torch.randint, torch.randn_like, torch.randn, torch.rand, random.choice,
             ref_mar.MAR.sample_orders)

    def fake_randint(*a, **k):
        v = q_int.pop(0)
        assert tuple(a[2]) == tuple(v.shape), (a, v.shape)
        return v

    def fake_randn_like(x, *a, **k):
        v = q_nrm.pop(0)
        assert v.shape == x.shape, (v.shape, x.shape)
        return v.to(x.dtype)

    def fake_randn(*shape, **k):
        v = q_eps.pop(0)
        shp = shape[0] if len(shape) == 1 and not isinstance(shape[0], int) else shape
        assert tuple(shp) == tuple(v.shape), (shp, v.shape)
        return v

    q_rand = [torch.from_numpy(rng["hist_u"])] if "hist_u" in rng else []

    def fake_rand(*shape, **k):
        if q_rand:  # the history-action drop draws first (:512-518), then the label drop
            v = q_rand.pop(0)
            assert tuple(shape) == tuple(v.shape), (shape, v.shape)
            return v
        return torch.from_numpy(rng["text_drop_u"])

    torch.randint, torch.randn_like, torch.randn, torch.rand = (
        fake_randint, fake_randn_like, fake_randn, fake_rand)
    if "task_mode" in rng:
        random.choice = lambda seq: rng["task_mode"]
    ref_mar.MAR.sample_orders = lambda self, bsz: torch.from_numpy(rng["orders"])
    try:
        yield
    finally:
        (torch.randint, torch.randn_like, torch.randn, torch.rand, random.choice,
         ref_mar.MAR.sample_orders) = saved
    assert not q_int and not q_nrm and not q_eps and not q_rand, "unconsumed injected draws"


def build_mar(variant):
    m = ref_mar.MAR(norm_layer=partial(nn.LayerNorm, eps=1e-6), **cases.MAR_GOLDEN,
                    **cases.mar_kwargs(variant))
    hash_init_(m, "mar.")
    m.train()
    return m


def mar_call(m, variant, mode, inp):
    v = cases.variant_def(variant)
    t = {k: torch.from_numpy(x) for k, x in inp.items()}
    prop = {}
    if v["use_proprioception"]:
        prop = {k: t[k] for k in t if k.startswith(("robot0_", "second_image", "pred_second_image"))}
    return m(t["z"], t["c"], t.get("history_nactions"), t["nactions"], t.get("text_latents"), task_mode=mode,
             proprioception_input=prop)


def gen_mar_extra():
    """g2_mar_<extra variant>_<mode>.npz for cases.EXTRA_VARIANTS (variants no shipped config selects)."""
    gen_mar(cases.EXTRA_VARIANTS)


def gen_mar(variants=None):
    for variant, v in (variants or cases.VARIANTS).items():
        inp = cases.mar_inputs(variant)
        for mode in v["modes"]:
            m = build_mar(variant)
            rng = cases.mar_rng(variant, mode)
            m.mask_ratio_generator = type("G", (), {"rvs": staticmethod(
                lambda n, r=rng["mask_rate"]: np.array([r]))})()
            with injected(rng), _amp():
                loss, lv, la = mar_call(m, variant, mode, inp)
            loss.float().backward()
            names, sums, heads = grad_table(m)
            _save(os.path.join(OUT, f"g2_mar_{variant}_{mode}.npz"),
                  loss=np.array([loss.item(), lv.item(), la.item()], np.float64),
                  grad_names=names, grad_sums=sums, grad_heads=heads, grad_sketch=sketch_table(m))
            print(f"mar {variant} {mode}: loss={loss.item():.6f} Lv={lv.item():.6f} "
                  f"La={la.item():.6f} ngrads={len(names)}")


def gen_policy_variants_all():
    """g2_policy_variants.npz from scratch: the fp32 run, then its bf16 extras."""
    gen_policy_variants()
    gen_bf16_extras(gens=(gen_policy_variants,))


def gen_bf16_extras(gens=None):
    """The reference's own bf16 error on every MAR case and policy mode: each generator re-run in
    fp32 (must reproduce its stored fixture; adds the gradient sketches) and under CPU bf16 autocast
    (bf16 linear / matmul / conv operands, fp32 norms and losses -- the reference's
    mixed_precision=bf16 training); the bf16 loss, gradient checksums and sketches are stored
    beside the fp32 ones ("<key>_bf16"), so the bf16 tests hold this build to the reference's own
    bf16 deviation."""
    global _CAPTURE, _AUTOCAST
    for gen in gens or (gen_mar, gen_policy, gen_policy_variants):
        _CAPTURE, _AUTOCAST = {}, False
        gen()
        fp = _CAPTURE
        _CAPTURE, _AUTOCAST = {}, True
        try:
            gen()
        finally:
            bf, _CAPTURE, _AUTOCAST = _CAPTURE, None, False
        for path, d in fp.items():
            old = dict(np.load(path))
            for k, v in d.items():
                if "sketch" not in k and k in old and np.asarray(v).dtype.kind == "f":
                    np.testing.assert_allclose(v, old[k], rtol=1e-9, atol=0, err_msg=f"{path} {k}")
            new = {k: v for k, v in old.items() if not k.endswith("_bf16")}
            new.update({k: v for k, v in d.items() if "sketch" in k})
            for k, v in bf[path].items():
                if k.endswith(("loss", "sums", "sketch")):
                    new[k + "_bf16"] = v
            np.savez(path, **new)
            print(f"bf16 extras -> {os.path.basename(path)}")


def gen_indexing():
    d = {}
    x = torch.arange(32).float().reshape(1, 32, 1, 1, 1)
    _, idx = data_utils.select_frames(x, 32, eval=False)
    d["frames_train"] = idx.numpy()
    _, idx = data_utils.select_frames(x, 32, eval=True)
    d["frames_eval"] = idx.numpy()
    d["history_combinations"] = np.array(data_utils.combinations, np.int64)
    na = torch.arange(32 * 3).float().reshape(1, 32, 3)
    h, tr = data_utils.get_trajectory(na, 32, True)
    d["traj_shift"] = tr.numpy()
    h, tr = data_utils.get_trajectory(na, 32, False)
    d["traj_noshift_hist"], d["traj_noshift"] = h.numpy(), tr.numpy()
    # masks for every (orders, rate) golden case
    m = build_mar("pusht")
    for mode in cases.ALL_MODES:
        rng = cases.mar_rng("pusht", mode)
        m.mask_ratio_generator = type("G", (), {"rvs": staticmethod(
            lambda n, r=rng["mask_rate"]: np.array([r]))})()
        mask = m.random_masking(torch.zeros(2, 4, 256, 8), torch.from_numpy(rng["orders"]))
        d[f"mask_{mode}"] = mask.numpy().astype(np.uint8)
    img = torch.arange(2 * 16 * 16 * 16).float().reshape(2, 16, 16, 16)
    d["patchify"] = m.patchify(img).numpy()
    np.savez(os.path.join(OUT, "g1_indexing.npz"), **d)
    print("indexing done")


def gen_block():
    from ref_shims import Block
    d = {}
    for n_tok in (1024, 1088):
        blk = Block(768, 12, 4.0, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6))
        hash_init_(blk, "blk.")
        x = torch.from_numpy(hash_normal(f"blk/x{n_tok}", (2, n_tok, 768))).requires_grad_(True)
        y = blk(x)
        gy = torch.from_numpy(hash_normal(f"blk/gy{n_tok}", (2, n_tok, 768)))
        y.backward(gy)
        names, sums, heads = grad_table(blk)
        d[f"y{n_tok}"] = checksum(y)
        d[f"y{n_tok}_rows"] = y.detach()[:, ::97].numpy()
        d[f"gx{n_tok}"] = checksum(x.grad)
        d[f"gx{n_tok}_rows"] = x.grad[:, ::97].numpy()
        d[f"gnames{n_tok}"], d[f"gsums{n_tok}"], d[f"gheads{n_tok}"] = names, sums, heads
    np.savez(os.path.join(OUT, "g3_block.npz"), **d)
    print("block done")


def gen_mlp():
    net = SimpleMLPAdaLN(16, 1024, 32, 768, 6)
    hash_init_(net, "mlp.")
    rows = 512
    x = torch.from_numpy(hash_normal("mlp/x", (rows, 16))).requires_grad_(True)
    c = torch.from_numpy(hash_normal("mlp/c", (rows, 768))).requires_grad_(True)
    t = torch.from_numpy(cases.t_steps("mlp", rows))
    y = net(x, t, c)
    gy = torch.from_numpy(hash_normal("mlp/gy", (rows, 32)))
    y.backward(gy)
    names, sums, heads = grad_table(net)
    np.savez(os.path.join(OUT, "g3_mlp.npz"), y=y.detach().numpy(), gx=x.grad.numpy(),
             gc=checksum(c.grad), gc_rows=c.grad[::16].numpy(), gnames=names, gsums=sums, gheads=heads)
    print("mlp done")


ACT_TRUNKS = ("conv_ori", "conv2", "fc2")


def gen_act_trunks():
    """g3_act_trunks.npz: the reference DiffActLoss with each off-config action trunk (act_model_type
    conv_ori / conv2 / fc2, diffusion_action_loss.py:63-89, 125-141) on hash weights, z [2, 1024, 64],
    target [2, 16, 2], injected t / noise: loss, dL/dz rows and every parameter gradient."""
    from unified_video_action.model.autoregressive.diffusion_action_loss import DiffActLoss
    d = {}
    for kind in ACT_TRUNKS:
        m = DiffActLoss(2, 64, 2, 64, "100", n_frames=4, act_model_type=kind, language_emb_model=None,
                        language_emb_model_type=1)
        hash_init_(m, f"act_{kind}.")
        m.train()
        z = torch.from_numpy(hash_normal(f"act_{kind}/z", (2, 1024, 64))).requires_grad_(True)
        target = torch.from_numpy(hash_normal(f"act_{kind}/target", (2, 16, 2)))
        rng = {"randint": [cases.t_steps(f"act_{kind}", 32)],
               "randn_like": [hash_normal(f"act_{kind}/noise", (32, 2))]}
        with injected(rng):
            loss = m(target, z)
        loss.backward()
        names, sums, heads = grad_table(m)
        d[f"{kind}_loss"] = np.array([loss.item()], np.float64)
        d[f"{kind}_gz_rows"] = z.grad[:, ::64].detach().numpy()
        d[f"{kind}_gz_sum"] = checksum(z.grad)
        d[f"{kind}_gnames"], d[f"{kind}_gsums"], d[f"{kind}_gheads"] = names, sums, heads
        print(f"act trunk {kind}: loss={loss.item():.6f} ngrads={len(names)}")
    np.savez(os.path.join(OUT, "g3_act_trunks.npz"), **d)


def gen_diffusion_math():
    d = {}
    for tag, C in (("video", 16), ("act", 2), ("act10", 10)):
        diff = create_diffusion(timestep_respacing="", noise_schedule="cosine")
        rows = 512
        x0 = torch.from_numpy(hash_tensor(f"dm/{tag}/x0", (rows, C)))
        out = torch.from_numpy(hash_tensor(f"dm/{tag}/out", (rows, 2 * C)))
        t = torch.from_numpy(cases.t_steps(f"dm/{tag}", rows))
        noise = torch.from_numpy(hash_normal(f"dm/{tag}/noise", (rows, C)))
        out.requires_grad_(True)
        terms = diff.training_losses(lambda xt, tt, **k: out, x0, t, {}, noise=noise)
        terms["loss"].sum().backward()
        d[f"{tag}_loss"] = terms["loss"].detach().numpy()
        d[f"{tag}_mse"] = terms["mse"].detach().numpy()
        d[f"{tag}_vb"] = terms["vb"].detach().numpy()
        d[f"{tag}_gout"] = out.grad.numpy()
    diff = create_diffusion(timestep_respacing="", noise_schedule="cosine")
    for k in ("betas", "alphas_cumprod", "posterior_log_variance_clipped",
              "posterior_mean_coef1", "posterior_mean_coef2", "sqrt_alphas_cumprod",
              "sqrt_one_minus_alphas_cumprod"):
        d[f"table_{k}"] = getattr(diff, k)
    np.savez(os.path.join(OUT, "g3_diffusion_math.npz"), **d)
    print("diffusion math done")


def gen_vae():
    class DD:
        vae_embed_dim = 16
        ch_mult = (1, 1, 2, 2, 4)

    ae = vaekl.AutoencoderKL(autoencoder_path=None, ddconfig=DD())
    hash_init_(ae, "vae.")
    x = torch.from_numpy(hash_tensor("vae/x", (1, 3, 256, 256)))
    eps = torch.from_numpy(hash_normal("vae/eps", (1, 16, 16, 16)))
    with torch.no_grad():
        h = ae.encoder(x)
        moments = ae.quant_conv(h)
        saved = torch.randn
        torch.randn = lambda *s, **k: eps
        try:
            z = ae.encode(x).sample().mul_(0.2325)
        finally:
            torch.randn = saved
    np.savez(os.path.join(OUT, "g3_vae.npz"), moments=moments.numpy(), z=z.numpy())
    print("vae done")


def gen_vae_decode():
    """AutoencoderKL.decode of the reference (vaekl.py:56-58, Decoder :276-397) on hash weights."""
    class DD:
        vae_embed_dim = 16
        ch_mult = (1, 1, 2, 2, 4)

    ae = vaekl.AutoencoderKL(autoencoder_path=None, ddconfig=DD())
    hash_init_(ae, "vae.")
    z = torch.from_numpy(hash_normal("vae/dec_z", (1, 16, 16, 16)))
    with torch.no_grad():
        img = ae.decode(z)
    np.savez(os.path.join(OUT, "g3_vae_decode.npz"), sub=img[:, :, ::8, ::8].numpy(),
             checksum=checksum(img), shape=np.array(img.shape))
    print("vae decode", tuple(img.shape), checksum(img))


def gen_resize():
    import torch.nn.functional as F
    d = {}
    for H in (96, 128, 224):
        x = torch.from_numpy((hash_tensor(f"resize/{H}", (2, 3, H, H)) + 1) * 0.5)
        y = F.interpolate(x, size=(256, 256), mode="bilinear", align_corners=False)
        d[f"y{H}"] = checksum(y)
        d[f"y{H}_rows"] = y[:, :, ::37].numpy()
    np.savez(os.path.join(OUT, "g3_resize.npz"), **d)
    print("resize done")


def gen_ema():
    ema = EMAModel(nn.Linear(2, 2), update_after_step=0, inv_gamma=1.0, power=0.75,
                   min_value=0.0, max_value=0.9999)
    dec = np.array([ema.get_decay(s) for s in range(2001)], np.float64)
    np.savez(os.path.join(OUT, "g4_ema.npz"), decay=dec)
    print("ema done")


def _ref_policy(cls, AD, amp):
    from unified_video_action.model.common.normalizer import LinearNormalizer
    pol = cls(
        vae_model_params=AD(autoencoder_path=None, ddconfig=AD(vae_embed_dim=16, ch_mult=[1, 1, 2, 2, 4])),
        autoregressive_model_params=AD(amp),
        action_model_params=AD(predict_action=True, act_model_type="conv_fc"),
        shape_meta=AD(action=AD(shape=[2])), n_action_steps=8, shift_action=True,
        language_emb_model=None, task_name="pusht", task_modes=[],
        normalizer_type="all", selected_training_mode=None, use_history_action=False,
        use_proprioception=False, action_mask_ratio=0.5, different_history_freq=False,
        predict_wrist_img=False, predict_proprioception=False, debug=False)
    hash_init_(pol.vae_model, "vae.")
    hash_init_(pol.model, "mar.")
    norm = LinearNormalizer()
    lim = torch.zeros(2, 2)
    lim[1] = 512.0
    norm.fit({"action": lim, "agent_pos": lim})
    pol.set_normalizer(norm)
    return pol


def gen_policy():
    from unified_video_action.policy.unified_video_action_policy import UnifiedVideoActionPolicy
    from unified_video_action.model.common.normalizer import LinearNormalizer

    class AD(dict):
        def __getattr__(self, k):
            v = self[k]
            return AD(v) if isinstance(v, dict) else v

    ref_mar.mar_golden = lambda **kw: ref_mar.MAR(
        norm_layer=partial(nn.LayerNorm, eps=1e-6), **cases.MAR_GOLDEN, **kw)
    amp = dict(pretrained_model_path=None, model_size="mar_golden")
    for k in cases.POLICY_AMP_KEYS:
        amp[k] = cases.MAR_KW[k]
    out = {}
    for mode in cases.POLICY_MODES:
        pol = _ref_policy(UnifiedVideoActionPolicy, AD, amp)
        pol.train()
        b = cases.policy_batch()
        batch = {"obs": {"image": torch.from_numpy(b["image"]),
                         "agent_pos": torch.from_numpy(b["agent_pos"])},
                 "action": torch.from_numpy(b["action"])}

        class Cfg:
            class task:
                name = "pusht"

        batch = data_utils.resize_image(Cfg, batch)
        rng = cases.policy_rng(mode)
        rng["task_mode"] = mode
        pol.model.mask_ratio_generator = type("G", (), {"rvs": staticmethod(
            lambda n, r=rng["mask_rate"]: np.array([r]))})()
        with injected(rng), _amp():
            loss, (lv, la) = pol.compute_loss(batch)
        loss.float().backward()
        names, sums, heads = grad_table(pol.model)
        out[f"{mode}_loss"] = np.array([loss.item(), lv.item(), la.item()], np.float64)
        out[f"{mode}_gnames"], out[f"{mode}_gsums"], out[f"{mode}_gheads"] = names, sums, heads
        out[f"{mode}_gsketch"] = sketch_table(pol.model)
        dec, nod = pol.add_weight_decay(pol.model, 0.02)[1], None
        print(f"policy {mode}: loss={loss.item():.6f} Lv={lv.item():.6f} La={la.item():.6f}")
    decay_names = [n for n, p in pol.model.named_parameters()
                   if p.requires_grad and not (len(p.shape) == 1 or n.endswith(".bias"))]
    out["decay_names"] = np.array(decay_names)
    _save(os.path.join(OUT, "g2_policy_pusht.npz"), **out)


def gen_sample():
    """sample_tokens(task_mode="policy_model") of the reference on every variant (eval mode),
    with the sampler's randn draws injected (cases.sample_rng)."""
    out = {}
    for variant, v in cases.VARIANTS.items():
        m = build_mar(variant)
        m.eval()
        inp = {k: torch.from_numpy(x) for k, x in cases.mar_inputs(variant).items()}
        rng = cases.sample_rng(variant)
        q = [torch.from_numpy(a) for a in rng["step_noise"]]
        saved = (torch.randn, torch.randn_like, torch.Tensor.cuda, ref_mar.MAR.sample_orders)

        def fake_randn(*shape, **k):
            assert tuple(shape) == rng["noise"].shape, shape
            return torch.from_numpy(rng["noise"])

        def fake_randn_like(x, *a, **k):
            return q.pop(0).to(x.dtype)

        torch.randn, torch.randn_like = fake_randn, fake_randn_like
        torch.Tensor.cuda = lambda self, *a, **k: self
        ref_mar.MAR.sample_orders = lambda self, bsz: torch.from_numpy(rng["orders"])
        try:
            prop = {k: inp[k] for k in inp if k.startswith(("robot0_", "second_image", "pred_second_image")) and not k.endswith("_pred")}
            _, act = m.sample_tokens(bsz=cases.B_MAR, cond=inp["c"], text_latents=inp.get("text_latents"),
                                     num_iter=1, cfg=1.0, temperature=cases.SAMPLE_TEMPERATURE,
                                     proprioception_input=prop, task_mode="policy_model")
            assert not q, "unconsumed step noise"
            q = [torch.from_numpy(a) for a in rng["step_noise"]]
            _, inv = m.sample_tokens(bsz=cases.B_MAR, cond=inp["c"], text_latents=inp.get("text_latents"),
                                     num_iter=1, cfg=1.0, temperature=cases.SAMPLE_TEMPERATURE,
                                     proprioception_input=prop, task_mode="inverse_model", x=inp["z"])
        finally:
            torch.randn, torch.randn_like, torch.Tensor.cuda, ref_mar.MAR.sample_orders = saved
        assert not q, "unconsumed step noise"
        out[f"{variant}_act"] = act.detach().double().numpy()
        out[f"{variant}_inverse_act"] = inv.detach().double().numpy()
        print(f"sample {variant}: act sum={act.sum().item():.6f} inverse sum={inv.sum().item():.6f}")
    np.savez(os.path.join(OUT, "g5_sample.npz"), **out)


def gen_video_sample():
    """sample_tokens(task_mode="video_model") of the reference (MaskGIT loop, mar_con_unified.py:
    1000-1151), eval mode, VIDEO_SAMPLE_ITERS iterations, draws injected (cases.video_sample_rng)."""
    out = {}
    for variant in ("pusht", "libero"):
        m = build_mar(variant)
        m.eval()
        inp = {k: torch.from_numpy(x) for k, x in cases.mar_inputs(variant).items()}
        rng = cases.video_sample_rng(variant)
        q_randn, q_like = [], []
        for i in range(cases.VIDEO_SAMPLE_ITERS):
            q_randn += [torch.from_numpy(rng["act_noise"][i]), torch.from_numpy(rng["video_noise"][i])]
            q_like += [torch.from_numpy(a) for a in rng["act_step_noise"][i]]
            q_like += [torch.from_numpy(a) for a in rng["video_step_noise"][i]]
        saved = (torch.randn, torch.randn_like, torch.Tensor.cuda, ref_mar.MAR.sample_orders)

        def fake_randn(*shape, **k):
            v = q_randn.pop(0)
            assert tuple(shape) == tuple(v.shape), (shape, v.shape)
            return v

        def fake_randn_like(x, *a, **k):
            v = q_like.pop(0)
            assert v.shape == x.shape, (v.shape, x.shape)
            return v.to(x.dtype)

        torch.randn, torch.randn_like = fake_randn, fake_randn_like
        torch.Tensor.cuda = lambda self, *a, **k: self
        ref_mar.MAR.sample_orders = lambda self, bsz: torch.from_numpy(rng["orders"])
        try:
            tok, act = m.sample_tokens(bsz=cases.B_MAR, cond=inp["c"], text_latents=inp.get("text_latents"),
                                       num_iter=cases.VIDEO_SAMPLE_ITERS, cfg=1.0,
                                       temperature=cases.SAMPLE_TEMPERATURE, task_mode="video_model")
        finally:
            torch.randn, torch.randn_like, torch.Tensor.cuda, ref_mar.MAR.sample_orders = saved
        assert not q_randn and not q_like, "unconsumed draws"
        out[f"{variant}_tokens"] = tok.detach().float().numpy()
        out[f"{variant}_act"] = act.detach().float().numpy()
        print(f"video sample {variant}: tokens {tuple(tok.shape)} sum={tok.sum().item():.5f}")
    np.savez(os.path.join(OUT, "g5_video_sample.npz"), **out)


def gen_video_sample_wrist():
    """sample_tokens(video_model) of the reference with the wrist-camera video stream
    (predict_wrist_img, toolhang_wrist): every MaskGIT iteration samples diffloss_wrist on the same
    rows as the video head and writes them into pred_second_image_z (:1118-1140); the call returns the
    unpatchified wrist tokens (:1143-1157).  Draws injected in the reference's order per iteration:
    action head, video head, wrist head (cases.video_sample_rng)."""
    variant = "toolhang_wrist"
    m = build_mar(variant)
    m.eval()
    inp = {k: torch.from_numpy(x) for k, x in cases.mar_inputs(variant).items()}
    rng = cases.video_sample_rng(variant)
    q_randn, q_like = [], []
    for i in range(cases.VIDEO_SAMPLE_ITERS):
        q_randn += [torch.from_numpy(rng["act_noise"][i]), torch.from_numpy(rng["video_noise"][i]),
                    torch.from_numpy(rng["wrist_noise"][i])]
        q_like += [torch.from_numpy(a) for a in rng["act_step_noise"][i]]
        q_like += [torch.from_numpy(a) for a in rng["video_step_noise"][i]]
        q_like += [torch.from_numpy(a) for a in rng["wrist_step_noise"][i]]
    saved = (torch.randn, torch.randn_like, torch.Tensor.cuda, ref_mar.MAR.sample_orders)

    def fake_randn(*shape, **k):
        v = q_randn.pop(0)
        assert tuple(shape) == tuple(v.shape), (shape, v.shape)
        return v

    def fake_randn_like(x, *a, **k):
        v = q_like.pop(0)
        assert v.shape == x.shape, (v.shape, x.shape)
        return v.to(x.dtype)

    torch.randn, torch.randn_like = fake_randn, fake_randn_like
    torch.Tensor.cuda = lambda self, *a, **k: self
    ref_mar.MAR.sample_orders = lambda self, bsz: torch.from_numpy(rng["orders"])
    prop = {k: inp[k] for k in inp if k.startswith(("robot0_", "second_image")) and not k.endswith("_pred")}
    try:
        tok, act = m.sample_tokens(bsz=cases.B_MAR, cond=inp["c"], text_latents=None,
                                   num_iter=cases.VIDEO_SAMPLE_ITERS, cfg=1.0,
                                   temperature=cases.SAMPLE_TEMPERATURE, task_mode="video_model",
                                   proprioception_input=prop)
    finally:
        torch.randn, torch.randn_like, torch.Tensor.cuda, ref_mar.MAR.sample_orders = saved
    assert not q_randn and not q_like, "unconsumed draws"
    out = {f"{variant}_wrist_tokens": tok.detach().float().numpy(), f"{variant}_act": act.detach().float().numpy()}
    print(f"video sample {variant}: wrist tokens {tuple(tok.shape)} sum={tok.sum().item():.5f}")
    np.savez(os.path.join(OUT, "g5_video_sample_wrist.npz"), **out)


def gen_predict():
    """UnifiedVideoActionPolicy.predict_action (policy:221-320) of the reference, eval mode, on the
    golden PushT policy (full KL-VAE, reduced MAR), draws injected (cases.predict_rng)."""
    from unified_video_action.policy.unified_video_action_policy import UnifiedVideoActionPolicy

    class AD(dict):
        def __getattr__(self, k):
            v = self[k]
            return AD(v) if isinstance(v, dict) else v

    ref_mar.mar_golden = lambda **kw: ref_mar.MAR(
        norm_layer=partial(nn.LayerNorm, eps=1e-6), **cases.MAR_GOLDEN, **kw)
    amp = dict(pretrained_model_path=None, model_size="mar_golden", num_iter=1, cfg=1,
               cfg_schedule="linear", temperature=cases.SAMPLE_TEMPERATURE)
    for k in cases.POLICY_AMP_KEYS:
        amp[k] = cases.MAR_KW[k]
    pol = _ref_policy(UnifiedVideoActionPolicy, AD, amp)
    pol.eval()
    b = cases.policy_batch()
    rng = cases.predict_rng()
    q_randn = [torch.from_numpy(rng["vae_eps"]), torch.from_numpy(rng["noise"])]
    q = [torch.from_numpy(a) for a in rng["step_noise"]]
    saved = (torch.randn, torch.randn_like, torch.Tensor.cuda, ref_mar.MAR.sample_orders)

    def fake_randn(*shape, **k):
        v = q_randn.pop(0)
        shp = shape[0] if len(shape) == 1 and not isinstance(shape[0], int) else shape
        assert tuple(shp) == tuple(v.shape), (shp, v.shape)
        return v

    torch.randn = fake_randn
    torch.randn_like = lambda x, *a, **k: q.pop(0).to(x.dtype)
    torch.Tensor.cuda = lambda self, *a, **k: self
    ref_mar.MAR.sample_orders = lambda self, bsz: torch.from_numpy(rng["orders"])
    try:
        with torch.no_grad():
            res = pol.predict_action({"image": torch.from_numpy(b["image"]),
                                      "agent_pos": torch.from_numpy(b["agent_pos"])})
    finally:
        torch.randn, torch.randn_like, torch.Tensor.cuda, ref_mar.MAR.sample_orders = saved
    assert not q and not q_randn, "unconsumed draws"
    np.savez(os.path.join(OUT, "g5_predict_pusht.npz"), action=res["action"].double().numpy(),
             action_pred=res["action_pred"].double().numpy())
    print("predict pusht: action_pred", tuple(res["action_pred"].shape), res["action_pred"][0, :3].tolist())


def gen_policy_variants():
    """compute_loss of the reference policy for the Libero (CLIP latents, Da = 10, 128-px agentview
    resized to 256) and UMI (proprioception in/out, img_indices gather, different_history_freq,
    8 frames at 224 px, no normalizer, shift_action False) variants: full KL-VAE, reduced MAR,
    draws injected; plus the UMI process_data gather itself (integer indexing, bit-exact)."""
    from unified_video_action.model.common.normalizer import LinearNormalizer
    from unified_video_action.policy.unified_video_action_policy import UnifiedVideoActionPolicy

    class AD(dict):
        def __getattr__(self, k):
            if k.startswith("__"):
                raise AttributeError(k)
            v = self[k]
            return AD(v) if isinstance(v, dict) else v

    ref_mar.mar_golden = lambda **kw: ref_mar.MAR(
        norm_layer=partial(nn.LayerNorm, eps=1e-6), **cases.MAR_GOLDEN, **kw)
    amp = dict(pretrained_model_path=None, model_size="mar_golden")
    for k in cases.POLICY_AMP_KEYS:
        amp[k] = cases.MAR_KW[k]
    out = {}
    for variant, modes in cases.POLICY_VARIANT_MODES.items():
        kw = cases.policy_variant_kwargs(variant)
        for mode in modes:
            pol = UnifiedVideoActionPolicy(
                vae_model_params=AD(autoencoder_path=None, ddconfig=AD(vae_embed_dim=16, ch_mult=[1, 1, 2, 2, 4])),
                autoregressive_model_params=AD(amp), action_model_params=AD(kw["action_model_params"]),
                shape_meta=AD(kw["shape_meta"]), **{k: v for k, v in kw.items()
                                                    if k not in ("action_model_params", "shape_meta")}, debug=False)
            hash_init_(pol.vae_model, "vae.")
            hash_init_(pol.model, "mar.")
            if variant == "libero":
                norm = LinearNormalizer()
                norm.fit({"action": torch.tensor([[-1.0] * 10, [1.0] * 10])})
                pol.set_normalizer(norm)
            pol.train()
            b = cases.policy_variant_batch(variant)
            batch = {"obs": {k: torch.from_numpy(v) for k, v in b["obs"].items()},
                     "action": torch.from_numpy(b["action"]),
                     "language_latents": torch.from_numpy(b["language_latents"])}

            class Cfg:
                class task:
                    name = kw["task_name"]

            batch = data_utils.resize_image(Cfg, batch)
            rng = cases.policy_variant_rng(variant, mode)
            pol.model.mask_ratio_generator = type("G", (), {"rvs": staticmethod(
                lambda n, r=rng["mask_rate"]: np.array([r]))})()
            with injected(rng), _amp():
                loss, (lv, la) = pol.compute_loss(batch)
            loss.float().backward()
            names, sums, heads = grad_table(pol.model)
            out[f"{variant}_{mode}_loss"] = np.array([loss.item(), float(lv), float(la)], np.float64)
            out[f"{variant}_{mode}_gnames"], out[f"{variant}_{mode}_gsums"], out[f"{variant}_{mode}_gheads"] = \
                names, sums, heads
            out[f"{variant}_{mode}_gsketch"] = sketch_table(pol.model)
            print(f"policy {variant} {mode}: loss={loss.item():.6f} Lv={float(lv):.6f} La={float(la):.6f}")
    # process_data's UMI gather (data_utils.py:214-219, 291-360), train and eval
    b = cases.policy_variant_batch("umi", B=3)
    batch = {"obs": {k: torch.from_numpy(v) for k, v in b["obs"].items()}}
    batch["obs"]["image"] = torch.zeros(3, 8, 3, 4, 4)
    for ev in (False, True):
        _, prop, idx = data_utils.process_data(batch, task_name="umi", eval=ev, use_proprioception=True,
                                               different_history_freq=True)
        tag = "eval" if ev else "train"
        out[f"umi_gather_{tag}_indices"] = idx.numpy()
        for k, v in prop.items():
            if v is not None:
                out[f"umi_gather_{tag}_{k}"] = v.numpy()
    _save(os.path.join(OUT, "g2_policy_variants.npz"), **out)


def gen_workspace_trace():
    """The reference's per-step training body (workspace:279-302) on the golden PushT policy
    (full KL-VAE, reduced MAR, joint model): deepcopy EMA policy, policy.get_optimizer (torch
    AdamW, two groups), cosine-with-warmup LambdaLR (diffusers restated: diffusers is absent),
    the reference EMAModel, step order fwd -> bwd -> opt.step -> zero_grad -> lr.step -> ema.step;
    draws injected per step (cases.trace_rng)."""
    import copy
    import math
    from unified_video_action.policy.unified_video_action_policy import UnifiedVideoActionPolicy

    class AD(dict):
        def __getattr__(self, k):
            if k.startswith("__"):
                raise AttributeError(k)
            v = self[k]
            return AD(v) if isinstance(v, dict) else v

    ref_mar.mar_golden = lambda **kw: ref_mar.MAR(
        norm_layer=partial(nn.LayerNorm, eps=1e-6), **cases.MAR_GOLDEN, **kw)
    amp = dict(pretrained_model_path=None, model_size="mar_golden")
    for k in cases.POLICY_AMP_KEYS:
        amp[k] = cases.MAR_KW[k]
    pol = _ref_policy(UnifiedVideoActionPolicy, AD, amp)
    pol.train()
    ema_model = copy.deepcopy(pol)
    L = cases.TRACE_LR
    opt = pol.get_optimizer(weight_decay=L["weight_decay"], learning_rate=L["lr"], betas=L["betas"])

    def cosine(step, warm=L["warmup"], total=L["total"]):
        if step < warm:
            return step / max(1, warm)
        prog = (step - warm) / max(1, total - warm)
        return max(0.0, 0.5 * (1.0 + math.cos(math.pi * 0.5 * 2.0 * prog)))

    sched = torch.optim.lr_scheduler.LambdaLR(opt, cosine, last_epoch=-1)
    ema = EMAModel(ema_model, **cases.TRACE_EMA)

    class Cfg:
        class task:
            name = "pusht"

    rows = []
    for step in range(cases.TRACE_STEPS):
        b = cases.trace_batch(step)
        batch = {"obs": {"image": torch.from_numpy(b["image"]), "agent_pos": torch.from_numpy(b["agent_pos"])},
                 "action": torch.from_numpy(b["action"])}
        batch = data_utils.resize_image(Cfg, batch)
        rng = cases.trace_rng(step)
        pol.model.mask_ratio_generator = type("G", (), {"rvs": staticmethod(
            lambda n, r=rng["mask_rate"]: np.array([r]))})()
        with injected(rng):
            loss, (lv, la) = pol(batch)
        loss.backward()
        opt.step()
        opt.zero_grad()
        sched.step()
        ema.step(pol)
        rows.append([loss.item(), float(lv), float(la), sched.get_last_lr()[0], ema.decay])
        print(f"trace step {step} {rng['task_mode']}: loss={loss.item():.6f} lr={rows[-1][3]:.3e} "
              f"decay={ema.decay:.6f}")
    live = dict(pol.named_parameters())
    avg = dict(ema_model.named_parameters())
    out = {"rows": np.array(rows, np.float64), "names": np.array(cases.TRACE_PARAMS)}
    out["live"] = np.stack([checksum(live[n]) for n in cases.TRACE_PARAMS])
    out["ema"] = np.stack([checksum(avg[n]) for n in cases.TRACE_PARAMS])
    def heads(d):
        h = np.zeros((len(cases.TRACE_PARAMS), 8), np.float64)
        for i, n in enumerate(cases.TRACE_PARAMS):
            v = d[n].detach().double().reshape(-1)[:8].numpy()
            h[i, :len(v)] = v
        return h

    out["live_heads"], out["ema_heads"] = heads(live), heads(avg)
    np.savez(os.path.join(OUT, "g6_workspace_trace.npz"), **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["indexing", "mar", "block", "mlp", "diffusion_math", "vae",
                             "resize", "ema", "policy", "sample", "predict", "vae_decode", "video_sample"]
    for w in which:
        globals()[f"gen_{w}"]()
