"""Golden-case definitions shared by make_golden.py (generation, reference side) and
the tests (replay, build side): model geometry, inputs and injected RNG draws.

All random draws of one reference training step (SURVEY §8c "RNG sources") are
replaced by deterministic hash streams so that the reference, the oracle and the
HIP path see identical values:
  orders      numpy shuffle per sample       mar_con_unified.py:414-422
  mask_rate   scipy truncnorm.rvs            mar_con_unified.py:428
  text_drop   torch.rand(B) (label drop)     mar_con_unified.py:629
  t_*/noise_* torch.randint / randn_like     diffusion_loss.py:51-56, gaussian_diffusion.py:761
  vae_eps_*   torch.randn (posterior.sample) vaekl.py:414-416
  task_mode   random.choice                  unified_video_action_policy.py:408
"""
import math

import numpy as np

from hashinit import hash_normal, hash_tensor, uniform_pm1

# Reduced MAR at FULL token geometry (4 frames x 256 tokens, 16-ch latents).
MAR_GOLDEN = dict(
    encoder_embed_dim=128, encoder_depth=1, encoder_num_heads=2,
    decoder_embed_dim=128, decoder_depth=1, decoder_num_heads=2, mlp_ratio=4,
)
MAR_KW = dict(
    img_size=256, vae_stride=16, patch_size=1, vae_embed_dim=16, mask_ratio_min=0.7,
    label_drop_prob=0.1, attn_dropout=0.0, proj_dropout=0.0, diffloss_d=2, diffloss_w=64,
    diffloss_act_d=2, diffloss_act_w=64, num_sampling_steps="100", diffusion_batch_mul=1,
    grad_checkpointing=False, predict_video=True, act_diff_training_steps=1000,
    act_diff_testing_steps="100", use_history_action=False, action_mask_ratio=0.5,
    predict_wrist_img=False,
)

ALL_MODES = ["video_model", "dynamic_model", "policy_model", "inverse_model", "full_dynamic_model"]

VARIANTS = {
    "pusht": dict(task_name="pusht", Da=2, clip=False, use_proprioception=False,
                  predict_proprioception=False, different_history_freq=False, modes=ALL_MODES),
    "libero": dict(task_name="libero_10", Da=10, clip=True, use_proprioception=False,
                   predict_proprioception=False, different_history_freq=False, modes=ALL_MODES),
    "umi": dict(task_name="umi", Da=10, clip=True, use_proprioception=True,
                predict_proprioception=True, different_history_freq=True,
                modes=["policy_model", "full_dynamic_model"]),
}
# variants outside every shipped config (uva.yaml: use_history_action null), pinned by their own
# reference runs (make_golden.py gen_mar_extra) and tests (test_mar_variants_gpu.py), not by the oracle
EXTRA_VARIANTS = {
    # input stream "mar/pusht_hist/e": with the first stream ("mar/pusht_hist") conv pre-activations of
    # the action trunk (262144 per case) lay within 8.6e-8 of their max from zero in policy_model, so
    # fp32 summation order alone flipped a ReLU between the reference and this build and moved the
    # gradients by up to 5e-3 (tools/hist_dbg2.py).  Among streams b-g (reference runs on the CPU),
    # "e" has the widest smallest margin over the three action modes, 1.06e-6 of max -- ~10x this
    # build's fp32 deviation from the reference on the trunk input
    "pusht_hist": dict(task_name="pusht", Da=2, clip=False, use_proprioception=False,
                       predict_proprioception=False, different_history_freq=False, use_history_action=True,
                       modes=ALL_MODES, input_tag="mar/pusht_hist/e"),
    # toolhang (config/task/toolhang.yaml) with the proprioception streams (second camera latents +
    # eef pos / quat / gripper, :126-147, 545-566) and the proprioception head (9-d, :331-344) ...
    "toolhang_prop": dict(task_name="toolhang", Da=10, clip=False, use_proprioception=True,
                          predict_proprioception=True, different_history_freq=False, modes=ALL_MODES),
    # ... and with the wrist-camera video stream + its video loss (predict_wrist_img, :97-114, 281-294, 738-776)
    "toolhang_wrist": dict(task_name="toolhang", Da=10, clip=False, use_proprioception=True,
                           predict_proprioception=True, different_history_freq=False, predict_wrist_img=True,
                           modes=ALL_MODES),
}
B_MAR = 2


def variant_def(variant):
    return VARIANTS[variant] if variant in VARIANTS else EXTRA_VARIANTS[variant]


def mar_kwargs(variant):
    v = variant_def(variant)
    kw = dict(MAR_KW)
    kw.update(
        use_history_action=v.get("use_history_action", False),
        predict_wrist_img=v.get("predict_wrist_img", False),
        task_name=v["task_name"], use_proprioception=v["use_proprioception"],
        predict_proprioception=v["predict_proprioception"],
        different_history_freq=v["different_history_freq"],
        language_emb_model="clip" if v["clip"] else None,
        action_model_params=dict(predict_action=True, act_model_type="conv_fc"),
        shape_meta={"action": {"shape": [v["Da"]]}},
    )
    return kw


def uses_video(mode):
    return mode in ("video_model", "dynamic_model", "full_dynamic_model")


def uses_action(mode):
    return mode in ("policy_model", "inverse_model", "full_dynamic_model")


def orders(tag, B, L=256):
    return np.stack([np.argsort(uniform_pm1(f"{tag}/orders/{b}", L), kind="stable")
                     for b in range(B)]).astype(np.int64)


def t_steps(tag, n, T=1000):
    u = (uniform_pm1(f"{tag}/t", n) + 1.0) * 0.5
    t = np.minimum((u * T).astype(np.int64), T - 1)
    t[:3] = [0, 1, T - 1]  # always exercise the t==0 decoder-NLL branch and both ends
    return t


def mask_rate(tag):
    u = (uniform_pm1(f"{tag}/rate", 1)[0] + 1.0) * 0.5
    return 0.7 + 0.3 * float(u)


def mar_inputs(variant, B=B_MAR):
    v = variant_def(variant)
    tag = v.get("input_tag", f"mar/{variant}")
    d = {
        "z": hash_normal(f"{tag}/z", (B, 4, 16, 16, 16)),
        "c": hash_normal(f"{tag}/c", (B, 4, 16, 16, 16)),
        "nactions": hash_tensor(f"{tag}/nactions", (B, 16, v["Da"])),
    }
    if v["clip"]:
        d["text_latents"] = hash_normal(f"{tag}/text", (B, 512))
    if v.get("use_history_action"):
        d["history_nactions"] = hash_tensor(f"{tag}/hist", (B, 16, v["Da"]))
    if v["use_proprioception"] and v["task_name"] != "umi":
        d["second_image_z"] = hash_normal(f"{tag}/z2", (B, 4, 16, 16, 16))
        for i, (k, n) in enumerate((("robot0_eef_pos", 3), ("robot0_eef_quat", 4), ("robot0_gripper_qpos", 2))):
            d[k] = hash_tensor(f"{tag}/s{i}", (B, 16, n))
            d[k + "_pred"] = hash_tensor(f"{tag}/s{i}p", (B, 16, n))
    if v.get("predict_wrist_img"):
        d["pred_second_image_z"] = hash_normal(f"{tag}/z2p", (B, 4, 16, 16, 16))
    if v["use_proprioception"] and v["task_name"] == "umi":
        d["robot0_eef_pos"] = hash_tensor(f"{tag}/p0", (B, 4, 3))
        d["robot0_eef_rot_axis_angle"] = hash_tensor(f"{tag}/p1", (B, 4, 6))
        d["robot0_gripper_width"] = hash_tensor(f"{tag}/p2", (B, 4, 1))
        d["robot0_eef_rot_axis_angle_wrt_start"] = hash_tensor(f"{tag}/p3", (B, 4, 6))
        d["robot0_eef_rot_axis_angle_wrt_start_pred"] = hash_tensor(f"{tag}/p4", (B, 16, 6))
    return d


def mar_rng(variant, mode, B=B_MAR):
    """Injected draws for one MAR.forward call, in the reference's call order."""
    v = variant_def(variant)
    tag = f"mar/{variant}/{mode}"
    r = {"orders": orders(tag, B), "mask_rate": mask_rate(tag), "randint": [], "randn_like": []}
    if v.get("use_history_action"):
        # torch.rand(B, T*4) of the history-action drop (:512-518); half the draws either side of 0.5
        r["hist_u"] = ((uniform_pm1(tag + "/hist_u", B * 16) + 1.0) * 0.5).astype(np.float32).reshape(B, 16)
    if v["clip"]:
        r["text_drop_u"] = np.array([0.05] + [0.5] * (B - 1), dtype=np.float32)  # sample 0 dropped
    if uses_video(mode):
        r["randint"].append(t_steps(tag + "/video", B * 1024))
        r["randn_like"].append(hash_normal(tag + "/video/noise", (B * 1024, 16)))
        if v.get("predict_wrist_img"):
            r["randint"].append(t_steps(tag + "/wrist", B * 1024))
            r["randn_like"].append(hash_normal(tag + "/wrist/noise", (B * 1024, 16)))
    if uses_action(mode):
        r["randint"].append(t_steps(tag + "/act", B * 16))
        r["randn_like"].append(hash_normal(tag + "/act/noise", (B * 16, v["Da"])))
    if v["predict_proprioception"]:
        r["randint"].append(t_steps(tag + "/prop", B * 16))
        r["randn_like"].append(hash_normal(tag + "/prop/noise", (B * 16, 6 if v["task_name"] == "umi" else 9)))
    return r


def num_masked(rate, L=256):
    return int(math.ceil(L * rate))


# ---- policy-level (config 1 semantics, B=1, full VAE, reduced MAR) -----------------
POLICY_B = 1
POLICY_MODES = ["full_dynamic_model", "video_model"]


def policy_batch(B=POLICY_B):
    img = (hash_tensor("policy/image", (B, 32, 3, 96, 96)) + 1.0) * 0.5
    pos = (hash_tensor("policy/agent_pos", (B, 32, 2)) + 1.0) * 256.0
    act = (hash_tensor("policy/action", (B, 32, 2)) + 1.0) * 256.0
    return {"image": img, "agent_pos": pos, "action": act}


def policy_rng(mode, B=POLICY_B):
    tag = f"policy/{mode}"
    r = mar_rng("pusht", mode, B)
    r["vae_eps_x"] = hash_normal(tag + "/eps_x", (B * 4, 16, 16, 16))
    r["vae_eps_c"] = hash_normal(tag + "/eps_c", (B * 4, 16, 16, 16))
    return r


SAMPLE_STEPS = 100  # act_diff_testing_steps="100"
SAMPLE_TEMPERATURE = 0.95  # config/model/uva.yaml:45


def sample_rng(variant, B=B_MAR):
    """Injected draws of one sample_tokens(policy_model) call, in the reference's order:
    orders (:994), x_T (diffusion_action_loss.py:212), then one randn_like per p_sample step
    (gaussian_diffusion.py:431)."""
    v = variant_def(variant)
    tag = f"sample/{variant}"
    rows = B * 16
    return {
        "orders": np.stack([np.random.default_rng(i).permutation(256) for i in range(B)]).astype(np.int64),
        "noise": hash_normal(f"{tag}/xT", (rows, v["Da"])),
        "step_noise": hash_normal(f"{tag}/steps", (SAMPLE_STEPS, rows, v["Da"])),
    }


def predict_rng(B=POLICY_B):
    """predict_action draws: posterior eps of the 4 eval frames ((b t) order, vaekl.py:414),
    then the sampler's x_T and per-step noise (sample_rng semantics)."""
    r = sample_rng("pusht", B)
    r["noise"] = hash_normal("predict/xT", (B * 16, 2))
    r["step_noise"] = hash_normal("predict/steps", (SAMPLE_STEPS, B * 16, 2))
    r["vae_eps"] = hash_normal("predict/eps", (B * 4, 16, 16, 16))
    return r


POLICY_AMP_KEYS = ("img_size", "vae_stride", "patch_size", "vae_embed_dim", "mask_ratio_min", "label_drop_prob",
                   "attn_dropout", "proj_dropout", "diffloss_d", "diffloss_w", "diffloss_act_d", "diffloss_act_w",
                   "num_sampling_steps", "diffusion_batch_mul", "grad_checkpointing", "predict_video",
                   "act_diff_training_steps", "act_diff_testing_steps")


VIDEO_SAMPLE_ITERS = 2


def video_sample_rng(variant, num_iter=VIDEO_SAMPLE_ITERS, B=B_MAR):
    """Draws of sample_tokens(video_model) over num_iter MaskGIT iterations: per iteration the
    action head (x_T, 100 steps) then the video head on the tokens predicted in that iteration
    (mar_con_unified.py:1026-1100; counts follow the cosine schedule, mask_by_order)."""
    import math
    v = variant_def(variant)
    tag = f"vsample/{variant}"
    r = {"orders": sample_rng(variant, B)["orders"], "act_noise": [], "act_step_noise": [],
         "video_noise": [], "video_step_noise": []}
    wrist = bool(v.get("predict_wrist_img"))
    if wrist:  # diffloss_wrist.sample after the video head, on the same rows (:1118-1140)
        r["wrist_noise"], r["wrist_step_noise"] = [], []
    cur = 256
    for step in range(num_iter):
        ml = max(1.0, min(cur - 1.0, float(np.floor(256 * np.cos(math.pi / 2.0 * (step + 1) / num_iter)))))
        pred = cur if step >= num_iter - 1 else cur - int(ml)
        cur = int(ml)
        rows = B * 4 * pred
        r["act_noise"].append(hash_normal(f"{tag}/{step}/axT", (B * 16, v["Da"])))
        r["act_step_noise"].append(hash_normal(f"{tag}/{step}/asteps", (SAMPLE_STEPS, B * 16, v["Da"])))
        r["video_noise"].append(hash_normal(f"{tag}/{step}/vxT", (rows, 16)))
        r["video_step_noise"].append(hash_normal(f"{tag}/{step}/vsteps", (SAMPLE_STEPS, rows, 16)))
        if wrist:
            r["wrist_noise"].append(hash_normal(f"{tag}/{step}/wxT", (rows, 16)))
            r["wrist_step_noise"].append(hash_normal(f"{tag}/{step}/wsteps", (SAMPLE_STEPS, rows, 16)))
    return r


# ---- workspace trace (reference per-step body, workspace:279-302) -------------------------
TRACE_STEPS = 4
TRACE_MODES = ["full_dynamic_model", "video_model", "policy_model", "full_dynamic_model"]
TRACE_LR = dict(name="cosine", warmup=1, total=10, lr=1e-4, betas=(0.9, 0.95), weight_decay=0.02)
TRACE_EMA = dict(update_after_step=0, inv_gamma=1.0, power=0.75, min_value=0.0, max_value=0.9999)
TRACE_PARAMS = ("model.z_proj.weight", "model.encoder_blocks.0.attn.qkv.weight", "model.decoder_norm.weight",
                "model.diffloss.net.res_blocks.0.mlp.0.weight", "model.diffactloss.net.final_layer.linear.bias")


def trace_batch(step, B=POLICY_B):
    img = (hash_tensor(f"trace/{step}/image", (B, 32, 3, 96, 96)) + 1.0) * 0.5
    pos = (hash_tensor(f"trace/{step}/agent_pos", (B, 32, 2)) + 1.0) * 256.0
    act = (hash_tensor(f"trace/{step}/action", (B, 32, 2)) + 1.0) * 256.0
    return {"image": img, "agent_pos": pos, "action": act}


def trace_rng(step, B=POLICY_B):
    mode = TRACE_MODES[step]
    tag = f"trace/{step}/{mode}"
    r = mar_rng("pusht", mode, B)
    # distinct draws per step (mar_rng is keyed by mode only)
    r["orders"] = orders(tag, B)
    r["mask_rate"] = mask_rate(tag)
    r["randint"] = [t_steps(f"{tag}/{i}", len(x)) for i, x in enumerate(r["randint"])]
    r["randn_like"] = [hash_normal(f"{tag}/{i}/noise", x.shape) for i, x in enumerate(r["randn_like"])]
    r["vae_eps_x"] = hash_normal(tag + "/eps_x", (B * 4, 16, 16, 16))
    r["vae_eps_c"] = hash_normal(tag + "/eps_c", (B * 4, 16, 16, 16))
    r["task_mode"] = mode
    return r


# ---- policy-level Libero / UMI cases (config 4 / 5 plumbing through compute_loss) ----------
POLICY_VARIANT_MODES = {"libero": ["full_dynamic_model", "policy_model"],
                        "umi": ["full_dynamic_model", "policy_model"],
                        # toolhang's second camera through the policy: wrist frames VAE-encoded with their own
                        # posterior draws (vae_eps_wrist), eef / gripper streams split into history / future
                        "toolhang_prop": ["full_dynamic_model", "policy_model"],
                        # ... and with the wrist-camera video stream + its loss (predict_wrist_img)
                        "toolhang_wrist": ["full_dynamic_model"]}


def umi_img_indices(tag, B):
    out = np.zeros((B, 8, 1), np.float32)
    for b in range(B):
        u = uniform_pm1(f"{tag}/idx/{b}", 16)
        hist = np.sort(np.argsort(u, kind="stable")[:4])
        out[b, :, 0] = np.concatenate([hist, [19, 23, 27, 31]])
    return out


REF_LATENT_KEYS = ("cup", "towel", "mouse")


def ref_language_latents(B, start=0):
    """[B, 512] rows of the reference's own prepared_data/language_latents.pkl,
    cycling cup / towel / mouse from `start`; extracted without unpickling by
    extract_ref_fixtures.py into ref_fixtures.npz."""
    import os
    f = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_fixtures.npz"))
    rows = [f["language_latents/" + REF_LATENT_KEYS[(start + i) % 3]] for i in range(B)]
    return np.stack(rows).astype(np.float32)


def policy_variant_batch(variant, B=POLICY_B):
    """Libero / UMI batches; the language latents are the reference's own CLIP latents (G6)."""
    tag = f"policy/{variant}"
    if variant.startswith("toolhang"):
        obs = {"sideview_image": (hash_tensor(tag + "/img", (B, 32, 3, 128, 128)) + 1.0) * 0.5,
               "robot0_eye_in_hand_image": (hash_tensor(tag + "/wrist", (B, 32, 3, 128, 128)) + 1.0) * 0.5}
        for k, d in (("robot0_eef_pos", 3), ("robot0_eef_quat", 4), ("robot0_gripper_qpos", 2)):
            obs[k] = hash_normal(f"{tag}/{k}", (B, 32, d))
        return {"obs": obs, "action": hash_tensor(tag + "/action", (B, 32, 10)),
                "language_latents": ref_language_latents(B, 2)}
    if variant == "libero":
        return {"obs": {"agentview_rgb": (hash_tensor(tag + "/img", (B, 32, 3, 128, 128)) + 1.0) * 0.5},
                "action": hash_tensor(tag + "/action", (B, 32, 10)),
                "language_latents": ref_language_latents(B, 0)}
    obs = {"camera0_rgb": (hash_tensor(tag + "/img", (B, 8, 3, 224, 224)) + 1.0) * 0.5,
           "img_indices": umi_img_indices(tag, B)}
    for k, d in (("robot0_eef_pos", 3), ("robot0_eef_rot_axis_angle", 6), ("robot0_gripper_width", 1),
                 ("robot0_eef_rot_axis_angle_wrt_start", 6)):
        obs[k] = hash_normal(f"{tag}/{k}", (B, 32, d))
    return {"obs": obs, "action": hash_normal(tag + "/action", (B, 32, 10)),
            "language_latents": ref_language_latents(B, 1)}


def policy_variant_rng(variant, mode, B=POLICY_B):
    tag = f"policy/{variant}/{mode}"
    r = mar_rng(variant, mode, B)
    r["vae_eps_x"] = hash_normal(tag + "/eps_x", (B * 4, 16, 16, 16))
    r["vae_eps_c"] = hash_normal(tag + "/eps_c", (B * 4, 16, 16, 16))
    r["task_mode"] = mode
    if variant.startswith("toolhang"):
        # the wrist frames' posterior draws, [future half | history half] as the policy encodes them; the
        # reference draws the history half first (get_vae_latent: second_image, then pred_second_image)
        r["vae_eps_wrist"] = hash_normal(tag + "/eps_w", (2 * B * 4, 16, 16, 16))
    # keep the text (no label drop): the batch carries the reference's own CLIP latents (G6); the
    # label-drop branch is pinned by the g2_mar goldens, whose sample 0 is dropped
    r["text_drop_u"] = np.full(B, 0.5, dtype=np.float32)
    return r


def policy_variant_kwargs(variant):
    """UnifiedVideoActionPolicy kwargs (besides vae / autoregressive params) of the variant."""
    v = variant_def(variant)
    umi = variant == "umi"
    return dict(action_model_params=dict(predict_action=True, act_model_type="conv_fc"),
                shape_meta={"action": {"shape": [v["Da"]]}}, n_action_steps=8, shift_action=not umi,
                language_emb_model="clip", task_name=v["task_name"],
                task_modes=["policy_model", "full_dynamic_model"] if umi else [],
                normalizer_type="none" if umi or "toolhang" in variant else "all", selected_training_mode=None, use_history_action=False,
                use_proprioception=v["use_proprioception"], action_mask_ratio=0.5,
                different_history_freq=v["different_history_freq"], predict_wrist_img=v.get("predict_wrist_img", False),
                predict_proprioception=v["predict_proprioception"])


GRAD_SKETCH_K = 4


def grad_sketch(name, a):
    """GRAD_SKETCH_K random +-1 projections of a flattened gradient (float64 numpy), signs drawn
    from the parameter's name.  Unlike the plain sum, a projection's error under per-element
    noise has the random-walk size rms(err) * sqrt(n) whatever the gradient's mean, so
    |sketch - ref| / (rms * sqrt(n)) is a well-conditioned relative error of the whole gradient."""
    import zlib
    a = np.asarray(a, np.float64).reshape(-1)
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    r = rng.integers(0, 2, size=(GRAD_SKETCH_K, a.size), dtype=np.int8).astype(np.float64) * 2 - 1
    return r @ a
