"""Training entry point with the reference's CLI (train.py:1-68):

    python train.py --config-name=uva_pusht [--config-dir=DIR] [key=value ...]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py --config-name=uva_pusht ...
    accelerate launch --num_processes=8 train.py --config-dir=. --config-name=uva_pusht.yaml ...

Composes the Hydra-style config (unified_video_action_amd/config.py: defaults, overrides,
${...} / ${eval:...} interpolation) from --config-dir (default: this package's config tree;
the reference's own config directory works too), applies the reference's adjustments
(train.py:35-56: top-k monitor for video-only runs, n_gpus, debug batch sizes) and runs
`get_class(cfg.model._target_)(cfg).run()`.
"""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse_argv(argv):
    config_dir = os.path.join(ROOT, "unified_video_action_amd", "config")
    config_name, overrides = None, []
    it = iter(argv)
    for a in it:
        if "local_rank" in a:  # deepspeed / legacy launchers (train.py:64-67)
            continue
        if a.startswith("--config-dir") or a.startswith("--config-path") or a.startswith("-cp"):
            v = a.split("=", 1)[1] if "=" in a else next(it)
            config_dir = os.path.abspath(v)
        elif a.startswith("--config-name") or a.startswith("-cn"):
            config_name = a.split("=", 1)[1] if "=" in a else next(it)
        else:
            overrides.append(a)
    if config_name is None:
        raise SystemExit("train.py: --config-name=<name> is required (e.g. uva_pusht)")
    return config_dir, config_name, overrides


def build_cfg(argv):
    from unified_video_action_amd import config as C
    config_dir, config_name, overrides = parse_argv(argv)
    cfg = C.compose(config_dir, config_name, overrides)
    if not cfg.model.policy.action_model_params.predict_action:
        topk = cfg.checkpoint.topk
        topk.monitor_key = "video_fvd"
        topk.format_str = "epoch={epoch:04d}-video_fvd={video_fvd:.3f}.ckpt"
        topk.mode = "min"
    try:
        import torch
        cfg.n_gpus = torch.cuda.device_count()
    except Exception:
        cfg.n_gpus = 0
    cfg.model.policy.debug = cfg.training.debug
    if cfg.training.debug:
        cfg.dataloader.batch_size = 2
        cfg.val_dataloader.batch_size = 2
        cfg.dataloader.shuffle = False
        cfg.val_dataloader.shuffle = False
        if "env_runner" in cfg.task:
            cfg.task.env_runner.max_steps = 20
        if "dataloader_cfg" in cfg.task.dataset:
            cfg.task.dataset.dataloader_cfg.batch_size = 2
    return cfg


def main(argv=None):
    from unified_video_action_amd import config as C
    cfg = build_cfg(sys.argv[1:] if argv is None else argv)
    cls = C.get_class(cfg.model._target_)
    workspace = cls(cfg)
    workspace.run()
    return workspace


if __name__ == "__main__":
    main()
