"""Inference latency of predict_action (PushT joint config, mar_base, full KL-VAE, 100-step action
sampler) and of the action sampler alone, graph vs eager.  Run on the GPU box:
    python tools/tools_infer_bench.py [--batches 1,32] [--iters 10]
Prints one JSON line per batch size."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,32")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--config", default="pusht_joint")
    a = ap.parse_args()
    from unified_video_action_amd import presets
    from unified_video_action_amd.policy.unified_video_action_policy import UnifiedVideoActionPolicy
    dev = torch.device("cuda:0")
    pol = UnifiedVideoActionPolicy(**presets.policy_kwargs(a.config)).to(dev).eval()
    presets.fit_normalizer(a.config, pol)
    dal = pol.model.diffactloss

    def timed(fn, iters):
        fn()
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters, (time.perf_counter() - t0) * 1e3 / iters

    for B in [int(x) for x in a.batches.split(",")]:
        obs = presets.synthetic_batch(a.config, B, dev, seed=B)["obs"]
        ms_pred, wall_pred = timed(lambda: pol.predict_action(obs), a.iters)
        z = torch.randn(B, 1024, pol.model.decoder_embed.weight.shape[0], device=dev)
        dal._sampler = None
        ms_samp, _ = timed(lambda: dal.sample(z, 0.95), a.iters)
        dal._sampler.use_graph = False
        dal._sampler._cache = None
        ms_eager, _ = timed(lambda: dal.sample(z, 0.95), max(2, a.iters // 2))
        dal._sampler = None
        print(json.dumps({"what": "predict_action", "config": a.config, "batch": B, "ms": round(ms_pred, 3),
                          "wall_ms": round(wall_pred, 3), "actions_per_s": round(B * 16 / ms_pred * 1e3, 1),
                          "sampler_graph_ms": round(ms_samp, 3), "sampler_eager_ms": round(ms_eager, 3),
                          "steps": dal.act_diff_testing_steps}), flush=True)


if __name__ == "__main__":
    main()
