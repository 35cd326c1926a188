"""UVA training-step throughput on MI355X (BASELINE.json metric: train samples/sec).

python bench.py --gpus N --steps K --warmup W        (N>1: launched by torch.distributed.run)

Workload (N=1 line = BASELINE configs[1]): PushT video_model, mar_base (24 blocks, D=768,
N=1024 tokens) + frozen KL-VAE encoder of 8 frames/sample, bf16 MFMA operands, dropout 0.1
as configured, batch 32 per GPU, synthetic device-resident batch of the dataset shape
([B,32,3,96,96] frames, resized on device).  One step = resize/select -> VAE encode ->
MAR fwd -> diffusion loss -> backward (-> RCCL bucket all-reduce) -> fused AdamW+EMA.
Weak scaling: batch per GPU fixed.  Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
# algorithmic GFLOP per sample per step (SURVEY §8d / BASELINE.md §3)
GFLOP_PER_SAMPLE = {"pusht_video": 2611.9, "pusht_joint": 2546.2, "libero10_joint": 2641.5, "umi_multi": 2674.2}
METRIC = "train samples/sec (video+action step) at 1/2/4/8 MI355X; loss parity"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--config", default="pusht_video", choices=sorted(GFLOP_PER_SAMPLE))
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-trace", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--trace-out", default="", help="write every traced kernel row (tag, launches, avg ms) here")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01f.json"))
    return ap.parse_args()


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def build(args, device, world):
    from unified_video_action_amd import presets
    from unified_video_action_amd.policy.unified_video_action_policy import UnifiedVideoActionPolicy
    from unified_video_action_amd.runtime import RT
    from unified_video_action_amd.workspace.optim import CosineWithWarmup, GradReducer, default_buckets
    RT.set_precision(args.precision)
    torch.manual_seed(42)  # identical init on every rank (the reference seeds every rank alike)
    pol = UnifiedVideoActionPolicy(**presets.policy_kwargs(args.config)).to(device)
    presets.fit_normalizer(args.config, pol)
    pol.train()
    opt = pol.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    opt.ema_cfg = dict(power=0.75, inv_gamma=1.0, min_value=0.0, max_value=0.9999, update_after_step=0)
    opt.grad_scale = 1.0 / world
    sched = CosineWithWarmup(opt, 1000, 100000)
    reducer = GradReducer(opt.store, default_buckets(pol.model))
    return pol, opt, sched, reducer


def step(pol, opt, sched, reducer, batch):
    loss, (lv, la) = pol(batch)
    loss.backward()
    reducer.finish()
    opt.step()
    opt.zero_grad()
    sched.step()
    return loss


def summarize_trace(trace):
    """tag -> (launches, avg ms, total ms, flops/launch); the dominant kernel by total time."""
    rows = []
    for tag, evs in trace.items():
        ms = [a.elapsed_time(b) for a, b, _ in evs]
        rows.append((sum(ms), tag, len(ms), sum(ms) / len(ms), evs[0][2]))
    rows.sort(reverse=True)
    return rows


def cpu_baseline(args):
    """oracle (PyTorch-CPU fp32 restatement, pinned to the reference) on a bounded sample:
    one full training step of the same workload at B=1."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import uva_oracle as O
    th = args.cpu_threads or torch.get_num_threads()
    torch.set_num_threads(th)
    torch.manual_seed(0)
    mar = O.mar_base(task_name="pusht", act_dim=2, predict_action=args.config != "pusht_video")
    O.set_dropout(mar, 0.1)
    vae = O.AutoencoderKLEncoder()
    pol = O.PolicyOracle(mar, vae, [2 / 512, 2 / 512], [-1.0, -1.0]).train()
    opt = torch.optim.AdamW(mar.parameters(), lr=1e-4, betas=(0.9, 0.95), weight_decay=0.02)
    B = 1
    img = torch.rand(B, 32, 3, 96, 96)
    act = torch.rand(B, 32, 2) * 512
    rng = {"orders": torch.stack([torch.randperm(256) for _ in range(B)]).numpy(), "mask_rate": 0.85,
           "randint": [torch.randint(0, 1000, (B * 1024,))], "randn_like": [torch.randn(B * 1024, 16)],
           "vae_eps_x": torch.randn(B * 4, 16, 16, 16), "vae_eps_c": torch.randn(B * 4, 16, 16, 16)}
    t0 = time.perf_counter()
    loss, _ = pol.compute_loss(img, act, "video_model", rng)
    loss.backward()
    opt.step()
    opt.zero_grad()
    dt = time.perf_counter() - t0
    return {"value": B / dt, "unit": "samples/s", "cores": th, "kind": "port",
            "sample": f"1 full training step (resize->KL-VAE->mar_base fwd/bwd->AdamW), B={B}, PushT video_model, "
                      f"fp32, dropout 0.1, oracle/uva_oracle.py; {dt:.1f} s"}


def main():
    args = parse()
    world, rank, local = setup_dist()
    device = torch.device("cuda", local)
    from unified_video_action_amd import presets
    from unified_video_action_amd.native import ops
    pol, opt, sched, reducer = build(args, device, world)
    batch = presets.synthetic_batch(args.config, args.batch, device, seed=1000 + rank)
    for _ in range(args.warmup):
        step(pol, opt, sched, reducer, batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if not args.no_trace:
        ops.TRACE = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step(pol, opt, sched, reducer, batch)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    trace, ops.TRACE = ops.TRACE, None
    final_loss = loss.item()
    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    samples = args.batch * world * args.steps
    value = samples / elapsed
    ms = elapsed / args.steps * 1e3
    gflop = GFLOP_PER_SAMPLE[args.config]
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16" if args.precision == "bf16" else "f32",
        "data": "synthetic (device-resident, dataset shapes; random-init weights)",
        "config": {"workload": f"{args.config}: PushT video_model step = frame select+resize -> KL-VAE encode "
                               f"(8 frames) -> mar_base MAR fwd/bwd (N=1024) -> diffusion loss -> AdamW+EMA; "
                               f"dropout 0.1", "model": "UVA mar_base + KL-VAE f16",
                   "global_batch": args.batch * world, "seq_len": 1024, "parallelism": f"dp{world}"},
        "step_tflops_per_gpu": round(gflop * args.batch / (ms / 1e3) / 1e3, 1),
        "step_mfma_frac": round(gflop * args.batch / (ms / 1e3) / 1e3 / PEAK_BF16_TFLOPS, 4),
        "final_loss": round(final_loss, 5),
    }
    if trace:
        rows = summarize_trace(trace)
        tot, tag, n, avg, fl = rows[0]
        ach = fl / (avg * 1e-3) / 1e12
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                traffic = json.load(open(args.traffic_json)).get(tag)
            except Exception:
                traffic = None
        out["roofline"] = {"bound": "mfma", "kernel": tag, "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS,
                           "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                           "launches_timed": n, "avg_ms": round(avg, 4),
                           "share_of_traced_time": round(tot / sum(r[0] for r in rows), 4)}
        if args.trace_out:
            with open(args.trace_out, "w") as f:
                json.dump([{"kernel": t_, "launches_per_step": n_ / args.steps, "total_ms_per_step": a / args.steps,
                            "avg_ms": av, "tflops": f_ / (av * 1e-3) / 1e12} for a, t_, n_, av, f_ in rows], f, indent=1)
        out["top_kernels"] = [{"kernel": t_, "total_ms_per_step": round(a / args.steps, 3),
                               "avg_ms": round(av, 4), "tflops": round(f_ / (av * 1e-3) / 1e12, 1)}
                              for a, t_, n_, av, f_ in rows[:8]]
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
