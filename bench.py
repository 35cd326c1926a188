"""UVA training-step throughput on MI355X (BASELINE.json metric: train samples/sec).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config pusht_video] [--batch 32]

N > 1: run under torch.distributed.run (RANK / WORLD_SIZE / LOCAL_RANK from the environment),
or -- when those are unset -- this process spawns N fresh worker processes (one per GPU,
RCCL over xGMI) before it touches the GPU, and exits with their status.

Workload (the N=1 line = BASELINE configs[1]): PushT video_model, mar_base (24 blocks, D=768,
N=1024 tokens) + frozen KL-VAE encoder of 8 frames/sample, bf16 MFMA operands, dropout 0.1 as
configured, batch 32 per GPU, synthetic device-resident batch of the dataset shape
([B,32,3,96,96] frames, resized on device).  One step = the reference workspace's per-step body
(workspace:283-302): policy(batch) [frame select+resize -> VAE encode -> MAR fwd -> diffusion
loss] -> backward (-> RCCL bucket all-reduce inside backward) -> optimizer.step (fused AdamW
+ EMA) -> zero_grad -> lr_scheduler.step -> ema.step.  Weak scaling: batch per GPU fixed.

Timing: W untimed warm-up steps, then exactly K steps between barrier + synchronize pairs, max
over ranks (`value`, `ms_per_step`), plus the median of the K per-step HIP-event times.  The
per-kernel trace for `roofline` (HIP events around the traced launches on their stream) runs
in a separate short pass afterwards, so its event overhead is not in `value`.  At N=1 the
default run also measures the PushT joint video+action step (BASELINE configs[2] at its
per-GPU batch 64) and reports it under "other_configs" in the same JSON line.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
# algorithmic GFLOP per sample per step (SURVEY §8d / BASELINE.md §3)
GFLOP_PER_SAMPLE = {"pusht_video": 2611.9, "pusht_joint": 2546.2, "libero10_joint": 2641.5, "umi_multi": 2674.2}
METRIC = "train samples/sec (video+action step) at 1/2/4/8 MI355X; loss parity"
# tokens per sample in the MAR (4 frames x 256 latent tokens, + 64 CLIP text tokens for Libero / UMI)
SEQ_LEN = {"pusht_video": 1024, "pusht_joint": 1024, "libero10_joint": 1088, "umi_multi": 1088}
WORKLOAD = {
    "pusht_video": "PushT video_model (BASELINE configs[1])",
    "pusht_joint": "PushT joint video+action, all 5 task modes (BASELINE configs[2] per-GPU batch)",
    "libero10_joint": "Libero10 joint + CLIP language latents, N=1088 (BASELINE configs[3] per-GPU batch)",
    "umi_multi": "UMI-multi proprio in/out, different_history_freq, 224px frames (BASELINE configs[4])",
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--config", default="pusht_video", choices=sorted(GFLOP_PER_SAMPLE))
    ap.add_argument("--precision", default="bf16", help="bf16 | fp8_attn (fp8 e4m3 attention) | fp32")
    ap.add_argument("--other-configs",
                    default="pusht_joint:64,libero10_joint:32,umi_multi:56:bf16,umi_multi:56:fp8_attn",
                    help="N=1 only: extra config:batch[:precision] entries measured after the main line "
                         "('' = none; precision defaults to --precision)")
    ap.add_argument("--other-steps", type=int, default=20)
    ap.add_argument("--launch-check", action="store_true",
                    help="check the --gpus N process wiring (gloo, no GPU work) and exit")
    ap.add_argument("--h2d-steps", type=int, default=10,
                    help="N=1: steps fed from host batches through the pinned prefetcher (0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=2, help="CPU baseline batch (BASELINE configs[0]: 2)")
    ap.add_argument("--cpu-warmup", type=int, default=5, help="CPU warm-up steps (BASELINE.md §4: 5)")
    ap.add_argument("--cpu-steps", type=int, default=10, help="timed CPU steps, median reported (BASELINE.md §4: 10)")
    ap.add_argument("--cpu-budget-s", type=float, default=200.0,
                    help="wall budget of the B=2 leg: fewer timed steps (stated in `sample`) when a step is slow")
    ap.add_argument("--no-trace", action="store_true")
    ap.add_argument("--trace-steps", type=int, default=3)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the host's physical cores, capped by this process's cgroup CPU quota")
    ap.add_argument("--no-cpu-batch-gpu", dest="cpu_batch_gpu", action="store_false",
                    help="skip the CPU baseline step at the config's per-GPU batch (~3.5 min at B=32)")
    ap.add_argument("--wall-budget-s", type=float, default=530.0,
                    help="the per-GPU-batch CPU step runs only if the whole bench is expected to end within this")
    ap.add_argument("--trace-out", default="", help="write every traced kernel row (tag, launches, avg ms) here")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r06_end.json"))
    return ap.parse_args(argv)


# ---- process launch --------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawned(local_rank, world, port, argv):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run(parse(argv))


def launch(args, argv):
    """--gpus N with no launcher environment: spawn N workers (fresh interpreters; this parent
    has not initialised the GPU) and return their exit status."""
    import torch.multiprocessing as mp
    ctx = mp.start_processes(_spawned, args=(args.gpus, _free_port(), argv), nprocs=args.gpus, join=False,
                             start_method="spawn")
    try:
        while not ctx.join():
            pass
    except Exception as e:  # a worker failed: its traceback is in the message
        print(f"bench.py: worker failed: {e}", file=sys.stderr, flush=True)
        return 1
    return 0


def setup_dist(args):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {dist.get_world_size()} ranks")
    elif args.gpus != 1:
        raise SystemExit(f"bench.py: --gpus {args.gpus} needs {args.gpus} processes")
    return world, rank, local


# ---- one training setup + step (the reference workspace's per-step body) ---------------------
def build(config, precision, device):
    import copy

    import torch
    from unified_video_action_amd import presets
    from unified_video_action_amd.model.autoregressive.ema_model import EMAModel
    from unified_video_action_amd.model.common.lr_scheduler import get_scheduler
    from unified_video_action_amd.policy.unified_video_action_policy import UnifiedVideoActionPolicy
    from unified_video_action_amd.runtime import RT
    RT.set_precision(precision)
    torch.manual_seed(42)  # identical init on every rank (the reference seeds every rank alike)
    pol = UnifiedVideoActionPolicy(**presets.policy_kwargs(config))
    presets.fit_normalizer(config, pol)
    ema_model = copy.deepcopy(pol)  # workspace:70-72 (before get_optimizer, as the reference)
    opt = pol.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    opt.overlap_tail = True  # step() follows backward directly: the DP tail reduces under AdamW
    pol.to(device).train()
    ema_model.to(device)
    sched = get_scheduler("cosine", opt, num_warmup_steps=1000, num_training_steps=100000)
    ema = EMAModel(ema_model, update_after_step=0, inv_gamma=1.0, power=0.75, min_value=0.0, max_value=0.9999)
    return pol, opt, sched, ema


def step(pol, opt, sched, ema, batch):
    loss, (lv, la) = pol(batch)
    loss.backward()  # the bucket reducer (world > 1) completes inside backward
    opt.step()
    opt.zero_grad()
    sched.step()
    ema.step(pol)
    return loss


def summarize_trace(trace):
    """tag -> (total ms, tag, launches, avg ms, flops/launch, side stream), by total time."""
    rows = []
    for tag, evs in trace.items():
        ms = [e[0].elapsed_time(e[1]) for e in evs]
        rows.append((sum(ms), tag, len(ms), sum(ms) / len(ms), evs[0][2], any(e[3] for e in evs)))
    rows.sort(reverse=True)
    return rows


def traced_pass(state, steps, only=None):
    """`steps` more training steps with HIP events around the library launches (all of them, or only the
    tags in `only`) -> (summarize_trace rows, mean step ms by events around each step)"""
    import torch
    from unified_video_action_amd.native import ops
    pol, opt, sched, ema, batch = state
    ops.TRACE, ops.TRACE_ONLY = {}, (set(only) if only else None)
    sev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    try:
        for a, b in sev:
            a.record()
            step(pol, opt, sched, ema, batch)
            b.record()
        torch.cuda.synchronize()
        trace = ops.TRACE
    finally:
        ops.TRACE, ops.TRACE_ONLY = None, None
    return summarize_trace(trace), sum(a.elapsed_time(b) for a, b in sev) / steps


def timed_run(config, batch_size, steps, warmup, precision, device, world, rank):
    """-> (elapsed s max over ranks, per-step ms list, final loss, (pol, opt, sched, ema, batch))."""
    import torch
    import torch.distributed as dist
    from unified_video_action_amd import presets
    pol, opt, sched, ema = build(config, precision, device)
    batch = presets.synthetic_batch(config, batch_size, device, seed=1000 + rank)
    for _ in range(warmup):
        step(pol, opt, sched, ema, batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        evs[i][0].record()
        loss = step(pol, opt, sched, ema, batch)
        evs[i][1].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    per_step = [a.elapsed_time(b) for a, b in evs]
    return elapsed, per_step, loss.item(), (pol, opt, sched, ema, batch)


def h2d_probe(state, device, steps):
    """PCIe-inclusive numbers beside `value` (which starts from HBM-resident inputs): the pinned
    host -> device copy of one batch alone, and steps fed through utils.prefetch.PinnedPrefetcher
    (copy of batch i+1 on a copy stream under step i) from pageable host batches."""
    import torch
    from unified_video_action_amd.utils.prefetch import PinnedPrefetcher, _leaves, _map
    pol, opt, sched, ema, batch = state
    host = _map(batch, lambda t: t.cpu())
    nbytes = sum(t.numel() * t.element_size() for t in _leaves(host, []))
    pinned = _map(host, lambda t: t.pin_memory())
    for _ in range(2):
        _map(pinned, lambda t: t.to(device, non_blocking=True))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        _map(pinned, lambda t: t.to(device, non_blocking=True))
    torch.cuda.synchronize()
    copy_ms = (time.perf_counter() - t0) / 5 * 1e3
    step(pol, opt, sched, ema, batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in PinnedPrefetcher([host] * steps, device, depth=2):
        step(pol, opt, sched, ema, b)
    torch.cuda.synchronize()
    fed_ms = (time.perf_counter() - t0) / steps * 1e3
    return {"bytes_per_batch": nbytes, "pinned_copy_ms": round(copy_ms, 3),
            "pinned_copy_GBps": round(nbytes / copy_ms / 1e6, 2), "steps_fed_from_host": steps,
            "ms_per_step_fed_from_host": round(fed_ms, 2)}


def cpu_quota():
    """CPUs this process may use by its cgroup (v2 cpu.max / v1 cfs quota), or None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def cpu_threads(args, info):
    """all host cores (physical), but never more than the cgroup quota allows (a
    thread pool over the quota only time-slices)."""
    if args.cpu_threads:
        return args.cpu_threads
    n = info.get("physical_cores") or info.get("usable") or os.cpu_count() or 1
    q = cpu_quota()
    if q is not None:
        n = min(n, q)
    return max(1, min(n, info.get("usable") or n))


def cpu_baseline(args):
    """oracle (PyTorch-CPU fp32 restatement, pinned to the reference) timed per BASELINE.md §4: all
    physical host cores (cgroup quota permitting), 5 warm-up steps + the median of 10 at BASELINE
    configs[0]'s batch (2), then one step at the config's per-GPU batch (within --wall-budget-s).  The B=2 leg keeps to
    --cpu-budget-s: if the warm-up shows a step too slow for 15 of them, fewer are timed (stated)."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import uva_oracle as O
    info = host_cpus()
    info["cgroup_quota_cpus"] = cpu_quota()
    th = cpu_threads(args, info)
    torch.set_num_threads(th)
    torch.manual_seed(0)
    mar = O.mar_base(task_name="pusht", act_dim=2, predict_action=args.config != "pusht_video")
    O.set_dropout(mar, 0.1)
    vae = O.AutoencoderKLEncoder()
    pol = O.PolicyOracle(mar, vae, [2 / 512, 2 / 512], [-1.0, -1.0]).train()
    opt = torch.optim.AdamW(mar.parameters(), lr=1e-4, betas=(0.9, 0.95), weight_decay=0.02)

    def one(B):
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
        print(f"[bench] cpu_baseline B={B} step {dt:.1f} s", file=sys.stderr, flush=True)
        return dt

    B = args.cpu_batch
    t_start = time.perf_counter()
    hb = _heartbeat("cpu_baseline")
    warm = [one(B)]
    nwarm, nsteps = args.cpu_warmup, args.cpu_steps
    if warm[0] * (nwarm + nsteps) > args.cpu_budget_s:  # keep the default bench within minutes
        nsteps = max(3, min(nsteps, int(args.cpu_budget_s / warm[0]) - 2))
        nwarm = max(1, min(nwarm, int(args.cpu_budget_s / warm[0]) - nsteps))
    warm += [one(B) for _ in range(nwarm - 1)]
    ts = [one(B) for _ in range(nsteps)]
    med = statistics.median(ts)
    proto = f"{nwarm} warm-up + median of {nsteps} steps"
    if (nwarm, nsteps) != (args.cpu_warmup, args.cpu_steps):
        proto += (f" (BASELINE.md §4 asks {args.cpu_warmup} + {args.cpu_steps}; cut to the "
                  f"{args.cpu_budget_s:.0f} s budget at {warm[0]:.1f} s per step)")
    out = {"value": round(B / med, 5), "unit": "samples/s", "cores": th, "kind": "port",
           "host_cpus": info,
           "sample": f"oracle/uva_oracle.py full training step (resize->KL-VAE->mar_base fwd/bwd->AdamW), "
                     f"PushT video_model, fp32, dropout 0.1, B={B}, torch.set_num_threads({th}): {proto} "
                     f"({', '.join(f'{t:.2f}' for t in ts)} s; B={B} leg {time.perf_counter() - t_start:.0f} s)"}
    if args.cpu_batch_gpu and args.batch != B:
        # also the per-GPU batch.  One step (the warm-ups above already paged in the weights
        # and kernels); its time is estimated from the B=2 median (x batch ratio x 1.2: round 4 measured
        # 1.14) and the step is skipped, with the reason stated, if the bench would overrun its wall budget
        est = med * args.batch / B * 1.2
        spent = time.perf_counter() - T_START
        if spent + est <= args.wall_budget_s:
            t = one(args.batch)
            out["per_gpu_batch"] = {"batch": args.batch, "value": round(args.batch / t, 5), "unit": "samples/s",
                                    "cores": th,
                                    "sample": f"one full training step at B={args.batch} after the B={B} runs "
                                              f"({t:.1f} s)"}
        else:
            out["per_gpu_batch"] = {"batch": args.batch, "value": None,
                                    "sample": f"skipped: ~{est:.0f} s estimated after {spent:.0f} s of bench "
                                              f"would pass the {args.wall_budget_s:.0f} s wall budget"}
    hb.set()
    return out


def _heartbeat(what, every=45.0):
    """a progress line on stderr every `every` s until the returned event is set (a single CPU step at
    the per-GPU batch runs for minutes; a silent process is taken for a hung one)"""
    import threading
    ev = threading.Event()
    t0 = time.perf_counter()

    def beat():
        while not ev.wait(every):
            print(f"[bench] {what}: {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()
    return ev


def host_cpus():
    """the host's CPU inventory as lscpu reports it: logical CPUs, physical cores (sockets x cores
    per socket), and the CPUs this process may run on"""
    info = {"logical": os.cpu_count()}
    try:
        info["usable"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        phys = set()
        cur = {}
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if not ln.strip():
                    if "physical id" in cur and "core id" in cur:
                        phys.add((cur["physical id"], cur["core id"]))
                    cur = {}
                    continue
                k, _, v = ln.partition(":")
                cur[k.strip()] = v.strip()
                if k.strip() == "model name":
                    info["model"] = v.strip()
        if phys:
            info["physical_cores"] = len(phys)
    except OSError:
        pass
    return info


def line_for(config, batch, world, steps, elapsed, per_step, loss):
    gflop = GFLOP_PER_SAMPLE[config]
    value = batch * world * steps / elapsed
    ms = elapsed / steps * 1e3
    med = statistics.median(per_step)
    return {"config": config, "workload": WORKLOAD[config], "global_batch": batch * world,
            "seq_len": SEQ_LEN[config], "value": round(value, 3),
            "ms_per_step": round(ms, 2), "ms_per_step_median": round(med, 2),
            "step_tflops_per_gpu": round(gflop * batch / (ms / 1e3) / 1e3, 1),
            "step_mfma_frac": round(gflop * batch / (ms / 1e3) / 1e3 / PEAK_BF16_TFLOPS, 4),
            "final_loss": round(loss, 5)}


def launch_check(args):
    """--launch-check: the N-process wiring of `--gpus N` (spawned workers or an external
    torchrun environment) without touching a GPU: gloo rendezvous, world size == --gpus, one
    all-reduce; rank 0 prints one JSON line."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
        t = torch.tensor([float(rank)])
        dist.all_reduce(t)
        ok = dist.get_world_size() == args.gpus
        dist.barrier()
        dist.destroy_process_group()
    else:
        t, ok = torch.tensor([0.0]), args.gpus == 1
    if rank == 0:
        print(json.dumps({"launch_check": ok, "world": world, "gpus": args.gpus, "rank_sum": t.item()}), flush=True)
    if not ok:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but {world} ranks")


def run(args):
    import torch
    import torch.distributed as dist
    if args.launch_check:
        launch_check(args)
        return
    world, rank, local = setup_dist(args)
    device = torch.device("cuda", local)
    from unified_video_action_amd.native import ops
    elapsed, per_step, loss, state = timed_run(args.config, args.batch, args.steps, args.warmup, args.precision,
                                               device, world, rank)
    if rank == 0:
        print(f"[bench] {args.config} B={args.batch}: {args.batch * world * args.steps / elapsed:.2f} samples/s",
              file=sys.stderr, flush=True)
    main = line_for(args.config, args.batch, world, args.steps, elapsed, per_step, loss)
    rows = None
    if not args.no_trace:
        # two short traced passes after the timed steps: (1) every library launch between HIP events, for
        # the per-kernel table (the per-launch events add idle time: its step is slower than the timed
        # one, and short kernels read long); (2) events around the roofline kernel's launches only, so
        # that pass runs at the timed step's speed and the roofline's avg_ms is measured in it
        state_ = state
        rows, traced_step_ms = traced_pass(state_, args.trace_steps)
        roof = next(r for r in rows if r[4] > 0)
        rrows, roof_step_ms = traced_pass(state_, args.trace_steps, only=[roof[1]])
        roof = rrows[0]
    h2d = h2d_probe(state, device, args.h2d_steps) if (world == 1 and args.h2d_steps > 0) else None
    del state
    others = []
    if world == 1 and args.other_configs:
        for item in args.other_configs.split(","):
            cfg, b, prec = (item.split(":") + ["", ""])[:3]
            b = int(b or args.batch)
            prec = prec or args.precision
            torch.cuda.empty_cache()
            e, ps, lo, st = timed_run(cfg, b, args.other_steps, args.warmup, prec, device, world, rank)
            del st
            others.append(dict(line_for(cfg, b, world, args.other_steps, e, ps, lo), steps=args.other_steps,
                               precision=prec))
            print(f"[bench] {cfg} B={b} {prec}: {others[-1]['value']} samples/s", file=sys.stderr, flush=True)
        from unified_video_action_amd.runtime import RT
        RT.set_precision(args.precision)
    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    out = {
        "metric": METRIC, "value": main["value"], "unit": "samples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": main["ms_per_step"], "ms_per_step_median": main["ms_per_step_median"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": {"bf16": "bf16", "fp8_attn": "bf16 (attention fp8 e4m3)"}.get(args.precision, "f32"),
        "data": "synthetic (device-resident, dataset shapes; random-init weights)",
        "config": {"workload": f"{args.config}: {WORKLOAD[args.config]}; step = frame select+resize -> KL-VAE "
                               f"encode (8 frames) -> mar_base MAR fwd/bwd (N=1024) -> diffusion loss -> backward "
                               f"-> fused AdamW + EMA -> LR step; dropout 0.1",
                   "model": "UVA mar_base + KL-VAE f16", "global_batch": args.batch * world,
                   "seq_len": SEQ_LEN[args.config],
                   "parallelism": f"dp{world}"},
        "rccl_world": world,
        "step_tflops_per_gpu": main["step_tflops_per_gpu"], "step_mfma_frac": main["step_mfma_frac"],
        "final_loss": main["final_loss"],
    }
    if rows:
        # every library launch is traced (ops._call tags the untagged entry points by name); the
        # roofline line is the dominant MFMA kernel (the traced kernel with a FLOP count and the
        # largest total time)
        tot, tag, n, avg, fl, _ = roof
        ach = fl / (avg * 1e-3) / 1e12
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                traffic = json.load(open(args.traffic_json)).get(tag)
            except (OSError, ValueError):
                traffic = None
        out["roofline"] = {"bound": "mfma", "kernel": tag, "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS,
                           "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                           "launches_timed": n, "avg_ms": round(avg, 4),
                           "timing_pass": {"events": "HIP events on the launching stream around this kernel's "
                                                     "launches only", "steps": args.trace_steps,
                                           "step_ms": round(roof_step_ms, 2),
                                           "vs_timed_step": round(roof_step_ms / main["ms_per_step"], 4)},
                           "share_of_main_stream_time": round(
                               tot / args.trace_steps / (sum(r[0] for r in rows if not r[5]) / args.trace_steps), 4)}
        if args.trace_out:
            with open(args.trace_out, "w") as f:
                json.dump([{"kernel": t_, "launches_per_step": n_ / args.trace_steps,
                            "total_ms_per_step": a / args.trace_steps, "avg_ms": av,
                            "tflops": f_ / (av * 1e-3) / 1e12, "side_stream": sd}
                           for a, t_, n_, av, f_, sd in rows], f, indent=1)
        out["top_kernels"] = [{"kernel": t_ + (" [side stream]" if sd else ""),
                               "total_ms_per_step": round(a / args.trace_steps, 3), "avg_ms": round(av, 4),
                               "tflops": round(f_ / (av * 1e-3) / 1e12, 1) if f_ > 0 else None}
                              for a, t_, n_, av, f_, sd in rows[:12]]
        main_ms = sum(r[0] for r in rows if not r[5]) / args.trace_steps
        side_ms = sum(r[0] for r in rows if r[5]) / args.trace_steps
        # GPU time of the fully traced step (events around each step on the main stream) against the time
        # inside main-stream library launches: what is left is torch glue (cat / copies / fills), launch
        # gaps and the per-launch event overhead -- no vendor-library kernel can hide in it unaccounted.
        # Side-stream launches (keep-mask planes, overlapping the VAE) are reported apart
        out["trace_accounting"] = {"events": "every library launch (top_kernels)",
                                   "traced_step_ms": round(traced_step_ms, 2),
                                   "timed_step_ms": main["ms_per_step"],
                                   "main_stream_library_ms": round(main_ms, 2),
                                   "outside_library_ms": round(traced_step_ms - main_ms, 2),
                                   "side_stream_library_ms": round(side_ms, 2),
                                   "library_entry_points": len(rows)}
    if h2d:
        out["h2d"] = h2d
    if others:
        out["other_configs"] = others
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


T_START = time.perf_counter()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args, argv))
    run(args)


if __name__ == "__main__":
    main()
