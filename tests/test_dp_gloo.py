"""Data-parallel reducer on the CPU with torch.distributed gloo, world_size 2:
  * the real policy (mar_base, PushT joint, fp32): get_optimizer's flat layout + default_buckets
    cover every trainable parameter exactly once (buckets + tail), every Block / diffusion trunk
    carries its bucket hook, and the reducer is created lazily once the process group exists; the
    26 real hooks fired in reverse order from inside a backward pass issue one collective per large
    range (the heads' remaining parameters with the last decoder Block, the decoder prelude with the
    last encoder Block; the small no-decay ranges merged into a few), the tail is only the encoder
    input side, and the reduced flat gradient equals the sum over ranks;
  * the reducer protocol on a small torch model: async per-bucket launches from backward, the
    end-of-backward completion callback, the tail bucket (also deferred to the optimizer's
    wait_tail), 1/world averaging -- equal to a single-process run on the concatenated batch;
  * the optimizer's AdamW split around a deferred tail tiles every group region once."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Tiny(nn.Module):
    def __init__(self):
        super().__init__()
        self.embed = nn.Linear(4, 8)
        self.blocks = nn.ModuleList([nn.Sequential(nn.Linear(8, 8), nn.LayerNorm(8)) for _ in range(3)])
        self.head = nn.Linear(8, 1)

    def forward(self, x):
        h = self.embed(x)
        for b in self.blocks:
            h = h + _Hook.apply(b(h), b)
        return self.head(h).square().mean()


class _Hook(torch.autograd.Function):
    """stands in for BlockFn's backward, which calls the bucket hook after its grads are enqueued."""

    @staticmethod
    def forward(ctx, x, mod):
        ctx.mod = mod
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        hook = getattr(ctx.mod, "_uva_bucket_hook", None)
        ctx.mod._pending_hook = hook  # fire once the module's own parameter grads exist (next step)
        return g, None


def _named_groups(m):
    from unified_video_action_amd.workspace.optim import is_no_decay
    named = [(n, p) for n, p in m.named_parameters()]
    return [[x for x in named if is_no_decay(*x)], [x for x in named if not is_no_decay(*x)]]


def _tiny_worker(rank, world, port, q, defer=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from unified_video_action_amd.runtime import RT
    from unified_video_action_amd.workspace.optim import GradReducer, ParamStore
    RT.set_precision("fp32")
    torch.manual_seed(0)
    m = Tiny()
    store = ParamStore(_named_groups(m))
    # the 8x8 weights (64 elements) are bucketed, the bias / LayerNorm ranges go to the tail
    red = GradReducer(store, [(b, b) for b in m.blocks], min_bucket_elems=32)
    assert len(red.buckets) == 3 and all(len(r) == 1 for r in red.buckets)
    assert int(red.coverage().min()) == 1 and int(red.coverage().max()) == 1
    g = torch.Generator().manual_seed(123)
    x = torch.randn(8, 4, generator=g)[rank * 4:(rank + 1) * 4]
    red.defer_tail = defer
    red.arm()

    # launch each block's bucket from inside backward, after its parameter grads are accumulated
    def post_hook(mod):
        def fn(*_):
            if getattr(mod, "_pending_hook", None) is not None:
                mod._pending_hook()
        return fn

    handles = [b[0].weight.register_post_accumulate_grad_hook(post_hook(b)) for b in m.blocks]
    m(x).backward()  # the queued end-of-backward callback completes the reduction
    assert not red.pending and not red.handles
    if defer:  # the tail's collectives are left in flight for the optimizer (wait_tail)
        assert len(red.tail_handles) == len(red.tail) > 0
        red.wait_tail()
    assert not red.tail_handles
    for h in handles:
        h.remove()
    # a numpy copy: a torch tensor crosses the queue as a shared-memory fd that the parent can only
    # attach while this process is alive (it may exit first)
    q.put((rank, (store.grad / world).numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("defer", [False, True])
def test_grad_reducer_world2_matches_single_process(defer):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tiny_worker, args=(r, world, port, q, defer)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: torch.from_numpy(a) for r, a in (q.get(timeout=100) for _ in range(world))}
    for p in procs:
        p.join(timeout=30)
    assert torch.allclose(res[0], res[1])
    from unified_video_action_amd.runtime import RT
    from unified_video_action_amd.workspace.optim import ParamStore
    RT.set_precision("fp32")
    torch.manual_seed(0)
    m = Tiny()
    store = ParamStore(_named_groups(m))
    g = torch.Generator().manual_seed(123)
    x = torch.randn(8, 4, generator=g)
    m(x[:4]).backward()
    m(x[4:]).backward()
    RT.set_precision("bf16")
    assert torch.allclose(res[0], store.grad / 2, atol=1e-6)


def _policy_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from unified_video_action_amd import presets
    from unified_video_action_amd.model.autoregressive.diffusion_loss import SimpleMLPAdaLN
    from unified_video_action_amd.model.autoregressive.mar_con_unified import Block
    from unified_video_action_amd.policy.unified_video_action_policy import UnifiedVideoActionPolicy
    from unified_video_action_amd.runtime import RT
    RT.set_precision("fp32")
    torch.manual_seed(0)
    pol = UnifiedVideoActionPolicy(**presets.policy_kwargs("pusht_joint"))
    opt = pol.get_optimizer(weight_decay=0.02, learning_rate=1e-4, betas=(0.9, 0.95))
    assert opt.maybe_init_reducer(pol.model) is None  # no process group yet (accelerate order)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    red = opt.maybe_init_reducer(pol.model)
    cov = red.coverage()
    st = opt.store
    inside = torch.zeros(st.total, dtype=torch.bool)
    for _, p in st.order:
        o, k = st.offsets[id(p)]
        inside[o:o + k] = True
    n_trainable = sum(p.numel() for p in pol.model.parameters() if p.requires_grad)
    hooked = [m for m in pol.model.modules() if isinstance(m, (Block, SimpleMLPAdaLN))]
    # the real hooks of the 26 modules fired from inside a backward pass in reverse order (as the
    # fused BlockFn / AdaLNTrunkFn backwards fire them), each launching ONE collective; the
    # end-of-backward callback reduces the tail (all no-decay ranges + the rest) and waits
    calls = []
    real_all_reduce = dist.all_reduce

    def counting_all_reduce(t, *a, **k):
        calls.append(t.numel())
        return real_all_reduce(t, *a, **k)

    dist.all_reduce = counting_all_reduce
    idx = torch.arange(st.total, dtype=torch.float32)
    st.grad.copy_((rank + 1) * torch.remainder(idx, 977.0))

    class FireHooks(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.clone()

        @staticmethod
        def backward(ctx, g):
            for m in reversed(hooked):
                m._uva_bucket_hook()
            return g

    red.arm()
    FireHooks.apply(torch.zeros(1, requires_grad=True)).sum().backward()
    dist.all_reduce = real_all_reduce
    ok = bool(torch.equal(st.grad[inside], 3.0 * torch.remainder(idx, 977.0)[inside]))
    n_bucket_calls = sum(1 for n in calls if n >= red.MIN_BUCKET_ELEMS)
    q.put((rank, int(cov[inside].min()), int(cov[inside].max()), int(cov.max()), st.n_params, n_trainable,
           len(hooked), sum(callable(getattr(m, "_uva_bucket_hook", None)) for m in hooked), opt.grad_scale,
           len(red.buckets), ok, len(calls), len(red.tail), sum(len(b) for b in red.buckets), n_bucket_calls,
           red.pending, sum(k for _, k in red.tail)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_mar_base_buckets_cover_every_param_once():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_policy_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=280) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for (rank, cmin, cmax, call, n_store, n_train, n_hooked, n_with_hook, scale, n_buckets, ok, n_calls, n_tail,
         n_ranges, n_bucket_calls, pending, tail_elems) in res:
        assert cmin == 1 and cmax == 1 and call == 1, (cmin, cmax, call)
        assert n_store == n_train == 261_079_156, n_store  # PushT joint MAR
        # 24 Blocks + 2 diffusion trunks, + the heads' remaining params (time / cond embeddings,
        # input_proj, the conv_fc trunk) fired by the last decoder Block, + the decoder prelude fired
        # by the last encoder Block
        assert n_hooked == 26 and n_with_hook == 26 and n_buckets == 28
        assert scale == 0.5
        assert ok, "reduced flat gradient != sum over ranks"
        assert n_ranges >= 28 and n_bucket_calls >= n_ranges, (n_ranges, n_bucket_calls)
        assert tail_elems < 2_100_000, tail_elems  # only the encoder input side (~8 MB) after backward
        # + the small no-decay ranges, merged with their neighbours into a handful of collectives
        assert n_tail <= 4 and 1 <= n_calls - n_ranges - n_tail <= 8, (n_calls, n_ranges, n_tail)
        assert not pending


def test_bench_gpus_n_spawns_n_ranks():
    """`bench.py --gpus 2` with no launcher environment spawns two workers that rendezvous on
    127.0.0.1 and agree on the world size (the driver's N>1 invocation path; gloo, no GPU)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launch-check"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line == {"launch_check": True, "world": 2, "gpus": 2, "rank_sum": 1.0}


def test_bench_under_torchrun_sees_the_launcher_world():
    """the driver's exact N>1 command line (torch.distributed.run, 127.0.0.1) reaches the same
    rendezvous check without spawning a second level of workers."""
    import json
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--launch-check"], cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines == [{"launch_check": True, "world": 2, "gpus": 2, "rank_sum": 1.0}]


def test_adamw_tail_segments_split():
    """the optimizer's two AdamW phases under a deferred tail: the widened (16-B aligned) tail
    segments and their complement tile every group region exactly once, every piece 16-B aligned."""
    from unified_video_action_amd.workspace.optim import GradReducer, _segments
    red = GradReducer.__new__(GradReducer)
    red.tail = [(5, 3), (9, 20), (101, 2), (300, 77)]
    segs = red.tail_segments()
    assert segs == [(4, 28), (100, 4), (300, 80)]
    for off, n in [(0, 64), (96, 256), (380, 1000)]:
        cnt = torch.zeros(off + n, dtype=torch.int32)
        for ph in (0, 1):
            for o, k in _segments(off, n, segs, ph):
                assert o % 4 == 0 and k > 0
                cnt[o:o + k] += 1
        assert bool((cnt[off:] == 1).all()) and int(cnt[:off].sum()) == 0
        assert _segments(off, n, segs, None) == [(off, n)]
    for o, k in red.tail:  # every tail element is in a phase-1 piece
        assert any(a <= o and o + k <= a + b for a, b in segs)
