"""Data-parallel reducer on CPU with torch.distributed gloo, world_size 2: bucket layout of
the flat gradient buffer, async per-bucket launches + tail bucket, 1/world averaging, and
equality with a single-process run on the concatenated batch."""
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
            h = h + b(h)
        return self.head(h).square().mean()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from unified_video_action_amd.runtime import RT
    from unified_video_action_amd.workspace.optim import GradReducer, ParamStore
    RT.set_precision("fp32")
    torch.manual_seed(0)
    m = Tiny()
    store = ParamStore(m)
    red = GradReducer(store, [(b, b) for b in m.blocks])
    assert len(red.buckets) == 3 and all(len(r) <= 2 for r in red.buckets)
    g = torch.Generator().manual_seed(123)
    x = torch.randn(8, 4, generator=g)[rank * 4:(rank + 1) * 4]
    loss = m(x)
    loss.backward()
    for i in reversed(range(3)):  # what the fused Block backward hooks do, in backward order
        m.blocks[i]._uva_bucket_hook()
    red.finish()
    q.put((rank, (store.grad / world).clone()))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_grad_reducer_world2_matches_single_process():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
    assert torch.allclose(res[0], res[1])
    # single process on the full batch = mean of the two half-batch gradients
    from unified_video_action_amd.runtime import RT
    from unified_video_action_amd.workspace.optim import ParamStore
    RT.set_precision("fp32")
    torch.manual_seed(0)
    m = Tiny()
    store = ParamStore(m)
    g = torch.Generator().manual_seed(123)
    x = torch.randn(8, 4, generator=g)
    m(x[:4]).backward()
    m(x[4:]).backward()
    RT.set_precision("bf16")
    assert torch.allclose(res[0], store.grad / 2, atol=1e-6)
