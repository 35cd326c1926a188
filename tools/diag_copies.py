"""Which Python call sites issue host->device / device->device copies in one bench step
(torch.profiler, CPU-side op events with stacks)."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from unified_video_action_amd import presets  # noqa: E402

pol, opt, sched, ema = bench.build("pusht_video", "bf16", "cuda")
batch = presets.synthetic_batch("pusht_video", 32, "cuda", seed=1)
for _ in range(2):
    bench.step(pol, opt, sched, ema, batch)
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    bench.step(pol, opt, sched, ema, batch)
    torch.cuda.synchronize()
cnt = collections.Counter()
for e in prof.events():
    if e.name in ("aten::copy_", "aten::_to_copy", "aten::to", "aten::clone", "aten::item", "aten::_local_scalar_dense",
                  "aten::index", "aten::index_put_", "aten::nonzero", "aten::masked_select", "aten::cat", "aten::zero_", "aten::fill_"):
        st = [f for f in (e.stack or []) if "unified_video_action_amd" in f or "bench.py" in f]
        cnt[(e.name, st[0] if st else "?")] += 1
for (n, s), v in cnt.most_common(40):
    print(f"{v:5d} {n:28s} {s}")
