"""Phase timeline of the persistent sampler from the ps_stamps diagnostic build (tools/conv_diag_build.py
ps_stamps; python tools/ab_run.py abx/diag_ps_stamps.so tools/ps_stamps.py): s_memtime deltas (shader cycles)
of workgroup 0 at step 50."""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests/golden")
from hashinit import hash_init_
from unified_video_action_amd.model.autoregressive.diffusion_loss import SimpleMLPAdaLN
from unified_video_action_amd.model.autoregressive.sampler import ActionSampler

net = SimpleMLPAdaLN(2, 1024, 4, 128, 6)
hash_init_(net, "sampler_net.")
net = net.to("cuda").eval()
R = 16
c = torch.randn(R, 128, device="cuda")
noise = torch.randn(R, 2, device="cuda")
steps = torch.randn(100, R, 2, device="cuda")
smp = ActionSampler(net, "100")
for _ in range(3):
    smp(c, noise, steps, 0.95)
torch.cuda.synchronize()
st = smp._cache["work"].view(torch.int64)[1024 // 8:1024 // 8 + 80].cpu().tolist()
names = ["step", "proj"]
for b in range(6):
    names += ([f"b{b}.fc1.wait"] if b else []) + [f"b{b}.fc1.ln", f"b{b}.fc1.pub", f"b{b}.fc2.wait", f"b{b}.fc2.pub"]
names += ["fin.wait"]
prev = st[0]
for n, t in zip(names, st):
    print(f"{n:14s} {t - prev:8d}")
    prev = t
