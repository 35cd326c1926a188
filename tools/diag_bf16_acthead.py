"""bf16 vs fp32 gradients at the action head's interfaces (trunk input z, trunk output c, the
diffusion net's output) on one golden MAR case: python tools/diag_bf16_acthead.py pusht policy_model"""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, ".")
import torch
import test_parity_gpu as T
from unified_video_action_amd.model.autoregressive import diffusion_action_loss as dal
from unified_video_action_amd.model.autoregressive import diffusion_loss as dl

variant, mode = sys.argv[1], sys.argv[2]
store = {}
orig_fwd = dal.DiffActLoss.forward
orig_trunk = dal.DiffActLoss.trunk


def _tap(name, t):
    store[name] = t.detach().double().clone()
    t.register_hook(lambda g: store.__setitem__("d" + name, g.detach().double().clone()))
    return t


def trunk(self, z):
    # DiffActLoss.trunk with every intermediate tapped
    B, N, D = z.shape
    _tap("z", z)
    f = z.reshape(B * 4, 16, 16, D)
    f = _tap("conv", dal.Conv3x3ReluFn.apply(f, self.conv[0].weight, self.conv[0].bias))
    f = _tap("pool", f.reshape(B * 4, 4, 4, 4, 4, D).mean(dim=(2, 4)))
    f = f.permute(0, 3, 1, 2).reshape(B * 4, D * 16)
    f = _tap("fc0", dal.linear(f, self.fc[0], act="relu", out_dtype=dal.cdt()))
    f = _tap("fc2", dal.linear(f, self.fc[2], out_dtype=dal.F32).reshape(B, 4, D))
    f = _tap("interp", dal.linear(f.transpose(1, 2), self.interpolate, out_dtype=dal.F32).transpose(1, 2))
    f = _tap("ref0", dal.linear(f, self.refine[0], act="relu", out_dtype=dal.cdt()))
    return _tap("c", dal.linear(f, self.refine[2], out_dtype=dal.F32))


dal.DiffActLoss.trunk = trunk
orig_hl = dl.diffusion_head_loss


def hl(net, sched, target, c, mask, t, noise):
    out = orig_hl(net, sched, target, c, mask, t, noise)
    return out


res = {}
for prec in ("fp32", "bf16"):
    T._precision(prec)
    store.clear()
    m, loss, lv, la = T.run_mar(variant, mode)
    loss.backward()
    res[prec] = dict(store)
for k in ("z", "conv", "pool", "fc0", "fc2", "interp", "ref0", "c", "dc", "dref0", "dinterp", "dfc2", "dfc0", "dpool", "dconv", "dz"):
    if k in res["fp32"]:
        a, b = res["fp32"][k], res["bf16"][k]
        print(k, tuple(a.shape), "rel L2 err %.4f" % ((b - a).norm() / a.norm()).item(), "|a| %.3e" % a.norm().item())
