"""debug: how close to zero the action trunk's ReLU pre-activations get in the pusht_hist / pusht policy
golden cases (fp32 torch on this build's trunk input) -- tools only"""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, ".")
import torch, torch.nn.functional as F
import test_parity_gpu as tp
tp._precision("fp32")
for variant, mode in (("pusht_hist", "policy_model"), ("pusht_hist", "inverse_model"), ("pusht_hist", "full_dynamic_model")):
    cap = {}
    m0 = tp.build_mar(variant)
    orig = m0.diffactloss.trunk
    def trunk(z, orig=orig):
        cap["z"] = z.detach().clone()
        return orig(z)
    tp.build_mar = (lambda v, m0=m0: m0)
    m0.diffactloss.trunk = trunk
    m, loss, lv, la = tp.run_mar(variant, mode)
    z = cap["z"].double()
    d = m.diffactloss
    B, N, D = z.shape
    x = z.reshape(B * 4, 16, 16, D).permute(0, 3, 1, 2)
    pre = F.conv2d(x, d.conv[0].weight.double(), d.conv[0].bias.double(), padding=1)
    post = F.adaptive_avg_pool2d(F.relu(pre), (4, 4)).reshape(B * 4, -1)
    pre2 = post @ d.fc[0].weight.double().t() + d.fc[0].bias.double()
    for name, t in (("conv", pre), ("fc0", pre2)):
        a = t.abs().flatten()
        print(variant, mode, name, "n", a.numel(), "min|pre| %.3e  scale %.3e  ratio %.3e  below 1e-6*scale: %d" % (
            a.min().item(), a.max().item(), a.min().item() / a.max().item(), int((a < 1e-6 * a.max()).sum())))
