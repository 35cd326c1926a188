"""Where does the bf16 path lose gradient precision?  One golden MAR case run twice on the GPU (fp32,
then bf16, same inputs and draws): per-parameter relative L2 error of the bf16 gradient against the
fp32 one (which matches the reference to 3e-3).  python tools/diag_bf16_layers.py pusht policy_model"""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, ".")
import torch
import test_parity_gpu as T

variant, mode = sys.argv[1], sys.argv[2]
grads = {}
for prec in ("fp32", "bf16"):
    T._precision(prec)
    m, loss, lv, la = T.run_mar(variant, mode)
    loss.backward()
    grads[prec] = {n: p.grad.detach().double().clone() for n, p in m.named_parameters() if p.grad is not None}
    print(prec, "loss", loss.item(), float(lv), float(la))
rows = []
for n, g in grads["fp32"].items():
    b = grads["bf16"][n]
    e = ((b - g).norm() / (g.norm() + 1e-30)).item()
    rows.append((e, n, tuple(g.shape), g.norm().item()))
for e, n, shp, nrm in sorted(rows, reverse=True)[:40]:
    print(f"{e:8.4f}  {n:60s} {str(shp):18s} |g|={nrm:.3e}")
