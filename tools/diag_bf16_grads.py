"""Per-case bf16 gradient checksum errors vs the reference goldens, beside the reference's own bf16
(autocast) error (diagnostic for test_parity_gpu): python tools/diag_bf16_grads.py"""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, ".")
import test_parity_gpu as T
import cases, replay
T._precision("bf16")
for v in cases.VARIANTS:
    for mode in cases.VARIANTS[v]["modes"]:
        g = replay.load(f"g2_mar_{v}_{mode}.npz")
        m, loss, lv, la = T.run_mar(v, mode)
        loss.backward()
        errs, ref = T.bf16_grad_errors(m.named_parameters(), g, "grad_names", "grad_sums", "grad_sketch")
        import numpy as np
        eo = np.sqrt(np.mean([e * e for e in errs.values()]))
        er = np.sqrt(np.mean([e * e for e in ref.values()]))
        top = sorted(errs.items(), key=lambda kv: -kv[1] / max(T.BF16_TOL, 3 * ref[kv[0]], 3 * er))[:2]
        print(v, mode, "rms ours %.4f ref %.4f" % (eo, er),
              [(n, round(e, 4), round(ref[n], 4)) for n, e in top], flush=True)
