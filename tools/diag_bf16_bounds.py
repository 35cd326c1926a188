"""Per-parameter bf16 gradient checksum errors of every bf16 parity case (tests/test_parity_gpu.py: the 27
MAR variant x mode cases and the policy cases), this build's error next to the reference's own bf16 run's
error for the same parameter -- the data behind assert_bf16_grads' bounds.  Runs each test body with the
bound check replaced by a recorder; writes one JSON (tools only).

    python tools/diag_bf16_bounds.py out.json"""
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

import test_parity_gpu as T  # noqa: E402
import cases  # noqa: E402

REC = []
CUR = {}


def record(errs, ref_errs):
    REC.append({"case": dict(CUR), "errs": errs, "ref_errs": ref_errs})


def main(out):
    T.assert_bf16_grads = record
    jobs = [("mar", dict(variant=v, mode=m), T.test_mar_bf16_loss_and_grads_match_reference) for v, m in T.MAR_CASES]
    jobs += [("policy", dict(mode=m, prec="bf16"), T.test_policy_compute_loss_end_to_end) for m in cases.POLICY_MODES]
    jobs += [("policy_variant", dict(variant=v, mode=m, prec="bf16"), T.test_policy_variants_compute_loss_vs_reference)
             for v, ms in cases.POLICY_VARIANT_MODES.items() for m in ms]
    for kind, kw, fn in jobs:
        CUR.clear()
        CUR.update(kind=kind, **kw)
        try:
            fn(**kw)
        except Exception:
            REC.append({"case": dict(CUR), "error": traceback.format_exc()[-800:]})
        print(kind, kw, "ok" if "error" not in REC[-1] else "ERROR", flush=True)
    json.dump(REC, open(out, "w"))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bf16_bounds.json")
