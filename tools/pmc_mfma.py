"""MFMA utilisation per kernel from one rocprofv3 --pmc pass over a short bench run
(tools/pmc_step.sh): counters SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, SQ_ACTIVE_INST_VALU,
SQ_WAVE_CYCLES, SQ_BUSY_CYCLES.

  kernel cycles     = GRBM_GUI_ACTIVE / 8          (rocprofv3 sums the 8 XCDs)
  mfma_busy_frac    = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles * 1024 SIMDs)
                      (SQ_VALU_MFMA_BUSY_CYCLES counts SIMD-cycles: 16 per v_mfma_f32_16x16x32_bf16,
                       MI355X_MICROARCH.md 'Per-instruction cycle constants')
  valu_per_mfma     = SQ_ACTIVE_INST_VALU * 4 / SQ_VALU_MFMA_BUSY_CYCLES   (quad-cycles -> cycles)

python tools/pmc_mfma.py gpurun_out/pmc_mfma/run_counter_collection.csv [out.json]
"""
import collections
import csv
import json
import sys

WANT = ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES")


def short(name):
    n = name.split("(")[0]
    for pre in ("void ", "__global__ "):
        n = n.replace(pre, "")
    return n[:90]


def main(path, out=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] in WANT:
            key = (short(r["Kernel_Name"]), r.get("Grid_Size", ""))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for (k, grid), c in acc.items():
        v = {n: sum(x) / len(x) for n, x in c.items()}
        launches = max(len(x) for x in c.values())
        cyc = v.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        if cyc <= 0:
            continue
        rows.append({"kernel": k, "grid": grid, "launches": launches, "kernel_cycles": cyc,
                     "mfma_busy_frac": busy / (cyc * 1024.0),
                     "valu_cycles_per_mfma_cycle": (v.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / busy) if busy else None,
                     "total_cycles": cyc * launches})
    rows.sort(key=lambda r: -r["total_cycles"])
    tot = sum(r["total_cycles"] for r in rows)
    wmf = sum(r["total_cycles"] * r["mfma_busy_frac"] for r in rows) / tot if tot else 0.0
    print(f"{'share':>6} {'mfma':>6} {'valu/mfma':>9} {'launch':>6}  kernel")
    for r in rows[:30]:
        vm = r["valu_cycles_per_mfma_cycle"]
        print(f"{r['total_cycles'] / tot:6.3f} {r['mfma_busy_frac']:6.3f} {vm if vm is not None else float('nan'):9.2f} "
              f"{r['launches']:6d}  {r['kernel']} [{r['grid']}]")
    print(f"time-weighted MFMA busy fraction over all kernels: {wmf:.3f}")
    if out:
        json.dump({"note": __doc__, "time_weighted_mfma_busy_frac": wmf, "kernels": rows[:60]}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:3])
