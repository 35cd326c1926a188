"""Summarise tools/pmc_kernel.sh: per kernel (name filtered by a substring) mean counters per launch
and the derived ratios (fractions of SQ_WAVE_CYCLES; MFMA busy of the launch's SIMD-cycles)."""
import collections
import csv
import glob
import os
import sys


def main(root, kf):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60] + f" g{r.get('Grid_Size', '')}"
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in sorted(acc.items()):
        if kf not in k:
            continue
        v = {n: sum(x) / len(x) for n, x in c.items()}
        wc = v.get("SQ_WAVE_CYCLES", 0) or 1
        cyc = v.get("GRBM_GUI_ACTIVE", 0) / 8
        print(k)
        line = [f"  cyc {cyc:9.0f}"]
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM", "SQ_INST_LEVEL_VMEM",
                  "SQ_VMEM_TA_ADDR_FIFO_FULL"):
            if n in v:
                line.append(f"{n[3:]} {v[n] / wc:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v and cyc:
            line.append(f"mfma_busy {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f}")
        if "SQ_VALU_MFMA_COEXEC_CYCLES" in v and cyc:
            line.append(f"coexec {v['SQ_VALU_MFMA_COEXEC_CYCLES'] / (cyc * 1024):.3f}")
        if "SQ_LDS_BANK_CONFLICT" in v and v.get("SQ_LDS_IDX_ACTIVE"):
            line.append(f"lds_conf {v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "SQ_LDS_IDX_ACTIVE" in v and cyc:
            line.append(f"lds_active {v['SQ_LDS_IDX_ACTIVE'] / (cyc * 256):.3f}")
        print("  ".join(line))
        line = ["  insts"]
        for n in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INST_CYCLES_VMEM_RD"):
            if n in v:
                line.append(f"{n[3:]} {v[n]:.4g}")
        print("  ".join(line))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
