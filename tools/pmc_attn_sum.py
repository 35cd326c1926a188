"""Summarise tools/pmc_attn.sh: per (build, kernel) mean counters per launch and derived ratios."""
import collections
import csv
import glob
import os
import sys


def main(root):
    for build in ("base", "new"):
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for f in glob.glob(os.path.join(root, f"{build}_*", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f"=== {build}")
        for k, c in sorted(acc.items()):
            if "attn" not in k:
                continue
            v = {n: sum(x) / len(x) for n, x in c.items()}
            wc = v.get("SQ_WAVE_CYCLES", 0) or 1
            cyc = v.get("GRBM_GUI_ACTIVE", 0) / 8
            line = [f"{k:48s}", f"cyc {cyc:9.0f}"]
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA"):
                if n in v:
                    line.append(f"{n[3:]} {v[n] / wc:.3f}")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in v and cyc:
                line.append(f"mfma_busy {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f}")
            if "SQ_LDS_BANK_CONFLICT" in v and v.get("SQ_LDS_IDX_ACTIVE"):
                line.append(f"lds_conf {v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']:.3f}")
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM"):
                if n in v:
                    line.append(f"{n[9:]} {v[n]:.3g}")
            print("  ".join(line))


if __name__ == "__main__":
    main(sys.argv[1])
