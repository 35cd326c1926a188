"""Per-kernel summary of rocprofv3 --pmc / --kernel-trace output directories (tools only):
counter means per dispatch, SQ wait / issue buckets as fractions of SQ_WAVE_CYCLES, mean traced duration.

    python tools/pmc_kernels.py <name-substring> <dir> [<dir> ...]"""
import collections
import csv
import glob
import sys


def main(sub, dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True):
            per = collections.defaultdict(float)
            for r in csv.DictReader(open(f)):
                if sub in r["Kernel_Name"]:
                    per[(r["Kernel_Name"][:80], r.get("Dispatch_Id", ""), r["Counter_Name"])] += float(r["Counter_Value"])
            for (k, _, c), v in per.items():
                agg[k][c].append(v)
        for f in glob.glob(d + "/**/run_kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if sub in r["Kernel_Name"]:
                    dur[r["Kernel_Name"][:80]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k in sorted(set(agg) | set(dur)):
        m = {c: sum(v) / len(v) for c, v in agg[k].items()}
        print(k)
        if dur[k]:
            print(f"  traced: {len(dur[k])} dispatches, mean {sum(dur[k]) / len(dur[k]):.1f} us")
        wc = m.get("SQ_WAVE_CYCLES")
        for c in sorted(m):
            extra = f"  ({m[c] / wc:.3f} of wave cycles)" if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
            print(f"  {c:28s} {m[c]:.4g}{extra}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
