"""rocprofv3 kernel trace CSV -> per (kernel, grid size) dispatch count and average / median
duration, so a shape-specific kernel (e.g. the level-0 VAE conv, grid 33554432) can be compared
with bench.py's HIP-event average.  usage: kt_by_grid.py <run_kernel_trace.csv> <out.csv>"""
import csv
import statistics
import sys
from collections import defaultdict


def main(src, dst):
    d = defaultdict(list)
    with open(src) as f:
        rd = csv.DictReader(f)
        cols = rd.fieldnames or []
        print("columns:", cols)
        gx = [c for c in ("Grid_Size", "Grid_Size_X") if c in cols]
        for r in rd:
            grid = r[gx[0]] if gx else ""
            if gx and gx[0] == "Grid_Size_X":
                grid = str(int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1))
            d[(r["Kernel_Name"], grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = sorted(((sum(v), k, v) for k, v in d.items()), reverse=True)
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Grid_Size", "Calls", "TotalDurationNs", "AverageNs", "MedianNs"])
        for tot, (name, grid), v in rows:
            w.writerow([name, grid, len(v), tot, round(tot / len(v), 1), statistics.median(v)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
