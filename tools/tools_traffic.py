"""Per-launch HBM traffic of the traced bench kernels from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, separate runs of bench.py --steps 1) -> profiles/traffic_*.json.

bytes/launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   (FETCH_SIZE counts half the bytes of
wide streaming reads on gfx950, MI355X_MICROARCH.md §HBM).  A bench tag that spans several
kernels (attn_bwd = pre + dK/dV + dQ) sums them; kernels shared by several tags are told
apart by grid size.

python tools/tools_traffic.py gpurun_out/prof/pmc_fetch gpurun_out/prof/pmc_write profiles/traffic_r01.json
"""
import collections
import csv
import json
import os
import sys

# bench tag -> list of (kernel-name substring, grid size or None); a tag whose launches run ONE of
# several kernels (the GN convs: with a residual on conv3x3_halo, without on the persistent
# conv3x3_gn_pt) is in MEAN: its per-launch traffic is the launch-weighted mean.  The persistent
# kernel's grid is the same at every level (2 workgroups per CU): its launches are told apart by
# size (("size", k): the k-th largest quarter... see split_pt)
MEAN = {"conv3x3/s1 bf16 256x256 Ci128 Co128 n256", "conv3x3/s1 bf16 128x128 Ci128 Co128 n256"}
TAGS = {
    "attn_bwd B32 N1024 H12": [("attn_bwd_dkdv", None), ("attn_bwd_dq", None),
                               ("attn_bwd_fused", None), ("attn_bwd_mask", None)],
    "attn_fwd B32 N1024 H12": [("attn_fwd", None), ("attn_mask", None)],
    "conv3x3/s1 bf16 256x256 Ci128 Co128 n256": [("conv3x3_halo", "33554432"), ("conv3x3_gn_pt", "hi")],
    "conv3x3/s1 bf16 128x128 Ci128 Co128 n256": [("conv3x3_halo", "8388608"), ("conv3x3_gn_pt", "lo")],
    "conv3x3/s1 bf16 64x64 Ci256 Co256 n256": [("conv3x3_halo", "4194304")],
}


def per_kernel(d, counter):
    """(kernel, grid) -> [(per-dispatch counter value) in dispatch order].  The persistent GN conv runs
    the same grid at 256x256 and 128x128: its dispatches are split into the larger half ("hi", level
    0: 4x the pixels) and the smaller half ("lo")."""
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            out[(r["Kernel_Name"], r["Grid_Size"])][r.get("Dispatch_Id", r.get("Correlation_Id", ""))] += float(
                r["Counter_Value"])
    res = {}
    for (name, g), by_disp in out.items():
        vals = list(by_disp.values())
        if "conv3x3_gn_pt" in name:
            vals.sort()
            half = len(vals) // 2
            if half:
                res[(name, "lo")] = sum(vals[:half]) / half
                res[(name, "hi")] = sum(vals[half:]) / (len(vals) - half)
            continue
        res[(name, g)] = sum(vals) / len(vals)
    return res


def main(fetch_dir, write_dir, out_path):
    f = per_kernel(fetch_dir, "FETCH_SIZE")
    w = per_kernel(write_dir, "WRITE_SIZE")
    res = {}
    for tag, parts in TAGS.items():
        tot, hit, nk = 0.0, False, 0
        for sub, grid in parts:
            for (name, g), v in f.items():
                if sub in name and (grid is None or g == grid):
                    tot += (2 * v + w.get((name, g), 0.0)) * 1024
                    hit = True
                    nk += 1
        if hit:
            res[tag] = int(tot / nk) if tag in MEAN else int(tot)
    res["_note"] = ("per-launch HBM bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE half-count "
                    "correction, MI355X_MICROARCH.md §HBM), rocprofv3 --pmc passes of bench.py --steps 1; "
                    "multi-kernel attention tags summed, GN-conv tags the mean of their residual / no-residual "
                    "kernels (tools_traffic.py)")
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
