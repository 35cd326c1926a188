"""Busy / idle time of the GPU over the last optimizer steps of a rocprofv3 kernel trace: the union
of kernel intervals (any stream) between consecutive fused-AdamW launches, vs the wall time between
them.  python tools/step_gaps.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
marks = [e for s, e, n in ev if "adamw_ema" in n]
# one adamw launch per param-group region: keep the last launch of each burst
steps = []
for m in marks:
    if steps and m - steps[-1] < 2_000_000:  # < 2 ms apart: same optimizer step
        steps[-1] = m
    else:
        steps.append(m)
print(f"optimizer steps in trace: {len(steps)}")
for a, b in zip(steps[-6:-1], steps[-5:]):
    iv = sorted((max(s, a), min(e, b)) for s, e, _ in ev if e > a and s < b)
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    gaps.sort(reverse=True)
    n = sum(1 for s, e, _ in ev if s >= a and s < b)
    print(f"step {(b - a) / 1e6:8.2f} ms  busy {busy / 1e6:8.2f} ms  idle {(b - a - busy) / 1e6:6.2f} ms  "
          f"launches {n}  largest gaps (us) {[round(g / 1e3, 1) for g in gaps[:6]]}")
