"""Per-step kernel time from a rocprofv3 kernel_stats.csv: python tools/kstats_per_step.py stats.csv [top]
(steps = launches of the fused AdamW+EMA kernel, one per optimizer step)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
steps = sum(int(r["Calls"]) for r in rows if "adamw_ema" in r["Name"])
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6 / steps
print(f"steps {steps}, kernel time {tot:.2f} ms/step")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms {int(r['Calls']) / steps:7.1f}/step "
          f"{float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:110]}")
