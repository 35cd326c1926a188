"""Summaries of rocprofv3 sqlite output (rocpd_*.db): per-kernel dispatch count / mean duration, and
per-kernel mean PMC values.  tools only.  python tools/rocpd_read.py file.db [...]"""
import sqlite3
import sys
from collections import defaultdict


def short(name, n=70):
    return name if len(name) <= n else name[:n] + "..."


def main(paths):
    for f in paths:
        c = sqlite3.connect(f)
        print(f"== {f}")
        rows = c.execute("""select s.display_name, d.end - d.start, d.id from rocpd_kernel_dispatch d
                            join rocpd_info_kernel_symbol s on d.kernel_id = s.id""").fetchall()
        dur = defaultdict(list)
        for name, t, _ in rows:
            dur[name].append(t)
        for name, ts in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
            print(f"  {len(ts):4d} x {sum(ts) / len(ts) / 1e3:9.1f} us  {short(name)}")
        try:
            pm = c.execute("""select s.display_name, i.name, p.value from rocpd_pmc_event p
                              join rocpd_info_pmc i on p.pmc_id = i.id
                              join rocpd_event e on p.event_id = e.id
                              join rocpd_kernel_dispatch d on d.event_id = e.id
                              join rocpd_info_kernel_symbol s on d.kernel_id = s.id""").fetchall()
        except sqlite3.Error as ex:
            print("  (pmc query failed:", ex, ")")
            pm = []
        agg = defaultdict(lambda: defaultdict(list))
        for name, ctr, v in pm:
            agg[name][ctr].append(v)
        for name, ctrs in agg.items():
            print(f"  pmc {short(name)}")
            for ctr, vs in sorted(ctrs.items()):
                print(f"      {ctr:28s} {sum(vs) / len(vs):16.0f}  (n={len(vs)})")


if __name__ == "__main__":
    main(sys.argv[1:])
