#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (the ROCm 7.2 default output, `<name>_results.db`)
into a markdown table: per kernel calls, mean / min / max us and share of GPU time.
usage: python tools/prof_db_summary.py gpurun_out/final/prof/bench_results.db "title" > profiles/x.md"""
import sqlite3
import sys

db, title = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else sys.argv[1])
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(duration), min(duration), max(duration), sum(duration) "
                 "from kernels group by name order by sum(duration) desc").fetchall()
total = sum(r[5] for r in rows) or 1
print(f"# rocprofv3 kernel summary: {title}\n")
print("| kernel | calls | mean us | min us | max us | % time |\n|---|---:|---:|---:|---:|---:|")
for name, n, avg, mn, mx, tot in rows:
    name = name.replace("|", "/")
    if len(name) > 90:
        name = name[:87] + "..."
    print(f"| `{name}` | {n} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | {100 * tot / total:.1f} |")
print("\nmxar kernels by launch shape (grid x / y, VGPRs, LDS bytes):\n")
print("| kernel | grid | VGPR | LDS | calls | median us |\n|---|---|---:|---:|---:|---:|")
shape = c.execute("select name, grid_x, grid_y, workgroup_x, vgpr_count, lds_size, duration from kernels "
                  "where name like '%mxar%'").fetchall()
groups: dict = {}
for name, gx, gy, wx, vg, lds, d in shape:
    groups.setdefault((name.split("(")[0], gx // max(wx, 1), gy, vg, lds), []).append(d)
for (name, gx, gy, vg, lds), ds in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
    ds.sort()
    print(f"| `{name}` | {gx} x {gy} | {vg} | {lds} | {len(ds)} | {ds[len(ds) // 2] / 1e3:.1f} |")
