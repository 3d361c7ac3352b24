#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace/--stats CSV run into a small markdown table
(per kernel: calls, mean/min/max us, share) plus per-dispatch groups of the comm kernels
by grid shape. usage: python tools/prof_summary.py gpurun_out/prof/local8 > profiles/x.md"""
import csv
import statistics
import sys
from collections import defaultdict

prefix = sys.argv[1]
title = sys.argv[2] if len(sys.argv) > 2 else prefix
stats = list(csv.DictReader(open(prefix + "_kernel_stats.csv")))
print(f"# rocprofv3 kernel summary: {title}\n")
print("| kernel | calls | mean us | min us | max us | % time |\n|---|---:|---:|---:|---:|---:|")
for r in stats:
    name = r["Name"].replace("|", "/")
    if len(name) > 90:
        name = name[:87] + "..."
    print(f"| `{name}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {float(r['MinNs'])/1e3:.1f} | "
          f"{float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
tr = list(csv.DictReader(open(prefix + "_kernel_trace.csv")))
groups = defaultdict(list)
meta = {}
for r in tr:
    if "mxar" not in r["Kernel_Name"]:
        continue
    key = (r["Kernel_Name"].split("(")[0], r["Grid_Size_X"], r["Grid_Size_Y"])
    groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    meta[key] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
print("\n## mxar dispatches by grid (threads)\n")
print("| kernel | grid x | grid y | n | median us | VGPR | SGPR | LDS | scratch |\n|---|---:|---:|---:|---:|---:|---:|---:|---:|")
for k, v in sorted(groups.items()):
    m = meta[k]
    print(f"| `{k[0]}` | {k[1]} | {k[2]} | {len(v)} | {statistics.median(v):.1f} | {m[0]} | {m[1]} | {m[2]} | {m[3]} |")
