#!/usr/bin/env python3
"""rocprofv3 summaries for profiles/ (one tool, three inputs):

    python tools/prof.py csv <prefix> [title]        --kernel-trace/--stats CSV run -> markdown
    python tools/prof.py db <results.db> [title]     rocpd database (ROCm 7.2 default) -> markdown
    python tools/prof.py pmc <counter_collection.csv> [--kernel twoshot] [--skip N]
                                                     --pmc run -> one JSON line per run of dispatches

csv / db: per kernel calls, mean / min / max us and share of GPU time, then the mxar kernels by
launch shape (grid, VGPRs, LDS, scratch). pmc: dispatches of kernels whose name contains
--kernel grouped into runs (a run ends at any other kernel); per run the median duration, the
effective core clock (GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH DVFS note) and the
median of every other counter, with EA request counters turned into derived columns:
  * *_LEVEL / * = mean cycles a fabric request is outstanding (Little's law);
  * *_DRAM / * = the share of L2-to-fabric requests that went to DRAM (not the Infinity Cache);
  * *_CREDIT_STALL / duration cycles = the share of cycles the L2 waited for DRAM credits.
(Replaces prof_summary.py, prof_db_summary.py and pmc_dispatch_summary.py - git history.)
"""
import argparse
import collections
import csv
import json
import sqlite3
import statistics
import sys
from collections import defaultdict


def _name(s: str) -> str:
    s = s.replace("|", "/")
    return s[:87] + "..." if len(s) > 90 else s


def summarise_csv(prefix: str, title: str) -> None:
    stats = list(csv.DictReader(open(prefix + "_kernel_stats.csv")))
    print(f"# rocprofv3 kernel summary: {title}\n")
    print("| kernel | calls | mean us | min us | max us | % time |\n|---|---:|---:|---:|---:|---:|")
    for r in stats:
        print(f"| `{_name(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {float(r['MinNs'])/1e3:.1f} | "
              f"{float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
    groups, meta = defaultdict(list), {}
    try:
        trace = list(csv.DictReader(open(prefix + "_kernel_trace.csv")))
    except OSError:  # tools/gpu.sh prof keeps only the stats (the trace runs to hundreds of MiB)
        return
    for r in trace:
        if "mxar" not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].split("(")[0], r["Grid_Size_X"], r["Grid_Size_Y"])
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        meta[key] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
    print("\n## mxar dispatches by grid (threads)\n")
    print("| kernel | grid x | grid y | n | median us | VGPR | SGPR | LDS | scratch |\n"
          "|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, v in sorted(groups.items()):
        m = meta[k]
        print(f"| `{k[0]}` | {k[1]} | {k[2]} | {len(v)} | {statistics.median(v):.1f} | {m[0]} | {m[1]} | {m[2]} | {m[3]} |")


def summarise_db(db: str, title: str) -> None:
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(duration), min(duration), max(duration), sum(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[5] for r in rows) or 1
    print(f"# rocprofv3 kernel summary: {title}\n")
    print("| kernel | calls | mean us | min us | max us | % time |\n|---|---:|---:|---:|---:|---:|")
    for name, n, avg, mn, mx, tot in rows:
        print(f"| `{_name(name)}` | {n} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | {100 * tot / total:.1f} |")
    print("\nmxar kernels by launch shape (grid x / y, VGPRs, LDS bytes):\n")
    print("| kernel | grid | VGPR | LDS | calls | median us |\n|---|---|---:|---:|---:|---:|")
    groups: dict = {}
    for name, gx, gy, wx, vg, lds, d in c.execute("select name, grid_x, grid_y, workgroup_x, vgpr_count, lds_size, "
                                                  "duration from kernels where name like '%mxar%'").fetchall():
        groups.setdefault((name.split("(")[0], gx // max(wx, 1), gy, vg, lds), []).append(d)
    for (name, gx, gy, vg, lds), ds in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        ds.sort()
        print(f"| `{name}` | {gx} x {gy} | {vg} | {lds} | {len(ds)} | {ds[len(ds) // 2] / 1e3:.1f} |")


def summarise_pmc(path: str, kernel: str, skip: int) -> None:
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        d = rows.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"]})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    runs, cur = [], []
    for i in sorted(rows):
        if kernel in rows[i]["name"]:
            cur.append(rows[i])
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)
    for k, run in enumerate(runs):
        run = run[skip:] or run
        med = {c: statistics.median(d[c] for d in run) for c in run[0] if c != "name"}
        out = {"run": k, "dispatches": len(run), "us": round(med["us"], 1)}
        if "GRBM_GUI_ACTIVE" in med:
            out["core_MHz"] = round(med["GRBM_GUI_ACTIVE"] / 8 / med["us"])
        cyc = med.get("GRBM_GUI_ACTIVE", 0) / 8
        for c, v in med.items():
            if c in ("us", "GRBM_GUI_ACTIVE"):
                continue
            out[c] = v
            base = c.replace("_LEVEL", "").replace("_DRAM_CREDIT_STALL", "").replace("_CREDIT_STALL", "")
            if c.endswith("_LEVEL_sum") and base in med and med[base]:
                # LEVEL accumulates in-flight requests per cycle summed over the 16 channels x 8 XCDs
                out[c.replace("_LEVEL_sum", "_cycles_in_flight")] = round(v / med[base], 1)
            if c.endswith("_DRAM_sum") and c.replace("_DRAM", "") in med and med[c.replace("_DRAM", "")]:
                out[c.replace("_sum", "_share")] = round(v / med[c.replace("_DRAM", "")], 3)
            if "CREDIT_STALL" in c and cyc:
                out[c.replace("_sum", "_per_cycle")] = round(v / cyc, 3)
        print(json.dumps(out))


def main() -> None:
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("csv")
    a.add_argument("prefix")
    a.add_argument("title", nargs="?")
    b = sub.add_parser("db")
    b.add_argument("db")
    b.add_argument("title", nargs="?")
    c = sub.add_parser("pmc")
    c.add_argument("csv")
    c.add_argument("--kernel", default="twoshot")
    c.add_argument("--skip", type=int, default=0, help="dispatches to drop at the start of each run (warm-up)")
    x = ap.parse_args()
    if x.cmd == "csv":
        summarise_csv(x.prefix, x.title or x.prefix)
    elif x.cmd == "db":
        summarise_db(x.db, x.title or x.db)
    else:
        summarise_pmc(x.csv, x.kernel, x.skip)


if __name__ == "__main__":
    sys.exit(main())
