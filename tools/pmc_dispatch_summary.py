"""Per-dispatch summary of a rocprofv3 `--pmc` counter_collection.csv (tools/gpu.sh pmc).

Groups the dispatches of kernels whose name contains `--kernel` into runs (a run ends at any
other kernel), and prints one JSON line per run: median duration, effective core clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH DVFS note), and the median of every
other counter. EA request counters are turned into derived columns where both halves are
present:
  * *_LEVEL / * = mean requests in flight per cycle / requests -> mean cycles a fabric
    request is outstanding (Little's law), the memory-side latency each request saw;
  * *_DRAM / * = the share of L2-to-fabric requests that went to DRAM (not the Infinity Cache);
  * *_CREDIT_STALL / duration cycles = the share of cycles the L2 waited for DRAM credits.

    python tools/pmc_dispatch_summary.py <counter_collection.csv> --kernel twoshot
"""
import argparse
import collections
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", default="twoshot")
    ap.add_argument("--skip", type=int, default=0, help="dispatches to drop at the start of each run (warm-up)")
    a = ap.parse_args()
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(a.csv)):
        d = rows.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"]})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    runs, cur = [], []
    for i in sorted(rows):
        if a.kernel in rows[i]["name"]:
            cur.append(rows[i])
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)
    for k, run in enumerate(runs):
        run = run[a.skip:] or run
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


if __name__ == "__main__":
    main()
