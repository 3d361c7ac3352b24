#!/usr/bin/env python3
"""Where a protocol round's time goes: P plane workers on one GPU run R
rounds of one size with the native tracer on; every round is cut into the hops of the
reference's round loop (AllreduceMaster.scala:58-67,91-97 -> AllreduceWorker.scala:84-104 ->
:180-192,253-268) from the trace's host timestamps:

    master start r  -> worker fetch r         master -> worker mailbox hop
    fetch r         -> launch r returned      source + plane launch (host)
    launch returned -> done r observed        GPU queue + kernel + completion detection
    done r          -> sink r begins          completion thread -> worker mailbox hop
    sink r                                     the dataSink
    sink r ends     -> master has complete r  worker -> master mailbox hop
    last complete   -> master start r + 1     the barrier's own work

plus the kernel's own duration from its phase stamps (GPU clock), so "GPU queue + detection"
is the launch-to-done interval minus the kernel. Medians over the timed rounds, per worker.

    python tools/round_breakdown.py --P 2 --size 40 --dtype f32 --chunk 2 --rounds 300
"""
from __future__ import annotations

import argparse
import json
import os
import re
import statistics
import sys


import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.engine import PlaneJob  # noqa: E402
from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402

_R = re.compile(r"^(start|complete|fetch|launch|done|sink) r(\d+)$")


def breakdown(events: list[dict], P: int, skip: int) -> dict:
    """Per-round hop intervals (us) from the tracer's events."""
    ms: dict[int, float] = {}
    per: dict[tuple[str, int, int], tuple[float, float]] = {}  # (kind, worker, round) -> (ts, end)
    for e in events:
        m = _R.match(e.get("name", ""))
        if not m:
            continue
        kind, r = m.group(1), int(m.group(2))
        ts = float(e["ts"])
        end = ts + float(e.get("dur", 0.0))
        if kind == "start":
            ms[r] = ts
            continue
        w = int((e.get("args") or {}).get("worker", -1))
        per[(kind, w, r)] = (ts, end)
    rounds = sorted(r for r in ms if r >= skip and r + 1 in ms)
    hops = {k: [] for k in ("master_to_fetch", "fetch_launch_host", "launch_to_done", "done_to_sink", "sink",
                            "sink_to_master", "barrier_to_next_start", "round_period")}
    per_worker = {w: {k: [] for k in ("master_to_fetch", "launch_to_done", "done_to_sink", "sink_to_master")}
                  for w in range(P)}
    for r in rounds:
        try:
            last_c = max(per[("complete", w, r)][0] for w in range(P))
            for w in range(P):
                f, l, d, s, c = (per[(k, w, r)] for k in ("fetch", "launch", "done", "sink", "complete"))
                vals = {"master_to_fetch": f[0] - ms[r], "fetch_launch_host": l[1] - f[0],
                        "launch_to_done": d[0] - l[1], "done_to_sink": s[0] - d[0], "sink": s[1] - s[0],
                        "sink_to_master": c[0] - s[1]}
                for k, v in vals.items():
                    hops[k].append(v)
                    if k in per_worker[w]:
                        per_worker[w][k].append(v)
        except KeyError:
            continue
        hops["barrier_to_next_start"].append(ms[r + 1] - last_c)
        hops["round_period"].append(ms[r + 1] - ms[r])
    med = lambda v: round(statistics.median(v), 2) if v else None  # noqa: E731
    # host spans nested in the launch path: source call, plane launch, the plane's round
    # setup + kernel launch, the kernel launch alone
    spans: dict[str, list[float]] = {}
    for e in events:
        if e.get("ph") != "X":
            continue
        name = e.get("name", "")
        key = re.sub(r" ?r?\d+B?$", "", name)
        spans.setdefault(key, []).append(float(e.get("dur", 0.0)))
    return {"rounds": len(hops["round_period"]), "median_us": {k: med(v) for k, v in hops.items()},
            "span_median_us": {k: med(v) for k, v in spans.items()},
            "p90_us": {k: round(sorted(v)[int(0.9 * (len(v) - 1))], 2) if v else None for k, v in hops.items()},
            "per_worker_median_us": {w: {k: med(v) for k, v in d.items()} for w, d in per_worker.items()}}


def parse_size(s: str) -> int:
    m = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(float(s[:-1]) * m[s[-1].upper()]) if s[-1].upper() in m else int(s)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=2)
    ap.add_argument("--size", default="1M")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--chunk", type=int, default=0, help="maxChunkSize (0: 1024 elements)")
    ap.add_argument("--rounds", type=int, default=300)
    ap.add_argument("--skip", type=int, default=20, help="warm-up rounds left out")
    ap.add_argument("--spin-us", type=int, default=1000)
    ap.add_argument("--trace-out", default=None, help="also write the Chrome trace here")
    ap.add_argument("--no-trace", action="store_true", help="round time only, without the tracer's own cost")
    ap.add_argument("--grid", type=int, default=0, help="workgroups per worker (0: PlaneJob's default)")
    ap.add_argument("--no-split", action="store_true", help="PlaneJob(split=False): one workgroup per chunk")
    ap.add_argument("--stamps-out", default=None, help="also write the last round's raw per-workgroup stamps here")
    a = ap.parse_args()
    from akka_allreduce_1_amd._native import C
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from plane_probe import phase_summary

    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    es = 2 if dtype == torch.bfloat16 else 4
    S = parse_size(a.size)
    n = max(1, S // es)
    xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=k) for k in range(a.P)]
    ref = sum(x.float() for x in xs).to(dtype)
    job = PlaneJob(a.P, n, max_chunk_size=a.chunk or 1024, dtype=dtype, max_round=a.rounds - 1, timeout_s=10.0,
                   spin_us=a.spin_us, sources=xs, keep_outputs=False, keep_last=True, split=not a.no_split,
                   grid=a.grid)
    bufs = [torch.zeros(job.grid * 8, dtype=torch.int64, device=dev) for _ in job.planes]
    for p, b in zip(job.planes, bufs):
        p.set_phase_stamps(b.data_ptr(), job.grid)
    C.trace.clear()
    C.trace.enable(not a.no_trace)
    row = {"P": a.P, "bytes": S, "dtype": a.dtype, "max_chunk_size": a.chunk or 1024, "rounds": a.rounds,
           "spin_us": a.spin_us, "split": not a.no_split, "grid": job.grid, "dispatch_spin_us": os.environ.get("MXAR_DISPATCH_SPIN_US", "default")}
    try:
        job.run(timeout=120.0)
        C.trace.enable(False)
        s = job.stamps
        if len(s) > a.skip + 2:
            row["ms_per_round"] = round((s[-1] - s[a.skip]) / (len(s) - 1 - a.skip) * 1e3, 4)
        ok = True
        for k in range(a.P):
            o = job.last_output(k)
            ok = ok and o is not None and torch.equal(o.data, ref)
        row["validated"] = ok
        try:
            ph = phase_summary([b.view(-1, 8).cpu() for b in bufs])
            row["kernel_last_round_us"] = {f"w{p['worker']}": round(p["end_max"] - p["start_first"], 1) for p in ph
                                           if "end_max" in p}
            row["kernel_phases"] = ph
            if a.stamps_out:
                with open(a.stamps_out, "w") as f:
                    json.dump([b.view(-1, 8).cpu().tolist() for b in bufs], f)
        except ValueError:  # no stamps written (e.g. a plane without a stamp buffer)
            row["kernel_last_round_us"] = None
        row["resident_rounds"] = [p.stats.resident_rounds for p in job.planes]
        tr = json.loads(C.trace.dump_json())
        row["traced"] = not a.no_trace
        if not a.no_trace:
            row["dropped_events"] = tr.get("otherData", {}).get("dropped")
            row.update(breakdown(tr["traceEvents"], a.P, a.skip))
        if a.trace_out:
            with open(a.trace_out, "w") as f:
                json.dump(tr, f)
    except Exception as e:  # noqa: BLE001
        row["error"] = repr(e)[:400]
    finally:
        C.trace.enable(False)
        job.shutdown()
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
