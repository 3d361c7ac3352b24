#!/usr/bin/env python3
"""Per-phase timing of the fused two-shot and ring kernels (verdict r1: where do the 8-rank
two-shot's microseconds go?). Every workgroup records s_memrealtime stamps (100 MHz) into a
debug buffer (xgmi_device.h PhaseStamps): start, end of the scatter (RS hops for the ring),
time spent waiting inside the reduce phase, end of the reduce phase, time spent waiting in
the gather (AG) phase, end. P logical ranks in ONE launch on one GPU (LocalCluster).

    python tools/phase_profile.py --P 8 --mib 256 --algos twoshot ring --iters 10 --json out.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402
from akka_allreduce_1_amd.utils.timing import hbm_bytes, percentile  # noqa: E402

SLOTS = 8


def stats(xs):
    xs = sorted(xs)
    return {"mean": round(sum(xs) / len(xs), 2), "p50": round(percentile(xs, 50), 2), "max": round(xs[-1], 2)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--algos", nargs="+", default=["twoshot", "ring"])
    ap.add_argument("--kib", type=int, default=0, help="bytes per rank in KiB (overrides --mib)")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--grid", type=int, default=512)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16
    S = (a.kib << 10) if a.kib else (a.mib << 20)
    n = S // 2
    # a lag ring for the threshold kernel (its stamps: [1] lag gate done, [3] reduce done,
    # [6] scatter done - see xgmi_threshold.hip)
    cl = LocalCluster(a.P, slot_bytes=-(-S // a.P) + (1 << 20), grid=a.grid, timeout_s=10.0,
                      max_lag=1 if "threshold" in a.algos else None)
    xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=k) for k in range(a.P)]
    ys = [torch.empty_like(t) for t in xs]
    buf = torch.zeros(a.grid * a.P * SLOTS, dtype=torch.int64, device=dev)
    out = {"P": a.P, "bytes_per_rank": S, "grid": a.grid, "algos": {}}
    for algo in a.algos:
        def run(algo=algo):
            if algo == "threshold":
                cl.allreduce_threshold(xs, ys, counts=False)
            else:
                cl.allreduce(xs, ys, algo=algo)

        for _ in range(3):
            run()
        rows = []
        for _ in range(a.iters):
            buf.zero_()
            cl.comms[0].set_phase_stamps(buf.data_ptr(), a.grid * a.P)
            run()
            torch.cuda.synchronize()
            cl.comms[0].set_phase_stamps(0, 0)
            st = buf.view(-1, SLOTS).cpu()
            used = st[st[:, 0] > 0]
            t0 = int(used[:, 0].min())
            # slot = blockIdx.y * gridDim.x + blockIdx.x = the linear workgroup id, which the
            # dispatcher deals round-robin over the 8 XCDs: XCD = slot % 8
            idx = torch.nonzero(st[:, 0] > 0).flatten()
            by_xcd = {}
            for x in range(8):
                sel = used[(idx % 8) == x]
                if len(sel):
                    by_xcd[x] = round(float((sel[:, 5] - sel[:, 0]).double().median()) / 100.0, 1)
            us = lambda v: float(v) / 100.0  # noqa: E731 - 100 MHz ticks -> us
            rows.append({
                "span_us": us(int(used[:, 5].max()) - t0),
                "start_skew_us": us(int(used[:, 0].max()) - t0),
                "scatter_end_us": [us(int(x) - t0) for x in used[:, 1]],
                "reduce_wait_us": [us(x) for x in used[:, 2]],
                "reduce_end_us": [us(int(x) - t0) for x in used[:, 3]],
                "gather_wait_us": [us(x) for x in used[:, 4]],
                "stamp6": [us(int(x) - t0) if algo == "threshold" else float(x) for x in used[:, 6]],
                "end_us": [us(int(x) - t0) for x in used[:, 5]],
                "workgroups": int(used.shape[0]),
                "span_by_xcd_us": by_xcd,
            })
        cl.check()
        span = [r["span_us"] for r in rows]
        best = rows[span.index(sorted(span)[len(span) // 2])]  # the median launch
        summ = {"span_us": stats(span), "start_skew_us": best["start_skew_us"], "workgroups": best["workgroups"],
                "span_by_xcd_us": best["span_by_xcd_us"]}
        for k in ("scatter_end_us", "reduce_wait_us", "reduce_end_us", "gather_wait_us", "end_us", "stamp6"):
            summ[k] = stats(best[k])
        summ["hbm_TBps_at_span_p50"] = round(hbm_bytes(S, a.P, "twoshot" if algo == "threshold" else algo, 2) / (summ["span_us"]["p50"] * 1e-6) / 1e12, 3)
        out["algos"][algo] = summ
        print(json.dumps({algo: summ}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
