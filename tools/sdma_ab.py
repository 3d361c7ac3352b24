"""SDMA allreduce A/B (verdict r4 #5): p50 of the copy-engine allreduce for P logical ranks on
one GPU at several reduce / gather grids, validated against fp32 first, plus the engines'
own copy time for the same bytes (what the engine schedule alone costs).

usage: python tools/sdma_ab.py [--mib 256] [--ranks 2] [--grids 32,128,256,512] [--reps 2]
prints one JSON line per (rep, grid) to stdout
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalSdmaCluster  # noqa: E402
from akka_allreduce_1_amd.utils.timing import percentile  # noqa: E402
from benchmarks.sections import device_times, rounding_check  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--grids", default="32,128,256,512")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16
    P, nbytes = a.ranks, a.mib << 20
    n = nbytes // 2
    xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=900 + k) for k in range(P)]
    ys = [torch.empty_like(x) for x in xs]
    ref = torch.zeros(n, device=dev)
    for x in xs:
        ref += x.float()
    for rep in range(a.reps):
        for g in [int(x) for x in a.grids.split(",")]:
            cl = LocalSdmaCluster(P, slot_bytes=-(-nbytes // P) + (1 << 20), grid=g, timeout_s=20.0)
            cl.allreduce(xs, ys)
            torch.cuda.synchronize(dev)
            cl.check()
            ok, err, _ = rounding_check(ys, ref, dtype, P)
            ts = device_times(lambda: cl.allreduce(xs, ys), a.iters, dev)
            cl.check()
            p50 = percentile(ts, 50)
            print(json.dumps({"rep": rep, "P": P, "mib": a.mib, "grid": g, "validated": ok, "max_abs_err": err,
                              "p50_ms": round(p50, 4), "algbw_GBps": round(nbytes / (p50 / 1e3) / 1e9, 1),
                              "engines_per_peer": cl.comms[0].engines_per_peer}), flush=True)
            del cl
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
