#!/usr/bin/env python3
"""Where the DP reducer's exposed time goes at world 1.

At world 1 the allreduce is the identity, so step - compute is pure reducer overhead.
Variants, timed INTERLEAVED (one step of each in turn, `--rounds` times, median per
variant) so that clock / thermal drift over a 30 ms step cancels:

  compute   synthetic backward + SGD update, no hook
  hook0     + a Python no-op hook per parameter (the callback cost itself)
  nolaunch  + the reducer's hook bookkeeping, buckets never handed off (overlap=False)
  events    + per-bucket compute->comm event hand-off, no allreduce call
  full      the reducer as bench.py runs it

    python tools/reducer_overhead.py --model llama3_8b --bucket-mib 1024
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.models.grad_sets import gradient_shapes  # noqa: E402
from akka_allreduce_1_amd.parallel import BucketedGradReducer, XgmiCommunicator  # noqa: E402
from akka_allreduce_1_amd.parallel.comm import init_distributed  # noqa: E402
from benchmarks.bench_dp import SyntheticBackward  # noqa: E402


class _NoComm:
    world = 1

    def allreduce_(self, t, **kw):
        return t


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["resnet50", "llama3_8b"], default="llama3_8b")
    ap.add_argument("--bucket-mib", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--event-scope", type=int, default=1)
    args = ap.parse_args()
    init_distributed("nccl")
    dev = torch.device("cuda", torch.cuda.current_device())
    comm = XgmiCommunicator(device=dev)
    params = [torch.nn.Parameter(torch.zeros(sh, dtype=torch.bfloat16, device=dev))
              for _, sh in gradient_shapes(args.model)]
    full = BucketedGradReducer(params, comm, bucket_bytes=args.bucket_mib << 20, op="avg",
                               event_scope=args.event_scope)
    full.remove_hooks()
    grads = [p.grad for p in params]
    lazy = BucketedGradReducer.__new__(BucketedGradReducer)
    lazy.__dict__.update(full.__dict__)
    lazy.overlap = False
    ev = BucketedGradReducer.__new__(BucketedGradReducer)
    ev.__dict__.update(full.__dict__)
    ev.comm = _NoComm()
    ev._raw_ok = False
    bwd = SyntheticBackward(params, 1024, torch.bfloat16, dev)

    def upd():
        torch._foreach_add_(params, grads, alpha=-1e-3)

    def v_compute():
        bwd.run(None)
        upd()

    def v_hook0():
        bwd.run(None, hook=lambda p: None)
        upd()

    def v_nolaunch():
        bwd.run(lazy)
        for b in lazy.buckets:
            b.pending = len(b.params)
            b.ready = False
        upd()

    def v_events():
        bwd.run(ev)
        ev.wait()
        upd()

    def v_full():
        bwd.run(full)
        full.wait()
        upd()

    variants = {"compute": v_compute, "hook0": v_hook0, "nolaunch": v_nolaunch, "events": v_events, "full": v_full}
    times: dict[str, list[float]] = {k: [] for k in variants}
    with torch.no_grad():
        for fn in variants.values():
            fn()
        torch.cuda.synchronize(dev)
        for _ in range(args.rounds):
            for k, fn in variants.items():
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize(dev)
                times[k].append((time.perf_counter() - t0) * 1e3)
    med = {k: statistics.median(v) for k, v in times.items()}
    row = {"model": args.model, "bucket_mib": args.bucket_mib, "buckets": len(full.buckets),
           "params": len(params), "rounds": args.rounds, "event_scope": args.event_scope,
           "median_ms": {k: round(v, 3) for k, v in med.items()},
           "over_compute_ms": {k: round(v - med["compute"], 3) for k, v in med.items() if k != "compute"}}
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
