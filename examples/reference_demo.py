#!/usr/bin/env python3
"""The reference's demo deployment in one process (README of the reference: one master and
two workers, dataSize 10, maxChunkSize 2), on the native actor runtime.

    python examples/reference_demo.py                 # host memory, the reference's thresholds
    python examples/reference_demo.py --plane gpu     # every round = one threshold-kernel launch on cuda:0

The data source is the reference's demo source: data[i] = i + iteration, worker k adds 1000 k
here so that the sum shows which workers contributed. The sink prints what the reference's
sink logs (AllreduceWorker.scala:285-301): the round, the output and the per-chunk counts.
"""
from __future__ import annotations

import argparse
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd._native import C  # noqa: E402
from akka_allreduce_1_amd.actors import make_master, make_plane_worker, make_worker  # noqa: E402
from akka_allreduce_1_amd.protocol import AllReduceInput, MemberUp  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--data-size", type=int, default=10)
    ap.add_argument("--max-chunk-size", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--th-reduce", type=float, default=0.9)
    ap.add_argument("--th-complete", type=float, default=0.8)
    ap.add_argument("--max-lag", type=int, default=1)
    ap.add_argument("--plane", choices=["host", "loopback", "gpu"], default="host",
                    help="host: the message-level protocol; loopback / gpu: the round engine")
    args = ap.parse_args()
    n, P = args.data_size, args.workers
    system = C.ActorSystem("ClusterSystem")
    done = threading.Event()
    lock = threading.Lock()

    def source(k):
        base = np.arange(n, dtype=np.float32) + np.float32(1000 * k)

        def f(req):
            if args.plane == "gpu":
                import torch

                return torch.from_numpy(base + np.float32(req.iteration)).to("cuda")
            return AllReduceInput(base + np.float32(req.iteration)) if args.plane == "host" else base + np.float32(req.iteration)
        return f

    def sink(k):
        def f(out):
            data = out.data.float().cpu().numpy() if hasattr(out.data, "cpu") else np.asarray(out.data)
            with lock:
                print(f"worker {k} round {out.iteration}: {data.tolist()} counts {list(out.count)}", flush=True)
        return f

    master = make_master(system, P, 1.0, args.th_reduce, args.th_complete, args.max_lag, n, args.rounds - 1,
                         args.max_chunk_size, on_finished=lambda r: done.set())
    planes = []
    for k in range(P):
        if args.plane == "host":
            w = make_worker(system, source(k), sink(k), f"worker{k}")
            master.tell(MemberUp(w, "worker", ""), None)
        else:
            kw = {"device": 0} if args.plane == "gpu" else {"hub": "demo"}
            w, plane = make_plane_worker(system, source(k), sink(k), data_size=n, name=f"worker{k}", **kw)
            planes.append(plane)
            master.tell(MemberUp(w, "worker", "", plane.descriptor), None)
    ok = done.wait(60)
    for p in planes:
        p.drain()
    system.await_idle(5.0)
    system.shutdown()
    print("finished" if ok else "timed out", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
