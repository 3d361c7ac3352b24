#!/usr/bin/env python3
"""Which allocations land a LocalCluster's slabs in the slow mode (placement_probe.py)? One
fresh process per mode; the 8 x 256 MiB two-shot p50 of three clusters created in order.
  inputs_first  torch inputs / outputs (4 GiB) allocated before the clusters (the bench's order)
  slabs_first   the clusters before the torch buffers
  ballast       a 2 GiB fine-grained ballast allocated (and kept) before anything else

    for m in inputs_first slabs_first ballast; do python tools/placement_probe2.py $m; done
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_1_amd._native import C  # noqa: E402
from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402


def p50(cl, xs, ys) -> float:
    for _ in range(3):
        cl.allreduce(xs, ys, algo="twoshot")
    ts = []
    for _ in range(15):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        cl.allreduce(xs, ys, algo="twoshot")
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    cl.check()
    return round(statistics.median(ts), 1)


def main() -> None:
    mode = sys.argv[1]
    dev = torch.device("cuda", 0)
    P, S = 8, 256 << 20
    n = S // 2
    keep = []
    if mode == "ballast":
        keep.append(C.hip.XgmiComm(0, 1, 0, 2 << 30, 512, 10.0, 0))  # a 2 GiB fine-grained slab
    xs = ys = None
    if mode != "slabs_first":
        xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=k) for k in range(P)]
        ys = [torch.empty_like(t) for t in xs]
    cls = [LocalCluster(P, slot_bytes=-(-S // P) + (1 << 20), grid=512, timeout_s=10.0) for _ in range(3)]
    if xs is None:
        xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=k) for k in range(P)]
        ys = [torch.empty_like(t) for t in xs]
    first = [p50(cl, xs, ys) for cl in cls]
    again = [p50(cl, xs, ys) for cl in cls]  # the same clusters once more: warm-up or placement?
    print(json.dumps({"mode": mode, "p50_us": first, "p50_us_again": again}), flush=True)


if __name__ == "__main__":
    main()
