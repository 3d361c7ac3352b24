#!/usr/bin/env python3
"""Does the allocation's placement set the 8 x 256 MiB two-shot's speed? Several LocalCluster
instances are created one after another (all kept alive), each timed on the SAME inputs; one
JSON line per instance with its p50 and the slabs' addresses (low bits in MiB / GiB). A
second pass times fresh input / output buffers on the first instance.

    python tools/placement_probe.py > gpurun_out/placement_probe.jsonl
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

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
    dev = torch.device("cuda", 0)
    P, S = 8, 256 << 20
    n = S // 2
    xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=k) for k in range(P)]
    ys = [torch.empty_like(t) for t in xs]
    keep = []
    for i in range(6):
        cl = LocalCluster(P, slot_bytes=-(-S // P) + (1 << 20), grid=512, timeout_s=10.0)
        keep.append(cl)
        addrs = [c.slab_address for c in cl.comms]
        print(json.dumps({"instance": i, "p50_us": p50(cl, xs, ys),
                          "slab_MiB_mod_1GiB": [(a >> 20) & 1023 for a in addrs],
                          "slab_GiB": [a >> 30 for a in addrs]}), flush=True)
    for j in range(4):
        xs2 = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=k) for k in range(P)]
        ys2 = [torch.empty_like(t) for t in xs2]
        print(json.dumps({"instance": 0, "fresh_buffers": j, "p50_us": p50(keep[0], xs2, ys2),
                          "in_MiB_mod_1GiB": [(t.data_ptr() >> 20) & 1023 for t in xs2]}), flush=True)
        del xs2, ys2


if __name__ == "__main__":
    main()
