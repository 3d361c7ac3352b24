#!/usr/bin/env python3
"""A/B of the device copy kernel variants (1-rank allreduce path) vs torch copy_, interleaved
rounds in one process (cdna_hip_programming.md §5.4 rule 24)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from akka_allreduce_1_amd._native import C  # noqa: E402
from akka_allreduce_1_amd.utils.timing import percentile  # noqa: E402

dev = torch.device("cuda", 0)
res = {}
for mib in (16, 64, 256, 1024):
    n = mib << 20
    x = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
    y = torch.empty_like(x)
    variants = {"torch": lambda: y.copy_(x)}
    for v in range(8):
        def f(v=v):
            C.hip.set_copy_variant(v)
            C.hip.copy(x.data_ptr(), y.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
        variants[f"v{v}"] = f
    times = {k: [] for k in variants}
    for _ in range(3):
        for f in variants.values():
            f()
    for rnd in range(15):
        for k, f in variants.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            torch.cuda.synchronize()
            times[k].append(a.elapsed_time(b))
    C.hip.set_copy_variant(-1)
    C.hip.copy(x.data_ptr(), y.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    res[mib] = {k: {"p50_us": round(percentile(v, 50) * 1e3, 1), "TBps": round(2 * n / (percentile(v, 50) / 1e3) / 1e12, 2)}
                for k, v in times.items()}
    print(mib, json.dumps(res[mib]), flush=True)
    del x, y
