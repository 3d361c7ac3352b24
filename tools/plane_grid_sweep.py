#!/usr/bin/env python3
"""Protocol rounds (PlaneJob, 2 workers sharing the GPU, thresholds 1) at several per-worker
workgroup budgets and round sizes: us per round from the master's barrier stamps. One JSON
line per (grid, size).

    python tools/plane_grid_sweep.py > gpurun_out/plane_grid_sweep.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_1_amd.engine import PlaneJob  # noqa: E402
from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    P = 2
    for nbytes, rounds in ((1 << 20, 1000), (16 << 20, 400), (64 << 20, 200), (256 << 20, 100)):
        n = nbytes // 2
        xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=k) for k in range(P)]
        for grid in (64, 128, 256):
            block = -(-n // P)
            chunk = max(1024, -(-block // 256))
            job = PlaneJob(P, n, max_chunk_size=chunk, dtype=torch.bfloat16, max_round=rounds - 1, sources=xs,
                           keep_outputs=False, keep_last=True, timeout_s=20.0, grid=grid)
            try:
                job.run(timeout=120)
                st = job.stamps
                warm = 10
                per = (st[-1] - st[warm - 1]) / (len(st) - warm)
                print(json.dumps({"bytes": nbytes, "grid_per_worker": grid, "us_per_round": round(per * 1e6, 1)}),
                      flush=True)
            finally:
                job.shutdown()


if __name__ == "__main__":
    main()
