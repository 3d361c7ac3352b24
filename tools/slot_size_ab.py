#!/usr/bin/env python3
"""Two-shot at 8 logical ranks x 256 MiB bf16 with slots of one block vs two blocks per source
(the bench's local_ranks section used two, for the fp32-wire ring): p50 us, interleaved.

    python tools/slot_size_ab.py > gpurun_out/slot_size_ab.jsonl
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    P, S = 8, 256 << 20
    n = S // 2
    xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=k) for k in range(P)]
    ys = [torch.empty_like(t) for t in xs]
    for rep in range(2):
        for blocks in (1, 2):
            cl = LocalCluster(P, slot_bytes=blocks * -(-S // P) + (1 << 20), grid=512, timeout_s=10.0)
            for algo in ("twoshot", "ring_native"):
                for _ in range(3):
                    cl.allreduce(xs, ys, algo=algo)
                ts = []
                for _ in range(20):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    cl.allreduce(xs, ys, algo=algo)
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                cl.check()
                print(json.dumps({"rep": rep, "slot_blocks": blocks, "algo": algo, "p50_us": round(statistics.median(ts), 1)}),
                      flush=True)
            del cl
            torch.cuda.synchronize()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
