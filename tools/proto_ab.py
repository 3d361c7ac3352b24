"""Protocol-round latency (verdict r4 #2): the reference's default job (10 floats, maxChunkSize
2, th = 1, maxLag 1) on the GPU round engine, in-process (2 PlaneWorkerActors) and as the
native deployment (mxar master + 2 mxar-gpu processes), us per round. One JSON line per run.

    python tools/proto_ab.py --tag new [--reps 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

if not os.environ.get("PYTHONPATH"):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.append(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.sections import native_deployment, protocol_sizes  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for rep in range(a.reps):
        p = protocol_sizes(dev, cases=((40, torch.float32, 2, 2000), (1 << 20, torch.bfloat16, 0, 2000)))
        nat = native_deployment(cases=((10, 2, 400),), budget_s=60.0)
        row = {"tag": a.tag, "rep": rep,
               "inproc_us": {k: v.get("us_per_round") for k, v in p.items() if isinstance(v, dict) and "us_per_round" in v},
               "inproc_ok": all(v.get("validated") for v in p.values() if isinstance(v, dict) and "validated" in v),
               "native_us": {k: v.get("us_per_round") for k, v in nat.items() if isinstance(v, dict) and "us_per_round" in v},
               "native_ok": all(v.get("validated") for v in nat.values() if isinstance(v, dict) and "validated" in v)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
