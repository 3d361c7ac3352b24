"""Threshold-round latency A/B (verdict r4 #2): p50 device time per call of the threshold
kernel next to the two-shot and the low-latency one-shot, P logical ranks in one launch on one
GPU, host ahead of the GPU (benchmarks/sections.py device_times), every cell validated first.
Run it once per build / setting and interleave the runs (boxes drift):

    MXAR_STUDY=1 MXAR_GATE_SHORTCUT=0 python tools/thr_ab.py --tag noshortcut
    PYTHONPATH=abtree/old python tools/thr_ab.py --tag old
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

if not os.environ.get("PYTHONPATH"):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import akka_allreduce_1_amd  # noqa: E402
from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402
from akka_allreduce_1_amd.utils.timing import percentile  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.sections import device_times, rounding_check  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--ranks", default="8,2")
    ap.add_argument("--kib", default="4,64,1024")
    ap.add_argument("--algos", default="ll,twoshot,threshold")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16
    for P in [int(x) for x in a.ranks.split(",")]:
        sizes = [int(x) << 10 for x in a.kib.split(",")]
        cl = LocalCluster(P, slot_bytes=-(-max(sizes) // P) + (1 << 20), grid=512, timeout_s=10.0, max_lag=1)
        for size in sizes:
            n = size // 2
            xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=900 + k) for k in range(P)]
            ys = [torch.empty_like(t) for t in xs]
            ref = torch.zeros(n, device=dev)
            for t in xs:
                ref += t.float()
            row = {"tag": a.tag, "P": P, "bytes": size, "pkg": os.path.dirname(akka_allreduce_1_amd.__file__)}
            for algo in a.algos.split(","):
                if algo == "threshold":
                    fn = lambda: cl.allreduce_threshold(xs, ys, counts=False)  # noqa: E731
                else:
                    fn = lambda algo=algo: cl.allreduce(xs, ys, algo=algo)  # noqa: E731
                fn()
                cl.check()
                ok, err, _ = rounding_check(ys, ref, dtype, P)
                for _ in range(5):
                    fn()
                t = device_times(fn, a.iters, dev)
                cl.check()
                row[algo] = round(percentile(t, 50) * 1e3, 2) if ok else f"INVALID {err}"
            print(json.dumps(row), flush=True)
        del cl
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
