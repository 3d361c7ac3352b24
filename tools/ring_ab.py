"""Ring A/B (verdict r4 #4): 8 logical ranks x 256 MiB bf16 in one launch (the bench's
local_ranks section), p50 and fraction of the same process's copy roofline for the exact
(fp32-wire) ring, the element-type-wire ring and the two-shot. Settings come from the
environment (study knobs need MXAR_STUDY=1), so interleave runs with different settings:

    MXAR_STUDY=1 MXAR_RING_U=4 python tools/ring_ab.py --tag u4
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

if not os.environ.get("PYTHONPATH"):  # PYTHONPATH=<tree>: that tree's package (A/B against an older build)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.append(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import akka_allreduce_1_amd  # noqa: E402
from akka_allreduce_1_amd._native import C  # noqa: E402
from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402
from akka_allreduce_1_amd.utils.timing import hbm_bytes, percentile  # noqa: E402
from benchmarks.sections import device_times, rounding_check  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--algos", default="ring,ring_native,twoshot")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    P, S = a.P, a.mib << 20
    n = S // 2
    st = torch.cuda.current_stream(dev).cuda_stream
    x = torch.empty(S, dtype=torch.uint8, device=dev)
    y = torch.empty_like(x)
    for _ in range(3):
        C.hip.copy(x.data_ptr(), y.data_ptr(), S, st)
    cms = percentile(device_times(lambda: C.hip.copy(x.data_ptr(), y.data_ptr(), S, st), a.iters, dev), 50)
    copy_tbps = 2 * S / (cms / 1e3) / 1e12
    del x, y
    cl = LocalCluster(P, slot_bytes=2 * -(-S // P) + (1 << 20), grid=512, timeout_s=10.0)
    xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=500 + k) for k in range(P)]
    ys = [torch.empty_like(t) for t in xs]
    ref = torch.zeros(n, device=dev)
    for t in xs:
        ref += t.float()
    row = {"tag": a.tag, "pkg": os.path.dirname(akka_allreduce_1_amd.__file__), "P": P, "mib": a.mib, "copy_TBps": round(copy_tbps, 3),
           "env": {k: v for k, v in os.environ.items() if k.startswith("MXAR_")}}
    for algo in a.algos.split(","):
        fn = lambda algo=algo: cl.allreduce(xs, ys, algo=algo)  # noqa: E731
        fn()
        cl.check()
        err = max((t.float() - ref).abs().max().item() for t in ys)
        for _ in range(3):
            fn()
        p50 = percentile(device_times(fn, a.iters, dev), 50)
        cl.check()
        tb = hbm_bytes(S, P, algo, 2) / (p50 / 1e3) / 1e12
        row[algo] = [round(p50, 4), round(tb / copy_tbps, 3), round(err, 4)]
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
