"""Co-located plane workers on the group kernel (csrc/hip/xgmi_plane.cc PlaneGroup): run one
PlaneJob shape and, if it stalls, print every plane's door / group / control words
(XgmiRoundPlane.debug_state) - the diagnosis of a stuck slice.

    python tools/group_probe.py --P 3 --n 600001 --chunk 100000 --rounds 8
    python tools/group_probe.py --shapes 2:1048583:524297,3:600001:100000 --repeat 10
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.engine import PlaneJob  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=3)
    ap.add_argument("--n", type=int, default=600001)
    ap.add_argument("--chunk", type=int, default=100000)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--timeout-s", type=float, default=4.0)
    ap.add_argument("--wait", type=float, default=20.0)
    ap.add_argument("--shapes", default="", help="P:n:chunk,... run in turn (default: --P/--n/--chunk)")
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args()
    shapes = [tuple(int(v) for v in s.split(":")) for s in a.shapes.split(",")] if a.shapes else [(a.P, a.n, a.chunk)]
    for i in range(a.repeat):
        for P, n, chunk in shapes:
            if not run(a, P, n, chunk, i):
                return


def run(a, P, n, chunk, i) -> bool:
    dtype = getattr(torch, a.dtype)
    job = PlaneJob(P, n, max_chunk_size=chunk, max_lag=1, max_round=a.rounds - 1, dtype=dtype,
                   timeout_s=a.timeout_s)
    t0 = time.perf_counter()
    ok = True
    try:
        job.run(timeout=a.wait)
    except TimeoutError:
        ok = False
    out = {"ok": ok, "iter": i, "P": P, "n": n, "chunk": chunk, "s": round(time.perf_counter() - t0, 3),
           "rounds": job.rounds["n"],
           "planes": [json.loads(p.debug_state()) for p in job.planes],
           "stats": [{"group_rounds": p.stats.group_rounds, "group_launches": p.stats.group_launches,
                      "group_size": p.stats.group_size, "chunk": p.chunk_elems} for p in job.planes]}
    if not ok or i == a.repeat - 1:
        print(json.dumps(out), flush=True)
    else:
        print(json.dumps({k: out[k] for k in ("ok", "iter", "P", "s", "rounds")}), flush=True)
    job.shutdown()
    return ok


if __name__ == "__main__":
    main()
