#!/usr/bin/env python3
"""A/B of resident protocol rounds (xgmi_plane.cc launch_resident) against one launch per
round (MXAR_PLANE_RESIDENT=0), interleaved on one box: the bench's in-process protocol rounds
(benchmarks.sections.protocol_sizes) and the native deployment's 40 B / 1 MiB rounds
(mxar master + 2 mxar-gpu workers). One JSON line per (mode, rep, section).

    python tools/resident_ab.py --reps 2 > gpurun_out/resident_ab.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--native", type=int, default=1)
    args = ap.parse_args()
    import torch

    from benchmarks.sections import native_deployment, protocol_sizes

    dev = torch.device("cuda", 0)
    for rep in range(args.reps):
        for mode in ("resident", "launched"):
            if mode == "launched":
                os.environ["MXAR_PLANE_RESIDENT"] = "0"
            else:
                os.environ.pop("MXAR_PLANE_RESIDENT", None)
            print(f"[resident_ab] rep {rep} {mode} in-process", file=sys.stderr, flush=True)
            r = protocol_sizes(dev, cases=((40, torch.float32, 2, 2000), (4096, torch.float32, 0, 2000),
                                           (65536, torch.bfloat16, 0, 2000), (1 << 20, torch.bfloat16, 0, 2000)))
            print(json.dumps({"mode": mode, "rep": rep, "section": "inproc", **{
                k: {f: v.get(f) for f in ("us_per_round", "round_interval_p50_us", "validated", "error")}
                for k, v in r.items() if isinstance(v, dict)}}), flush=True)
            if args.native:
                print(f"[resident_ab] rep {rep} {mode} native", file=sys.stderr, flush=True)
                r = native_deployment(cases=((10, 2, 400), (16384, 1024, 400)), budget_s=60.0)
                print(json.dumps({"mode": mode, "rep": rep, "section": "native", **{
                    k: {f: v.get(f) for f in ("us_per_round", "validated", "validated_timed", "error")}
                    for k, v in r.items() if isinstance(v, dict)}}), flush=True)
    os.environ.pop("MXAR_PLANE_RESIDENT", None)


if __name__ == "__main__":
    main()
