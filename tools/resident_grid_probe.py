#!/usr/bin/env python3
"""Protocol rounds (benchmarks.sections.protocol_sizes: 2 plane workers on one GPU, th 1, bench
geometry) at the sizes given; run once per configuration of MXAR_PLANE_RESIDENT /
MXAR_PLANE_RESIDENT_GRID (read when a plane is built). One JSON line per run.

    MXAR_PLANE_RESIDENT=8388608 MXAR_PLANE_RESIDENT_GRID=64 \
        python tools/resident_grid_probe.py R64 --sizes 256K 1M 4M >> gpurun_out/resident_grid_ab.jsonl
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from benchmarks.sections import protocol_sizes  # noqa: E402


def parse_size(s: str) -> int:
    m = {"K": 1 << 10, "M": 1 << 20}
    return int(float(s[:-1]) * m[s[-1]]) if s[-1] in m else int(s)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg")
    ap.add_argument("--sizes", nargs="+", default=["256K", "1M", "4M"])
    args = ap.parse_args()
    cases = tuple((parse_size(s), torch.bfloat16, 0, 3000 if parse_size(s) <= 4 << 20 else 400) for s in args.sizes)
    r = protocol_sizes(torch.device("cuda", 0), cases=cases)
    print(json.dumps({"cfg": args.cfg, **{k: {f: v.get(f) for f in ("us_per_round", "round_interval_p50_us", "validated",
                                                                       "error")}
                                          for k, v in r.items() if isinstance(v, dict)}}), flush=True)


if __name__ == "__main__":
    main()
