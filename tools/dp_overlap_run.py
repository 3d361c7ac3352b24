"""The bench's dp.overlap_rehearsal section alone (benchmarks/sections.py dp_overlap): BASELINE
config 5 (and 4) on one GPU with real 2-rank comm kernels beside the GEMMs, every schedule
variant (CU grids, serial, CU-sliced streams, SDMA). One JSON line.

    python tools/dp_overlap_run.py [--models llama3_8b]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from benchmarks.sections import dp_overlap  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="+", default=["resnet50", "llama3_8b"])
    a = ap.parse_args()
    print(json.dumps(dp_overlap(torch.device("cuda", 0), models=tuple(a.models))), flush=True)
