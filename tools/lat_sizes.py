#!/usr/bin/env python3
"""The bench's latency_vs_size section alone (benchmarks/sections.py): per logical-rank count
and size, every kernel's p50 and which one `auto` picks. One JSON line.

    python tools/lat_sizes.py > gpurun_out/lat_sizes.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from benchmarks.sections import latency_vs_size  # noqa: E402

if __name__ == "__main__":
    r = latency_vs_size(torch.device("cuda", 0), torch.bfloat16, max_bytes=256 << 20)
    print(json.dumps(r), flush=True)
