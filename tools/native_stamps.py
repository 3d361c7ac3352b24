#!/usr/bin/env python3
"""Phase stamps of the native deployment's last round (mxar-gpu workers run with
MXAR_PLANE_STAMPS=<file>), summarised like tools/plane_probe.py --stamps: per worker, when its
kernel started, passed the lag gate, finished scatter / reduce / gather (us from the first
workgroup start of either worker; s_memrealtime is one clock for every process on the GPU).

    python tools/native_stamps.py gpurun_out/native_stamps.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from plane_probe import phase_summary  # noqa: E402

rows = [json.loads(line) for line in open(sys.argv[1]) if line.strip()]
per = [torch.tensor(r["stamps"], dtype=torch.int64).view(-1, 8) for r in rows]
print(json.dumps({"workers": len(per), "phases_last_round": phase_summary(per)}))
