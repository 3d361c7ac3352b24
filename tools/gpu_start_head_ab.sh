#!/bin/bash
# Same-box A/B of the round engine over this session: commit 7f8489d (abtest/start, the
# state at the start of round-2 work on the engine) vs HEAD, P = 2 plane workers,
# 1 / 64 / 256 MiB, 300 rounds, alternated x3, GPU_MAX_HW_QUEUES=8 for both.
set -o pipefail
mkdir -p gpurun_out/ab2
export HSA_ENABLE_IPC_MODE_LEGACY=0 GPU_MAX_HW_QUEUES=8
O=gpurun_out/ab2
rm -f $O/*.jsonl
for rep in 1 2 3; do
  timeout -k 10 200 python -u abtest/start/tools/plane_probe.py --P 2 --sizes 1M 64M 256M --rounds 300 --timeout 10 >> $O/start.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 200 python -u tools/plane_probe.py --P 2 --sizes 1M 64M 256M --rounds 300 --timeout 10 >> $O/head.jsonl 2>> $O/err.log || exit 1
done
python - <<'PY'
import json, collections, glob, os
for f in sorted(glob.glob("gpurun_out/ab2/*.jsonl")):
    d = collections.defaultdict(list)
    for l in open(f):
        x = json.loads(l); d[x["bytes"] >> 20].append((x.get("ms_per_round"), x.get("lat_p50_ms", [None])[0]))
    print(os.path.basename(f)[:-6], dict(d))
PY
