#!/bin/bash
# Round-output release on the default stream (default) vs behind an event at the next launch
# (MXAR_PLANE_RELEASE=event): plane tests, then 2 plane workers x 1 / 64 MiB, 300 rounds, x3.
set -o pipefail
mkdir -p gpurun_out/rel
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/rel
rm -f $O/*.jsonl
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_plane_gpu.py > $O/t.log 2>&1
rc=$?; echo "plane tests rc=$rc $(tail -1 $O/t.log)"; if [ $rc -ne 0 ]; then tail -30 $O/t.log; exit $rc; fi
for rep in 1 2 3; do
  MXAR_PLANE_RELEASE=event timeout -k 10 200 python -u tools/plane_probe.py --P 2 --sizes 1M 64M --rounds 300 --timeout 10 >> $O/event.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 200 python -u tools/plane_probe.py --P 2 --sizes 1M 64M --rounds 300 --timeout 10 >> $O/null.jsonl 2>> $O/err.log || exit 1
done
python - <<'PY'
import json, collections, glob, os
for f in sorted(glob.glob("gpurun_out/rel/*.jsonl")):
    d = collections.defaultdict(list)
    for l in open(f):
        x = json.loads(l); d[x["bytes"] >> 20].append((x.get("ms_per_round"), x.get("lat_p50_ms", [None])[0]))
    print(os.path.basename(f)[:-6], dict(d))
PY
