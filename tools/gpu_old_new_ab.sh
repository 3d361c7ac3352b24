#!/bin/bash
# Same-box A/B of the round engine: commit 5eb21cf (abtest/old) vs HEAD, P = 2 plane workers,
# 1 / 64 / 256 MiB, 300 rounds, alternated x3, plus the plane GPU tests on HEAD.
set -o pipefail
mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab
rm -f $O/*.jsonl
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_plane_gpu.py tests/test_threshold_gpu.py > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/t.log)"; if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2 3; do
  timeout -k 10 200 python -u abtest/old/tools/plane_probe.py --P 2 --sizes 1M 64M 256M --rounds 300 --timeout 10 >> $O/old.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 200 python -u tools/plane_probe.py --P 2 --sizes 1M 64M 256M --rounds 300 --timeout 10 >> $O/new.jsonl 2>> $O/err.log || exit 1
done
python - <<'PY'
import json, collections, glob, os
for f in sorted(glob.glob("gpurun_out/ab/*.jsonl")):
    d = collections.defaultdict(list)
    for l in open(f):
        x = json.loads(l); d[x["bytes"] >> 20].append(x.get("ms_per_round"))
    print(os.path.basename(f)[:-6], dict(d))
PY
