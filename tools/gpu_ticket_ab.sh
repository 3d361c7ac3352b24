#!/bin/bash
# Same-box A/B of the threshold kernel's round-end ticket: abtest/prev (acq_rel ticket, the
# commit before; built in-tree, not committed) vs HEAD (relaxed ticket, sc1 counts), alternated.
set -o pipefail
mkdir -p gpurun_out/ticket
O=gpurun_out/ticket
rm -f $O/ab.jsonl
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  for b in prev head; do
    s=tools/plane_probe.py; [ $b = prev ] && s=abtest/prev/tools/plane_probe.py
    timeout -k 10 200 python -u $s --P 2 --sizes 1M 64M 256M --rounds 300 --units 64 2>> $O/ab.err | sed "s/^{/{\"build\": \"$b\", /" >> $O/ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ticket/ab.jsonl"):
    r = json.loads(l); d[(r["bytes"], r["build"])].append((r["ms_per_round"], r["validated"]))
for k, v in sorted(d.items()): print(k, v)
PY
