#!/bin/bash
# Same-box A/B of the slab-copy unroll (scatter / gather phases): abtest/prev (U = 4) vs HEAD
# (U = 8), 8 logical ranks on one GPU, two-shot / ring / all-gather, alternated 3 times.
set -o pipefail
mkdir -p gpurun_out/copyu
O=gpurun_out/copyu
rm -f $O/ab.jsonl
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  for b in prev head; do
    s=tools/bench_local.py; [ $b = prev ] && s=abtest/prev/tools/bench_local.py
    timeout -k 10 200 python -u $s --ranks 8 2 --sizes 1M 64M 256M --algos twoshot ring all_gather --iters 20 2>> $O/ab.err | sed "s/^{/{\"build\": \"$b\", /" >> $O/ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/copyu/ab.jsonl"):
    r = json.loads(l)
    if "algo" in r: d[(r["algo"], r["P"], r["bytes"], r["build"])].append(r["p50_us"])
for k, v in sorted(d.items()): print(k, v)
PY
