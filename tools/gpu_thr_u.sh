#!/bin/bash
# Threshold-kernel reduce loads, same-box A/B in ONE launch (LocalCluster: no launch skew):
# U = 0 (one source at a time), 2 and 4 (sources in groups of 4), two-shot alongside as the
# reference; 2 / 8 logical ranks x 64 / 256 MiB bf16, alternated 0/2/4 twice.
set -o pipefail
mkdir -p gpurun_out/thru
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/thru
rm -f $O/l*.jsonl
for rep in 1 2; do
  for u in 0 2 4; do
    MXAR_THRESHOLD_U=$u timeout -k 10 200 python -u tools/bench_local.py --ranks 2 8 --sizes 64M 256M --algos twoshot threshold --iters 20 > $O/tmp.txt 2>&1 || { tail $O/tmp.txt; exit 1; }
    grep '^{"P"' $O/tmp.txt | sed "s/^/{\"U\": $u, \"rep\": $rep, \"r\": /; s/$/}/" >> $O/l.jsonl
  done
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/thru/l.jsonl"):
    x = json.loads(l); r = x["r"]
    d[(r["P"], r["bytes"] >> 20, r["algo"], x["U"])].append(r["p50_us"])
for k in sorted(d): print(k, d[k])
PY
