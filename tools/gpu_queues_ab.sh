#!/bin/bash
# Same-box A/B: 8 logical ranks x 256 MiB two-shot / ring under GPU_MAX_HW_QUEUES 4 vs 8.
set -o pipefail
mkdir -p gpurun_out/qab
O=gpurun_out/qab
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python -u tools/bench_local.py --ranks 8 --sizes 256M --algos twoshot ring --iters 30 > $O/q$q.txt 2>&1 || { echo "rc=$?"; tail $O/q$q.txt; exit 1; }
  echo "queues=$q"; grep -v "^\[" $O/q$q.txt | tail -4
done
