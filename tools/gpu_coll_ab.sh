#!/bin/bash
# Same-box A/B of the collectives' finish barrier: abtest/prev (acq_rel ticket) vs HEAD
# (relaxed ticket after a drain), 8 logical ranks on one GPU, alternated; then the tests.
set -o pipefail
mkdir -p gpurun_out/coll
O=gpurun_out/coll
rm -f $O/ab.jsonl
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_coll_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for b in prev head; do
    s=tools/bench_local.py; [ $b = prev ] && s=abtest/prev/tools/bench_local.py
    timeout -k 10 200 python -u $s --ranks 8 --sizes 1M 64M 256M --algos all_gather reduce_scatter all_to_all --iters 20 2>> $O/ab.err | sed "s/^{/{\"build\": \"$b\", /" >> $O/ab.jsonl || exit $?
  done
done
cat $O/ab.jsonl | head -40
