#!/bin/bash
# Plane GPU tests (raised hardware queues) + actor-runtime rates (BASELINE config 1) on the
# box's CPUs, alternating the pre-MPSC build (abtest/old, not committed) with HEAD.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_plane_gpu.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/plane_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/plane_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for b in old new; do
    if [ $b = old ]; then s=abtest/old/benchmarks/bench_actors.py; else s=benchmarks/bench_actors.py; fi
    [ -f $s ] || continue
    timeout -k 10 120 python $s --rounds 4000 --transport all 2>> gpurun_out/actors.err | sed "s/^{/{\"build\": \"$b\", /" >> gpurun_out/actors_mpsc_ab.jsonl || exit $?
  done
done
cat gpurun_out/actors_mpsc_ab.jsonl
