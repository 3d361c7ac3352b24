#!/bin/bash
# Full GPU test suite, then mxar-bench sweeps of every fused algorithm with P logical ranks
# on one MI355X (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A25 "Error\|error" gpurun_out/pytest_gpu.log | head -60; exit $rc; }
for P in 2 4 8; do
  timeout -k 10 300 python -m akka_allreduce_1_amd bench --local $P --algos oneshot twoshot ring threshold --sizes 4K..256M --iters 10 --json gpurun_out/sweep_local_p$P.jsonl 2> gpurun_out/sweep_local_p$P.txt || { tail gpurun_out/sweep_local_p$P.txt; exit 1; }
done
cat gpurun_out/sweep_local_p8.txt
