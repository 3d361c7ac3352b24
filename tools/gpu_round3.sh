#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_local.py --ranks 2 8 --sizes 64K 1M 16M 256M --algos twoshot oneshot --fence 3 1 2 0 --out gpurun_out/local_bench2.json > gpurun_out/local_bench2.log 2>&1; rc=$?
grep -v Warn gpurun_out/local_bench2.log | tail -60; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { echo "bench failed"; tail -20 gpurun_out/bench_n1.err; exit 1; }
cat gpurun_out/bench_n1.json
