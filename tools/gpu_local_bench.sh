#!/bin/bash
# GPU tests + single-GPU multi-rank kernel bench with both fence modes (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -m5 "Failed:\|Error" gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 400 python tools/bench_local.py --ranks 2 8 --sizes 64K 1M 16M 256M --algos twoshot oneshot --fence 3 2 --out gpurun_out/local_bench_fine.json > gpurun_out/local_bench_fine.log 2>&1; rc=$?
grep -v Warn gpurun_out/local_bench_fine.log | tail -30; exit $rc
