#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B2 -A8 "Error" gpurun_out/pytest_gpu.log | head -40; exit $rc; }
timeout -k 10 400 python tools/bench_local.py --ranks 2 8 --sizes 64K 1M 16M 256M --algos twoshot oneshot --fence 2 3 --out gpurun_out/local_bench3.json > gpurun_out/local_bench3.log 2>&1; rc=$?
grep -v Warn gpurun_out/local_bench3.log | tail -40; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o local8 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_local.py --ranks 8 --sizes 16M 256M --algos twoshot --iters 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_local.log 2>&1; rc=$?
tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof_local.log
exit $rc
