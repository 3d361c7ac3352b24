#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_comm_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_comm.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_comm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_local.py --ranks 2 4 8 --sizes 64K 1M 16M 64M 256M --fence 3 0 --out gpurun_out/local_bench.json > gpurun_out/local_bench.log 2>&1; rc=$?
cat gpurun_out/local_bench.log | tail -60; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o local8 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_local.py --ranks 8 --sizes 256M --algos twoshot --iters 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_local.log 2>&1; rc=$?
tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_local.log
exit $rc
