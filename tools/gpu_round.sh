#!/bin/bash
# GPU suite + 1-GPU bench + rocprofv3 kernel summary of the bench (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|error\|FAIL" gpurun_out/pytest_gpu.log | head -80; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { echo "bench failed"; tail -20 gpurun_out/bench_n1.err; exit 1; }
cut -c1-700 gpurun_out/bench_n1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 50 --warmup 5 --no-tune > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
echo prof ok
