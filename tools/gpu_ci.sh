#!/bin/bash
# GPU CI: the MI355X test suite, smoke() and the 1-GPU bench (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A25 "Error\|error" gpurun_out/pytest_gpu.log | head -60; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { echo "bench failed"; tail -20 gpurun_out/bench_n1.err; exit 1; }
cat gpurun_out/bench_n1.json
