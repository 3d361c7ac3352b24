set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAIL" gpurun_out/pytest_gpu.log | head -60; exit $rc; }
timeout -k 10 300 python tools/bench_local.py --ranks 2 8 --sizes 1M 256M --algos twoshot ring oneshot --out gpurun_out/local_guard.json > gpurun_out/local_guard.log 2>&1 || { tail -20 gpurun_out/local_guard.log; exit 1; }
grep -v Warn gpurun_out/local_guard.log | tail -12
REHEARSAL_NS=8 bash tools/gpu_rehearsal.sh
