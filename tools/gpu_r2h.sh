#!/bin/bash
# Split-slice counter relaxed: plane + threshold GPU tests, then the prev/head rate A/B with
# few chunks per block (--units 64: split slices in play).
set -o pipefail
mkdir -p gpurun_out/r2h
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_plane_gpu.py tests/test_threshold_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2h/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r2h/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ticket_ab.sh
