#!/bin/bash
# GPU tests of the examples (reference demo on the round engine, 1-GPU DP training).
set -o pipefail
mkdir -p gpurun_out/ex
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_examples.py > gpurun_out/ex/t.log 2>&1
rc=$?; tail -5 gpurun_out/ex/t.log; exit $rc
