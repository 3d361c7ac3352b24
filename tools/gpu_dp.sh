#!/bin/bash
# GPU tests + data-parallel step benchmark at N=1 (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -m5 "Failed:\|Error" gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python benchmarks/bench_dp.py --model resnet50 > gpurun_out/dp_resnet50_n1.json 2> gpurun_out/dp_resnet50.err || { tail -20 gpurun_out/dp_resnet50.err; exit 1; }
cat gpurun_out/dp_resnet50_n1.json
timeout -k 10 600 python benchmarks/bench_dp.py --model llama3_8b --steps 3 --warmup 1 > gpurun_out/dp_llama_n1.json 2> gpurun_out/dp_llama.err || { tail -20 gpurun_out/dp_llama.err; exit 1; }
cat gpurun_out/dp_llama_n1.json
