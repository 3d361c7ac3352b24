#!/bin/bash
# BASELINE configs measurable on one MI355X (run via gpurun):
#   config 2  - in-place reduce kernel, 1 GiB fp32 (+ bf16), with a rocprofv3 kernel summary
#   configs 4/5 at N=1 - DP step (ResNet-50 / Llama-3-8B gradient sets, synthetic backward)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python benchmarks/bench_reduce.py > gpurun_out/reduce_fp32.json 2> gpurun_out/reduce.err || { tail -20 gpurun_out/reduce.err; exit 1; }
cat gpurun_out/reduce_fp32.json
timeout -k 10 300 python benchmarks/bench_reduce.py --dtype bf16 --mib 512 > gpurun_out/reduce_bf16.json 2>> gpurun_out/reduce.err || { tail -20 gpurun_out/reduce.err; exit 1; }
cat gpurun_out/reduce_bf16.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_reduce -o run -- python3 benchmarks/bench_reduce.py --iters 10 > gpurun_out/prof_reduce.log 2>&1 || { tail -20 gpurun_out/prof_reduce.log; exit 1; }
timeout -k 10 300 python benchmarks/bench_dp.py --model resnet50 > gpurun_out/dp_resnet50_n1.json 2> gpurun_out/dp_resnet50.err || { tail -20 gpurun_out/dp_resnet50.err; exit 1; }
tail -1 gpurun_out/dp_resnet50_n1.json
timeout -k 10 600 python benchmarks/bench_dp.py --model llama3_8b --steps 3 --warmup 1 > gpurun_out/dp_llama_n1.json 2> gpurun_out/dp_llama.err || { tail -20 gpurun_out/dp_llama.err; exit 1; }
tail -1 gpurun_out/dp_llama_n1.json
