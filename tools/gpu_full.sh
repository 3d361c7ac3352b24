#!/bin/bash
# Full GPU regression: every gpu-marked test, then the plane probe and the N=1 bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/full_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 gpurun_out/full_gpu.log; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/plane_probe.py --P 2 --sizes 1M 64M 256M --rounds 40 --timeout 8 > gpurun_out/probe3.jsonl 2> gpurun_out/probe3.err || exit $?
cat gpurun_out/probe3.jsonl
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit $?
echo bench ok
