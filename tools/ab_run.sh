# ad-hoc GPU A/B driver (fused AdamW layout + PMC bytes); see tools/bench_adamw.py, tools/adam_stream_probe.hip
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh tests tests/test_adamw_gpu.py tests/test_ddp_gpu.py || exit 1
for rep in 1 2; do
  MXAR_STUDY=1 MXAR_ADAM_STREAM=0 timeout -k 10 120 python tools/bench_adamw.py --ranks 1 8 --mib 256 --grid 256 --fused-only | sed 's/^/{"layout": "lane_pairs", "r": /;s/$/}/' >> gpurun_out/adam_ab.jsonl || exit 1
  timeout -k 10 120 python tools/bench_adamw.py --ranks 1 8 --mib 256 --grid 256 --fused-only | sed 's/^/{"layout": "halves", "r": /;s/$/}/' >> gpurun_out/adam_ab.jsonl || exit 1
done
timeout -k 10 120 ./tools/adam_stream_probe.bin > gpurun_out/adam_probe.jsonl || exit 1
for cnt in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $cnt --output-format csv -d gpurun_out/pmc_adam_$cnt -o run -- python3 tools/bench_adamw.py --ranks 1 --mib 256 --grid 256 --fused-only --iters 5 > gpurun_out/pmc_adam_$cnt.log 2>&1 || exit 1
  MXAR_STUDY=1 MXAR_ADAM_STREAM=0 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $cnt --output-format csv -d gpurun_out/pmc_adam0_$cnt -o run -- python3 tools/bench_adamw.py --ranks 1 --mib 256 --grid 256 --fused-only --iters 5 > gpurun_out/pmc_adam0_$cnt.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $cnt --output-format csv -d gpurun_out/pmc_probe_$cnt -o run -- ./tools/adam_stream_probe.bin > gpurun_out/pmc_probe_$cnt.log 2>&1 || exit 1
done
echo ab done
