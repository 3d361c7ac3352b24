bash tools/gpu.sh tests tests/test_comm_gpu.py tests/test_plane_gpu.py tests/test_threshold_gpu.py && bash tools/gpu.sh bench --steps 20 --warmup 5 --no-dp && \
for cfg in "8 64" "2 64" "8 16" "8 1"; do set -- $cfg; timeout -k 10 120 python tools/phase_profile.py --P $1 --mib $2 --algos twoshot threshold --iters 10 > gpurun_out/phase_P$1_$2.json 2>gpurun_out/phase.err || exit 1; done && \
timeout -k 10 120 python tools/plane_probe.py --P 2 --sizes 1M --rounds 300 --trace gpurun_out/round_trace_1m.json > gpurun_out/probe_1m.jsonl 2> gpurun_out/probe_1m.err
