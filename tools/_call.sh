# same-box A/B: abtest/prev = sc1 / plain loads (round-2 kernels), in-tree = nt loads + grouped threshold scatter
bash tools/gpu.sh tests tests/test_comm_gpu.py tests/test_threshold_gpu.py tests/test_coll_gpu.py tests/test_adamw_gpu.py tests/test_plane_gpu.py && \
for rep in 1 2; do for v in prev head; do
  B=. ; [ $v = prev ] && B=abtest/prev
  timeout -k 10 200 python $B/tools/bench_local.py --ranks 8 2 --sizes 1M 16M 64M 256M --algos twoshot ring oneshot --fence 3 --iters 15 > gpurun_out/ab_local_${v}_$rep.jsonl 2>>gpurun_out/ab.err || exit 1
  echo "$v $rep ok"
done; done && \
timeout -k 10 120 tools/api_cost_probe > gpurun_out/api_cost.json 2>&1 && \
timeout -k 10 120 python tools/plane_probe.py --P 2 --sizes 1M --rounds 300 --trace gpurun_out/round_trace_1m.json > gpurun_out/probe_1m.jsonl 2> gpurun_out/probe_1m.err && \
for cfg in "8 64" "2 64" "8 16"; do set -- $cfg; timeout -k 10 120 python tools/phase_profile.py --P $1 --mib $2 --algos twoshot threshold --iters 10 > gpurun_out/phase_P$1_$2.json 2>gpurun_out/phase.err || exit 1; done && \
bash tools/gpu.sh bench --steps 20 --warmup 5 --no-dp
