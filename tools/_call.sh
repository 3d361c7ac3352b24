for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-dp --no-local --no-protocol --no-sizes > gpurun_out/adam_default_$rep.json 2>>gpurun_out/adam.err || exit 1
  MXAR_ADAM_STREAM=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-dp --no-local --no-protocol --no-sizes > gpurun_out/adam_env0_$rep.json 2>>gpurun_out/adam.err || exit 1
  timeout -k 10 200 python abtest/prev/tools/bench_adamw.py --ranks 1 2 --mib 256 > gpurun_out/adam_prevtool_$rep.jsonl 2>>gpurun_out/adam.err || exit 1
  echo "rep $rep ok"
done && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-local --no-protocol > gpurun_out/bench_dp.json 2> gpurun_out/bench_dp.err && echo dp ok
