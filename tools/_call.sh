# two-shot geometry A/B on one box: coarse / fine / flat (+ the threshold kernel for reference)
bash tools/gpu.sh tests tests/test_comm_gpu.py tests/test_adamw_gpu.py tests/test_ddp_gpu.py && \
for rep in 1 2; do for g in coarse fine flat; do
  MXAR_TWOSHOT_GEOM=$g timeout -k 10 200 python tools/bench_local.py --ranks 8 4 2 --sizes 1M 4M 16M 64M 256M --algos twoshot --fence 3 --iters 15 > gpurun_out/geom_${g}_$rep.jsonl 2>>gpurun_out/ab.err || exit 1
  echo "$g $rep ok"
done; done && \
MXAR_TWOSHOT_GEOM=flat timeout -k 10 120 python tools/phase_profile.py --P 8 --mib 256 --algos twoshot threshold --iters 10 > gpurun_out/phase_flat_P8_256.json 2>gpurun_out/phase.err && \
for rep in 1 2; do for v in 1 0; do
  MXAR_ADAM_STREAM=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-dp --no-local --no-protocol --no-sizes > gpurun_out/adam_stream${v}_$rep.json 2>>gpurun_out/adam.err || exit 1
  echo "adam stream=$v rep $rep ok"
done; done
