#!/bin/bash
# two-shot chunk granularity study: MXAR_TWOSHOT_UNITS = scatter units per workgroup
export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
for u in 1 2 4 8; do
  MXAR_TWOSHOT_UNITS=$u timeout -k 10 120 python tools/bench_local.py --ranks 8 --sizes 16M 256M --algos twoshot --fence 3 > gpurun_out/units_local_$u.log 2>&1 || exit 1
  echo "local u=$u: $(grep '"P"' gpurun_out/units_local_$u.log | python3 -c 'import sys,json; print([ (json.loads(l)["bytes"]>>20, json.loads(l)["p50_us"]) for l in sys.stdin])')"
done
for u in 1 4; do
  MXAR_TWOSHOT_UNITS=$u timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29650 + u)) bench.py --gpus 8 --steps 10 --warmup 3 --share-device --no-tune --no-threshold --algo twoshot > gpurun_out/units_reh_$u.json 2> gpurun_out/units_reh_$u.err || { tail -5 gpurun_out/units_reh_$u.err; exit 1; }
  echo "rehearsal8 u=$u: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/units_reh_$u.json | head -1)"
done
