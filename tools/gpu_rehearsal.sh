#!/bin/bash
# Multi-rank rehearsal of bench.py on ONE GPU: 2 and 4 ranks (torch.distributed.run, gloo,
# every rank on cuda:0, IPC-mapped slabs, split workgroup budget). Same code path as the
# driver's N-GPU run minus xGMI and RCCL. (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for N in ${REHEARSAL_NS:-2 4 8}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29600 + N)) bench.py --gpus $N --steps 10 --warmup 3 --share-device ${BENCH_ARGS:-} \
    > gpurun_out/rehearsal_n$N.json 2> gpurun_out/rehearsal_n$N.err || { echo "rehearsal N=$N failed"; tail -30 gpurun_out/rehearsal_n$N.err; exit 1; }
  cut -c1-600 gpurun_out/rehearsal_n$N.json
done
