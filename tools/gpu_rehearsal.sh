#!/bin/bash
# Multi-process rehearsal of the whole N>1 bench path on ONE GPU (--share-device: gloo for the
# CPU group, IPC-mapped slabs and plane arenas, split workgroup budget): N = 4, then N = 8.
set -o pipefail
mkdir -p gpurun_out/rehearsal
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/rehearsal
for n in 4 8; do
  timeout -k 10 420 python -u -m torch.distributed.run --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29540 + n)) \
      bench.py --gpus $n --share-device --steps 10 --warmup 3 --dp-rehearsal > $O/bench_share_n$n.json 2> $O/bench_share_n$n.err
  rc=$?; echo "n=$n rc=$rc"; cat $O/bench_share_n$n.json; if [ $rc -ne 0 ]; then tail -20 $O/bench_share_n$n.err; exit $rc; fi
done
echo done
