#!/bin/bash
# One-GPU rehearsal of the N>1 bench path at 2 and 8 processes (no dp sections).
set -o pipefail
mkdir -p gpurun_out/r2e
O=gpurun_out/r2e
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in ${NS:-2 8}; do
  timeout -k 10 500 python -u -m torch.distributed.run --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29550 + n)) \
      bench.py --gpus $n --share-device --steps 10 --warmup 3 --no-dp > $O/bench_share_n$n.json 2> $O/bench_share_n$n.err
  rc=$?; echo "n=$n rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_share_n$n.err; exit $rc; }
  python -c "import json;d=json.loads(open('$O/bench_share_n$n.json').read().strip().splitlines()[-1]);print(d['value'], d['config']['algo'], d.get('status'), d.get('validated'), d.get('protocol',{}).get('validated'), d.get('protocol',{}).get('ms_per_round'))"
done
