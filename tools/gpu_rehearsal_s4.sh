#!/bin/bash
# N > 1 bench path as 2 / 4 / 8 processes on ONE GPU (--share-device --no-dp): every algorithm
# and the protocol section (master on rank 0, plane descriptors in the TCP join) validated.
set -o pipefail
O=gpurun_out/rehearsal_s4
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 4 8; do
  timeout -k 10 400 python -u -m torch.distributed.run --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29640 + n)) \
      bench.py --gpus $n --share-device --no-dp --steps 10 --warmup 3 > $O/bench_share_n$n.json 2> $O/bench_share_n$n.err
  rc=$?; echo "n=$n rc=$rc"
  python -c "import json;d=json.loads(open('$O/bench_share_n$n.json').read().strip().splitlines()[-1]);p=d.get('protocol',{});print(d['value'], d['config']['algo'], all(v.get('validated') for v in d.get('validation',{}).values()), p.get('validated'), p.get('ms_per_round'), p.get('bridge'), p.get('error'))" || true
  [ $rc -eq 0 ] || { tail -20 $O/bench_share_n$n.err; exit $rc; }
done
echo done
