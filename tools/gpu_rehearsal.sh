#!/bin/bash
# Multi-process rehearsal of the whole N>1 bench path on ONE GPU (--share-device: gloo for the
# CPU group, IPC-mapped slabs and plane arenas, split workgroup budget): N = 4 with the DP
# section, N = 8 with the DP section under a 60 s watchdog (8 ranks' comm kernels and GEMMs
# on one GPU are an artefact of sharing; the watchdog must still produce the result line).
set -o pipefail
mkdir -p gpurun_out/rehearsal
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/rehearsal
for n in 4 8; do
  extra="--dp-rehearsal"; [ $n = 8 ] && extra="--dp-rehearsal --dp-timeout 60"
  timeout -k 10 420 python -u -m torch.distributed.run --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29540 + n)) \
      bench.py --gpus $n --share-device --steps 10 --warmup 3 $extra > $O/bench_share_n$n.json 2> $O/bench_share_n$n.err
  rc=$?; echo "n=$n rc=$rc"; python -c "import json;d=json.load(open('$O/bench_share_n$n.json'));print(d['value'], d['status'], json.dumps(d.get('protocol',{}))[:300], json.dumps(d.get('dp'))[:300])" || true
  if [ $rc -ne 0 ]; then tail -20 $O/bench_share_n$n.err; exit $rc; fi
done
echo done
