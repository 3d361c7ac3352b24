#!/bin/bash
# A/B of the idle-dispatcher spin (MXAR_DISPATCH_SPIN_US 0 / 50, alternated) on BASELINE config
# 1 in-process and on the GPU round engine (2 plane workers, 1 MiB / 64 MiB, 400 rounds).
set -o pipefail
mkdir -p gpurun_out/rates
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/rates
for s in 0 50 0 50; do
  MXAR_DISPATCH_SPIN_US=$s timeout -k 10 120 python -u benchmarks/bench_actors.py --rounds 3000 --transport inproc > $O/a$s.jsonl 2>> $O/actors.err || exit 1
  echo "spin=$s $(cut -c1-200 $O/a$s.jsonl)"
  MXAR_DISPATCH_SPIN_US=$s timeout -k 10 120 python -u tools/plane_probe.py --P 2 --sizes 1M 64M --rounds 400 --timeout 10 > $O/p$s.jsonl 2>> $O/plane.err || exit 1
  echo "spin=$s"; cut -c1-40,150-260 $O/p$s.jsonl
done
