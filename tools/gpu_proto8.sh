#!/bin/bash
# The protocol engine at P = 8 in one process (plane_probe, both stream priorities, hardware
# queues raised to 20), then the full N = 1 bench with its hardware-queue setting.
set -o pipefail
mkdir -p gpurun_out/proto8
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/proto8
for pr in normal high; do
  timeout -k 10 120 python -u tools/plane_probe.py --P 8 --sizes 16M 256M --rounds 13 --timeout 10 --priority $pr >> $O/probe8.jsonl 2>> $O/probe8.err || { echo "probe rc=$?"; tail -5 $O/probe8.err; exit 1; }
done
cut -c1-400 $O/probe8.jsonl
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || { echo "bench rc=$?"; tail -20 $O/bench_n1.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_n1.json'));print(d['value'], json.dumps(d.get('protocol')), json.dumps(d.get('local_ranks')), json.dumps(d.get('dp')))"
