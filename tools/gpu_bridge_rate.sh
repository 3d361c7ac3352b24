#!/bin/bash
# master-driven vs bridge lock-step vs bridge pipelined round rate on the xGMI round engine
set -o pipefail
O=gpurun_out/bridge
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u tools/bridge_rate.py --plane xgmi --rounds 300 --mib 1 64 256 > $O/rate2.jsonl 2> $O/rate2.err || { echo rate failed; tail -5 $O/rate2.err; exit 1; }
cat $O/rate2.jsonl
