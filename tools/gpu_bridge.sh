#!/bin/bash
# Control bridge on the GPU: the GPU test (bridge client drives the xGMI round engine) and
# the master-driven vs bridge-driven round rate (tools/bridge_rate.py).
set -o pipefail
O=gpurun_out/bridge
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_plane_gpu.py -k "bridge or exact_at_threshold_one" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bridge_rate.py --plane xgmi --rounds 300 --mib 1 64 256 > $O/rate.jsonl 2> $O/rate.err || { echo rate failed; tail -5 $O/rate.err; exit 1; }
cat $O/rate.jsonl
