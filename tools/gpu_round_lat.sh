#!/bin/bash
# Plane + threshold GPU tests, then the protocol round-time A/B (round outputs released behind
# the default stream at the next launch, or directly); P = 2, 1 MiB / 64 MiB, alternated.
set -o pipefail
mkdir -p gpurun_out/lat
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/lat
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_plane_gpu.py tests/test_threshold_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for v in on off on off; do
  f=""; [ $v = off ] && f="--no-order-release"
  timeout -k 10 120 python -u tools/plane_probe.py --P 2 --sizes 1M 64M --rounds 400 --timeout 10 $f >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
cut -c1-230 $O/ab.jsonl
