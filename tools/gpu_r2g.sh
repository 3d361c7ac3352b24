#!/bin/bash
# Threshold kernel without the lag-gate acquire: its GPU tests, then phase stamps and round
# rates of the protocol probe (compare profiles/round2 stamps: gate_p50 3.7 us at 1 MiB).
set -o pipefail
mkdir -p gpurun_out/r2g; rm -f gpurun_out/r2g/*.jsonl
O=gpurun_out/r2g
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_plane_gpu.py tests/test_threshold_gpu.py tests/test_ddp_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/plane_probe.py --P 2 --sizes 1M 64K --rounds 200 --stamps > $O/stamps.jsonl 2> $O/stamps.err || exit $?
for i in 1 2; do
  timeout -k 10 200 python -u tools/plane_probe.py --P 2 --sizes 1M 64M 256M --rounds 300 >> $O/rates.jsonl 2>> $O/rates.err || exit $?
done
cat $O/stamps.jsonl $O/rates.jsonl
