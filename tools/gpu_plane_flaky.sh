#!/bin/bash
# Is the catch-up test's 30 s lag-gate wait a hardware-queue effect? The plane tests twice
# under the box's GPU_MAX_HW_QUEUES (4) and twice with 8, alternated (no fault involved: a
# stuck gate ends at the kernel's own deadline).
set -o pipefail
mkdir -p gpurun_out/flaky
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/flaky
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_plane_gpu.py -k "catchup or reinit or straggler" > $O/q$q.log 2>&1
  rc=$?; echo "queues=$q rc=$rc $(tail -1 $O/q$q.log)"; grep "error word" $O/q$q.log | head -3
  if [ $rc -gt 1 ]; then exit $rc; fi
done
