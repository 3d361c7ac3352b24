#!/bin/bash
# The whole plane GPU test file three times in a row (box default hardware queues): does the
# catch-up test's lag-gate wait come back? A stuck gate ends at the kernel's own deadline.
set -o pipefail
mkdir -p gpurun_out/flaky
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/flaky
for i in 1 2 3; do
  timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_plane_gpu.py > $O/full$i.log 2>&1
  rc=$?; echo "run $i rc=$rc $(tail -1 $O/full$i.log)"; grep -h "error word\|PASSED\|FAILED" $O/full$i.log | cut -c1-120
  if [ $rc -gt 1 ]; then exit $rc; fi
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
