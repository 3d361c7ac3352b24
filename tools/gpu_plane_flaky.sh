#!/bin/bash
# Plane GPU tests (incl. worker loss / re-init) twice, threshold tests once, then smoke().
set -o pipefail
mkdir -p gpurun_out/flaky
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/flaky
for i in 1 2; do
  timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_plane_gpu.py > $O/full$i.log 2>&1
  rc=$?; echo "run $i rc=$rc $(tail -1 $O/full$i.log)"; grep -h "error word\|FAILED\|Error" $O/full$i.log | cut -c1-160 | head -8
  if [ $rc -gt 1 ]; then exit $rc; fi
done
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_threshold_gpu.py > $O/thr.log 2>&1
rc=$?; echo "threshold rc=$rc $(tail -1 $O/thr.log)"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
