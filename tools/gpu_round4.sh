#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for mem in uncached fine coarse; do
  MXAR_SLAB_MEM=$mem timeout -k 10 300 python -m pytest tests/test_comm_gpu.py -q -p no:cacheprovider -k "local_cluster" > gpurun_out/pytest_comm_$mem.log 2>&1; rc=$?
  echo "== $mem rc=$rc"; grep -E "passed|failed|AssertionError: \(" gpurun_out/pytest_comm_$mem.log | head -8
  [ $rc -le 1 ] || exit $rc
done
