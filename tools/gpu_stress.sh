#!/bin/bash
# Memory-ordering study: the churn stress test under each fence / slab-memory setting.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in "3 uncached" "2 uncached" "3 fine" "2 fine"; do
  set -- $cfg
  for rep in 1 2; do
    MXAR_FENCE=$1 MXAR_SLAB_MEM=$2 timeout -k 10 300 python -m pytest tests/test_comm_gpu.py -q -p no:cacheprovider \
      -k "stress or local_cluster_allreduce" > gpurun_out/stress_$1_$2_$rep.log 2>&1; rc=$?
    echo "fence=$1 mem=$2 rep=$rep rc=$rc: $(tail -1 gpurun_out/stress_$1_$2_$rep.log)"
    grep -m2 "Failed:" gpurun_out/stress_$1_$2_$rep.log
    [ $rc -le 1 ] || exit $rc
  done
done
