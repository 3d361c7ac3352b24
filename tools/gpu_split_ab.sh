#!/bin/bash
# Split chunks on / off (MXAR_PLANE_SPLIT), alternated on one box: the in-process protocol
# probe at the bench geometry (chunk = bytes / 1024) and the native deployment with 8
# chunks per vector (mxar master + 2 mxar-gpu workers).
set -o pipefail
mkdir -p gpurun_out/split
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/split
for sp in 1 0 1 0; do
  MXAR_PLANE_SPLIT=$sp timeout -k 10 150 python -u tools/plane_probe.py --P 2 --sizes 1M 64M 256M --rounds 200 --timeout 10 > $O/probe_$sp.jsonl 2>> $O/probe.err || exit 1
  echo "split=$sp"; cut -c1-60,150-260 $O/probe_$sp.jsonl
  MXAR_PLANE_SPLIT=$sp GRIDS=0 SIZES="16777216 67108864" NO_PROBE=1 bash tools/gpu_native_rate.sh || exit 1
done
