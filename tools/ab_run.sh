# ad-hoc GPU A/B driver (ring partial layout, protocol rounds); see tools/ring_ab.py, tools/proto_ab.py
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for rep in 1 2; do
  PYTHONPATH=abtree/old timeout -k 10 120 python tools/ring_ab.py --tag old >> gpurun_out/ring_ab4.jsonl || exit 1
  timeout -k 10 120 python tools/ring_ab.py --tag planar >> gpurun_out/ring_ab4.jsonl || exit 1
  PYTHONPATH=abtree/old timeout -k 10 200 python tools/proto_ab.py --tag old >> gpurun_out/proto_ab2.jsonl || exit 1
  timeout -k 10 200 python tools/proto_ab.py --tag new >> gpurun_out/proto_ab2.jsonl || exit 1
done
echo ab done
