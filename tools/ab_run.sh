# ad-hoc GPU A/B driver (this round's threshold / protocol-round work); see tools/thr_ab.py, tools/proto_ab.py
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for rep in 1 2; do
  PYTHONPATH=abtree/old timeout -k 10 200 python tools/proto_ab.py --tag old >> gpurun_out/proto_ab.jsonl || exit 1
  timeout -k 10 200 python tools/proto_ab.py --tag new >> gpurun_out/proto_ab.jsonl || exit 1
done
echo ab done
