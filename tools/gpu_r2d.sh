#!/bin/bash
# Multi-process IPC allreduce test (incl. the coarse two-shot labels) + the 4-process one-GPU
# rehearsal of the N>1 bench path (tuner with "~1" geometry candidates, post-tune validation).
set -o pipefail
mkdir -p gpurun_out/r2d
O=gpurun_out/r2d
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_comm_gpu.py -k "multiprocess_ipc" -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/mp.log 2>&1
rc=$?; tail -3 $O/mp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29544 \
    bench.py --gpus 4 --share-device --steps 10 --warmup 3 --no-dp > $O/bench_share_n4.json 2> $O/bench_share_n4.err
rc=$?; echo "rehearsal rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_share_n4.err; exit $rc; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r2d/bench_share_n4.json").read().strip().splitlines()[-1])
print(d["value"], d["config"]["algo"], d.get("status"))
for r in d.get("sweep") or []:
    if r["bytes"] >= 64 << 20:
        print({k: v for k, v in r.items() if "p50" in k or k in ("bytes", "choice")})
PY
