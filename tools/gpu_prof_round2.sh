#!/bin/bash
# Round-2 profiles: (1) kernel trace + stats of the N=1 bench (all sections but dp), (2) PMC
# HBM bytes of the protocol round kernel (threshold_kernel) at 2 workers x 256 MiB bf16.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/prof2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_conformance.py tests/test_device_actors_gpu.py > $O/conf.log 2>&1
rc=$?; echo "device-plane tests rc=$rc $(tail -1 $O/conf.log)"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bench -o bench -- python3 bench.py --steps 20 --warmup 5 --no-dp \
  > $O/bench.json 2> $O/bench.err || { echo "bench trace failed"; tail -5 $O/bench.err; exit 1; }
echo "bench trace ok"
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d $O/$pmc -o run -- \
    python3 tools/plane_probe.py --P 2 --sizes 256M --rounds 8 --timeout 10 > $O/$pmc.log 2>&1 || { echo "pmc $pmc failed"; tail -5 $O/$pmc.log; exit 1; }
  echo "pass $pmc ok"
done
