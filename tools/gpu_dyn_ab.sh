#!/bin/bash
# Two-shot static vs dynamic unit assignment (MXAR_TWOSHOT_DYNAMIC): correctness (comm GPU
# tests with the knob on), then 8 / 2 logical ranks x 64 / 256 MiB bf16 alternated 0/1/0/1.
set -o pipefail
mkdir -p gpurun_out/dyn
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/dyn
MXAR_TWOSHOT_DYNAMIC=1 timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_comm_gpu.py > $O/tests.log 2>&1
rc=$?; echo "comm tests (dynamic) rc=$rc $(tail -1 $O/tests.log)"; if [ $rc -ne 0 ]; then tail -30 $O/tests.log; exit $rc; fi
for d in 0 1 0 1; do
  MXAR_TWOSHOT_DYNAMIC=$d timeout -k 10 180 python -u tools/bench_local.py --ranks 8 2 --sizes 64M 256M --algos twoshot --iters 30 > $O/d$d.txt 2>&1 || { echo "bench rc=$?"; tail $O/d$d.txt; exit 1; }
  echo "dynamic=$d"; grep '^{' $O/d$d.txt | cut -c1-160
done
MXAR_TWOSHOT_DYNAMIC=1 timeout -k 10 180 python -u tools/phase_profile.py --P 8 --mib 256 --algos twoshot --iters 10 --json $O/phases_dyn.json > $O/ph.log 2>&1 || exit 1
python -c "import json;d=json.load(open('$O/phases_dyn.json'));print(json.dumps(d['algos']['twoshot'])[:600])"
