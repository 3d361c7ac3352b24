#!/bin/bash
# GPU session script (round 2): plane-engine tests, the bench at N=1, a 2-process
# share-device rehearsal of the distributed protocol section, and a kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_plane_gpu.py > gpurun_out/r2_plane.log 2>&1
rc=$?; echo "plane tests rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi  # 1 = failed tests; anything else: stop
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench_n1.json 2> gpurun_out/r2_bench_n1.err || { echo "bench rc=$?"; exit 1; }
timeout -k 10 300 python -u -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --share-device --steps 10 --warmup 3 --no-dp --no-tune --no-fused-step > gpurun_out/r2_rehearsal_n2.json 2> gpurun_out/r2_rehearsal_n2.err || { echo "rehearsal rc=$?"; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2 -o bench -- python3 bench.py --steps 10 --warmup 3 --no-dp --no-tune > gpurun_out/r2_prof_bench.json 2> gpurun_out/r2_prof_bench.err || { echo "prof rc=$?"; exit 1; }
echo done
