#!/bin/bash
# rocprofv3 PMC passes over bench.py's fused AdamW section (1 rank, 134 M params:
# twoshot_adamw_kernel = grad reduce + AdamW on the fp32 master + bf16 param write in one
# launch): HBM bytes fetched / written per dispatch vs the 28 B/param minimum.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_adamw
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d gpurun_out/pmc_adamw/$pmc -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-tune --no-rccl --no-threshold --no-collectives --no-dp \
    > gpurun_out/pmc_adamw/$pmc.log 2>&1 || { echo "pmc $pmc failed"; tail -5 gpurun_out/pmc_adamw/$pmc.log; exit 1; }
  echo "pass $pmc ok"
done
