#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, kernel trace only) over the P=4 reduce
# kernel and the 8-logical-rank fused two-shot: HBM bytes fetched / written and SQ activity.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R="python3 benchmarks/bench_reduce.py --mib 256 --slots 4 --iters 3"
L="python3 tools/bench_local.py --ranks 8 --sizes 64M --algos twoshot --iters 3"
i=0
for cmd in "$R" "$L"; do
  i=$((i+1))
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"; do
    tag=$(echo $pmc | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d gpurun_out/pmc/c${i}_$tag -o run -- $cmd > gpurun_out/pmc/c${i}_$tag.log 2>&1 || { echo "pmc $i $pmc failed"; tail -5 gpurun_out/pmc/c${i}_$tag.log; exit 1; }
    echo "pass $i $tag ok"
  done
done
