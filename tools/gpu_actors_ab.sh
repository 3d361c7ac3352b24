#!/bin/bash
# Actor-runtime rates (BASELINE config 1) on the GPU box's CPUs: the pre-MPSC build
# (abtest/old, built in-tree from an older commit, not committed) alternated with HEAD.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/${1:-actors_ab}.jsonl
for i in 1 2 3 4 5; do
  for b in old new; do
    if [ $b = old ]; then s=abtest/old/benchmarks/bench_actors.py; else s=benchmarks/bench_actors.py; fi
    [ -f $s ] || continue
    timeout -k 10 120 python $s --rounds 6000 --transport ${2:-all} 2>> gpurun_out/actors.err | sed "s/^{/{\"build\": \"$b\", /" >> $out || exit $?
  done
done
cat $out
