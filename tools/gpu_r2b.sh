#!/bin/bash
# Round-2 follow-ups: reducer overhead breakdown, fused AdamW in-bench vs standalone (same box).
set -o pipefail
mkdir -p gpurun_out/r2b
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/r2b
timeout -k 10 240 python -u tools/reducer_overhead.py --model llama3_8b --bucket-mib 1024 --rounds 8 > $O/reducer_llama.jsonl 2> $O/reducer.err || exit $?
timeout -k 10 240 python -u tools/reducer_overhead.py --model llama3_8b --bucket-mib 1024 --rounds 8 --event-scope 2 >> $O/reducer_llama.jsonl 2>> $O/reducer.err || exit $?
timeout -k 10 120 python -u tools/reducer_overhead.py --model resnet50 --bucket-mib 25 --rounds 20 > $O/reducer_resnet.jsonl 2>> $O/reducer.err || exit $?
cat $O/reducer_llama.jsonl $O/reducer_resnet.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_ab -o ab -- python3 tools/adam_state_ab.py separate 40 > $O/adam_ab.jsonl 2> $O/adam_ab.err || exit $?
cat $O/adam_ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o bench -- python3 bench.py --steps 40 --warmup 5 --no-tune --no-threshold --no-collectives --no-dp --no-local --no-protocol --no-rccl > $O/bench_adam.json 2> $O/bench_adam.err || exit $?
cat $O/bench_adam.json
echo done
