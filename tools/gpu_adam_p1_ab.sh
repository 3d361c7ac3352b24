#!/bin/bash
# Fused AdamW at P = 1 (the N = 1 optimizer step): PT = 1 template instantiation (HEAD) vs
# the runtime-P loop (abtest/old = c82cc1b, built in-tree, not committed), alternated.
set -o pipefail
mkdir -p gpurun_out/adam
O=gpurun_out/adam
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_adamw_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for b in old new; do
    s=tools/adam_state_ab.py; [ $b = old ] && s=abtest/old/tools/adam_state_ab.py
    timeout -k 10 120 python -u $s separate 40 2>> $O/ab.err | sed "s/^{/{\"build\": \"$b\", /" >> $O/ab.jsonl || exit $?
  done
done
cat $O/ab.jsonl
