#!/bin/bash
# Slot-reuse guard study (run through gpurun from the repo root):
#   1. the slow-reader test with the guard (must pass) and without it (MXAR_SLOT_GUARD=0:
#      the negative control - expected to fail with a mismatch, never a fault);
#   2. same-box A/B of the bench's kernel sections: this tree, this tree with the guard off,
#      and the previous commit built in ./ab_old (a git worktree), alternated twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=tests/test_comm_gpu.py::test_multiprocess_slot_reuse_slow_reader
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider $T \
  > $O/guard_test.log 2>&1 || { echo "guarded test failed"; tail -20 $O/guard_test.log; exit 1; }
echo "guarded test ok"
MXAR_SLOT_GUARD=0 timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider $T > $O/guard_negative.log 2>&1
rc=$?
echo "negative control rc=$rc (1 = the hazard showed)"
[ $rc -le 1 ] || exit 1
ARGS="--no-dp --no-protocol --no-native --no-tune --no-rccl --no-threshold --steps 20 --warmup 5"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py $ARGS > $O/ab_new_$i.json 2> $O/ab_new_$i.err || { echo "new failed"; exit 1; }
  MXAR_SLOT_GUARD=0 timeout -k 10 400 python -u bench.py $ARGS > $O/ab_noguard_$i.json 2> $O/ab_noguard_$i.err \
    || { echo "noguard failed"; exit 1; }
  if [ -d ab_old ]; then
    (cd ab_old && timeout -k 10 400 python -u bench.py $ARGS) > $O/ab_old_$i.json 2> $O/ab_old_$i.err \
      || { echo "old failed"; exit 1; }
  fi
  echo "round $i done"
done
