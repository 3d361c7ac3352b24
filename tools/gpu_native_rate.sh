#!/bin/bash
# Round rates of the Python-free deployment: `mxar master` + 2 `mxar-gpu worker --device 0`
# processes (TCP cluster control, xGMI-arena data plane, th = 1), 400 rounds per size; the
# master prints its steady round rate. Then the in-process Python PlaneJob at the same sizes.
set -o pipefail
mkdir -p gpurun_out/native
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/native
X=akka_allreduce_1_amd
for g in ${GRIDS:-0}; do
for n in ${SIZES:-262144 16777216 67108864}; do
  port=$((20000 + RANDOM % 20000))
  seeds="--seeds mxar.tcp://ClusterSystem@127.0.0.1:$port --loglevel ERROR --quiet"
  timeout -k 5 150 $X/mxar-gpu worker 0 $n --device 0 --max-peers 2 --plane-timeout 20 --grid $g $seeds > $O/w0_$n.log 2>&1 &
  w0=$!
  timeout -k 5 150 $X/mxar-gpu worker 0 $n --device 0 --max-peers 2 --plane-timeout 20 --grid $g $seeds > $O/w1_$n.log 2>&1 &
  w1=$!
  timeout -k 10 120 $X/mxar master $port 2 $n $((n / 8)) --th-reduce 1 --th-complete 1 --max-lag 2 --max-round 399 $seeds > $O/m_$n.log 2>&1
  rc=$?
  wait $w0; r0=$?
  wait $w1; r1=$?
  echo "grid=$g n=$n master rc=$rc workers rc=$r0,$r1: $(grep steady $O/m_$n.log)"
  [ $rc -eq 0 ] && [ $r0 -eq 0 ] && [ $r1 -eq 0 ] || exit 1
done
done
[ -n "$NO_PROBE" ] && exit 0
timeout -k 10 150 python -u tools/plane_probe.py --P 2 --sizes 1M 64M 256M --rounds 400 --timeout 10 > $O/probe.jsonl 2> $O/probe.err || exit 1
cut -c1-300 $O/probe.jsonl
