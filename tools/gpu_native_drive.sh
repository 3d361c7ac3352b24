#!/bin/bash
# Python-free deployment on one MI355X: `mxar master` + 2 `mxar-gpu worker --device 0` (th = 1,
# 400 rounds), rounds driven (a) by the master itself, (b) by `mxar drive` over the control
# bridge, pipelined, (c) the same, lock-step. Alternated twice per size.
set -o pipefail
O=gpurun_out/native_drive
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
X=akka_allreduce_1_amd
for rep in 1 2; do
for n in 262144 16777216 67108864; do
for mode in master pipelined lockstep; do
  port=$((20000 + RANDOM % 20000)); bport=$((port + 1))
  seeds="--seeds mxar.tcp://ClusterSystem@127.0.0.1:$port --loglevel ERROR --quiet"
  ext=""; [ $mode != master ] && ext="--bridge $bport --external-rounds"
  timeout -k 5 150 $X/mxar-gpu worker 0 $n --device 0 --max-peers 2 --plane-timeout 20 $seeds > $O/w0.log 2>&1 &
  w0=$!
  timeout -k 5 150 $X/mxar-gpu worker 0 $n --device 0 --max-peers 2 --plane-timeout 20 $seeds > $O/w1.log 2>&1 &
  w1=$!
  timeout -k 10 120 $X/mxar master $port 2 $n $((n / 256)) --th-reduce 1 --th-complete 1 --max-lag 2 --max-round 399 $ext $seeds > $O/m.log 2>&1 &
  m=$!
  drc=0
  if [ $mode != master ]; then
    ls=""; [ $mode = lockstep ] && ls="--lockstep"
    timeout -k 5 110 $X/mxar drive 127.0.0.1:$bport $ls > $O/d.log 2>&1; drc=$?
  fi
  wait $m; rc=$?
  wait $w0; r0=$?
  wait $w1; r1=$?
  echo "{\"rep\": $rep, \"n_f32\": $n, \"mode\": \"$mode\", \"master\": $(grep steady $O/m.log || echo null), \"drive\": $( [ $mode != master ] && (grep driver $O/d.log || echo null) || echo null)}" | tee -a $O/rates.jsonl
  [ $rc -eq 0 ] && [ $r0 -eq 0 ] && [ $r1 -eq 0 ] && [ $drc -eq 0 ] || { echo "failed rc=$rc,$r0,$r1,$drc"; tail -5 $O/*.log; exit 1; }
done
done
done
