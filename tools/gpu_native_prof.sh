#!/bin/bash
# Kernel trace of one `mxar-gpu` worker (the other runs unprofiled) at 256 MiB per round.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/nprof
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/nprof
X=akka_allreduce_1_amd
n=${N:-67108864}
port=$((20000 + RANDOM % 20000))
seeds="--seeds mxar.tcp://ClusterSystem@127.0.0.1:$port --loglevel ERROR --quiet"
timeout -k 5 150 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/p${MXAR_PLANE_SPLIT:-x} -o w0 -- $X/mxar-gpu worker 0 $n --device 0 --max-peers 2 --plane-timeout 20 $seeds > $O/w0.log 2>&1 &
w0=$!
sleep 3
timeout -k 5 150 $X/mxar-gpu worker 0 $n --device 0 --max-peers 2 --plane-timeout 20 $seeds > $O/w1.log 2>&1 &
w1=$!
timeout -k 10 120 $X/mxar master $port 2 $n $((n / 8)) --th-reduce 1 --th-complete 1 --max-lag 2 --max-round 60 $seeds > $O/m.log 2>&1
rc=$?
wait $w0; r0=$?
wait $w1; r1=$?
echo "master rc=$rc workers rc=$r0,$r1: $(grep steady $O/m.log)"
find $O/p${MXAR_PLANE_SPLIT:-x} -name '*stats*' | head
