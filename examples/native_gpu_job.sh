#!/bin/bash
# The reference's deployment (AllreduceMaster / AllreduceWorker processes, README.md of the
# reference: `runMain ...AllreduceMaster 2551 2 10 2` + workers) with every worker's rounds on a
# GPU and no Python anywhere: one `mxar-gpu worker --device k` process per GPU, the master on
# the same host, control over TCP, data over xGMI (IPC-mapped arenas).
#
#   examples/native_gpu_job.sh [workers=8] [dataSize=67108864] [maxChunkSize=131072] [rounds=100]
#   SHARE_DEVICE=1 examples/native_gpu_job.sh 2      # every worker on GPU 0 (one-GPU boxes)
#   DTYPE=bf16 examples/native_gpu_job.sh             # bf16 rounds (fp32 sums, one rounding)
#
# Workers print nothing per round (--quiet); the master prints its steady round rate. Drop
# --quiet from WOPTS to see every round's output sum, as the reference's demo sink does.
set -o pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
X="$HERE/akka_allreduce_1_amd"
P=${1:-8}
N=${2:-67108864}
CHUNK=${3:-131072}
ROUNDS=${4:-100}
PORT=${PORT:-$((20000 + RANDOM % 20000))}
export HSA_ENABLE_IPC_MODE_LEGACY=0
SEEDS="--seeds mxar.tcp://ClusterSystem@127.0.0.1:$PORT --loglevel ERROR"
GRID=0
[ "${SHARE_DEVICE:-0}" = 1 ] && GRID=$((512 / P))
pids=()
for k in $(seq 0 $((P - 1))); do
  dev=$k
  [ "${SHARE_DEVICE:-0}" = 1 ] && dev=0
  # --source iota: data[i] = i + round (the reference's demo source); --spin-us defaults to 500
  "$X/mxar-gpu" worker 0 "$N" --device $dev --max-peers $P --grid $GRID --source iota --dtype ${DTYPE:-fp32} \
    --quiet $SEEDS &
  pids+=($!)
done
"$X/mxar" master $PORT $P $N $CHUNK --th-reduce 1 --th-complete 1 --max-lag 1 --max-round $((ROUNDS - 1)) \
  --spin-us 500 --quiet $SEEDS
rc=$?
for p in "${pids[@]}"; do
  wait "$p" || rc=1
done
exit $rc
