#!/bin/bash
# hipIpcOpenMemHandle vs slab size (profiles/ipc_size_probe.md): 2 processes on one GPU map
# each other's XgmiComm slab and run a two-shot allreduce that fills it. (run via gpurun)
export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
probe() { # slot_mib nproc [env]
  env $3 timeout -k 5 60 python -m torch.distributed.run --nnodes=1 --nproc-per-node $2 --master-addr 127.0.0.1 \
    --master-port $((29800 + RANDOM % 100)) tools/ipc_size_probe.py $1 > gpurun_out/ipc_$1_$2.out 2>&1
  echo "slot=$1 np=$2 $3 rc=$? $(grep '^slot' gpurun_out/ipc_$1_$2.out)"
}
probe 500 2     # 1.97 GiB
probe 700 2     # 2.75 GiB: bit 31 set, padded to 4 GiB
probe 1030 2    # 4.05 GiB
probe 1700 2    # 6.68 GiB: padded to 8 GiB
probe 96 8      # 8 ranks, 1.5 GiB
