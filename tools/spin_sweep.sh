#!/bin/bash
# Host CPU vs round latency of the protocol engine: the plane's completion
# thread spin budget (spin_us) x the actor dispatchers' idle spin (MXAR_DISPATCH_SPIN_US),
# 2 plane workers, 1 MiB and 40 B rounds. Output: gpurun_out/spin_sweep.jsonl
O=gpurun_out/spin_sweep.jsonl
: > $O
for rep in 1 2; do
for d in 50 0; do
for s in 1000 100 0; do
  MXAR_DISPATCH_SPIN_US=$d timeout -k 10 120 python tools/plane_probe.py --P 2 --sizes 1M 40 --rounds 300 --spin-us $s \
    2>>gpurun_out/spin_sweep.err | sed "s/^{/{\"dispatch_spin_us\": $d, \"rep\": $rep, /" >> $O || exit 1
done; done; done
echo spin sweep ok
