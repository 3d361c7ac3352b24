#!/bin/bash
# two-shot geometry: automatic (by block size) vs the old fixed one-unit-per-workgroup geometry
export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
for mode in auto fixed; do
  if [ $mode = fixed ]; then export MXAR_TWOSHOT_UNITS=1 MXAR_TWOSHOT_SUB=64; fi
  timeout -k 10 200 python -m akka_allreduce_1_amd bench --local 4 --algos twoshot threshold --sizes 16M 64M 256M --iters 10 > gpurun_out/geo4_$mode.txt 2>&1 || exit 1
  timeout -k 10 200 python -m akka_allreduce_1_amd bench --local 8 --algos twoshot threshold --sizes 16M 64M 256M --iters 10 > gpurun_out/geo8_$mode.txt 2>&1 || exit 1
  for P in 4 8; do echo "$mode P=$P: $(grep -E '^ +[0-9]+ +(twoshot|threshold)' gpurun_out/geo${P}_$mode.txt | awk '{printf "%s/%s=%sus ", $1/1048576, $2, $3}')"; done
done
