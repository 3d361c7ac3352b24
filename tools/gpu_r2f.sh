#!/bin/bash
# Native round IO (tensor dataSource, keep-last dataSink, native master stamps): plane GPU
# tests, then the in-process protocol probe alternating Python IO / native IO on one box.
set -o pipefail
mkdir -p gpurun_out/r2f
O=gpurun_out/r2f
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_plane_gpu.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/plane_gpu.log 2>&1
rc=$?; tail -3 $O/plane_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for io in python native; do
    f=""; [ $io = python ] && f="--python-io"
    timeout -k 10 200 python -u tools/plane_probe.py --P 2 --sizes 1M 64M 256M --rounds 300 $f >> $O/io_ab.jsonl 2>> $O/io_ab.err || exit $?
  done
done
cat $O/io_ab.jsonl
