#!/bin/bash
# End-of-session evidence: every gpu test, smoke(), the N=1 bench line, and a rocprofv3
# kernel trace + stats of the bench (dp sections off: they are GEMM traces).
set -o pipefail
mkdir -p gpurun_out/final
O=gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || { echo bench failed; tail $O/bench_n1.err; exit 1; }
echo bench ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --no-dp \
  > $O/bench_traced.json 2> $O/bench_traced.err || { echo "bench trace failed"; tail -5 $O/bench_traced.err; exit 1; }
echo trace ok
