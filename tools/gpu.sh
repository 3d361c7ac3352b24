#!/bin/bash
# One entry point for GPU-box work (run through gpurun from the repo root):
#
#   gpurun -- 'bash tools/gpu.sh ci'                      gpu tests + smoke() + the N=1 bench line
#   gpurun -- 'bash tools/gpu.sh tests [pytest args]'     gpu-marked tests (default: all of them)
#   gpurun -- 'bash tools/gpu.sh bench [bench.py args]'   the N=1 bench line -> gpurun_out/bench_n1.json
#   gpurun -- 'bash tools/gpu.sh prof [bench.py args]'    rocprofv3 kernel trace + stats of the bench
#   gpurun -- 'bash tools/gpu.sh pmc "<counters>" <cmd>'  one rocprofv3 PMC pass (kernel trace only)
#   gpurun -- 'bash tools/gpu.sh rehearsal [2 4 8]'       N>1 bench path as N processes on ONE GPU
#   gpurun -- 'bash tools/gpu.sh native [sizes]'          Python-free mxar master + 2 mxar-gpu workers
#   gpurun -- 'bash tools/gpu.sh run <tag> <cmd...>'      any python tool under a time limit, output
#                                                         in gpurun_out/<tag>.{out,err}
#
# Every GPU step runs under its own `timeout -k`, steps are chained so that the first failure
# (fault, abort, time limit) ends the script: nothing more touches the GPU after it.
# (The round-1/2 session scripts this replaces are in git history before round 3.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
task=${1:-ci}
shift || true

tests() {
  local args=("$@")
  [ ${#args[@]} -eq 0 ] && args=(tests)
  timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider \
    "${args[@]}" > $O/gpu_tests.log 2>&1
  local rc=$?
  echo "gpu tests rc=$rc: $(tail -1 $O/gpu_tests.log)"
  [ $rc -eq 0 ] || grep -E "FAILED|ERROR|Error" $O/gpu_tests.log | head -30
  return $rc
}

bench() {
  timeout -k 10 900 python -u bench.py "$@" > $O/bench_n1.json 2> $O/bench_n1.err
  local rc=$?
  echo "bench rc=$rc"
  [ $rc -eq 0 ] || tail -20 $O/bench_n1.err
  return $rc
}

case $task in
  ci)
    tests && {
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
      echo "smoke ok"
    } && bench --steps 20 --warmup 5
    ;;
  tests) tests "$@" ;;
  bench) bench "$@" ;;
  prof)
    # (no native-deployment section: its child processes would run under the profiler too)
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-native "$@" \
      > $O/prof_bench.json 2> $O/prof_bench.err
    rc=$?
    f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
    # the raw kernel trace runs to hundreds of MiB (gpurun copies back <= 64 MiB): keep the stats
    find $O/prof -name '*kernel_trace.csv' -delete
    [ -n "$f" ] || { echo "profiled bench failed (rc=$rc, no stats)"; tail -20 $O/prof_bench.err; exit 1; }
    python3 tools/prof.py csv "${f%_kernel_stats.csv}" "bench.py $*" > $O/prof_summary.md
    # a non-zero status after the profiler wrote its stats (e.g. a crash in process teardown
    # under the profiler's library) is reported, the stats are kept
    echo "prof ok (bench rc=$rc)"
    ;;
  pmc)
    counters=$1
    shift
    tag=$(echo "$counters" | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $counters --output-format csv -d $O/pmc_$tag -o run -- "$@" \
      > $O/pmc_$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $O/pmc_$tag.log; exit 1; }
    echo "pmc $tag ok"
    ;;
  rehearsal)
    ns=("$@")
    [ ${#ns[@]} -eq 0 ] && ns=(2 4 8)
    for n in "${ns[@]}"; do
      timeout -k 10 400 python -u -m torch.distributed.run --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $((29640 + n)) bench.py --gpus $n --share-device --no-dp --steps 10 --warmup 3 \
        > $O/rehearsal_n$n.json 2> $O/rehearsal_n$n.err
      rc=$?
      echo "rehearsal n=$n rc=$rc"
      [ $rc -eq 0 ] || { tail -20 $O/rehearsal_n$n.err; exit $rc; }
    done
    ;;
  native)
    # NATIVE_SOURCE=iota|static (per-round demo fill, or the same input every round),
    # NATIVE_GRID (workgroups per worker; 256 = half the GPU each: separate kernels, one per process)
    sizes=("$@")
    [ ${#sizes[@]} -eq 0 ] && sizes=(262144 16777216 67108864)
    src=${NATIVE_SOURCE:-iota}
    grid=${NATIVE_GRID:-256}
    X=akka_allreduce_1_amd
    for n in "${sizes[@]}"; do
      port=$((20000 + RANDOM % 20000))
      seeds="--seeds mxar.tcp://ClusterSystem@127.0.0.1:$port --loglevel ERROR --quiet"
      wopt="--device 0 --max-peers 2 --plane-timeout 20 --grid $grid --source $src"
      timeout -k 5 150 $X/mxar-gpu worker 0 $n $wopt $seeds > $O/w0.log 2>&1 &
      w0=$!
      timeout -k 5 150 $X/mxar-gpu worker 0 $n $wopt $seeds > $O/w1.log 2>&1 &
      w1=$!
      timeout -k 10 120 $X/mxar master $port 2 $n $((n > 524288 ? n / 512 : 1024)) --th-reduce 1 --th-complete 1 \
        --max-lag 1 --max-round 399 --spin-us ${NATIVE_MASTER_SPIN:-500} $seeds > $O/m.log 2>&1
      rc=$?
      wait $w0; r0=$?
      wait $w1; r1=$?
      echo "{\"n_f32\": $n, \"source\": \"$src\", \"grid\": $grid, \"master\": $(grep steady $O/m.log || echo null)}" | tee -a $O/native_rates.jsonl
      [ $rc -eq 0 ] && [ $r0 -eq 0 ] && [ $r1 -eq 0 ] || { echo "failed rc=$rc,$r0,$r1"; tail -5 $O/*.log; exit 1; }
    done
    ;;
  run)
    tag=$1
    shift
    timeout -k 10 900 "$@" > $O/$tag.out 2> $O/$tag.err
    rc=$?
    echo "$tag rc=$rc"
    [ $rc -eq 0 ] || tail -20 $O/$tag.err
    exit $rc
    ;;
  *) echo "unknown task $task"; exit 2 ;;
esac
