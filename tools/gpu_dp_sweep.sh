set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_ddp_gpu.py -q -x > gpurun_out/pt_ddp.log 2>&1 || { tail -30 gpurun_out/pt_ddp.log; exit 1; }
tail -1 gpurun_out/pt_ddp.log
for cfg in "--sync torch" "--sync native --event-scope 0" "--sync native --event-scope 1" "--sync native --event-scope 2" "--sync native --event-scope 1 --bucket-mib 256"; do
  timeout -k 10 300 python benchmarks/bench_dp.py --model llama3_8b --steps 3 --warmup 1 $cfg 2> /dev/null | tail -1 >> gpurun_out/dp_sweep.jsonl || exit 1
done
cat gpurun_out/dp_sweep.jsonl
