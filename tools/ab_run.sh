# ad-hoc GPU run: SDMA child section (test + N=2 rehearsal)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh tests tests/test_sdma_gpu.py -k "xdev" -s || exit 1
timeout -k 10 400 python -u -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29642 bench.py --gpus 2 --share-device --no-dp --no-protocol --no-collectives --no-fused-step --no-tune --steps 5 --warmup 2 > gpurun_out/rehearsal_sdma_n2.json 2> gpurun_out/rehearsal_sdma_n2.err || exit 1
echo ab done
