# ad-hoc GPU A/B driver (this round's threshold / reduce work); see tools/thr_ab.py
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
bash tools/gpu.sh tests tests/test_threshold_gpu.py tests/test_sdma_gpu.py tests/test_plane_gpu.py tests/test_comm_gpu.py || exit 1
for rep in 1 2; do
  PYTHONPATH=abtree/old timeout -k 10 120 python tools/thr_ab.py --tag old >> gpurun_out/thr_ab3.jsonl || exit 1
  timeout -k 10 120 python tools/thr_ab.py --tag new >> gpurun_out/thr_ab3.jsonl || exit 1
done
timeout -k 10 120 python tools/phase_profile.py --P 8 --kib 4 --algos twoshot threshold --iters 20 > gpurun_out/phase_p8.jsonl || exit 1
timeout -k 10 120 python tools/phase_profile.py --P 2 --kib 4 --algos twoshot threshold --iters 20 > gpurun_out/phase_p2.jsonl || exit 1
echo ab done
