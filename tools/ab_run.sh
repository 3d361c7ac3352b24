# ad-hoc GPU run: DP overlap rehearsal with CU splits
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/dp_overlap_run.py --models llama3_8b > gpurun_out/dp_overlap2.json 2> gpurun_out/dp_overlap2.err || exit 1
echo ab done
