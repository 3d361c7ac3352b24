# ad-hoc GPU run: ring flag-ownership negative controls
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/negative_controls.py late_forward_protected late_forward_ring_hop_rows late_forward_no_guard late_forward_hop_rows_no_guard > gpurun_out/negative_controls_r5.jsonl 2> gpurun_out/negative_controls_r5.err || exit 1
echo ab done
