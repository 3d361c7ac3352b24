# ad-hoc GPU run: protocol-round maxChunkSize sweep at 64 MiB bf16 (2 co-located workers)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/chunk64m.jsonl
for size in 64M 16M; do
  for c in 16384 32768 65536 131072 262144 1048576; do
    timeout -k 10 120 python -u tools/round_breakdown.py --P 2 --size $size --dtype bf16 --chunk $c --rounds 120 --no-trace > /tmp/o.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('/tmp/o.json'));print(json.dumps({'size':'$size','chunk':$c,'ms':d.get('ms_per_round'),'ok':d.get('validated'),'k':d.get('kernel_last_round_us')}))" >> gpurun_out/chunk64m.jsonl
  done
done
cat gpurun_out/chunk64m.jsonl
