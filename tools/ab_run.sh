# ad-hoc GPU run: final settings - 2 co-located workers (group kernel) and the 8-process rehearsal protocol
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in 64M:65536 16M:16384; do
  IFS=: read size c <<< "$cfg"
  timeout -k 10 120 python -u tools/round_breakdown.py --P 2 --size $size --dtype bf16 --chunk $c --rounds 200 --no-trace > /tmp/o.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/o.json'));print(json.dumps({'size':'$size','grid':d.get('grid'),'ms':d.get('ms_per_round'),'ok':d.get('validated')}))"
done
skip="--no-dp --no-tune --no-rccl --no-threshold --no-collectives --no-fused-step --no-links --no-sdma --no-native --no-sizes"
timeout -k 10 300 python -u -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $((29700 + RANDOM % 200)) bench.py --gpus 8 --share-device --steps 10 --warmup 3 $skip \
    > /tmp/r.json 2> gpurun_out/rg_final.err || exit 1
python3 -c "import json;d=json.load(open('/tmp/r.json'));print(json.dumps({'rehearsal8':d.get('protocol_us'),'value':d.get('value')}))"
