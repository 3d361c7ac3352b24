# ad-hoc GPU run: 8 co-located workers x 64 MiB, new default grid (32) vs the old 64
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/p8_64m_grid.jsonl
rm -f $out
for rep in 0 1; do
  for g in 0 64; do
    timeout -k 10 150 python -u tools/round_breakdown.py --P 8 --size 64M --dtype bf16 --chunk 16384 --grid $g --rounds 100 --no-trace > /tmp/o.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('/tmp/o.json'));print(json.dumps({'rep':$rep,'P':8,'size':'64M','chunk':16384,'grid':d.get('grid'),'ms':d.get('ms_per_round'),'ok':d.get('validated'),'err':d.get('error')}))" >> $out
  done
done
cat $out
