# ad-hoc GPU run: co-located plane grid, new default (CUs / workers + one chunk per workgroup) vs the old 512 / workers
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/grid_default_ab.jsonl
rm -f $out
for rep in 0 1; do
  for cfg in 2:1M:1024 2:16M:16384 2:64M:65536 2:256M:262144 4:16M:8192 8:16M:4096 4:64M:32768; do
    IFS=: read P size c <<< "$cfg"
    for g in 0 $((512 / P)); do
      r=200; [ $size = 256M ] && r=100; [ $size = 1M ] && r=400
      timeout -k 10 150 python -u tools/round_breakdown.py --P $P --size $size --dtype bf16 --chunk $c --grid $g --rounds $r --no-trace > /tmp/o.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.load(open('/tmp/o.json'));print(json.dumps({'rep':$rep,'P':$P,'size':'$size','chunk':$c,'grid':d.get('grid'),'ms':d.get('ms_per_round'),'ok':d.get('validated'),'k':d.get('kernel_last_round_us'),'err':d.get('error')}))" >> $out
    done
  done
done
cat $out
