# ad-hoc GPU run: protocol round (2 co-located workers, group kernel) vs the 2-rank single launch, same box
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/protocol_vs_launch.jsonl
rm -f $out
for rep in 0 1; do
  for cfg in 16M:16384:16 64M:65536:64 256M:262144:256; do
    IFS=: read size c mib <<< "$cfg"
    r=200; [ $size = 256M ] && r=100
    timeout -k 10 120 python -u tools/round_breakdown.py --P 2 --size $size --dtype bf16 --chunk $c --rounds $r --no-trace > /tmp/o.json 2>/dev/null || exit 1
    timeout -k 10 120 python -u tools/phase_profile.py --P 2 --mib $mib --algos threshold twoshot --iters 8 > /tmp/p.jsonl 2>/dev/null || exit 1
    python3 -c "
import json
d=json.load(open('/tmp/o.json'))
row={'rep':$rep,'size':'$size','protocol_round_us':round(d['ms_per_round']*1e3,1),'protocol_kernel_us':d.get('kernel_last_round_us')}
for l in open('/tmp/p.jsonl'):
    for k,v in json.loads(l).items(): row[k+'_single_launch_span_us']=v['span_us']['p50']
print(json.dumps(row))" >> $out
  done
done
cat $out
