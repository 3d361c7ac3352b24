# ad-hoc GPU run: default-grid LocalCluster launches after the shared-launch cap
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/shared_cap.jsonl
rm -f $out
for rep in 0 1; do
  for cfg in 2:256 2:128 4:128 4:256 8:256 2:64; do
    IFS=: read P mib <<< "$cfg"
    timeout -k 10 120 python -u tools/phase_profile.py --P $P --mib $mib --grid 512 --algos twoshot threshold --iters 8 > /tmp/o.jsonl 2>/dev/null || exit 1
    python3 -c "
import json
for l in open('/tmp/o.jsonl'):
    d=json.loads(l)
    for k,v in d.items(): print(json.dumps({'rep':$rep,'P':$P,'mib':$mib,'grid':'default','algo':k,'span_p50':v['span_us']['p50'],'wgs':v['workgroups'],'TBps':v['hbm_TBps_at_span_p50']}))
" >> $out
  done
done
cat $out
