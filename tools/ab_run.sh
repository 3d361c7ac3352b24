# ad-hoc GPU run: 40 B protocol round breakdown, dispatcher spin budget default vs 500 us
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/spin_ab.jsonl
rm -f $out
for rep in 0 1; do
  for spin in default 500; do
    if [ $spin = default ]; then unset MXAR_DISPATCH_SPIN_US; else export MXAR_DISPATCH_SPIN_US=$spin; fi
    timeout -k 10 120 python -u tools/round_breakdown.py --P 2 --size 40 --dtype f32 --chunk 2 --rounds 600 > /tmp/o.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('/tmp/o.json'));print(json.dumps({'rep':$rep,'spin':'$spin','ms':d.get('ms_per_round'),'med':d.get('median_us')}))" >> $out
  done
done
cat $out
