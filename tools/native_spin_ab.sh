#!/bin/bash
# Native deployment (mxar master + 2 mxar-gpu processes, static source, f32): round time with
# the actor dispatchers' idle spin and the cluster readers' socket poll at their defaults vs
# long enough to cover a round's kernel (every hop of the round then lands on a running
# thread instead of waking a sleeping one). Interleaved reps; gpurun_out/native_spin_ab.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/native_spin_ab.jsonl
: > $O
for rep in 1 2 3; do
  for v in "default:" "dispatch:MXAR_DISPATCH_SPIN_US=500" "tcp:MXAR_TCP_SPIN_US=500" "both:MXAR_DISPATCH_SPIN_US=500,MXAR_TCP_SPIN_US=500"; do
    name=${v%%:*}
    IFS=, read -r -a env <<< "${v#*:}"
    : > gpurun_out/native_rates.jsonl
    env "${env[@]}" NATIVE_SOURCE=static bash tools/gpu.sh native 262144 16777216 > /dev/null || exit 1
    sed "s/^{/{\"variant\": \"$name\", \"rep\": $rep, /" gpurun_out/native_rates.jsonl >> $O
  done
done
python3 - <<'PY'
import json, collections
per = collections.defaultdict(list)
for l in open("gpurun_out/native_spin_ab.jsonl"):
    d = json.loads(l)
    per[(d["n_f32"] * 4, d["variant"])].append(round(1e6 / d["master"]["steady_rounds_per_s"], 1))
for k, v in sorted(per.items()):
    print(json.dumps({"bytes": k[0], "variant": k[1], "mean_round_us": v}))
PY
