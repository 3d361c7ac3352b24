#!/bin/bash
# Same-box comparison of the reference's deployment shape (mxar master + 2 mxar-gpu worker
# processes on GPU 0, arenas IPC-mapped, control over TCP) with the in-process protocol engine
# (2 plane workers + master in one process): f32, maxChunkSize = n / 512, 256 workgroups per
# worker, the same input every round; 1 / 64 / 256 MiB, interleaved over reps. Both sides are
# MEAN round intervals (native: 1 / the master's steady rounds/s; in-process: plane_probe).
# Output: gpurun_out/native_vs_inproc.jsonl
#   bash tools/native_vs_inproc.sh [reps]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/native_vs_inproc.jsonl
: > $O
reps=${1:-2}
for rep in $(seq 1 "$reps"); do
  : > gpurun_out/native_rates.jsonl
  NATIVE_SOURCE=static bash tools/gpu.sh native 262144 16777216 67108864 > /dev/null || exit 1
  sed "s/^{/{\"shape\": \"native\", \"rep\": $rep, /" gpurun_out/native_rates.jsonl >> $O
  timeout -k 10 200 python tools/plane_probe.py --P 2 --dtype f32 --sizes 1M 64M 256M --rounds 400 \
    2>> gpurun_out/native_vs_inproc.err | sed "s/^{/{\"shape\": \"in-process\", \"rep\": $rep, /" >> $O || exit 1
done
python3 - <<'EOF'
import json, collections
per = collections.defaultdict(list)
for l in open("gpurun_out/native_vs_inproc.jsonl"):
    d = json.loads(l)
    if d["shape"] == "native":
        per[(d["n_f32"] * 4, "native")].append(round(1e6 / d["master"]["steady_rounds_per_s"], 1))  # mean
    else:
        per[(d["bytes"], "in-process")].append(round(d["ms_per_round"] * 1e3, 1))
for b in sorted({k[0] for k in per}):
    nat, inp = per[(b, "native")], per[(b, "in-process")]
    print(json.dumps({"bytes": b, "native_us": nat, "in_process_us": inp,
                      "native_over_in_process": round(sorted(nat)[len(nat) // 2] / sorted(inp)[len(inp) // 2], 3)}))
EOF
