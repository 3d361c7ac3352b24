#!/bin/bash
# The reference's deployment shape on the GPU - `mxar master` + 2 `mxar-gpu worker` processes
# sharing GPU 0, arenas IPC-mapped, control over TCP - studied against the in-process protocol
# engine (master + 2 plane workers in one process). f32, maxChunkSize = n / 512, 256
# workgroups per worker, the same input every round (`--source static`). Output under gpurun_out/.
#
#   bash tools/native_study.sh compare [reps]   mean round interval of both shapes at 1 / 64 / 256 MiB,
#                                               interleaved reps -> native_vs_inproc.jsonl
#   bash tools/native_study.sh prof [n_f32]     rocprofv3 kernel traces of both shapes -> native_prof.json
#   bash tools/native_study.sh stamps [n_f32]   phase stamps of both shapes' last round (MXAR_PLANE_STAMPS)
#                                               -> stamps_{native,inproc}.json
#   bash tools/native_study.sh spin             host polling A/B (dispatcher / cluster reader spin)
#                                               -> native_spin_ab.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mode=${1:-compare}
shift || true
case $mode in
  compare)
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
;;
  prof)
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out
n=${1:-16777216}
X=akka_allreduce_1_amd
port=$((20000 + RANDOM % 20000))
seeds="--seeds mxar.tcp://ClusterSystem@127.0.0.1:$port --loglevel ERROR --quiet"
wopt="--device 0 --max-peers 2 --plane-timeout 20 --grid 256 --source static"
rm -rf $O/nat $O/inp
timeout -k 5 150 rocprofv3 --kernel-trace --output-format csv -d $O/nat -o w0 -- $X/mxar-gpu worker 0 $n $wopt $seeds \
  > $O/nat_w0.log 2>&1 &
w0=$!
sleep 3  # the profiler's start-up before the job's rounds
timeout -k 5 150 $X/mxar-gpu worker 0 $n $wopt $seeds > $O/nat_w1.log 2>&1 &
w1=$!
timeout -k 10 120 $X/mxar master $port 2 $n $((n / 512)) --th-reduce 1 --th-complete 1 --max-lag 1 --max-round 399 \
  $seeds > $O/nat_m.log 2>&1
rc=$?
wait $w0; r0=$?
wait $w1; r1=$?
[ $rc -eq 0 ] && [ $r0 -eq 0 ] && [ $r1 -eq 0 ] || { echo "native failed rc=$rc,$r0,$r1"; tail -5 $O/nat_*.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/inp -o inp -- python3 tools/plane_probe.py --P 2 \
  --dtype f32 --sizes $((n * 4)) --rounds 400 > $O/inp.out 2> $O/inp.err || { echo "in-process failed"; tail -5 $O/inp.err; exit 1; }
python3 - "$n" <<'EOF' > $O/native_prof.json
import csv, glob, json, statistics, sys
def ks(d):
    p = glob.glob(f"gpurun_out/{d}/**/*kernel_trace.csv", recursive=True)
    rows = list(csv.DictReader(open(p[0])))
    th = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "threshold" in r["Kernel_Name"])
    # a round's kernels on one worker: in-process both workers' kernels are traced (pair by start)
    return th
out = {"n_f32": int(sys.argv[1])}
m = open("gpurun_out/nat_m.log").read()
for line in m.splitlines():
    if "steady" in line:
        out["native_master"] = json.loads(line[line.index("{"):]) if "{" in line else line
for d in ("nat", "inp"):
    th = ks(d)[40:]  # past warm-up
    dur = [(e - s) / 1e3 for s, e in th]
    gaps = [(th[i + 1][0] - th[i][1]) / 1e3 for i in range(len(th) - 1)]
    out[d] = {"kernels": len(th), "kernel_us_p50": round(statistics.median(dur), 1),
              "kernel_us_p90": round(sorted(dur)[int(0.9 * (len(dur) - 1))], 1),
              "gap_to_next_kernel_us_p50": round(statistics.median(gaps), 1) if gaps else None}
out["inproc_probe"] = json.loads(open("gpurun_out/inp.out").read().splitlines()[-1])["ms_per_round"]
print(json.dumps(out))
EOF
cat $O/native_prof.json
;;
  stamps)
n=${1:-16777216}
rm -f gpurun_out/native_stamps.jsonl
MXAR_PLANE_STAMPS=$PWD/gpurun_out/native_stamps.jsonl NATIVE_SOURCE=static bash tools/gpu.sh native $n || exit 1
timeout -k 10 60 python tools/native_stamps.py gpurun_out/native_stamps.jsonl > gpurun_out/stamps_native.json || exit 1
timeout -k 10 200 python tools/plane_probe.py --P 2 --dtype f32 --sizes $((n * 4)) --rounds 400 --stamps \
  > gpurun_out/stamps_inproc.json 2> gpurun_out/stamps_inproc.err || exit 1
cat gpurun_out/stamps_native.json gpurun_out/stamps_inproc.json
;;
  spin)
O=gpurun_out/native_spin_ab.jsonl
: > $O
for rep in 1 2 3; do
  # explicit MXAR_* values win over the executables' --spin-us (mxar_main.cc apply_spin)
  for v in "builtin:MXAR_DISPATCH_SPIN_US=50,MXAR_TCP_SPIN_US=0" "dispatch:MXAR_DISPATCH_SPIN_US=500,MXAR_TCP_SPIN_US=0" \
           "tcp:MXAR_DISPATCH_SPIN_US=50,MXAR_TCP_SPIN_US=500" "both:MXAR_DISPATCH_SPIN_US=500,MXAR_TCP_SPIN_US=500"; do
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
;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
