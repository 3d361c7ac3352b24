#!/bin/bash
# Kernel-level comparison of the native deployment (mxar master + 2 mxar-gpu worker processes
# sharing GPU 0, IPC-mapped arenas) with the in-process protocol engine (2 plane workers in one
# process, arenas shared by pointer): the same f32 size, geometry (maxChunkSize = n / 512),
# grid (256 workgroups per worker) and static source; worker 0 / the in-process run under
# rocprofv3 --kernel-trace. Output: gpurun_out/nat/*, gpurun_out/inp/*, native_prof.json.
#   bash tools/native_prof.sh [n_f32]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
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
