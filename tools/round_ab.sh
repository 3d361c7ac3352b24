#!/bin/bash
# Same-box A/B of the protocol round's host path (tools/round_breakdown.py): P = 2 plane
# workers, 40 B (the reference's default job) and 1 MiB rounds, each traced (hop breakdown)
# and untraced (clean round time), variants interleaved over 2 reps.
#
#   bash tools/round_ab.sh default "events:MXAR_PLANE_EVENTS=1" "old:MXAR_DISPATCH_LIFO=0,MXAR_DISPATCH_YIELD=1"
#
# A variant is NAME or NAME:VAR=VAL[,VAR=VAL...]. Knobs: MXAR_PLANE_EVENTS=1 (per-round event
# confirms completion), MXAR_DISPATCH_NOTIFY=always (futex wake on every schedule),
# MXAR_DISPATCH_LIFO=0 (no run-next slot), MXAR_DISPATCH_YIELD=1 (yield-only idle spin).
# Output: gpurun_out/round_ab.jsonl
O=gpurun_out/round_ab.jsonl
: > $O
variants=("$@")
[ ${#variants[@]} -eq 0 ] && variants=(default)
for rep in 1 2; do
  for spec in "${variants[@]}"; do
    name=${spec%%:*}
    env=()
    if [[ $spec == *:* ]]; then IFS=, read -r -a env <<< "${spec#*:}"; fi
    for sz in "40 --dtype f32 --chunk 2" "1M"; do
      for tr in "" "--no-trace"; do
        env "${env[@]}" timeout -k 10 120 python tools/round_breakdown.py --P 2 --size $sz --rounds 400 $tr \
          2>>gpurun_out/round_ab.err | sed "s/^{/{\"variant\": \"$name\", \"rep\": $rep, /" >> $O || exit 1
      done
    done
  done
done
echo round ab ok
