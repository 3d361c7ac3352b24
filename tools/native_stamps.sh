#!/bin/bash
# Phase stamps of one size in both deployment shapes on the same box (same f32 geometry as
# tools/native_vs_inproc.sh): the native master + 2 mxar-gpu processes (MXAR_PLANE_STAMPS),
# then the in-process engine (plane_probe --stamps). Output: gpurun_out/stamps_{native,inproc}.json
#   bash tools/native_stamps.sh [n_f32]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
n=${1:-16777216}
rm -f gpurun_out/native_stamps.jsonl
MXAR_PLANE_STAMPS=$PWD/gpurun_out/native_stamps.jsonl NATIVE_SOURCE=static bash tools/gpu.sh native $n || exit 1
timeout -k 10 60 python tools/native_stamps.py gpurun_out/native_stamps.jsonl > gpurun_out/stamps_native.json || exit 1
timeout -k 10 200 python tools/plane_probe.py --P 2 --dtype f32 --sizes $((n * 4)) --rounds 400 --stamps \
  > gpurun_out/stamps_inproc.json 2> gpurun_out/stamps_inproc.err || exit 1
cat gpurun_out/stamps_native.json gpurun_out/stamps_inproc.json
