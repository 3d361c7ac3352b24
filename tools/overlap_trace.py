#!/usr/bin/env python3
"""Why the one-GPU DP overlap rehearsal loses to the serial schedule (bench dp.overlap_rehearsal):
a kernel-level look, run under rocprofv3 --kernel-trace.

Three phases, separated by idle gaps of 20 ms that the analysis splits on:
  A  compute only: the synthetic backward (weight-gradient GEMMs) + SGD update
  B  overlap:      the same with each bucket's 2-rank allreduce on the comm stream as it fills
  C  serial:       backward first, then every bucket's allreduce
Each phase runs `--reps` steps. `--analyze PREFIX` reads the kernel trace and reports per phase
the GEMM time (sum and per-kernel median), the comm kernels' time, the wall span and how much
of the comm kernels' time overlapped a GEMM.

    rocprofv3 --kernel-trace -d gpurun_out/ovl -o ovl -- python3 tools/overlap_trace.py --layers 4
    python3 tools/overlap_trace.py --analyze gpurun_out/ovl/<host>/ovl
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a) -> None:
    import torch

    from akka_allreduce_1_amd.models.grad_sets import gradient_shapes, llama3_8b_shapes
    from akka_allreduce_1_amd.parallel import BucketedGradReducer
    from benchmarks.bench_dp import SyntheticBackward
    from benchmarks.sections import PairRehearsalComm, _Placeholder

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    shapes = llama3_8b_shapes(a.layers) if a.model == "llama3_8b" else gradient_shapes(a.model)
    params = [torch.nn.Parameter(torch.zeros(sh, dtype=torch.bfloat16, device=dev)) for _, sh in shapes]
    reducer = BucketedGradReducer(params, _Placeholder(), op="avg", bucket_bytes=a.bucket_mib << 20)
    reducer.remove_hooks()
    comm = PairRehearsalComm(reducer.buckets, max(a.grid, 8))
    for c in comm.cl.comms:
        c.grid = a.grid
    reducer.comm = comm
    reducer._raw_ok = True
    bwd = SyntheticBackward(params, a.tokens, torch.bfloat16, dev)
    grads = [q.grad for q in params]

    def compute():
        bwd.run(None)
        torch._foreach_add_(params, grads, alpha=-1e-3)

    def overlap():
        reducer.overlap = True
        bwd.run(reducer)
        reducer.wait()
        torch._foreach_add_(params, grads, alpha=-1e-3)

    def serial():
        reducer.overlap = False
        bwd.run(reducer)
        reducer.wait()
        torch._foreach_add_(params, grads, alpha=-1e-3)

    from akka_allreduce_1_amd._native import C

    out = {"model": a.model, "layers": a.layers, "tokens": a.tokens, "grid": a.grid, "buckets": len(reducer.buckets),
           "bucket_bytes": [b.nbytes for b in reducer.buckets][:4]}
    probe_stream = torch.cuda.Stream(device=dev)
    interval = 5000  # 50 us at 100 MHz

    def clock_mhz(samples: torch.Tensor, dur_s: float) -> float | None:
        """Median shader clock over the samples inside the phase's first 90 %."""
        v = samples.view(-1, 2).cpu().tolist()
        v = [x for x in v if x[1] > 0]
        if len(v) < 3:
            return None
        t_end = v[0][1] + 0.9 * dur_s * 1e8
        f = [(v[i + 1][0] - v[i][0]) / (v[i + 1][1] - v[i][1]) * 100.0 for i in range(len(v) - 1)
             if v[i + 1][1] <= t_end and v[i + 1][1] > v[i][1]]
        return round(statistics.median(f), 1) if f else None

    with torch.no_grad():
        est = {}
        for name, fn in (("A", compute), ("B", overlap), ("C", serial)):  # warm-up outside the phases
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            est[name] = time.perf_counter() - t0
        torch.cuda.synchronize()
        # the idle clock: the probe alone
        buf = torch.zeros(2 * 200, dtype=torch.int64, device=dev)
        C.hip.clock_probe(buf.data_ptr(), 200, interval, probe_stream.cuda_stream)
        torch.cuda.synchronize()
        out["idle_clock_mhz"] = clock_mhz(buf, 200 * interval / 1e8)
        for name, fn in (("A", compute), ("B", overlap), ("C", serial)):
            time.sleep(0.02)
            n = int(est[name] * a.reps * 1.2 * 1e8 / interval) + 4
            buf = torch.zeros(2 * n, dtype=torch.int64, device=dev)
            C.hip.clock_probe(buf.data_ptr(), n, interval, probe_stream.cuda_stream)
            t0 = time.perf_counter()
            for _ in range(a.reps):
                fn()
            torch.cuda.current_stream(dev).synchronize()  # the phase (its comm joined in), not the probe
            dur = time.perf_counter() - t0
            probe_stream.synchronize()
            out[f"{name}_wall_ms_per_step"] = round(dur / a.reps * 1e3, 3)
            out[f"{name}_clock_mhz"] = clock_mhz(buf, dur)
    comm.check()
    print(json.dumps(out), flush=True)


def analyze(prefix: str, reps: int) -> dict:
    paths = glob.glob(prefix + "_kernel_trace.csv") or glob.glob(os.path.join(prefix, "**", "*kernel_trace.csv"),
                                                                    recursive=True)
    rows = list(csv.DictReader(open(paths[0])))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    # phases: the last three runs of kernels separated by >= 10 ms of idle
    segs, cur, last_end = [], [], None
    for s, e, n in ks:
        if last_end is not None and s - last_end > 10_000_000:
            segs.append(cur)
            cur = []
        cur.append((s, e, n))
        last_end = e if last_end is None else max(last_end, e)
    segs.append(cur)
    phases = dict(zip("ABC", segs[-3:]))

    def is_comm(n):
        return "mxar" in n and ("twoshot" in n or "oneshot" in n or "ring" in n or "threshold" in n or "ll_" in n)

    def is_gemm(n):
        low = n.lower()
        return "gemm" in low or "cijk" in low or "matmul" in low or "mfma" in low

    res = {}
    for name, ev in phases.items():
        gem = [(s, e) for s, e, n in ev if is_gemm(n)]
        com = [(s, e) for s, e, n in ev if is_comm(n)]
        span = (max(e for _, e, _ in ev) - min(s for s, _, _ in ev)) / 1e6
        overl = 0
        for cs, ce in com:  # comm time that ran while some GEMM ran
            for gs, ge in gem:
                lo, hi = max(cs, gs), min(ce, ge)
                if hi > lo:
                    overl += hi - lo
        res[name] = {"kernels": len(ev), "span_ms_per_step": round(span / reps, 3),
                     "gemm_ms_per_step": round(sum(e - s for s, e in gem) / 1e6 / reps, 3),
                     "gemm_median_us": round(statistics.median([(e - s) / 1e3 for s, e in gem]), 1) if gem else None,
                     "gemm_n": len(gem),
                     "comm_ms_per_step": round(sum(e - s for s, e in com) / 1e6 / reps, 3),
                     "comm_median_us": round(statistics.median([(e - s) / 1e3 for s, e in com]), 1) if com else None,
                     "comm_n": len(com),
                     "comm_overlapping_gemm_ms_per_step": round(overl / 1e6 / reps, 3),
                     "other_kernels": sorted({n.split("(")[0][:60] for _, _, n in ev if not is_gemm(n) and not is_comm(n)})[:8]}
    return res


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--tokens", type=int, default=1024)
    ap.add_argument("--bucket-mib", type=int, default=256)
    ap.add_argument("--grid", type=int, default=256, help="workgroups per bucket launch (both logical ranks)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--analyze", default=None, help="kernel-trace prefix (or directory) to analyse instead of running")
    a = ap.parse_args()
    if a.analyze:
        print(json.dumps(analyze(a.analyze, a.reps), indent=1))
    else:
        run(a)


if __name__ == "__main__":
    main()
