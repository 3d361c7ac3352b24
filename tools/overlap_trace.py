#!/usr/bin/env python3
"""Why the one-GPU DP overlap rehearsal loses to the serial schedule (bench dp.overlap_rehearsal):
a kernel-level look, run under rocprofv3 --kernel-trace (and `--contention`: the memory-system
counters of one GEMM beside the comm, for PMC passes). The comm is one rank of an 8-GPU
two-shot (benchmarks/sections.py SoloRehearsalComm: a real rank's per-GPU HBM bytes).

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
    from benchmarks.sections import SoloRehearsalComm, _Placeholder

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    shapes = llama3_8b_shapes(a.layers) if a.model == "llama3_8b" else gradient_shapes(a.model)
    params = [torch.nn.Parameter(torch.zeros(sh, dtype=torch.bfloat16, device=dev)) for _, sh in shapes]
    reducer = BucketedGradReducer(params, _Placeholder(8), op="avg", bucket_bytes=a.bucket_mib << 20)
    reducer.remove_hooks()
    comm = SoloRehearsalComm(reducer.buckets, 8, max(a.grid, 8))  # one rank of an 8-GPU two-shot
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


def contention(a) -> None:
    """The memory-system side of the overlap loss, for a PMC pass: the weight-gradient GEMM of
    a Llama-3-8B MLP projection (dW[4096 x 14336] = X^T dY, K = `--tokens`) alone (phase A),
    then beside a continuous one-rank 8-GPU two-shot of 1 GiB buckets on a side stream at the
    full grid (phase B) and at a paced grid of 32 (phase C). Phases are separated by a sleep
    kernel (the `spin_kernel` marker `--analyze-pmc` splits on). The TCC counters are
    device-wide: during a GEMM of phase B they count the comm's traffic too.

        tools/gpu.sh pmc "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" python tools/overlap_trace.py --contention
        python tools/overlap_trace.py --analyze-pmc gpurun_out/pmc_GRBM_GUI_ACTIVE/run_counter_collection.csv
    """
    import torch

    from benchmarks.sections import SoloRehearsalComm

    class _B:
        def __init__(self, t):
            self.buffer, self.nbytes = t, t.numel() * t.element_size()

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    x = torch.randn(a.tokens, 4096, dtype=torch.bfloat16, device=dev)
    dy = torch.randn(a.tokens, 14336, dtype=torch.bfloat16, device=dev)
    dw = torch.empty(4096, 14336, dtype=torch.bfloat16, device=dev)
    bucket = torch.zeros((1 << 30) // 2, dtype=torch.bfloat16, device=dev)
    comm = SoloRehearsalComm([_B(bucket)], 8, 512)
    side = torch.cuda.Stream(device=dev, priority=-1)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    out: dict = {"tokens": a.tokens, "gemm": "dW[4096 x 14336] = X^T dY (bf16)"}

    def gemms(n: int) -> float:
        ev[0].record()
        for _ in range(n):
            torch.matmul(x.t(), dy, out=dw)
        ev[1].record()
        torch.cuda.synchronize(dev)
        return ev[0].elapsed_time(ev[1]) / n

    gemms(5)
    for phase, grid in (("A", 0), ("B", 512), ("C", 32)):
        torch.cuda._sleep(2_000_000)  # the phase marker (spin_kernel)
        torch.cuda.synchronize(dev)
        if grid:
            for c in comm.comms:
                c.grid = grid
            with torch.cuda.stream(side):  # enough comm to cover the GEMMs
                for _ in range(a.comm_calls if grid == 512 else max(2, a.comm_calls // 3)):
                    comm.allreduce_(bucket, op="avg", stream=side.cuda_stream)
        out[f"{phase}_gemm_ms"] = round(gemms(a.gemms), 4)
        torch.cuda.synchronize(dev)
    comm.check()
    print(json.dumps(out), flush=True)


def analyze_pmc(path: str) -> dict:
    """Per phase (split on spin_kernel dispatches): medians of the GEMM dispatches' counters."""
    rows: dict = {}
    for r in csv.DictReader(open(path)):
        d = rows.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"],
                                                     "us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    phase, per = -1, {}
    for i in sorted(rows):
        n = rows[i]["name"]
        if "spin_kernel" in n:
            phase += 1
            continue
        low = n.lower()
        if phase >= 0 and ("gemm" in low or "cijk" in low):
            per.setdefault("ABC"[min(phase, 2)], []).append(rows[i])
    res = {}
    for ph, ds in per.items():
        cs = [k for k in ds[0] if k not in ("name",)]
        med = {k: statistics.median(d[k] for d in ds if k in d) for k in cs}
        cell = {"gemms": len(ds), "us": round(med["us"], 1)}
        cyc = med.get("GRBM_GUI_ACTIVE")
        for k, v in med.items():
            if k != "us":
                cell[k] = v
        if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in med:  # per SIMD-cycle: 1024 SIMDs x GUI cycles / 8 XCDs
            cell["mfma_busy_frac"] = round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc / 8), 4)
        if "TCC_HIT_sum" in med and "TCC_MISS_sum" in med:
            cell["l2_hit"] = round(med["TCC_HIT_sum"] / max(1.0, med["TCC_HIT_sum"] + med["TCC_MISS_sum"]), 4)
        if "TCC_EA0_RDREQ_sum" in med and "TCC_EA0_WRREQ_sum" in med:  # 64-B requests (device-wide)
            cell["hbm_TBps_device"] = round((med["TCC_EA0_RDREQ_sum"] + med["TCC_EA0_WRREQ_sum"]) * 64 /
                                            (med["us"] * 1e-6) / 1e12, 3)
        if "TCP_TCC_READ_REQ_LATENCY_sum" in med and med.get("TCP_TCC_READ_REQ_sum"):
            cell["l1_to_l2_read_latency_cycles"] = round(med["TCP_TCC_READ_REQ_LATENCY_sum"] / med["TCP_TCC_READ_REQ_sum"], 1)
        if "TCC_EA0_RDREQ_LEVEL_sum" in med and med.get("TCC_EA0_RDREQ_sum"):
            cell["ea_read_cycles_in_flight"] = round(med["TCC_EA0_RDREQ_LEVEL_sum"] / med["TCC_EA0_RDREQ_sum"], 1)
        res[ph] = cell
    return res


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
    ap.add_argument("--contention", action="store_true", help="the GEMM-beside-comm probe for PMC passes")
    ap.add_argument("--gemms", type=int, default=30)
    ap.add_argument("--comm-calls", type=int, default=24)
    ap.add_argument("--analyze-pmc", default=None, help="a PMC pass's counter_collection.csv of --contention")
    a = ap.parse_args()
    if a.analyze_pmc:
        print(json.dumps(analyze_pmc(a.analyze_pmc)))
    elif a.contention:
        contention(a)
    elif a.analyze:
        print(json.dumps(analyze(a.analyze, a.reps), indent=1))
    else:
        run(a)


if __name__ == "__main__":
    main()
