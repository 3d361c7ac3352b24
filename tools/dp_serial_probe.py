"""Why does the DP rehearsal's SERIAL schedule report a slower backward (verdict r4 #3)?

dp.overlap_rehearsal `serial_grid512` (Llama-3-8B, every bucket allreduced after backward)
reported backward 27.2 ms vs 19.5 ms alone - a schedule with nothing beside the backward.
Candidates: (a) the previous step's comm leaks into the next backward, (b) the reducer's hooks
cost host time the GPU waits for, (c) the GPU runs the backward at a lower clock after the
previous step's ~27 ms of full-bandwidth comm (power management), not because of any overlap.

Cases, each timed by events around the backward only (ms, medians of `--steps`), with the
shader clock sampled by a one-wave probe on a side stream during the backward (MHz):
  alone            backward without hooks (the rehearsal's `compute`)
  hooks            backward with the reducer's hooks, serial schedule, NO comm afterwards
  serial           backward + hooks, then every bucket allreduced (the rehearsal's serial step)
  serial_idle      as serial, with --idle-ms of host sleep (GPU idle) before each step
  after_comm       backward without hooks right after a comm-only burst of every bucket

    python tools/dp_serial_probe.py --model llama3_8b --steps 5
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd._native import C  # noqa: E402
from akka_allreduce_1_amd.models.grad_sets import gradient_shapes  # noqa: E402
from akka_allreduce_1_amd.parallel import BucketedGradReducer  # noqa: E402
from benchmarks.bench_dp import SyntheticBackward  # noqa: E402
from benchmarks.sections import PairRehearsalComm, _Placeholder  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--grid", type=int, default=512)
    ap.add_argument("--idle-ms", type=float, default=100.0)
    ap.add_argument("--tokens", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    shapes = gradient_shapes(a.model)
    params = [torch.nn.Parameter(torch.zeros(sh, dtype=torch.bfloat16, device=dev)) for _, sh in shapes]
    big = a.model == "llama3_8b"
    kw = dict(bucket_bytes=1 << 30, first_bucket_bytes=64 << 20) if big else dict(bucket_bytes=25 << 20)
    reducer = BucketedGradReducer(params, _Placeholder(), op="avg", **kw)
    reducer.remove_hooks()
    comm = PairRehearsalComm(reducer.buckets, a.grid)
    reducer.comm = comm
    reducer._raw_ok = True
    reducer.overlap = False
    bwd = SyntheticBackward(params, a.tokens, torch.bfloat16, dev)
    grads = [q.grad for q in params]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    side = torch.cuda.Stream(device=dev, priority=0)
    samples = 400
    clk = torch.zeros(2 * samples, dtype=torch.int64, device=dev)

    def probe_start():  # one wave on a side stream, a sample every 0.25 ms for 100 ms
        with torch.cuda.stream(side):
            clk.zero_()
        C.hip.clock_probe(clk.data_ptr(), samples, 25_000, side.cuda_stream)

    def clock_mhz(t0_ms: float, t1_ms: float) -> float | None:
        torch.cuda.synchronize(dev)
        v = clk.view(samples, 2).cpu()
        ct, rt = v[:, 0].double(), v[:, 1].double()
        ok = rt > 0
        if ok.sum() < 3:
            return None
        ct, rt = ct[ok], rt[ok]
        # samples inside the backward window (realtime ticks of 10 ns relative to the first)
        dt = (rt - rt[0]) / 1e5  # ms
        sel = (dt >= t0_ms) & (dt <= t1_ms)
        if sel.sum() < 3:
            sel = torch.ones_like(dt, dtype=torch.bool)
        c, r = ct[sel], rt[sel]
        return round(float((c[-1] - c[0]) / (r[-1] - r[0]) * 100.0), 1)  # s_memtime ticks per us

    def backward(hooks: bool):
        ev[0].record()
        bwd.run(reducer if hooks else None)
        ev[1].record()

    def step(kind: str):
        if kind == "serial_idle":
            torch.cuda.synchronize(dev)
            time.sleep(a.idle_ms / 1e3)
        if kind == "after_comm":
            for b in reducer.buckets:
                comm.allreduce_(b.buffer, op="avg", stream=reducer._comm_raw)
            torch.cuda.current_stream(dev).wait_stream(reducer.stream)
        probe_start()
        backward(kind in ("hooks", "serial", "serial_idle"))
        if kind in ("serial", "serial_idle"):
            reducer.wait()
        elif kind == "hooks":
            for b in reducer.buckets:  # reset the reducer's per-step state without comm
                b.pending = len(b.params)
                b.ready = b.launched = False
            reducer._next = 0
        torch._foreach_add_(params, grads, alpha=-1e-3)

    kinds = ["alone", "hooks", "serial", "serial_idle", "after_comm"]
    res = {k: {"bwd_ms": [], "clock_MHz": []} for k in kinds}
    with torch.no_grad():
        for k in kinds:
            step(k)
        torch.cuda.synchronize(dev)
        for _ in range(a.steps):
            for k in kinds:  # interleaved
                torch.cuda.synchronize(dev)
                step(k)
                torch.cuda.synchronize(dev)
                ms = ev[0].elapsed_time(ev[1])
                res[k]["bwd_ms"].append(ms)
                res[k]["clock_MHz"].append(clock_mhz(0.0, ms))
    comm.check()
    out = {"model": a.model, "tokens": a.tokens, "grid": a.grid, "idle_ms": a.idle_ms}
    base = statistics.median(res["alone"]["bwd_ms"])
    for k in kinds:
        m = statistics.median(res[k]["bwd_ms"])
        clocks = [c for c in res[k]["clock_MHz"] if c]
        out[k] = {"bwd_ms": round(m, 3), "vs_alone": round(m / base, 3),
                  "clock_MHz": round(statistics.median(clocks), 1) if clocks else None,
                  "all_ms": [round(x, 2) for x in res[k]["bwd_ms"]]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
