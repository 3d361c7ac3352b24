#!/usr/bin/env python3
"""GPU probe of the protocol engine in one process: P plane workers on one GPU, fixed
synthetic inputs, sizes from small to the bench's 256 MiB; prints one JSON row per size
(round time at the master's barrier, validation) as it goes.

    python tools/plane_probe.py --P 2 --sizes 1M 16M 64M 256M --rounds 8
"""
from __future__ import annotations

import argparse
import resource
import json
import os
import sys
import time


import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.engine import PlaneJob  # noqa: E402
from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402


def parse_size(s: str) -> int:
    m = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(float(s[:-1]) * m[s[-1].upper()]) if s[-1].upper() in m else int(s)


def phase_summary(per_worker) -> list[dict]:
    """Threshold-kernel stamps (xgmi_threshold.hip layout) of one round per worker, in us
    from the earliest workgroup start of ANY worker: when each worker's kernel started, got
    through the snapshot / lag gate, finished scatter / reduce / gather, and how long its
    workgroups waited."""
    used = [st[st[:, 0] > 0] for st in per_worker]
    t0 = min(int(u[:, 0].min()) for u in used if len(u))

    def us(v):
        return round(float(v) / 100.0, 1)

    out = []
    for k, u in enumerate(used):
        if not len(u):
            out.append({"worker": k})
            continue
        med = lambda col: int(u[:, col].median().item())  # noqa: E731 - int64: ticks exceed float32
        out.append({"worker": k, "wgs": int(u.shape[0]), "start_first": us(int(u[:, 0].min()) - t0),
                    "start_last": us(int(u[:, 0].max()) - t0), "gate_p50": us(med(1) - t0),
                    "scatter_p50": us(med(6) - t0), "reduce_wait_mean": us(float(u[:, 2].float().mean())),
                    "reduce_p50": us(med(3) - t0), "gather_wait_mean": us(float(u[:, 4].float().mean())),
                    "end_p50": us(med(5) - t0), "end_max": us(int(u[:, 5].max()) - t0)})
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=2)
    ap.add_argument("--sizes", nargs="+", default=["1M", "16M", "64M", "256M"])
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--units", type=int, default=256, help="reduce units (chunks) per block")
    ap.add_argument("--timeout", type=float, default=10.0)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--trace", default=None, help="write a Chrome trace of the last size here")
    ap.add_argument("--priority", choices=["high", "normal"], default="high", help="plane stream priority")
    ap.add_argument("--spin-us", type=int, default=1000, help="completion-thread polling before blocking")
    ap.add_argument("--no-order-release", action="store_true",
                    help="release round outputs without waiting for the default stream (A/B knob)")
    ap.add_argument("--python-io", action="store_true",
                    help="Python dataSource / dataSink callables (default: tensor sources + native keep-last sink)")
    ap.add_argument("--stamps", action="store_true",
                    help="phase stamps of every worker's LAST round kernel (same GPU clock for all workers)")
    a = ap.parse_args()
    from akka_allreduce_1_amd._native import C
    if a.trace:
        C.trace.enable(True)
    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    es = 2 if dtype == torch.bfloat16 else 4
    for sz in a.sizes:
        S = parse_size(sz)
        n = S // es
        xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=k) for k in range(a.P)]
        ref = sum(x.float() for x in xs).to(dtype)
        chunk = max(1024, -(-(-(-n // a.P)) // a.units))
        last = {}

        def on_output(k, out, rounds=a.rounds):
            if out.iteration == rounds - 1:
                last[k] = out.data.clone()

        if a.python_io:  # Python dataSource / dataSink every round (GIL on the round path)
            io = dict(sources=[(lambda req, x=x: x) for x in xs], keep_outputs=False, on_output=on_output)
        else:  # native: the tensors as sources, a native keep-last sink
            io = dict(sources=xs, keep_outputs=False, keep_last=True)
        job = PlaneJob(a.P, n, max_chunk_size=chunk, dtype=dtype, max_round=a.rounds - 1, timeout_s=a.timeout,
                       high_priority=a.priority == "high", order_release=not a.no_order_release, spin_us=a.spin_us,
                       **io)
        row = {"P": a.P, "bytes": S, "chunk": chunk, "priority": a.priority, "order_release": not a.no_order_release, "spin_us": a.spin_us,
               "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "io": "python" if a.python_io else "native"}
        bufs = []
        if a.stamps:
            bufs = [torch.zeros(job.grid * 8, dtype=torch.int64, device=dev) for _ in job.planes]
            for p, b in zip(job.planes, bufs):
                p.set_phase_stamps(b.data_ptr(), job.grid)
        t0 = time.perf_counter()
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        try:
            job.run(timeout=max(60.0, 4 * a.timeout))
            ru1 = resource.getrusage(resource.RUSAGE_SELF)
            st = job.state()
            row["wall_s"] = round(time.perf_counter() - t0, 3)
            # host CPU the job's threads burned (dispatchers, completion pollers, master), per
            # round: what the busy-polls cost
            cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
            row["cpu_us_per_round"] = round(cpu / a.rounds * 1e6, 1)
            row["cpu_cores_busy"] = round(cpu / max(1e-9, time.perf_counter() - t0), 2)
            s = job.stamps
            if len(s) > 2:
                per = (s[-1] - s[1]) / (len(s) - 2)
                row["ms_per_round"] = round(per * 1e3, 4)
                row["algbw_GBps"] = round(S / per / 1e9, 2)
            row["errors"] = [w["stats"]["plane_errors"] for w in st["workers"]]
            if not a.python_io:
                for k in range(a.P):
                    o = job.last_output(k)
                    if o is not None and o.iteration == a.rounds - 1:
                        last[k] = o.data.clone()
            row["validated"] = all(torch.equal(last.get(k, torch.empty(0)), ref) for k in range(a.P))
            row["lat_p50_ms"] = [round(w["round_latency"]["p50_ms"], 3) for w in st["workers"]]
            if bufs:
                row["phases_last_round"] = phase_summary([b.view(-1, 8).cpu() for b in bufs])
        except Exception as e:  # noqa: BLE001
            row["error"] = repr(e)[:400]
        finally:
            job.shutdown()
        print(json.dumps(row), flush=True)
        if a.trace:
            with open(a.trace, "w") as f:
                f.write(C.trace.dump_json())
            C.trace.clear()
        del xs, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
