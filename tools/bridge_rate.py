#!/usr/bin/env python3
"""Round rate of the round engine when the master drives the rounds vs when a control-bridge
client drives them (docs/BRIDGE.md): what an external driver (e.g. a JVM Akka actor) costs per
round. Two plane workers, thresholds 1, tensor sources, native keep-last sinks.

usage: python tools/bridge_rate.py [--plane xgmi|loopback] [--rounds 200] [--mib 1 64 256]
One JSON line per (size, mode) on stdout."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_1_amd.bridge import BridgeClient  # noqa: E402
from akka_allreduce_1_amd.engine import PlaneJob  # noqa: E402


def run(plane, n, rounds, warm, external, chunk, pipeline=False):
    P = 2
    if plane == "xgmi":
        dev = torch.device("cuda", 0)
        sources = [torch.full((n,), float(k + 1), dtype=torch.bfloat16, device=dev) for k in range(P)]
        kw = dict(dtype=torch.bfloat16, sources=sources, keep_last=True)
    else:
        kw = dict(plane="loopback", keep_outputs=False)
    job = PlaneJob(P, n, max_chunk_size=chunk, max_round=rounds - 1, timeout_s=30.0,
                   bridge_port=0 if external else None, external_rounds=external, **kw)
    try:
        if not external:
            job.run(timeout=300)
            st = job.stamps
        else:
            job.start()
            st = []
            with BridgeClient("127.0.0.1", job.bridge_port, timeout=60) as b:
                b.wait_for("InitWorkers")
                if pipeline:  # the next start is queued while the round runs (BridgeClient.drive)
                    b.start(0)
                    for r in range(rounds):
                        if r + 1 < rounds:
                            b.start(r + 1)
                        b.wait_for("RoundComplete", round=r)
                        st.append(time.perf_counter())
                else:  # lock-step: start, wait for the barrier, start the next
                    for r in range(rounds):
                        b.send({"type": "StartAllreduce", "round": r})
                        b.wait_for("RoundComplete", round=r)
                        st.append(time.perf_counter())
            assert job.finished.wait(30)
            for p in job.planes:
                p.drain()
        st = st[warm:]
        ms = 1e3 * (st[-1] - st[0]) / (len(st) - 1)
        return ms
    finally:
        job.shutdown()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plane", default="xgmi")
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mib", type=float, nargs="+", default=[1, 64, 256])
    a = ap.parse_args()
    for mib in a.mib:
        n = int(mib * 2 ** 20) // (2 if a.plane == "xgmi" else 4)
        chunk = max(1, -(-n // 2) // 128)  # 128 chunks per block (the bench's geometry)
        for mode in ("master", "bridge lock-step", "bridge pipelined") * 2:
            ms = run(a.plane, n, a.rounds, a.warmup, mode != "master", chunk, pipeline=mode == "bridge pipelined")
            print(json.dumps({"plane": a.plane, "MiB_per_worker": mib, "driver": mode,
                              "rounds": a.rounds, "ms_per_round": round(ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
