"""The copy-engine (SDMA) allreduce across the bench's GPUs, run in CHILD processes (bench.py,
N > 1): SDMA copies into another GPU's memory have not run on a multi-GPU node before, and a
fault there would take the process down - so the bench runs them here first, in a job of its
own (one child per bench rank, a gloo group on a port of its own), and only when every child
validated does it let its own DP tuner use the candidate (parallel/sdma.py
mark_xdev_validated). Reference: SURVEY §2.4 K2 - the scatter copies of
AllreduceWorker.scala:200-206 as engine transfers.

Child (one per rank; env SDMA_RANK, SDMA_WORLD, SDMA_PORT, SDMA_DEVICE, SDMA_MIB): validates a
small and the full-size allreduce against the exact fp32-ordered sum, then times p50 of the
full size; prints ONE JSON line.
Parent helper: run_children(rank, world, device, port, mib, timeout) -> this rank's row.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child() -> None:
    import datetime

    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    from akka_allreduce_1_amd.ops import fill_uniform
    from akka_allreduce_1_amd.parallel.sdma import SdmaCommunicator
    from akka_allreduce_1_amd.utils.timing import percentile

    rank, world = int(os.environ["SDMA_RANK"]), int(os.environ["SDMA_WORLD"])
    dev = torch.device("cuda", int(os.environ["SDMA_DEVICE"]))
    mib = int(os.environ.get("SDMA_MIB", "256"))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{os.environ['SDMA_PORT']}", rank=rank,
                            world_size=world, timeout=datetime.timedelta(seconds=60))
    row: dict = {"rank": rank, "world": world}

    def note(msg: str) -> None:
        print(f"[sdma_xdev rank {rank}] {msg}", file=sys.stderr, flush=True)

    try:
        nbytes = mib << 20
        note("constructing + small validation")
        comm = SdmaCommunicator(device=dev, slot_bytes=-(-nbytes // world) + (1 << 20), grid=256, timeout_s=20.0)
        row["cross_gpu"] = comm.cross_gpu
        note("full-size allreduce")
        n = nbytes // 2
        xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=900 + k) for k in range(world)]
        ref = torch.zeros(n, device=dev)
        for x in xs:
            ref += x.float()
        y = comm.allreduce(xs[rank])
        torch.cuda.synchronize(dev)
        comm.check()
        err = (y.float() - ref).abs().max().item()
        del ref
        ok = err <= 2e-2 * world
        flags: list = [None] * world
        dist.all_gather_object(flags, ok)
        row.update(max_abs_err=err, validated=all(flags))
        if row["validated"]:
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
            for _ in range(3):
                comm.allreduce(xs[rank], y)
            torch.cuda.synchronize(dev)
            dist.barrier()
            for a, b in evs:
                a.record()
                comm.allreduce(xs[rank], y)
                b.record()
            torch.cuda.synchronize(dev)
            comm.check()
            p50 = percentile([a.elapsed_time(b) for a, b in evs], 50)
            row.update(p50_ms=round(p50, 4), algbw_GBps=round(nbytes / (p50 / 1e3) / 1e9, 2))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        row["error"] = repr(e)[:300]
        row["validated"] = False
    print(json.dumps(row), flush=True)
    try:
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass


def run_children(rank: int, world: int, device: int, port: int, mib: int = 256, timeout: float = 120.0) -> dict:
    """Start this rank's child (every bench rank calls it at the same point) and return its row;
    a child that crashed or timed out is reported, never raised."""
    env = dict(os.environ, SDMA_RANK=str(rank), SDMA_WORLD=str(world), SDMA_PORT=str(port), SDMA_DEVICE=str(device),
               SDMA_MIB=str(mib), MXAR_SDMA_XDEV="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    # a job of its own: none of torchrun's rendezvous variables (with TORCHELASTIC_USE_AGENT_STORE
    # the child's init would look for the parent job's store)
    for k in list(env):
        if k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK",
                 "ROLE_NAME", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT") or k.startswith("TORCHELASTIC_"):
            env.pop(k)
    t0 = time.perf_counter()
    try:
        p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "child"], env=env, capture_output=True,
                           text=True, timeout=timeout, cwd=ROOT)
    except subprocess.TimeoutExpired as e:
        err = e.stderr or b""
        err = err.decode(errors="replace") if isinstance(err, bytes) else err
        head = next((ln for ln in err.splitlines() if "Error" in ln or "error" in ln), err[:300])
        return {"rank": rank, "validated": False, "error": f"child timed out after {timeout:g} s: {head[:300]}"}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"rank": rank, "validated": False,
                "error": f"child rc={p.returncode}: {(p.stderr or p.stdout)[-300:]}"}
    row = json.loads(lines[-1])
    row["child_s"] = round(time.perf_counter() - t0, 1)
    return row


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "child":
    child()
