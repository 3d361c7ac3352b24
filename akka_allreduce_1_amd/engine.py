"""The protocol-driven GPU round engine, in one process.

The reference runs one master actor and N worker actors (AllreduceMaster.scala:15-98,
AllreduceWorker.scala:9-270). `PlaneJob` builds exactly that on the native actor runtime,
with every worker a `PlaneWorkerActor` (csrc/runtime/plane_worker.h) over its own xGMI round
plane (csrc/hip/xgmi_plane.h): StartAllreduce(r) from the master becomes ONE threshold-kernel
launch per worker, the sink gets the GPU output tensor and the real per-chunk counts, and
CompleteAllreduce goes back to the master. Registration carries each worker's plane
descriptor (its HBM arena's IPC handle) in MemberUp.meta; the master relays them to all
workers in InitWorkers.planes.

Multi-process deployments use the CLIs instead (`mxar-master` + `mxar-worker --device k`);
the plane descriptor then travels in the cluster join (ClusterConfig.meta).

    job = PlaneJob(3, 1 << 20, max_chunk_size=1 << 14, th_reduce=1.0, th_complete=1.0, max_round=20)
    job.run()
    out, counts = job.outputs[0][20]   # worker 0, round 20
"""
from __future__ import annotations

import threading
import time
from typing import Callable, Sequence

import torch

from ._native import C
from .ops.kernels import dtype_code


def iota_source(n: int, device: torch.device, dtype: torch.dtype, offset: float = 0.0) -> Callable:
    """The reference's demo dataSource (AllreduceWorker.scala:285-291), data[i] = i + iteration
    (+ offset), produced on the GPU by the fill_iota kernel on torch's current stream."""
    code = dtype_code(dtype)

    def source(req):
        x = torch.empty(n, dtype=dtype, device=device)
        C.hip.fill_iota(x.data_ptr(), n, float(req.iteration) + offset, code, torch.cuda.current_stream(device).cuda_stream)
        return x

    return source


class PlaneJob:
    """Master + P plane workers in one process (threaded actor system)."""

    def __init__(self, P: int, data_size: int, *, max_chunk_size: int, th_allreduce: float = 1.0,
                 th_reduce: float = 1.0, th_complete: float = 1.0, max_lag: int = 1, max_round: int = 10,
                 devices: Sequence[int] | None = None, dtype: torch.dtype = torch.float32, grid: int = 0,
                 sources: Sequence[Callable] | None = None, keep_outputs: bool = True, round_timeout_ms: int = 0,
                 timeout_s: float = 60.0, order_ref: bool = True, on_output: Callable | None = None):
        self.P = P
        self.n = data_size
        self.dtype = dtype
        self.devices = list(devices) if devices is not None else [torch.cuda.current_device()] * P
        if len(self.devices) != P:
            raise ValueError("one device per worker")
        if grid <= 0:  # workers sharing a GPU split its workgroups so every kernel stays resident
            share = max(self.devices.count(d) for d in set(self.devices))
            grid = max(8, 512 // share)
        self.system = C.ActorSystem("ClusterSystem", False)
        self.finished = threading.Event()
        self.rounds = {"n": 0}
        self.outputs: list[dict[int, tuple]] = [dict() for _ in range(P)]
        self.keep = keep_outputs
        self.on_output = on_output
        self.planes = [C.hip.xgmi_plane(d, dtype_code(dtype), data_size, max_peers=max(P, 1), max_lag=max_lag,
                                        grid=grid, timeout_s=timeout_s, order_ref=order_ref) for d in self.devices]
        if sources is None:
            sources = [iota_source(data_size, torch.device("cuda", d), dtype, 1000.0 * k)
                       for k, d in enumerate(self.devices)]
        self.sources = list(sources)

        def fin(r):
            self.rounds["n"] = r
            self.finished.set()

        self.master = self.system.master(P, th_allreduce, th_reduce, th_complete, max_lag, data_size, max_round,
                                         max_chunk_size, on_finished=fin, roundTimeoutMs=round_timeout_ms)
        self.workers = [self.system.plane_worker(self.sources[k], self._sink(k), self.planes[k], f"worker{k}")
                        for k in range(P)]

    def _sink(self, k: int) -> Callable:
        def sink(out):
            if self.keep:
                self.outputs[k][out.iteration] = (out.data, list(out.count))
            if self.on_output is not None:
                self.on_output(k, out)
        return sink

    def start(self) -> None:
        """Register the workers with the master (MemberUp carrying the plane descriptor, in
        worker order: worker k gets id k)."""
        for w, p in zip(self.workers, self.planes):
            self.master.tell(C.MemberUp(w, "worker", "", p.descriptor), None)

    def run(self, timeout: float = 120.0) -> float:
        """start() and wait until the master finished every round; returns the wall time."""
        t0 = time.perf_counter()
        self.start()
        if not self.finished.wait(timeout):
            raise TimeoutError(f"plane job did not finish in {timeout} s: {self.state()}")
        for p in self.planes:  # the last round's sinks run after the master's last barrier
            p.drain()
        self.system.await_idle(10.0)
        return time.perf_counter() - t0

    def state(self) -> dict:
        return {"master": self.system.master_state(self.master),
                "workers": [self.system.plane_worker_state(w) for w in self.workers]}

    def shutdown(self) -> None:
        self.system.shutdown()
        self.planes = []
