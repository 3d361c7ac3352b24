"""Actor API: the reference's master/worker actors on the native actor runtime.

    system = ActorSystem("ClusterSystem")                      # threaded dispatcher
    worker = system.worker(data_source, data_sink, "worker")   # AllreduceWorker(dataSource, dataSink)
    master = system.master(totalWorkers=2, thAllreduce=1.0, thReduce=0.9, thComplete=0.8,
                           maxLag=1, dataSize=10, maxRound=100, maxChunkSize=2)
    master.tell(MemberUp(worker, "worker"))                    # cluster membership event

`data_source(AllReduceInputRequest) -> AllReduceInput | array` and
`data_sink(AllReduceOutput) -> None` have the reference's signatures
(`AllreduceWorker.scala:9-10`). Reference: `AllreduceWorker.scala:9-270`,
`AllreduceMaster.scala:15-98`; the protocol cores are C++ (`csrc/core`).

The round engine's worker (`make_plane_worker`) keeps the same messages but runs each
round's data exchange in a RoundPlane: one threshold-kernel launch over xGMI on a GPU
(`device=k`), or the host loopback plane for workers of one process (`hub=...`).
"""
from __future__ import annotations

from ._native import C

ActorSystem = C.ActorSystem
ActorRef = C.ActorRef
ProbeRef = C.ProbeRef
host_plane = C.host_plane


def make_worker(system, data_source, data_sink=None, name: str = "worker", plane=None):
    """AllreduceWorker actor (`AllreduceWorker.scala:9`), registered as /user/<name>."""
    return system.worker(data_source, data_sink, name, plane)


def make_master(system, total_workers: int, th_allreduce: float, th_reduce: float, th_complete: float,
                max_lag: int, data_size: int, max_round: int, max_chunk_size: int, *,
                live_barrier: bool = False, on_finished=None, name: str = "master"):
    """AllreduceMaster actor (`AllreduceMaster.scala:15-24`), registered as /user/<name>."""
    return system.master(total_workers, th_allreduce, th_reduce, th_complete, max_lag, data_size,
                         max_round, max_chunk_size, live_barrier, on_finished, name)


def make_plane_worker(system, data_source, data_sink=None, *, data_size: int, name: str = "worker",
                      device: int | None = None, hub: str | None = None, dtype=None, max_peers: int = 8,
                      max_lag: int = 4, grid: int = 0, timeout_s: float = 60.0):
    """Round-granular AllreduceWorker (csrc/runtime/plane_worker.h) and its plane.

    device=k: an XgmiRoundPlane on GPU k holding up to `data_size` elements per round
    (dtype: torch.float32 / bfloat16 / float16); hub="name": a LoopbackRoundPlane (host
    memory; every worker of the job in this process names the same hub). Returns
    (worker_ref, plane). Announce `plane.descriptor` when the worker registers -
    `MemberUp(worker_ref, "worker", "", plane.descriptor)` in process, or
    `ClusterConfig.meta` over TCP - so the master can relay it in InitWorkers.planes.
    """
    if (device is None) == (hub is None):
        raise ValueError("give exactly one of device= (xGMI plane) or hub= (loopback plane)")
    if device is not None:
        import torch

        from .ops.kernels import dtype_code

        plane = C.hip.xgmi_plane(device, dtype_code(dtype or torch.float32), data_size, max_peers=max_peers,
                                 max_lag=max_lag, grid=grid, timeout_s=timeout_s)
    else:
        plane = C.loopback_plane(hub)
    return system.plane_worker(data_source, data_sink, plane, name), plane
