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
