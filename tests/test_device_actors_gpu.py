"""The full actor protocol (master + P workers, threaded runtime) with every worker's
DataBuffers and payloads in MI355X HBM: sources hand in torch CUDA tensors (zero-copy
DLPack), sinks receive torch CUDA tensors."""
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu

from akka_allreduce_1_amd._native import C  # noqa: E402
from akka_allreduce_1_amd.protocol import AllReduceInput, MemberUp  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("P,N,chunk", [(2, 10, 2), (4, 1000, 64), (3, 4097, 256)])
def test_actor_cluster_on_device_plane(P, N, chunk):
    rounds = 6
    system = C.ActorSystem("ClusterSystem", False)
    done = threading.Event()
    master = system.master(P, 1.0, 1.0, 1.0, 2, N, rounds - 1, chunk, on_finished=lambda r: done.set())
    outs = {k: {} for k in range(P)}
    planes = [C.hip.device_plane(0) for _ in range(P)]
    lock = threading.Lock()

    def make(k):
        def src(req):
            t = torch.arange(N, device=DEV, dtype=torch.float32) * (k + 1) + req.iteration
            return AllReduceInput(t)

        def sink(o):
            assert isinstance(o.data, torch.Tensor) and o.data.is_cuda
            with lock:
                outs[k][o.iteration] = o.data.clone()

        return src, sink

    workers = []
    for k in range(P):
        src, sink = make(k)
        workers.append(system.worker(src, sink, f"worker{k}", planes[k]))
    for w in workers:
        master.tell(MemberUp(w, "worker", ""), None)
    try:
        assert done.wait(60), "allreduce rounds did not finish"
        assert system.await_idle(10.0)
        base = torch.arange(N, device=DEV, dtype=torch.float32)
        for k in range(P):
            for r in range(rounds):
                exp = base * sum(range(1, P + 1)) + P * r
                assert torch.equal(outs[k][r], exp), (k, r)
        assert all(p.kernels > 0 for p in planes)
    finally:
        system.shutdown()
