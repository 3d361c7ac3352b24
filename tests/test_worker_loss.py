"""A worker that dies mid-job. With `reinitOnLoss` the master re-initialises
the survivors as a new membership epoch that resumes at the current round, and the barrier
counts live workers. The reference would instead wait forever at thAllreduce = 1 (Q4),
because it only re-initialises on MemberUp. Message-level workers (host) and round-engine
workers (loopback plane) are covered here. tests/test_plane_gpu.py covers the xGMI plane.
"""
import threading
import time

import numpy as np
import pytest

from akka_allreduce_1_amd._native import C
from akka_allreduce_1_amd.engine import host_iota_source
from akka_allreduce_1_amd.protocol import AllReduceInput, MemberUp, PoisonPill

F = np.float32


def expected(n, it, ranks):
    i = np.arange(n, dtype=np.float64)
    return sum(i + it + 1000.0 * k for k in ranks)


@pytest.mark.parametrize("kind", ["host", "loopback"])
def test_survivors_are_reinitialised_and_finish(kind):
    P, n, chunk, rounds, victim = 3, 24, 4, 30, 2
    system = C.ActorSystem("Loss", False)
    fin = threading.Event()
    outs = [dict() for _ in range(P)]
    lock = threading.Lock()
    started = threading.Event()

    def src(k):
        base = host_iota_source(n, 1000.0 * k)

        def f(req):
            time.sleep(0.01)  # rounds slow enough to lose the victim mid-job
            if req.iteration >= 5:
                started.set()
            v = base(req)
            return AllReduceInput(v) if kind == "host" else v
        return f

    def sink(k):
        def f(out):
            with lock:
                outs[k][out.iteration] = (np.asarray(out.data).copy(), list(out.count))
        return f

    master = system.master(P, 1.0, 1.0, 1.0, 1, n, rounds - 1, chunk, on_finished=lambda r: fin.set(),
                           reinitOnLoss=True)
    ws, planes = [], []
    for k in range(P):
        if kind == "host":
            ws.append(system.worker(src(k), sink(k), f"w{k}"))
            master.tell(MemberUp(ws[k], "worker", ""), None)
        else:
            planes.append(C.loopback_plane("loss-hub"))
            ws.append(system.plane_worker(src(k), sink(k), planes[k], f"w{k}"))
            master.tell(MemberUp(ws[k], "worker", "", planes[k].descriptor), None)
    try:
        assert started.wait(20)
        ws[victim].tell(PoisonPill(), None)  # the victim stops; the master's DeathWatch fires
        assert fin.wait(30), system.master_state(master)
        st = system.master_state(master)
        assert st["loss_reinits"] == 1 and st["numWorkers"] == 2, st
        # the survivors finished every round; after the re-init their sums hold exactly the two of them
        for k in (0, 1):
            assert max(outs[k]) == rounds - 1
            data, counts = outs[k][rounds - 1]
            np.testing.assert_array_equal(data, expected(n, rounds - 1, (0, 1)).astype(F))
            assert all(c == 2 for c in counts), counts
    finally:
        system.shutdown()


@pytest.mark.parametrize("kind", ["host", "loopback"])
def test_lost_worker_replaced_mid_job(kind):
    """Elastic membership: worker 2 dies (the survivors are re-initialised, reinitOnLoss), then
    a replacement joins (resumeOnJoin). Everyone is re-initialised at the CURRENT round, not
    restarted at round 0 as in the reference (Q2), and the job finishes with three workers."""
    P, n, chunk, rounds = 3, 24, 4, 60
    system = C.ActorSystem("Elastic", False)
    fin = threading.Event()
    outs = [dict() for _ in range(P + 1)]
    lock = threading.Lock()
    progressed = {"r": -1}

    def src(k):
        base = host_iota_source(n, 1000.0 * min(k, 2))  # the replacement contributes as worker 2 did

        def f(req):
            time.sleep(0.01)
            progressed["r"] = max(progressed["r"], req.iteration)
            v = base(req)
            return AllReduceInput(v) if kind == "host" else v
        return f

    def sink(k):
        def f(out):
            with lock:
                outs[k][out.iteration] = (np.asarray(out.data).copy(), list(out.count))
        return f

    master = system.master(P, 1.0, 1.0, 1.0, 1, n, rounds - 1, chunk, on_finished=lambda r: fin.set(),
                           reinitOnLoss=True, resumeOnJoin=True)
    planes = []

    def join(k):
        if kind == "host":
            w = system.worker(src(k), sink(k), f"w{k}")
            master.tell(MemberUp(w, "worker", ""), None)
        else:
            planes.append(C.loopback_plane("elastic-hub"))
            w = system.plane_worker(src(k), sink(k), planes[-1], f"w{k}")
            master.tell(MemberUp(w, "worker", "", planes[-1].descriptor), None)
        return w

    try:
        ws = [join(k) for k in range(P)]
        t0 = time.time()
        while progressed["r"] < 5 and time.time() - t0 < 20:
            time.sleep(0.01)
        ws[2].tell(PoisonPill(), None)
        while system.master_state(master)["loss_reinits"] < 1 and time.time() - t0 < 20:
            time.sleep(0.01)
        resumed_at = progressed["r"]
        join(3)  # the replacement
        assert fin.wait(30), system.master_state(master)
        st = system.master_state(master)
        assert st["loss_reinits"] == 1 and st["join_reinits"] == 1 and st["numWorkers"] == 3, st
        assert st["inits"] == 3, st  # start, loss, join - never a restart from round 0
        last, counts = outs[0][rounds - 1]
        np.testing.assert_array_equal(last, expected(n, rounds - 1, (0, 1, 2)).astype(F))
        assert all(c == 3 for c in counts), counts
        assert min(outs[3]) >= resumed_at  # the replacement started at the current round
    finally:
        system.shutdown()
