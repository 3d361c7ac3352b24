"""Cluster layer over real TCP on 127.0.0.1 (csrc/cluster): membership through seed nodes,
MemberUp -> master, the full allreduce protocol between nodes, remote DeathWatch +
auto-down. Mirrors the reference's multi-JVM deployment (README.md:3-7) in one process."""
import threading
import time

import numpy as np

from akka_allreduce_1_amd._native import C
from akka_allreduce_1_amd.parallel.comm import free_port


def _cfg(port, roles, seeds, fast=True):
    c = C.ClusterConfig()
    c.host = "127.0.0.1"
    c.port = port
    c.roles = roles
    c.seed_nodes = seeds
    if fast:
        c.heartbeat_interval_s = 0.1
        c.acceptable_heartbeat_pause_s = 0.5
        c.auto_down_unreachable_after_s = 0.3
    return c


def _wait(pred, timeout=10.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_codec_address_helpers():
    assert C.normalize_address("akka.tcp://ClusterSystem@127.0.0.1:2551") == "mxar.tcp://ClusterSystem@127.0.0.1:2551"
    assert C.make_address("S", "h", 7) == "mxar.tcp://S@h:7"


def test_membership_and_allreduce_over_tcp():
    P, N, C_, rounds = 2, 10, 2, 4
    mport = free_port()
    seed = f"akka.tcp://ClusterSystem@127.0.0.1:{mport}"  # reference-style seed URI accepted
    msys = C.ActorSystem("ClusterSystem", False)
    done = threading.Event()
    master = msys.master(P, 1.0, 1.0, 1.0, 1, N, rounds - 1, C_, on_finished=lambda r: done.set())
    mnode = C.ClusterNode.start(msys, _cfg(mport, ["master"], [seed]))
    mnode.subscribe(master)
    outs = {0: [], 1: []}
    wsys, wnodes = [], []
    for k in range(P):
        s = C.ActorSystem("ClusterSystem", False)

        def src(req, k=k):
            return C.AllReduceInput(np.arange(N, dtype=np.float32) + req.iteration + k)

        def sink(o, k=k):
            outs[k].append((o.iteration, np.asarray(o.data).copy()))

        s.worker(src, sink, "worker")
        wsys.append(s)
        wnodes.append(C.ClusterNode.start(s, _cfg(0, ["worker"], [seed])))
    try:
        assert _wait(lambda: len(mnode.members()) == P + 1), mnode.members()
        assert _wait(lambda: all(len(v) >= rounds for v in outs.values()), 20), outs
        assert done.wait(10)
        for k in range(P):
            got = dict(outs[k])
            for r in range(rounds):
                exp = 2 * (np.arange(N) + r) + 1  # (i + r + 0) + (i + r + 1)
                np.testing.assert_array_equal(got[r], exp)
        st = mnode.stats()
        assert st.frames_in > 0 and st.decode_errors == 0
        assert mnode.leader() == min(m["address"] for m in mnode.members())
    finally:
        for n in wnodes:
            n.shutdown()
        mnode.shutdown()
        for s in wsys:
            s.shutdown()
        msys.shutdown()


def test_failure_detection_auto_down_and_deathwatch():
    mport = free_port()
    seed = f"mxar.tcp://ClusterSystem@127.0.0.1:{mport}"
    msys = C.ActorSystem("ClusterSystem", False)
    probe = msys.probe("watcher")
    mnode = C.ClusterNode.start(msys, _cfg(mport, ["master"], [seed]))
    mnode.subscribe(probe)
    wsys = C.ActorSystem("ClusterSystem", False)
    wsys.worker(lambda req: C.AllReduceInput(np.zeros(4, np.float32)), None, "worker")
    wnode = C.ClusterNode.start(wsys, _cfg(0, ["worker"], [seed]))
    try:
        ups = []
        assert _wait(lambda: len(mnode.members()) == 2)
        while True:
            m = probe.receive(2.0)
            assert m is not None, "no MemberUp for the worker"
            if isinstance(m[0], C.MemberUp) and m[0].role == "worker":
                ups.append(m[0])
                break
        worker_ref = ups[0].ref
        assert worker_ref.path.endswith("/user/worker")
        # a master-like watcher: the master actor watches on MemberUp (AllreduceMaster.scala:74)
        master = msys.master(1, 1.0, 1.0, 1.0, 1, 4, 0, 2, name="m2")
        master.tell(ups[0], None)
        # kill the worker node abruptly (no Leave): heartbeats stop -> unreachable -> downed
        wnode.shutdown()
        assert _wait(lambda: len(mnode.members()) == 1, 10), mnode.members()
        assert mnode.stats().members_removed >= 1
    finally:
        wnode.shutdown()
        mnode.shutdown()
        wsys.shutdown()
        msys.shutdown()


def test_graceful_leave():
    mport = free_port()
    seed = f"mxar.tcp://ClusterSystem@127.0.0.1:{mport}"
    msys = C.ActorSystem("ClusterSystem", False)
    mnode = C.ClusterNode.start(msys, _cfg(mport, ["master"], [seed], fast=False))
    wsys = C.ActorSystem("ClusterSystem", False)
    wnode = C.ClusterNode.start(wsys, _cfg(0, ["worker"], [seed], fast=False))
    try:
        assert _wait(lambda: len(mnode.members()) == 2)
        wnode.leave()
        assert _wait(lambda: len(mnode.members()) == 1, 5)
    finally:
        wnode.shutdown()
        mnode.shutdown()
        wsys.shutdown()
        msys.shutdown()
