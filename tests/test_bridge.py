"""Control bridge (csrc/runtime/control_bridge.h, docs/BRIDGE.md): the reference's control
messages as JSON lines over TCP, so a non-native client (e.g. a JVM Akka actor with a socket)
can watch a job or drive its rounds.

Driving mode mirrors AllreduceMaster.scala:58-67,91-97 from outside: the client sends
StartAllreduce(r), the master forwards it to the workers and reports the barrier.
"""
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from akka_allreduce_1_amd._native import C
from akka_allreduce_1_amd.bridge import BridgeClient, BridgeError
from akka_allreduce_1_amd.engine import host_iota_source
from akka_allreduce_1_amd.protocol import AllReduceInput, MemberUp

F = np.float32


def expected(n, it, P):
    i = np.arange(n, dtype=np.float64)
    return sum(i + it + 1000.0 * k for k in range(P))


def _job(P, n, chunk, rounds, kind="host", external=True, name="Bridge"):
    system = C.ActorSystem(name, False)
    fin = threading.Event()
    outs = [dict() for _ in range(P)]
    lock = threading.Lock()

    def src(k):
        base = host_iota_source(n, 1000.0 * k)

        def f(req):
            v = base(req)
            return AllReduceInput(v) if kind == "host" else v
        return f

    def sink(k):
        def f(out):
            with lock:
                outs[k][out.iteration] = (np.asarray(out.data).copy(), list(out.count))
        return f

    master = system.master(P, 1.0, 1.0, 1.0, 1, n, rounds - 1, chunk, on_finished=lambda r: fin.set(),
                           externalRounds=external, bridgePort=0)
    port = system.master_bridge_port(master)
    assert port > 0
    ws = []
    for k in range(P):
        if kind == "host":
            ws.append(system.worker(src(k), sink(k), f"w{k}"))
            master.tell(MemberUp(ws[k], "worker", ""), None)
        else:
            plane = C.loopback_plane(name + "-hub")
            ws.append(system.plane_worker(src(k), sink(k), plane, f"w{k}"))
            master.tell(MemberUp(ws[k], "worker", "", plane.descriptor), None)
    return system, master, port, outs, fin


@pytest.mark.parametrize("kind", ["host", "loopback"])
def test_client_drives_every_round(kind):
    P, n, chunk, rounds = 2, 40, 6, 12
    system, master, port, outs, fin = _job(P, n, chunk, rounds, kind, name=f"Drive{kind}")
    try:
        with BridgeClient("127.0.0.1", port) as b:
            assert b.hello["protocol"] == "mxar-bridge/1"
            init = b.wait_for("InitWorkers")
            assert init["workers"] == [0, 1] and init["dataSize"] == n and init["maxChunkSize"] == chunk
            assert init["externalRounds"] is True
            # nothing runs until the client starts a round
            time.sleep(0.2)
            assert all(not o for o in outs)
            st = b.status()
            assert st["awaiting"] is True and st["workers"] == P
            done = b.drive(range(rounds))
            assert [d["round"] for d in done] == list(range(rounds))
            assert fin.wait(10)
            b.wait_for("AllreduceFinished", rounds=rounds)
            completes = [e for e in b.events if e["type"] == "CompleteAllreduce" and e["counted"]]
            assert sorted((e["round"], e["srcId"]) for e in completes) == [(r, i) for r in range(rounds) for i in range(P)]
        deadline = time.time() + 5
        while time.time() < deadline and any(len(o) < rounds for o in outs):
            time.sleep(0.01)
        for k in range(P):
            for it in range(rounds):
                data, counts = outs[k][it]
                np.testing.assert_array_equal(data, expected(n, it, P).astype(F))
    finally:
        system.shutdown()


def test_refused_commands_and_malformed_lines():
    P, n, chunk, rounds = 2, 12, 3, 6
    system, master, port, outs, fin = _job(P, n, chunk, rounds, name="Refuse")
    try:
        with BridgeClient("127.0.0.1", port) as b:
            b.wait_for("InitWorkers")
            b.send_raw("not json")
            assert "malformed" in b.wait_for("Error")["reason"]
            b.send_raw('{"type": "StartAllreduce", "round": {"nested": 1}}')
            b.wait_for("Error")
            b.send_raw('{"type":"StartAllreduce","round":-3}')
            assert "non-negative" in b.wait_for("Error")["reason"]
            b.send({"type": "Reboot"})
            assert b.wait_for("Error")["reason"] == "unknown command"
            with pytest.raises(BridgeError, match="maxRound"):
                b.start(rounds + 5)
            b.start(2)  # skipping ahead is allowed (the client owns the round numbering)
            b.wait_for("RoundComplete", round=2)
            with pytest.raises(BridgeError, match="not after"):
                b.start(1)  # never backwards
            with pytest.raises(BridgeError, match="not after"):
                b.start(2)
            # the connection survived all of it
            assert b.status()["round"] == 2
    finally:
        system.shutdown()


def test_start_during_a_round_is_queued_once():
    """A start while a round is in flight is queued (ONE at a time) and runs the moment the
    barrier is reached; rounds never overlap, as with the reference master
    (AllreduceMaster.scala:62-66)."""
    P, n, chunk, rounds = 2, 8, 2, 4
    system = C.ActorSystem("Inflight", False)
    gate = threading.Event()

    def src(k):
        base = host_iota_source(n, 0.0)

        def f(req):
            gate.wait(10)  # hold round 0 in flight
            return AllReduceInput(base(req))
        return f

    master = system.master(P, 1.0, 1.0, 1.0, 1, n, rounds - 1, chunk, externalRounds=True, bridgePort=0)
    port = system.master_bridge_port(master)
    for k in range(P):
        w = system.worker(src(k), None, f"w{k}")
        master.tell(MemberUp(w, "worker", ""), None)
    try:
        with BridgeClient("127.0.0.1", port) as b:
            b.wait_for("InitWorkers")
            assert b.start(0)["type"] == "Accepted"
            assert b.start(1)["type"] == "Queued"
            with pytest.raises(BridgeError, match="already queued"):
                b.start(2)
            st = b.status()
            assert st["round"] == 0 and st["queued"] == 1, st
            gate.set()
            b.wait_for("RoundComplete", round=0)
            b.wait_for("Accepted", round=1)  # started at round 0's barrier
            b.wait_for("RoundComplete", round=1)
            assert b.status()["awaiting"] is True
    finally:
        gate.set()
        system.shutdown()


@pytest.mark.parametrize("pipeline", [True, False])
def test_drive_pipelined_and_lockstep(pipeline):
    P, n, chunk, rounds = 3, 50, 7, 20
    system, master, port, outs, fin = _job(P, n, chunk, rounds, name=f"Pipe{int(pipeline)}")
    try:
        with BridgeClient("127.0.0.1", port) as b:
            b.wait_for("InitWorkers")
            done = b.drive(range(rounds), pipeline=pipeline)
            assert [d["round"] for d in done] == list(range(rounds))
            b.wait_for("AllreduceFinished", rounds=rounds)
            if pipeline:
                assert any(e["type"] == "Queued" for e in b.events)
            else:
                assert not any(e["type"] == "Queued" for e in b.events)
        deadline = time.time() + 5
        while time.time() < deadline and any(len(o) < rounds for o in outs):
            time.sleep(0.01)
        for k in range(P):
            for it in range(rounds):
                np.testing.assert_array_equal(outs[k][it][0], expected(n, it, P).astype(F))
    finally:
        system.shutdown()


def test_observer_mode_and_late_client():
    """Without externalRounds the master drives itself; a client only watches. A client that
    connects after the init still gets the InitWorkers line first."""
    P, n, chunk, rounds = 2, 10, 5, 30
    system, master, port, outs, fin = _job(P, n, chunk, rounds, external=False, name="Observe")
    try:
        assert fin.wait(20)
        with BridgeClient("127.0.0.1", port) as b:
            init = b.wait_for("InitWorkers")
            assert init["externalRounds"] is False and init["workers"] == [0, 1]
            with pytest.raises(BridgeError, match="externalRounds"):
                b.start(0)
            assert b.status()["finished"] is True
    finally:
        system.shutdown()


def test_two_clients_see_the_same_events():
    P, n, chunk, rounds = 2, 16, 4, 5
    system, master, port, outs, fin = _job(P, n, chunk, rounds, name="TwoClients")
    try:
        with BridgeClient("127.0.0.1", port) as a, BridgeClient("127.0.0.1", port) as w:
            a.wait_for("InitWorkers")
            w.wait_for("InitWorkers")
            a.drive(range(rounds))
            w.wait_for("AllreduceFinished")
            seen = [e["round"] for e in w.events if e["type"] == "RoundComplete"]
            assert seen == list(range(rounds))
            # replies go only to the sender
            assert not any(e["type"] == "Accepted" for e in w.events)
    finally:
        system.shutdown()


def test_flat_json_parser():
    p = C.parse_flat_json
    assert p('{"type":"StartAllreduce","round":7}') == {"type": "StartAllreduce", "round": "7"}
    assert p(' { "a" : "x\\"y\\\\z\\n" , "b" : true } ') == {"a": 'x"y\\z\n', "b": "true"}
    assert p("{}") == {}
    assert p('{"a":"\\u0041"}') == {"a": "A"}
    for bad in ["", "[]", '{"a":1', '{"a":1}x', '{"a":[1]}', '{"a":{"b":1}}', '{a:1}', '{"a":"x}', '{"a":1,}']:
        assert p(bad) is None, bad


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["python", "native"])
def test_master_cli_bridge_external_rounds(kind):
    """mxar-master --bridge PORT --external-rounds + 2 worker processes over TCP (Python CLIs,
    or the Python-free `mxar` executable): the bridge client is the only round driver."""
    from akka_allreduce_1_amd.parallel.comm import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    mport, bport = free_port(), free_port()
    rounds = 8
    if kind == "python":
        seed = ["--set", f"mxar.cluster.seed-nodes=mxar.tcp://ClusterSystem@127.0.0.1:{mport}",
                "--set", "mxar.loglevel=WARNING"]
        py = [sys.executable, "-m", "akka_allreduce_1_amd"]
        mcmd = py + ["master", str(mport), "2", "10", "2", "--bridge", str(bport), "--external-rounds",
                     "--set", f"mxar.allreduce.max-round={rounds - 1}"] + seed
    else:
        exe = os.path.join(root, "akka_allreduce_1_amd", "mxar")
        if not os.path.exists(exe):
            pytest.skip("native executable not built (tools/build_native.py)")
        seed = ["--seeds", f"mxar.tcp://ClusterSystem@127.0.0.1:{mport}", "--loglevel", "ERROR"]
        py = [exe]
        mcmd = [exe, "master", str(mport), "2", "10", "2", "--bridge", str(bport), "--external-rounds",
                "--max-round", str(rounds - 1)] + seed
    master = subprocess.Popen(mcmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    workers = []
    try:
        deadline = time.time() + 60
        b = None
        while b is None and time.time() < deadline:
            try:
                b = BridgeClient("127.0.0.1", bport, timeout=60)
            except OSError:
                time.sleep(0.2)
        assert b is not None, "bridge did not come up"
        workers = [subprocess.Popen(py + ["worker", "0", "10"] + seed, env=env, stdout=subprocess.PIPE,
                                    stderr=subprocess.STDOUT, text=True) for _ in range(2)]
        with b:
            init = b.wait_for("InitWorkers", timeout=60)
            assert init["workers"] == [0, 1]
            done = b.drive(range(rounds), timeout=30)
            assert len(done) == rounds
            b.wait_for("AllreduceFinished", timeout=30)
        assert master.wait(30) == 0
    finally:
        for p in workers + [master]:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(10)
                except subprocess.TimeoutExpired:
                    p.kill()


def test_planejob_loopback_driven_through_the_bridge():
    """PlaneJob(bridge_port=0, external_rounds=True) on the loopback round engine: the same
    job shape the GPU test drives on the xGMI plane."""
    from akka_allreduce_1_amd.engine import PlaneJob

    P, n, chunk, rounds = 3, 301, 17, 10
    job = PlaneJob(P, n, max_chunk_size=chunk, max_round=rounds - 1, plane="loopback", bridge_port=0,
                   external_rounds=True)
    try:
        job.start()
        with BridgeClient("127.0.0.1", job.bridge_port) as b:
            assert b.wait_for("InitWorkers")["workers"] == list(range(P))
            b.drive(range(rounds))
            b.wait_for("AllreduceFinished", rounds=rounds)
        assert job.finished.wait(10)
        for p in job.planes:
            p.drain()
        job.system.await_idle(10.0)
        for k in range(P):
            for it in range(rounds):
                data, counts = job.outputs[k][it]
                np.testing.assert_array_equal(np.asarray(data), expected(n, it, P).astype(F))
                assert all(c == P for c in counts)
    finally:
        job.shutdown()


def test_worker_loss_while_the_client_drives():
    """externalRounds + reinitOnLoss: a worker dies between two client-driven rounds. The
    master re-initialises the survivors (a new InitWorkers epoch) WITHOUT starting a round by
    itself; the client's next StartAllreduce runs on the survivors only."""
    from akka_allreduce_1_amd.protocol import PoisonPill

    P, n, chunk, rounds = 3, 30, 4, 10
    system = C.ActorSystem("LossDrive", False)
    outs = [dict() for _ in range(P)]
    delivered = [[] for _ in range(P)]
    lock = threading.Lock()

    def src(k):
        base = host_iota_source(n, 1000.0 * k)
        return lambda req: AllReduceInput(base(req))

    def sink(k):
        def f(out):
            with lock:
                outs[k][out.iteration] = (np.asarray(out.data).copy(), list(out.count))
                delivered[k].append(out.iteration)
        return f

    master = system.master(P, 1.0, 1.0, 1.0, 1, n, rounds - 1, chunk, reinitOnLoss=True, externalRounds=True,
                           bridgePort=0)
    ws = [system.worker(src(k), sink(k), f"w{k}") for k in range(P)]
    for w in ws:
        master.tell(MemberUp(w, "worker", ""), None)
    try:
        with BridgeClient("127.0.0.1", system.master_bridge_port(master)) as b:
            e1 = b.wait_for("InitWorkers", workers=[0, 1, 2])
            b.drive(range(3))
            ws[2].tell(PoisonPill(), None)
            e2 = b.wait_for("InitWorkers", workers=[0, 1])
            assert e2["epoch"] > e1["epoch"]
            time.sleep(0.2)
            st = b.status()
            assert st["awaiting"] is True and st["round"] == 2, st  # no round started by the re-init
            b.drive(range(3, rounds))
            b.wait_for("AllreduceFinished", rounds=rounds)
        deadline = time.time() + 5
        while time.time() < deadline and any(len(outs[k]) < rounds for k in (0, 1)):
            time.sleep(0.01)
        for k in (0, 1):
            assert delivered[k] == list(range(rounds)), delivered[k]  # every round exactly once
            np.testing.assert_array_equal(outs[k][2][0], expected(n, 2, 3).astype(F))
            data, counts = outs[k][rounds - 1]
            i = np.arange(n, dtype=np.float64)
            np.testing.assert_array_equal(data, sum(i + rounds - 1 + 1000.0 * j for j in (0, 1)).astype(F))
            assert all(c == 2 for c in counts)
    finally:
        system.shutdown()


@pytest.mark.slow
@pytest.mark.parametrize("lockstep", [False, True])
def test_native_drive_client(lockstep):
    """No Python anywhere: `mxar master --bridge --external-rounds`, two `mxar worker`s and the
    `mxar drive` bridge client (pipelined, or lock-step) run the whole job."""
    from akka_allreduce_1_amd.parallel.comm import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "akka_allreduce_1_amd", "mxar")
    if not os.path.exists(exe):
        pytest.skip("native executable not built (tools/build_native.py)")
    mport, bport = free_port(), free_port()
    seed = ["--seeds", f"mxar.tcp://ClusterSystem@127.0.0.1:{mport}", "--loglevel", "ERROR"]
    rounds = 40
    procs = [subprocess.Popen([exe, "master", str(mport), "2", "12", "2", "--th-reduce", "1", "--th-complete", "1",
                               "--bridge", str(bport), "--external-rounds", "--max-round", str(rounds - 1)] + seed,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)]
    try:
        procs += [subprocess.Popen([exe, "worker", "0", "12"] + seed, stdout=subprocess.DEVNULL,
                                   stderr=subprocess.DEVNULL) for _ in range(2)]
        drive = subprocess.run([exe, "drive", f"127.0.0.1:{bport}"] + (["--lockstep"] if lockstep else []),
                               capture_output=True, text=True, timeout=120)
        assert drive.returncode == 0, (drive.stdout, drive.stderr)
        line = json.loads(drive.stdout.strip().splitlines()[-1])
        assert line["rounds"] == rounds and line["rounds_per_s"] > 0, line
        assert line["driver"] == ("bridge lock-step" if lockstep else "bridge pipelined")
        out, _ = procs[0].communicate(timeout=30)
        assert procs[0].returncode == 0 and f"finished {rounds} rounds" in out, out
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(10)
                except subprocess.TimeoutExpired:
                    p.kill()


def test_client_churn_while_rounds_publish():
    """Observers connect, read a little and vanish (some mid-line) while the master publishes
    every CompleteAllreduce / RoundComplete: the job is unaffected and the bridge keeps
    serving (reap / close / publish never race on a reused fd)."""
    import socket as pysock

    P, n, chunk, rounds = 2, 64, 8, 400
    system, master, port, outs, fin = _job(P, n, chunk, rounds, external=False, name="Churn")
    try:
        t_end = time.time() + 20
        churned = 0
        while not fin.is_set() and time.time() < t_end:
            s = pysock.create_connection(("127.0.0.1", port), timeout=5)
            s.recv(64)  # part of Hello / InitWorkers / events
            if churned % 3 == 0:
                s.sendall(b'{"type":"Sta')  # half a command, then gone
            s.close()
            churned += 1
        assert fin.wait(30)
        assert churned > 5
        with BridgeClient("127.0.0.1", port) as b:
            st = b.status()
            assert st["finished"] is True
        for k in range(P):
            np.testing.assert_array_equal(outs[k][rounds - 1][0], expected(n, rounds - 1, P).astype(F))
    finally:
        system.shutdown()


def test_client_that_never_reads_does_not_stall_the_master():
    """publish() used to block the master actor in send() once a connected client
    stopped reading. Events now go through a bounded per-client queue drained by a writer
    thread: a watcher that never reads its socket is disconnected when its queue overflows
    (4 MiB), and the job's rounds run at their own pace meanwhile."""
    import socket

    P, n, chunk, rounds = 2, 8, 2, 3000
    system, master, port, outs, fin = _job(P, n, chunk, rounds, external=False, name="Stall")
    lazy = socket.create_connection(("127.0.0.1", port))
    lazy.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)  # and never reads
    try:
        assert fin.wait(120), "rounds stalled behind a client that never reads"
        assert len(outs[0]) == rounds and len(outs[1]) == rounds
    finally:
        lazy.close()
        system.shutdown()


@pytest.mark.parametrize("init_workers", [0, 2])
def test_init_workers_waits_for_the_whole_membership(init_workers):
    """MasterParams.initWorkers: below thAllreduce = 1 the reference initialises with the first
    workers up (AllreduceMaster.scala:42) and restarts at round 0 when the next one joins;
    initWorkers = N makes the first init wait for N workers."""
    n, chunk, rounds = 8, 2, 6
    system = C.ActorSystem(f"InitW{init_workers}", False)
    fin = threading.Event()
    outs = [dict(), dict()]

    def sink(k):
        return lambda out: outs[k].__setitem__(out.iteration, list(out.count))

    try:
        master = system.master(2, 0.5, 1.0, 1.0, 1, n, rounds - 1, chunk, on_finished=lambda r: fin.set(),
                               initWorkers=init_workers)
        w0 = system.worker(lambda req: AllReduceInput(host_iota_source(n, 0.0)(req)), sink(0), "w0")
        master.tell(MemberUp(w0, "worker", ""), None)
        time.sleep(0.3)
        if init_workers == 2:
            assert not outs[0] and not fin.is_set()  # nothing runs with one of two workers
        else:
            assert outs[0]  # the reference: the lone worker's job already ran
        w1 = system.worker(lambda req: AllReduceInput(host_iota_source(n, 1000.0)(req)), sink(1), "w1")
        master.tell(MemberUp(w1, "worker", ""), None)
        if init_workers == 2:
            assert fin.wait(10)
            deadline = time.time() + 5
            while time.time() < deadline and len(outs[1]) < rounds:
                time.sleep(0.01)
            assert sorted(outs[1]) == list(range(rounds))
            assert all(c == [2] * len(c) for c in outs[1].values())
    finally:
        system.shutdown()
