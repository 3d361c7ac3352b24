"""Akka classic remoting on the wire (csrc/cluster/akka_wire.h, csrc/runtime/akka_endpoint.h,
docs/AKKA_WIRE.md): an Akka 2.5 client - the reference's own stack (build.sbt:3,
application.conf:5-9) - drives the master's rounds with the reference's messages
(AllreduceMessage.scala:17-19) over akka.tcp.

Each layer of the C++ codec is checked against an independent encoder:
* protobuf: google.protobuf classes built from the akka-remote 2.5 schemas
  (akka_allreduce_1_amd/akka_remote.py), byte for byte both ways;
* Java serialization: a Python ObjectOutputStream writer / reader;
* SHA-1: hashlib; serialVersionUID: a Python computeDefaultSUID.
Parity unpinned: no JVM exists here, so no test can say what a real Akka system emits; the
schemas, the stream format and the scalac 2.12 member list are written from their
specifications (docs/AKKA_WIRE.md lists what a JVM run would pin).
"""
import hashlib
import os
import random
import socket
import struct
import threading
import time

import numpy as np
import pytest

from akka_allreduce_1_amd import akka_remote as ar
from akka_allreduce_1_amd._native import C
from akka_allreduce_1_amd.engine import host_iota_source
from akka_allreduce_1_amd.protocol import AllReduceInput, MemberUp

A = C.akka
START = ar.REF_PACKAGE + ".StartAllreduce"
COMPLETE = ar.REF_PACKAGE + ".CompleteAllreduce"


# ---- codec layers -------------------------------------------------------------------------

def test_sha1_matches_hashlib():
    rng = random.Random(3)
    for n in (0, 1, 55, 56, 63, 64, 65, 119, 1000):
        b = bytes(rng.getrandbits(8) for _ in range(n))
        assert A.sha1(b) == hashlib.sha1(b).digest(), n


def test_associate_and_control_pdus_match_protobuf():
    P = ar.pb()
    m = P.AkkaProtocolMessage()
    m.instruction.commandType = 1
    o = m.instruction.handshakeInfo.origin
    o.system, o.hostname, o.port, o.protocol = "ClusterSystem", "10.0.0.7", 2551, "akka.tcp"
    m.instruction.handshakeInfo.uid = 0xFEDCBA9876543210
    assert A.encode_associate("ClusterSystem", "10.0.0.7", 2551, 0xFEDCBA9876543210) == m.SerializeToString()
    m.instruction.handshakeInfo.cookie = "secret"
    assert A.encode_associate("ClusterSystem", "10.0.0.7", 2551, 0xFEDCBA9876543210, "secret") == m.SerializeToString()
    d = A.decode_pdu(m.SerializeToString())
    assert d["command"] == 1 and d["uid"] == 0xFEDCBA9876543210 and d["cookie"] == "secret"
    assert d["origin"] == {"system": "ClusterSystem", "hostname": "10.0.0.7", "port": 2551, "protocol": "akka.tcp"}
    for cmd in (2, 3, 4, 5):
        h = P.AkkaProtocolMessage()
        h.instruction.commandType = cmd
        assert A.encode_control(cmd) == h.SerializeToString()
        assert A.decode_pdu(h.SerializeToString()) == {"command": cmd}
    p = P.AkkaProtocolMessage(payload=b"\x01\x02\x03")
    assert A.encode_payload_pdu(b"\x01\x02\x03") == p.SerializeToString()
    assert A.decode_pdu(p.SerializeToString()) == {"payload": b"\x01\x02\x03"}
    with pytest.raises(ValueError):
        A.decode_pdu(b"\x12\x05\x08")  # truncated


@pytest.mark.parametrize("serializer", [1, 6, 16, -7])
def test_envelope_container_matches_protobuf(serializer):
    P = ar.pb()
    c = P.AckAndEnvelopeContainer()
    c.ack.cumulativeAck = 41
    c.ack.nacks.extend([38, 40])
    e = c.envelope
    e.recipient.path = "akka.tcp://ClusterSystem@127.0.0.1:2551/user/master#-1234"
    e.message.message = bytes(range(200))
    e.message.serializerId = serializer
    e.message.messageManifest = b"RH"
    e.sender.path = "akka.tcp://Client@127.0.0.1:25520/temp/$a"
    e.seq = 9
    d = {"ack": {"cumulativeAck": 41, "nacks": [38, 40]},
         "envelope": {"recipient": e.recipient.path, "sender": e.sender.path, "seq": 9,
                      "message": {"message": bytes(range(200)), "serializerId": serializer, "messageManifest": b"RH"}}}
    assert A.encode_container(d) == c.SerializeToString()
    assert A.decode_container(c.SerializeToString()) == d
    # optional parts absent
    c2 = P.AckAndEnvelopeContainer()
    c2.envelope.recipient.path = "akka.tcp://S@h:1/"
    c2.envelope.message.message = b""
    c2.envelope.message.serializerId = serializer
    d2 = {"envelope": {"recipient": "akka.tcp://S@h:1/", "sender": None, "seq": None,
                       "message": {"message": b"", "serializerId": serializer, "messageManifest": None}}}
    assert A.encode_container(d2) == c2.SerializeToString()
    assert A.decode_container(c2.SerializeToString()) == d2


def test_selection_envelope_matches_protobuf():
    P = ar.pb()
    s = P.SelectionEnvelope(enclosedMessage=b"xyz", serializerId=1)
    s.pattern.add(type=1, matcher="user")
    s.pattern.add(type=2, matcher="mas*")
    s.pattern.add(type=0)
    s.messageManifest = b"M"
    s.wildcardFanOut = True
    b = A.encode_selection({"message": b"xyz", "serializerId": 1, "messageManifest": b"M"},
                           [(1, "user"), (2, "mas*"), (0, "")], True)
    assert b == s.SerializeToString()
    inner, pattern, wc = A.decode_selection(s.SerializeToString())
    assert inner == {"message": b"xyz", "serializerId": 1, "messageManifest": b"M"}
    assert pattern == [(1, "user"), (2, "mas*"), (0, "")] and wc is True


def test_actor_paths():
    a, el = A.parse_actor_path("akka.tcp://ClusterSystem@127.0.0.1:2551/user/master#-77")
    assert a == {"system": "ClusterSystem", "hostname": "127.0.0.1", "port": 2551, "protocol": "akka.tcp"}
    assert el == ["user", "master"]
    assert A.parse_actor_path("akka.tcp://S@h:7/")[1] == []
    assert A.parse_actor_path("akka://local/user/x") is None  # no host: not a remote path
    assert A.parse_actor_path("akka.tcp://S@h:99999/user") is None


def test_java_serialization_matches_python_writer():
    suid = -6180218149226146171
    fields = [("I", "srcId", 3), ("I", "round", -7)]
    b = A.java_serialize(COMPLETE, suid, fields)
    assert b == ar.java_serialize(COMPLETE, suid, fields)
    # stream layout: magic, TC_OBJECT, TC_CLASSDESC, name, SUID, SC_SERIALIZABLE, 2 fields in
    # ObjectStreamField order (round before srcId), TC_ENDBLOCKDATA, TC_NULL, the values
    name = COMPLETE.encode()
    head = b"\xac\xed\x00\x05\x73\x72" + struct.pack(">H", len(name)) + name + struct.pack(">q", suid) + b"\x02\x00\x02"
    assert b.startswith(head)
    assert b[len(head):] == b"I\x00\x05roundI\x00\x05srcId\x78\x70" + struct.pack(">ii", -7, 3)
    assert A.java_deserialize(b) == (COMPLETE, suid, [("I", "round", -7), ("I", "srcId", 3)])
    assert ar.java_deserialize(b) == (COMPLETE, suid, {"round": -7, "srcId": 3})
    mixed = [("J", "a", -(1 << 40)), ("Z", "b", 1), ("D", "c", 2.5), ("F", "d", -0.75), ("S", "e", -3), ("B", "f", 7),
             ("C", "g", 65)]
    assert A.java_serialize("x.Y", 1, mixed) == ar.java_serialize("x.Y", 1, mixed)
    assert [v for _, _, v in A.java_deserialize(A.java_serialize("x.Y", 1, mixed))[2]] == [-(1 << 40), 1, 2.5, -0.75,
                                                                                         -3, 7, 65]
    with pytest.raises(ValueError):
        A.java_deserialize(b[:-3])
    with pytest.raises(ValueError, match="object fields"):
        A.java_deserialize(b"\xac\xed\x00\x05\x73\x72\x00\x01X" + b"\x00" * 8 + b"\x02\x00\x01L\x00\x01s\x74\x00\x01L\x78\x70")


def test_default_suid_algorithm():
    # the same class model hashed by the C++ and the Python computeDefaultSUID
    rng = random.Random(5)
    for k in range(20):
        name = f"p.q.C{k}"
        fields = [(f"f{i}", rng.choice([0x2 | 0x10, 0x1, 0x2 | 0x8, 0x4 | 0x80]), rng.choice("IJZ")) for i in range(3)]
        ctors = [(0x1, "(I)V"), (0x2, "()V")]
        methods = [(rng.choice(["a", "b", "run"]), rng.choice([0x1, 0x9, 0x2, 0x11]), "(Lp/q/X;)V") for _ in range(4)]
        ifs = ["java.io.Serializable", "a.B"]
        cpp = A.class_suid(name, 0x11 | 0x20, ifs, fields, ctors, methods, bool(k % 2))
        py = ar.default_suid(ar.ClassModel(name, 0x11 | 0x20, ifs, fields, ctors, methods, bool(k % 2)))
        assert cpp == py
    # private static / private transient fields and private members do not count
    base = A.class_suid("p.D", 0x1, [], [("a", 0x1, "I")], [(0x1, "()V")], [])
    assert A.class_suid("p.D", 0x1, [], [("a", 0x1, "I"), ("z", 0x2 | 0x8, "J")], [(0x1, "()V"), (0x2, "(I)V")],
                        [("m", 0x2, "()V")]) == base
    assert A.class_suid("p.D", 0x1, [], [("a", 0x1, "I"), ("z", 0x2, "J")], [(0x1, "()V")], []) != base


def test_reference_case_class_suids():
    # parity unpinned (no JVM): the C++ and Python models of scalac 2.12's output agree, the
    # SUID changes with the package (it hashes the class name), and the member lists carry
    # what the JVM's computeDefaultSUID reads
    for fqcn, params in ((START, [("round", "I")]), (COMPLETE, [("srcId", "I"), ("round", "I")])):
        assert A.case_class_suid(fqcn, params) == ar.case_class_suid(fqcn, params)
        assert A.case_class_suid("other.pkg." + fqcn.rsplit(".", 1)[1], params) != A.case_class_suid(fqcn, params)
    m = ar.case_class_model(COMPLETE, [("srcId", "I"), ("round", "I")])
    names = sorted(n for n, _, _ in m.methods)
    assert names == sorted(["srcId", "round", "copy", "copy$default$1", "copy$default$2", "productPrefix",
                            "productArity", "productElement", "productIterator", "canEqual", "hashCode", "toString",
                            "equals", "apply", "unapply", "tupled", "curried"])
    assert m.fields == [("srcId", 0x12, "I"), ("round", 0x12, "I")]


# ---- the endpoint ---------------------------------------------------------------------------

def expected(n, it, P):
    i = np.arange(n, dtype=np.float64)
    return sum(i + it + 1000.0 * k for k in range(P))


def _job(P, n, chunk, rounds, name, **akka):
    system = C.ActorSystem(name, False)
    fin = threading.Event()
    outs = [dict() for _ in range(P)]
    lock = threading.Lock()

    def src(k):
        base = host_iota_source(n, 1000.0 * k)
        return lambda req: AllReduceInput(base(req))

    def sink(k):
        def f(out):
            with lock:
                outs[k][out.iteration] = (np.asarray(out.data).copy(), list(out.count))
        return f

    master = system.master(P, 1.0, 1.0, 1.0, 1, n, rounds - 1, chunk, on_finished=lambda r: fin.set(),
                           externalRounds=True, bridgePort=0)
    ep = A.start_endpoint(master, **akka)
    for k in range(P):
        w = system.worker(src(k), sink(k), f"w{k}")
        master.tell(MemberUp(w, "worker", ""), None)
    return system, master, ep, outs, fin


def test_akka_client_drives_the_reference_round_loop():
    """The reference master's loop (AllreduceMaster.scala:58-67,91-97) run by an Akka client:
    resolve /user/master, StartAllreduce(r), count CompleteAllreduce(srcId, r) until every
    worker completed, then r + 1."""
    P, n, chunk, rounds = 3, 30, 4, 8
    system, master, ep, outs, fin = _job(P, n, chunk, rounds, "AkkaDrive")
    try:
        assert ep.address == f"akka.tcp://ClusterSystem@127.0.0.1:{ep.port}"
        with ar.AkkaClient("127.0.0.1", ep.port) as cl:
            assert cl.remote_origin.system == "ClusterSystem" and cl.remote_origin.port == ep.port
            ref = cl.identify(["user", "master"])
            assert ref == ep.master_path and ref.startswith(ep.address + "/user/master#")
            assert cl.identify(["user", "nobody"]) is None
            assert cl.identify(["user", "ma*"]) == ref  # CHILD_PATTERN selection
            got = []
            for r in range(rounds):
                # even rounds by ActorRef (the resolved path), odd ones by ActorSelection
                cl.start_allreduce(r, to=ref if r % 2 == 0 else None)
                seen = set()
                while len(seen) < P:
                    src_id, rr, cls, suid = cl.complete_allreduce()
                    assert cls == COMPLETE and suid == ep.suid_complete
                    if rr == r:
                        seen.add(src_id)
                got.append(sorted(seen))
            assert got == [list(range(P))] * rounds
            assert fin.wait(10)
        st = ep.stats()
        assert st["starts"] == rounds and st["identifies"] == 3 and st["suid_mismatches"] == 0
        assert st["completes_sent"] >= rounds * P and st["client_suid_start"] == ep.suid_start
        deadline = time.time() + 5
        while time.time() < deadline and any(len(o) < rounds for o in outs):
            time.sleep(0.01)
        for k in range(P):
            for it in range(rounds):
                np.testing.assert_array_equal(outs[k][it][0], expected(n, it, P).astype(np.float32))
                assert outs[k][it][1] == [P] * len(outs[k][it][1])
    finally:
        system.shutdown()


def test_heartbeats_watch_and_system_messages():
    system, master, ep, outs, fin = _job(2, 8, 2, 4, "AkkaHb", heartbeat_s=0.05)
    try:
        with ar.AkkaClient("127.0.0.1", ep.port) as cl:
            # a sequenced system message (e.g. Watch) is acknowledged cumulatively
            cl.tell(ep.address + "/user/master", b"\x00", serializer=22, sender=cl.local + "/user/w", seq=1)
            r = cl.receive(lambda m: getattr(m, "ack", None) == 1)
            assert r.ack == 1
            # the remote watcher's heartbeat gets HeartbeatRsp(uid) (misc serializer, "RHR")
            watcher = cl.local + "/system/remote-watcher"
            cl.tell(ep.address + "/system/remote-watcher", b"", serializer=16, manifest=b"RH", sender=watcher)
            rsp = cl.receive(lambda m: m.recipient == watcher)
            assert rsp.serializer == 16 and rsp.manifest == b"RHR"
            hb = ar.pb().WatcherHeartbeatResponse()
            hb.ParseFromString(rsp.message)
            assert hb.uid == cl.remote_uid & 0xFFFFFFFF  # the Int address uid (positive)
            time.sleep(0.3)
            with pytest.raises(TimeoutError):
                cl.receive(lambda m: False, timeout=0.3)
            assert cl.heartbeats >= 3  # transport heartbeats keep coming
            st = ep.stats()
            assert st["system_messages"] == 1 and st["watcher_heartbeats"] == 1
    finally:
        system.shutdown()


def test_refusals_suid_mismatch_and_shutdown():
    system, master, ep, outs, fin = _job(2, 8, 2, 4, "AkkaRefuse", cookie="s3cret")
    try:
        # no handshake: a payload first closes the connection
        s = socket.create_connection(("127.0.0.1", ep.port), timeout=5)
        body = A.encode_payload_pdu(b"")
        s.sendall(struct.pack(">I", len(body)) + body)
        s.settimeout(5)
        assert s.recv(16) == b""
        s.close()
        # wrong cookie (akka.remote.require-cookie)
        with pytest.raises((ConnectionError, TimeoutError, OSError)):
            ar.AkkaClient("127.0.0.1", ep.port, cookie="wrong", timeout=3)
        with ar.AkkaClient("127.0.0.1", ep.port, cookie="s3cret") as cl:
            # an oversized frame is refused and the association dropped
            cl2 = ar.AkkaClient("127.0.0.1", ep.port, cookie="s3cret")
            cl2.sock.sendall(struct.pack(">I", A.MAX_FRAME + 10000))
            with pytest.raises((ConnectionError, OSError)):
                cl2.receive(timeout=5)
            cl2.sock.close()
            # a client whose StartAllreduce carries another SUID is reported (its classes
            # disagree with the model), the start still runs
            cl.start_allreduce(0, suid=12345)
            src_id, r, _, _ = cl.complete_allreduce()
            assert r == 0
            # unsupported messages are dropped, the association stays up
            cl.tell(ep.address + "/user/master", ar.java_serialize(ar.REF_PACKAGE + ".Other", 1, [("I", "x", 1)]),
                    sender=cl.local + "/user/driver")
            cl.tell(ep.address + "/user/master", b"junk", serializer=99, sender=cl.local + "/user/driver")
            cl.start_allreduce(1)
            while True:
                _, r, _, _ = cl.complete_allreduce()
                if r == 1:
                    break
            st = ep.stats()
            assert st["suid_mismatches"] == 1 and st["client_suid_start"] == ep.suid_start
            assert st["unsupported"] == 2 and st["rejected"] >= 2
            assert ep.associations() == 1
            # the master's shutdown tells the client (DISASSOCIATE_SHUTTING_DOWN)
            system.shutdown()
            with pytest.raises(ConnectionError):
                while True:
                    cl.receive(timeout=5)
            assert cl.closed_by_peer in (ar.SHUTTING_DOWN, None)
    finally:
        system.shutdown()


def test_cli_master_serves_akka(tmp_path):
    """`mxar master ... --akka-port P --external-rounds` with native workers: an Akka client
    drives every round of the reference's default job over akka.tcp."""
    import subprocess

    import akka_allreduce_1_amd

    exe = os.path.join(os.path.dirname(akka_allreduce_1_amd.__file__), "mxar")

    def free_port():
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            return so.getsockname()[1]

    port, aport = free_port(), free_port()
    seeds = ["--seeds", f"mxar.tcp://ClusterSystem@127.0.0.1:{port}", "--loglevel", "WARNING"]
    rounds = 5
    m = subprocess.Popen([exe, "master", str(port), "2", "10", "2", "--external-rounds", "--akka-port", str(aport),
                          "--max-round", str(rounds - 1)] + seeds, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         text=True)
    ws = [subprocess.Popen([exe, "worker", "0", "10"] + seeds, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
          for _ in range(2)]
    try:
        deadline = time.time() + 20
        cl = None
        while cl is None and time.time() < deadline:
            try:
                cl = ar.AkkaClient("127.0.0.1", aport, timeout=10)
            except OSError:
                time.sleep(0.1)
        assert cl is not None
        with cl:
            assert cl.identify(["user", "master"]).startswith(f"akka.tcp://ClusterSystem@127.0.0.1:{aport}/user/master#")
            for r in range(rounds):
                while True:  # the first start may come before the workers are initialised
                    cl.start_allreduce(r)
                    try:
                        seen = set()
                        while len(seen) < 2:
                            s, rr, _, _ = cl.complete_allreduce(timeout=2 if r == 0 and not seen else 10)
                            if rr == r:
                                seen.add(s)
                        break
                    except TimeoutError:
                        assert r == 0 and time.time() < deadline
        out, _ = m.communicate(timeout=20)
        assert m.returncode == 0, out
        assert f"finished {rounds} rounds" in out or f"finished {rounds - 1} rounds" in out, out
    finally:
        for p in [m] + ws:
            if p.poll() is None:
                p.kill()
                p.wait()


def test_python_cli_master_serves_akka():
    """`python -m akka_allreduce_1_amd master ... --akka-port P --external-rounds` with two
    Python worker processes: the Akka client drives every round (exact thresholds)."""
    import subprocess
    import sys

    from akka_allreduce_1_amd.parallel.comm import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port, aport = free_port(), free_port()
    common = ["--set", f"mxar.cluster.seed-nodes=mxar.tcp://ClusterSystem@127.0.0.1:{port}",
              "--set", "mxar.loglevel=WARNING"]
    exact = ["--set", "mxar.allreduce.th-reduce=1.0", "--set", "mxar.allreduce.th-complete=1.0",
             "--set", "mxar.allreduce.max-round=3"]
    env = dict(os.environ, PYTHONPATH=root)
    py = [sys.executable, "-m", "akka_allreduce_1_amd"]
    m = subprocess.Popen(py + ["master", str(port), "2", "10", "2", "--akka-port", str(aport), "--external-rounds"]
                         + common + exact, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    ws = [subprocess.Popen(py + ["worker", "0", "10"] + common, env=env, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL) for _ in range(2)]
    try:
        deadline = time.time() + 60
        cl = None
        while cl is None and time.time() < deadline:
            try:
                cl = ar.AkkaClient("127.0.0.1", aport, timeout=10)
            except OSError:
                time.sleep(0.2)
        assert cl is not None
        with cl:
            for r in range(4):
                while True:  # a start before the workers are initialised is refused: retry
                    cl.start_allreduce(r)
                    try:
                        seen = set()
                        while len(seen) < 2:
                            s, rr, _, _ = cl.complete_allreduce(timeout=2 if r == 0 and not seen else 20)
                            if rr == r:
                                seen.add(s)
                        break
                    except TimeoutError:
                        assert r == 0 and time.time() < deadline
        out, _ = m.communicate(timeout=30)
        assert m.returncode == 0, out
        assert "akka.tcp endpoint" in out and "finished 4 rounds" in out, out
    finally:
        for p in [m] + ws:
            if p.poll() is None:
                p.kill()
                p.wait()
