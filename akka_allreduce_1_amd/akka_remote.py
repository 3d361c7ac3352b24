"""A minimal Akka classic-remoting client in Python, for the master's akka.tcp endpoint
(csrc/runtime/akka_endpoint.h, docs/AKKA_WIRE.md).

It does what an Akka 2.5 actor system does when one of its actors talks to the reference's
master (``/root/reference/src/main/scala/sample/cluster/allreduce/AllreduceMaster.scala``):
associate over ``akka.tcp`` (the reference's transport, ``application.conf:5-9``), resolve
``/user/master`` with ``Identify`` (``actorSelection(...).resolveOne``), send
``StartAllreduce(round)`` Java-serialized and receive ``CompleteAllreduce(srcId, round)``
(``AllreduceMessage.scala:17-19``).

Every layer here is written independently of the C++ codec it talks to, so the tests check
one against the other:

* protobuf: google.protobuf message classes built at import from the akka-remote 2.5 schemas
  (``WireFormats.proto``, ``ContainerFormats.proto``), not the hand-rolled C++ encoder;
* Java serialization: a Python ``ObjectOutputStream`` writer / reader for flat classes;
* serialVersionUID: a Python ``ObjectStreamClass.computeDefaultSUID`` over the scalac 2.12
  member list of a final case class.

No JVM exists in this image: where only a JVM could say what the bytes must be (the default
SUIDs above all), the result is parity-unpinned and the endpoint lets a user override it.
"""
from __future__ import annotations

import hashlib
import random
import socket
import struct
import time
from dataclasses import dataclass, field

__all__ = ["AkkaClient", "pb", "java_serialize", "java_deserialize", "default_suid", "case_class_model",
           "case_class_suid", "REF_PACKAGE"]

REF_PACKAGE = "sample.cluster.allreduce"  # AllreduceMessage.scala:1

ASSOCIATE, DISASSOCIATE, HEARTBEAT, SHUTTING_DOWN, QUARANTINED = 1, 2, 3, 4, 5
JAVA, CONTAINER, MISC = 1, 6, 16


# ---- protobuf schemas ---------------------------------------------------------------------

class _Schemas:
    """akka-remote 2.5 message classes (proto2), built from descriptors at first use."""

    def __init__(self):
        from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

        fd = descriptor_pb2.FileDescriptorProto(name="mxar_akka_wire.proto", package="akka", syntax="proto2")
        F = descriptor_pb2.FieldDescriptorProto
        REQ, OPT, REP = F.LABEL_REQUIRED, F.LABEL_OPTIONAL, F.LABEL_REPEATED

        def msg(name, *fields):
            m = fd.message_type.add(name=name)
            for fname, num, label, ftype, tname in fields:
                f = m.field.add(name=fname, number=num, label=label, type=ftype)
                if tname:
                    f.type_name = ".akka." + tname
            return m

        e = fd.enum_type.add(name="CommandType")
        for n, v in (("ASSOCIATE", 1), ("DISASSOCIATE", 2), ("HEARTBEAT", 3), ("DISASSOCIATE_SHUTTING_DOWN", 4),
                     ("DISASSOCIATE_QUARANTINED", 5)):
            e.value.add(name=n, number=v)
        e = fd.enum_type.add(name="PatternType")
        for n, v in (("PARENT", 0), ("CHILD_NAME", 1), ("CHILD_PATTERN", 2)):
            e.value.add(name=n, number=v)
        T = F
        # WireFormats.proto
        msg("AckAndEnvelopeContainer", ("ack", 1, OPT, T.TYPE_MESSAGE, "AcknowledgementInfo"),
            ("envelope", 2, OPT, T.TYPE_MESSAGE, "RemoteEnvelope"))
        msg("RemoteEnvelope", ("recipient", 1, REQ, T.TYPE_MESSAGE, "ActorRefData"),
            ("message", 2, REQ, T.TYPE_MESSAGE, "SerializedMessage"),
            ("sender", 4, OPT, T.TYPE_MESSAGE, "ActorRefData"), ("seq", 5, OPT, T.TYPE_FIXED64, None))
        msg("AcknowledgementInfo", ("cumulativeAck", 1, REQ, T.TYPE_FIXED64, None),
            ("nacks", 2, REP, T.TYPE_FIXED64, None))
        msg("ActorRefData", ("path", 1, REQ, T.TYPE_STRING, None))
        msg("SerializedMessage", ("message", 1, REQ, T.TYPE_BYTES, None), ("serializerId", 2, REQ, T.TYPE_INT32, None),
            ("messageManifest", 3, OPT, T.TYPE_BYTES, None))
        msg("AkkaProtocolMessage", ("payload", 1, OPT, T.TYPE_BYTES, None),
            ("instruction", 2, OPT, T.TYPE_MESSAGE, "AkkaControlMessage"))
        m = msg("AkkaControlMessage", ("handshakeInfo", 2, OPT, T.TYPE_MESSAGE, "AkkaHandshakeInfo"))
        m.field.add(name="commandType", number=1, label=REQ, type=T.TYPE_ENUM, type_name=".akka.CommandType")
        msg("AkkaHandshakeInfo", ("origin", 1, REQ, T.TYPE_MESSAGE, "AddressData"), ("uid", 2, REQ, T.TYPE_FIXED64, None),
            ("cookie", 3, OPT, T.TYPE_STRING, None))
        msg("AddressData", ("system", 1, REQ, T.TYPE_STRING, None), ("hostname", 2, REQ, T.TYPE_STRING, None),
            ("port", 3, REQ, T.TYPE_UINT32, None), ("protocol", 4, OPT, T.TYPE_STRING, None))
        # ContainerFormats.proto
        msg("SelectionEnvelope", ("enclosedMessage", 1, REQ, T.TYPE_BYTES, None),
            ("serializerId", 2, REQ, T.TYPE_INT32, None), ("pattern", 3, REP, T.TYPE_MESSAGE, "Selection"),
            ("messageManifest", 4, OPT, T.TYPE_BYTES, None), ("wildcardFanOut", 5, OPT, T.TYPE_BOOL, None))
        m = msg("Selection", ("matcher", 2, OPT, T.TYPE_STRING, None))
        m.field.add(name="type", number=1, label=REQ, type=T.TYPE_ENUM, type_name=".akka.PatternType")
        msg("Payload", ("enclosedMessage", 1, REQ, T.TYPE_BYTES, None), ("serializerId", 2, REQ, T.TYPE_INT32, None),
            ("messageManifest", 4, OPT, T.TYPE_BYTES, None))
        msg("Identify", ("messageId", 1, REQ, T.TYPE_MESSAGE, "Payload"))
        msg("ActorIdentity", ("correlationId", 1, REQ, T.TYPE_MESSAGE, "Payload"),
            ("ref", 2, OPT, T.TYPE_MESSAGE, "ActorRef"))
        msg("ActorRef", ("path", 1, REQ, T.TYPE_STRING, None))
        msg("Option", ("value", 1, OPT, T.TYPE_MESSAGE, "Payload"))
        msg("WatcherHeartbeatResponse", ("uid", 1, REQ, T.TYPE_UINT64, None))
        pool = descriptor_pool.DescriptorPool()
        pool.Add(fd)
        for m in fd.message_type:
            setattr(self, m.name, message_factory.GetMessageClass(pool.FindMessageTypeByName("akka." + m.name)))


_SCHEMAS: _Schemas | None = None


def pb() -> _Schemas:
    global _SCHEMAS
    if _SCHEMAS is None:
        _SCHEMAS = _Schemas()
    return _SCHEMAS


# ---- Java serialization (java.io.ObjectOutputStream, flat classes of primitive fields) ------

_PRIM = {"B": ">b", "C": ">H", "D": ">d", "F": ">f", "I": ">i", "J": ">q", "S": ">h", "Z": ">?"}


def _utf(s: str) -> bytes:
    b = s.encode("utf-8")
    return struct.pack(">H", len(b)) + b


def java_serialize(fqcn: str, suid: int, fields: list[tuple[str, str, object]]) -> bytes:
    """ObjectOutputStream.writeObject of a class with primitive fields [(type, name, value)]."""
    fs = sorted(fields, key=lambda f: f[1])  # ObjectStreamField order: primitives by name
    out = bytearray(b"\xac\xed\x00\x05\x73\x72")  # magic, version, TC_OBJECT, TC_CLASSDESC
    out += _utf(fqcn) + struct.pack(">q", suid) + b"\x02" + struct.pack(">H", len(fs))
    for t, name, _ in fs:
        out += t.encode() + _utf(name)
    out += b"\x78\x70"  # TC_ENDBLOCKDATA, superclass TC_NULL
    for t, _, v in fs:
        out += struct.pack(_PRIM[t], v)
    return bytes(out)


def java_deserialize(b: bytes) -> tuple[str, int, dict]:
    """(class name, SUID, {field: value}) of one flat object (the most-derived class)."""
    if b[:4] != b"\xac\xed\x00\x05" or b[4] != 0x73 or b[5] != 0x72:
        raise ValueError("not a serialized object with a class descriptor")
    i = 6
    (n,) = struct.unpack_from(">H", b, i)
    name = b[i + 2:i + 2 + n].decode()
    i += 2 + n
    (suid,) = struct.unpack_from(">q", b, i)
    i += 9  # suid + flags
    (nf,) = struct.unpack_from(">H", b, i)
    i += 2
    fs = []
    for _ in range(nf):
        t = chr(b[i])
        (n,) = struct.unpack_from(">H", b, i + 1)
        fs.append((t, b[i + 3:i + 3 + n].decode()))
        i += 3 + n
    if b[i:i + 2] != b"\x78\x70":
        raise ValueError("annotations or a serializable superclass are not supported")
    i += 2
    vals = {}
    for t, fname in fs:
        (v,) = struct.unpack_from(_PRIM[t], b, i)
        vals[fname] = v
        i += struct.calcsize(_PRIM[t])
    return name, suid, vals


# ---- serialVersionUID ---------------------------------------------------------------------

PUBLIC, PRIVATE, PROTECTED, STATIC, FINAL = 0x1, 0x2, 0x4, 0x8, 0x10
_FIELD_MASK = 0x1 | 0x2 | 0x4 | 0x8 | 0x10 | 0x40 | 0x80
_METHOD_MASK = 0x1 | 0x2 | 0x4 | 0x8 | 0x10 | 0x20 | 0x100 | 0x400 | 0x800


@dataclass
class ClassModel:
    name: str
    mods: int
    interfaces: list = field(default_factory=list)
    fields: list = field(default_factory=list)    # (name, mods, descriptor)
    ctors: list = field(default_factory=list)     # (mods, descriptor)
    methods: list = field(default_factory=list)   # (name, mods, descriptor)
    clinit: bool = False


def default_suid(c: ClassModel) -> int:
    """java.io.ObjectStreamClass.computeDefaultSUID."""
    d = bytearray(_utf(c.name))
    cm = c.mods & (0x1 | 0x10 | 0x200 | 0x400)
    if cm & 0x200:
        cm = (cm | 0x400) if c.methods else (cm & ~0x400)
    d += struct.pack(">i", cm)
    for i in sorted(c.interfaces):
        d += _utf(i)
    for name, mods, desc in sorted(c.fields, key=lambda f: f[0]):
        m = mods & _FIELD_MASK
        if not (m & PRIVATE) or not (m & (STATIC | 0x80)):
            d += _utf(name) + struct.pack(">i", m) + _utf(desc)
    if c.clinit:
        d += _utf("<clinit>") + struct.pack(">i", STATIC) + _utf("()V")
    for mods, desc in sorted(c.ctors, key=lambda k: k[1]):
        m = mods & _METHOD_MASK
        if not m & PRIVATE:
            d += _utf("<init>") + struct.pack(">i", m) + _utf(desc.replace("/", "."))
    for name, mods, desc in sorted(c.methods, key=lambda x: (x[0], x[2])):
        m = mods & _METHOD_MASK
        if not m & PRIVATE:
            d += _utf(name) + struct.pack(">i", m) + _utf(desc.replace("/", "."))
    h = hashlib.sha1(bytes(d)).digest()
    return struct.unpack("<q", h[:8])[0]


def case_class_model(fqcn: str, params: list[tuple[str, str]]) -> ClassModel:
    """What scalac 2.12 emits for ``final case class Name(p: T, ...)`` with primitive T."""
    self_t = "L" + fqcn.replace(".", "/") + ";"
    args = "".join(t for _, t in params)
    c = ClassModel(fqcn, PUBLIC | FINAL, ["scala.Product", "scala.Serializable"])
    c.fields = [(n, PRIVATE | FINAL, t) for n, t in params]
    c.ctors = [(PUBLIC, f"({args})V")]
    c.methods = [(n, PUBLIC, "()" + t) for n, t in params]
    c.methods += [("copy", PUBLIC, f"({args}){self_t}")]
    c.methods += [(f"copy$default${k + 1}", PUBLIC, "()" + t) for k, (_, t) in enumerate(params)]
    c.methods += [("productPrefix", PUBLIC, "()Ljava/lang/String;"), ("productArity", PUBLIC, "()I"),
                  ("productElement", PUBLIC, "(I)Ljava/lang/Object;"),
                  ("productIterator", PUBLIC, "()Lscala/collection/Iterator;"),
                  ("canEqual", PUBLIC, "(Ljava/lang/Object;)Z"), ("hashCode", PUBLIC, "()I"),
                  ("toString", PUBLIC, "()Ljava/lang/String;"), ("equals", PUBLIC, "(Ljava/lang/Object;)Z")]
    ps = PUBLIC | STATIC  # the synthetic companion's static forwarders
    c.methods += [("apply", ps, f"({args}){self_t}"), ("unapply", ps, f"({self_t})Lscala/Option;")]
    if len(params) == 1:
        c.methods += [("andThen", ps, "(Lscala/Function1;)Lscala/Function1;"),
                      ("compose", ps, "(Lscala/Function1;)Lscala/Function1;")]
    else:
        c.methods += [("tupled", ps, "()Lscala/Function1;"), ("curried", ps, "()Lscala/Function1;")]
    return c


def case_class_suid(fqcn: str, params: list[tuple[str, str]]) -> int:
    return default_suid(case_class_model(fqcn, params))


# ---- the client -----------------------------------------------------------------------------

@dataclass
class Received:
    recipient: str
    sender: str | None
    serializer: int
    manifest: bytes | None
    message: bytes
    seq: int | None = None


class AkkaClient:
    """An Akka 2.5 actor system as seen on the wire, with one association to ``host:port``.

    ``local`` is the address this client claims in its handshake; replies addressed to actors
    under it come back over the same connection (akka.remote.use-passive-connections)."""

    def __init__(self, host: str, port: int, system: str = "ClusterSystem", local_system: str = "Client",
                 local_port: int = 25520, uid: int | None = None, cookie: str = "", timeout: float = 10.0):
        self.remote = f"akka.tcp://{system}@{host}:{port}"
        self.local = f"akka.tcp://{local_system}@127.0.0.1:{local_port}"
        self.uid = uid if uid is not None else random.getrandbits(63)
        self.timeout = timeout
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.buf = b""
        self.heartbeats = 0
        self.remote_uid = None
        self.remote_origin = None
        self.closed_by_peer = None
        self._temp = 0
        P = pb()
        m = P.AkkaProtocolMessage()
        m.instruction.commandType = ASSOCIATE
        o = m.instruction.handshakeInfo.origin
        o.system, o.hostname, o.port, o.protocol = local_system, "127.0.0.1", local_port, "akka.tcp"
        m.instruction.handshakeInfo.uid = self.uid
        if cookie:
            m.instruction.handshakeInfo.cookie = cookie
        self._send_pdu(m.SerializeToString())
        # the passive side answers with its own ASSOCIATE (ProtocolStateActor, inbound WaitHandshake)
        pdu = self._read_pdu()
        if not pdu.HasField("instruction") or pdu.instruction.commandType != ASSOCIATE:
            raise ConnectionError(f"no ASSOCIATE reply: {pdu}")
        self.remote_uid = pdu.instruction.handshakeInfo.uid
        self.remote_origin = pdu.instruction.handshakeInfo.origin

    # framing
    def _send_pdu(self, body: bytes) -> None:
        self.sock.sendall(struct.pack(">I", len(body)) + body)

    def send_raw_frame(self, body: bytes) -> None:
        self._send_pdu(body)

    def _read_exact(self, n: int, deadline: float) -> bytes:
        while len(self.buf) < n:
            left = deadline - time.monotonic()
            if left <= 0:
                raise TimeoutError("no frame from the endpoint")
            self.sock.settimeout(left)
            chunk = self.sock.recv(65536)
            if not chunk:
                raise ConnectionError("endpoint closed the connection")
            self.buf += chunk
        out, self.buf = self.buf[:n], self.buf[n:]
        return out

    def _read_pdu(self, timeout: float | None = None):
        deadline = time.monotonic() + (timeout or self.timeout)
        (n,) = struct.unpack(">I", self._read_exact(4, deadline))
        m = pb().AkkaProtocolMessage()
        m.ParseFromString(self._read_exact(n, deadline))
        return m

    # messages
    def _envelope(self, recipient: str, message: bytes, serializer: int, manifest: bytes | None,
                  sender: str | None, seq: int | None = None) -> bytes:
        P = pb()
        c = P.AckAndEnvelopeContainer()
        e = c.envelope
        e.recipient.path = recipient
        e.message.message = message
        e.message.serializerId = serializer
        if manifest is not None:
            e.message.messageManifest = manifest
        if sender is not None:
            e.sender.path = sender
        if seq is not None:
            e.seq = seq
        m = P.AkkaProtocolMessage(payload=c.SerializeToString())
        return m.SerializeToString()

    def tell(self, recipient: str, message: bytes, serializer: int = JAVA, manifest: bytes | None = None,
             sender: str | None = None, seq: int | None = None) -> None:
        """ActorRef.tell to a full path (``akka.tcp://Sys@h:p/user/master[#uid]``)."""
        self._send_pdu(self._envelope(recipient, message, serializer, manifest, sender, seq))

    def tell_selection(self, elements: list[str], message: bytes, serializer: int = JAVA,
                       manifest: bytes | None = None, sender: str | None = None, patterns: bool = True) -> None:
        """ActorSelection ``remote/user/master ! msg``: a SelectionEnvelope sent to the root (an
        element with ``*`` or ``?`` becomes a CHILD_PATTERN, as ActorSelection parses it)."""
        P = pb()
        s = P.SelectionEnvelope(enclosedMessage=message, serializerId=serializer)
        if manifest is not None:
            s.messageManifest = manifest
        for el in elements:
            wild = patterns and any(ch in el for ch in "*?")
            s.pattern.add(type=2 if wild else 1, matcher=el)
        self.tell(self.remote + "/", s.SerializeToString(), CONTAINER, None, sender)

    def temp_path(self) -> str:
        self._temp += 1
        return f"{self.local}/temp/${chr(ord('a') + self._temp - 1)}"

    def identify(self, elements: list[str], timeout: float | None = None) -> str | None:
        """``actorSelection(remote/elements).resolveOne()``: Identify(None) from a temp actor,
        the ActorIdentity's ref path (None when nothing lives there)."""
        P = pb()
        none = P.Option().SerializeToString()  # scala.None via the misc serializer (manifest "C")
        ident = P.Identify()
        ident.messageId.enclosedMessage = none
        ident.messageId.serializerId = MISC
        ident.messageId.messageManifest = b"C"
        temp = self.temp_path()
        self.tell_selection(elements, ident.SerializeToString(), MISC, b"A", temp)
        r = self.receive(lambda m: m.recipient == temp, timeout)
        if r.serializer != MISC or r.manifest != b"B":
            raise ValueError(f"expected ActorIdentity, got serializer {r.serializer} manifest {r.manifest!r}")
        a = P.ActorIdentity()
        a.ParseFromString(r.message)
        if a.correlationId.SerializeToString() != ident.messageId.SerializeToString():
            raise ValueError("ActorIdentity does not echo the Identify's messageId")
        return a.ref.path if a.HasField("ref") else None

    def start_allreduce(self, round_: int, to: str | None = None, sender: str | None = None,
                        package: str = REF_PACKAGE, suid: int | None = None) -> None:
        """``master ! StartAllreduce(round)`` (by ref path ``to``, else by selection)."""
        cls = package + ".StartAllreduce"
        body = java_serialize(cls, case_class_suid(cls, [("round", "I")]) if suid is None else suid,
                              [("I", "round", round_)])
        sender = sender or f"{self.local}/user/driver"
        if to:
            self.tell(to, body, JAVA, None, sender)
        else:
            self.tell_selection(["user", "master"], body, JAVA, None, sender)

    def receive(self, predicate=None, timeout: float | None = None) -> Received:
        """The next user message (heartbeats counted and skipped) matching predicate."""
        deadline = time.monotonic() + (timeout or self.timeout)
        while True:
            left = deadline - time.monotonic()
            if left <= 0:
                raise TimeoutError("no matching message")
            pdu = self._read_pdu(left)
            if pdu.HasField("instruction"):
                c = pdu.instruction.commandType
                if c == HEARTBEAT:
                    self.heartbeats += 1
                    continue
                if c != ASSOCIATE:
                    self.closed_by_peer = c
                    raise ConnectionError(f"endpoint disassociated (command {c})")
                continue
            c = pb().AckAndEnvelopeContainer()
            c.ParseFromString(pdu.payload)
            if not c.HasField("envelope"):
                r = Received("", None, 0, None, b"", None)
                r.ack = c.ack.cumulativeAck
                if predicate is None or predicate(r):
                    return r
                continue
            e = c.envelope
            r = Received(e.recipient.path, e.sender.path if e.HasField("sender") else None, e.message.serializerId,
                         e.message.messageManifest if e.message.HasField("messageManifest") else None,
                         e.message.message, e.seq if e.HasField("seq") else None)
            if predicate is None or predicate(r):
                return r

    def complete_allreduce(self, timeout: float | None = None) -> tuple[int, int, str, int]:
        """The next CompleteAllreduce: (srcId, round, class name, its SUID)."""
        r = self.receive(lambda m: m.serializer == JAVA, timeout)
        name, suid, vals = java_deserialize(r.message)
        if not name.endswith("CompleteAllreduce"):
            raise ValueError(f"unexpected message {name}")
        return vals["srcId"], vals["round"], name, suid

    def close(self, command: int = DISASSOCIATE) -> None:
        try:
            m = pb().AkkaProtocolMessage()
            m.instruction.commandType = command
            self._send_pdu(m.SerializeToString())
        except OSError:
            pass
        self.sock.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
