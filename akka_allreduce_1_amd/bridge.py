"""Client of the master's control bridge (csrc/runtime/control_bridge.h, docs/BRIDGE.md).

The bridge carries the reference's control messages -- ``InitWorkers``, ``StartAllreduce``,
``CompleteAllreduce`` (``/root/reference/src/main/scala/sample/cluster/allreduce/
AllreduceMessage.scala:7-20``) -- as one JSON object per line over TCP, so any client with a
socket can watch or drive a job. With the master in ``externalRounds`` mode the client is the
round driver of ``AllreduceMaster.scala:58-67,91-97``: it sends ``StartAllreduce(r)``, the
master forwards it to every worker, counts their ``CompleteAllreduce`` and reports
``RoundComplete(r)`` once ``numComplete >= totalWorkers * thAllreduce``.

    with BridgeClient("127.0.0.1", port) as b:
        b.wait_for("InitWorkers")
        b.drive(range(0, 101))          # the reference master's loop, from outside
"""
from __future__ import annotations

import json
import socket
import time
from typing import Iterable


class BridgeError(RuntimeError):
    """The master refused a command (``{"type": "Error", ...}``) or the bridge went away."""


class BridgeClient:
    def __init__(self, host: str, port: int, timeout: float = 30.0) -> None:
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.timeout = timeout
        self._buf = b""
        self.events: list[dict] = []  # every event line received, in order
        self._inbox: list[dict] = []  # received but not yet matched by a wait
        self.hello = self.wait_for("Hello")

    # ------------------------------------------------------------------ wire
    def send(self, msg: dict) -> None:
        self.sock.sendall((json.dumps(msg, separators=(",", ":")) + "\n").encode())

    def send_raw(self, line: str) -> None:
        self.sock.sendall(line.encode() + b"\n")

    def recv(self, timeout: float | None = None) -> dict:
        deadline = time.monotonic() + (self.timeout if timeout is None else timeout)
        while b"\n" not in self._buf:
            left = deadline - time.monotonic()
            if left <= 0:
                raise TimeoutError("no line from the control bridge")
            self.sock.settimeout(left)
            chunk = self.sock.recv(65536)
            if not chunk:
                raise BridgeError("control bridge closed the connection")
            self._buf += chunk
        line, self._buf = self._buf.split(b"\n", 1)
        msg = json.loads(line)
        self.events.append(msg)
        return msg

    def _next(self, pred, timeout: float | None) -> dict:
        """First unmatched message satisfying pred (an Error raises); unmatched lines stay
        in the inbox for later waits, so interleaved replies and events are never lost."""
        for i, m in enumerate(self._inbox):
            if m.get("type") == "Error" or pred(m):
                del self._inbox[i]
                if m.get("type") == "Error" and not pred(m):
                    raise BridgeError(f"{m.get('cmd')}: {m.get('reason')}")
                return m
        deadline = time.monotonic() + (self.timeout if timeout is None else timeout)
        while True:
            m = self.recv(max(0.0, deadline - time.monotonic()))
            if pred(m):
                return m
            if m.get("type") == "Error":
                raise BridgeError(f"{m.get('cmd')}: {m.get('reason')}")
            self._inbox.append(m)
            if len(self._inbox) > 100000:  # a watcher that never waits: keep the newest
                del self._inbox[:50000]

    def wait_for(self, type_: str, timeout: float | None = None, **fields) -> dict:
        """Next message of ``type_`` whose fields match; Error replies raise."""
        return self._next(lambda m: m.get("type") == type_ and all(m.get(k) == v for k, v in fields.items()),
                          timeout)

    def wait_for_any(self, types, timeout: float | None = None, **fields) -> dict:
        return self._next(lambda m: m.get("type") in types and all(m.get(k) == v for k, v in fields.items()),
                          timeout)

    # -------------------------------------------------------------- commands
    def start(self, round_: int) -> dict:
        """StartAllreduce(round) -> the reply: Accepted (started now) or Queued (runs when the
        round in flight reaches its barrier; its Accepted follows then). BridgeError when refused."""
        self.send({"type": "StartAllreduce", "round": int(round_)})
        return self._start_reply(int(round_))

    def _start_reply(self, r: int) -> dict:
        return self.wait_for_any(("Accepted", "Queued"), round=r)

    def status(self) -> dict:
        self.send({"type": "Status"})
        return self.wait_for("Status")

    def drive(self, rounds: Iterable[int], timeout: float | None = None, pipeline: bool = True) -> list[dict]:
        """The reference master's round loop (AllreduceMaster.scala:58-67,91-97) from outside:
        start each round, wait for its barrier. Returns the RoundComplete events.
        pipeline: the next round's start is sent as soon as the current one is running, so
        the master starts it at the barrier without waiting for this client (one start is
        queued at a time; rounds never overlap)."""
        rs = [int(r) for r in rounds]
        done: list[dict] = []
        if not rs:
            return done
        self.start(rs[0])
        for i, r in enumerate(rs):
            if pipeline and i + 1 < len(rs):
                self.start(rs[i + 1])  # Queued behind r (or Accepted if r already finished)
            done.append(self.wait_for("RoundComplete", timeout=timeout, round=r))
            if not pipeline and i + 1 < len(rs):
                self.start(rs[i + 1])
        return done

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass

    def __enter__(self) -> "BridgeClient":
        return self

    def __exit__(self, *exc) -> None:
        self.close()
