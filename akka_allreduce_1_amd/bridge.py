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

    def wait_for(self, type_: str, timeout: float | None = None, **fields) -> dict:
        """Next message of ``type_`` whose fields match; Error replies raise."""
        deadline = time.monotonic() + (self.timeout if timeout is None else timeout)
        while True:
            m = self.recv(max(0.0, deadline - time.monotonic()))
            if m.get("type") == "Error" and type_ != "Error":
                raise BridgeError(f"{m.get('cmd')}: {m.get('reason')}")
            if m.get("type") == type_ and all(m.get(k) == v for k, v in fields.items()):
                return m

    # -------------------------------------------------------------- commands
    def start(self, round_: int) -> dict:
        """StartAllreduce(round) -> the Accepted reply (BridgeError when refused)."""
        self.send({"type": "StartAllreduce", "round": int(round_)})
        return self.wait_for("Accepted", round=int(round_))

    def status(self) -> dict:
        self.send({"type": "Status"})
        return self.wait_for("Status")

    def drive(self, rounds: Iterable[int], timeout: float | None = None) -> list[dict]:
        """The reference master's round loop (AllreduceMaster.scala:58-67,91-97) from outside:
        start each round, wait for its barrier. Returns the RoundComplete events."""
        done = []
        for r in rounds:
            self.start(r)
            done.append(self.wait_for("RoundComplete", timeout=timeout, round=int(r)))
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
