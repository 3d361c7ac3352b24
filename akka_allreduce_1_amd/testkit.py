"""TestKit for actor-level tests, modelled on Akka TestKit + ImplicitSender as used by
the reference spec (`src/test/scala/AllreduceSpec.scala:8-12, 715-763`).

The probe (`test_actor`) impersonates every peer AND the master ("fake-cluster trick",
SURVEY §4.2): the worker under test sends all its traffic to the probe, and the test
injects what the other P-1 peers would send.

By default the system is *deterministic*: `tell` only enqueues, and every expectation
first drains the system to quiescence ("batch then drain"), so message
order is reproducible. `TestKit(deterministic=False)` runs the threaded dispatcher and
expectations wait with a timeout, like Akka's `remainingOrDefault`.
"""
from __future__ import annotations

import random
import string
from typing import Callable, Iterable

import numpy as np

from ._native import C
from .protocol import AllReduceInput, ReduceBlock, ScatterBlock


class ExpectationError(AssertionError):
    pass


def to_host(v) -> np.ndarray:
    """Payload -> numpy (device payloads arrive as torch tensors on the GPU)."""
    if hasattr(v, "detach") and hasattr(v, "cpu"):
        return v.detach().cpu().numpy()
    return np.asarray(v)


class TestKit:
    __test__ = False  # not a pytest class

    def __init__(self, name: str = "MySpec", deterministic: bool = True, timeout: float = 3.0, plane=None):
        self.system = C.ActorSystem(name, deterministic)
        self.test_actor = self.system.probe("testActor")
        self.timeout = timeout
        self.plane = plane  # default DataPlane of created workers (None = host)

    # ImplicitSender: `self` in the Scala spec
    @property
    def self_ref(self):
        return self.test_actor

    def shutdown(self) -> None:
        self.system.shutdown()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.shutdown()

    # ----------------------------------------------------------------- actors
    def create_new_worker(self, source, sink=None, plane=None):
        """AllreduceSpec.scala:746-755 (random actor name)."""
        name = "".join(random.choice(string.ascii_letters + string.digits) for _ in range(10))
        return self.system.worker(source, sink, name, plane if plane is not None else self.plane)

    def initialize_workers_as_self(self, size: int) -> dict:
        """AllreduceSpec.scala:757-763: every peer id points at the probe."""
        return {i: self.test_actor for i in range(size)}

    def tell(self, ref, msg) -> None:
        ref.tell(msg, self.test_actor)

    # ----------------------------------------------------------------- receive
    def receive_one(self, timeout: float | None = None):
        r = self.test_actor.receive(self.timeout if timeout is None else timeout)
        return None if r is None else r[0]

    def expect_msg(self, expected, timeout: float | None = None):
        m = self.receive_one(timeout)
        if m is None:
            raise ExpectationError(f"timeout waiting for {expected!r}")
        if m != expected:
            raise ExpectationError(f"expected {expected!r}, found {m!r}")
        return m

    def expect_msg_type(self, cls, timeout: float | None = None):
        m = self.receive_one(timeout)
        if m is None:
            raise ExpectationError(f"timeout waiting for a {cls.__name__}")
        if not isinstance(m, cls):
            raise ExpectationError(f"expected a {cls.__name__}, found {m!r}")
        return m

    def expect_scatter(self, expected: ScatterBlock):
        """AllreduceSpec.scala:719-728: field-wise, arrays compared element-wise."""
        s = self.expect_msg_type(ScatterBlock)
        for f in ("srcId", "destId", "round", "chunkId"):
            if getattr(s, f) != getattr(expected, f):
                raise ExpectationError(f"ScatterBlock.{f}: expected {expected!r}, found {s!r}")
        if list(to_host(s.value)) != list(to_host(expected.value)):
            raise ExpectationError(f"ScatterBlock.value: expected {expected!r}, found {s!r}")
        return s

    def expect_reduce(self, expected: ReduceBlock):
        """AllreduceSpec.scala:734-744."""
        r = self.expect_msg_type(ReduceBlock)
        for f in ("srcId", "destId", "round", "chunkId", "count"):
            if getattr(r, f) != getattr(expected, f):
                raise ExpectationError(f"ReduceBlock.{f}: expected {expected!r}, found {r!r}")
        if list(to_host(r.value)) != list(to_host(expected.value)):
            raise ExpectationError(f"ReduceBlock.value: expected {expected!r}, found {r!r}")
        return r

    def expect_no_msg(self, timeout: float = 0.1):
        m = self.receive_one(timeout)
        if m is not None:
            raise ExpectationError(f"expected no message, received {m!r}")

    def fish_for_message(self, pred: Callable[[object], bool], timeout: float | None = None):
        """Akka fishForMessage: skip messages until pred returns True."""
        while True:
            m = self.receive_one(timeout)
            if m is None:
                raise ExpectationError("timeout while fishing for message")
            if pred(m):
                return m


# ---------------------------------------------------------------------- data sources
def create_custom_data_source(size: int, gen: Callable[[int, int], float]):
    """AllreduceSpec.scala:29-35."""

    def source(req):
        return AllReduceInput(np.array([gen(i, req.iteration) for i in range(size)], dtype=np.float32))

    return source


def create_basic_data_source(size: int):
    """AllreduceSpec.scala:23-27: data[i] = i + iteration."""
    return create_custom_data_source(size, lambda idx, it: float(idx + it))


def assertive_data_sink(expected: list[list[float]], iterations: Iterable[int], seen: list | None = None):
    """AllreduceSpec.scala:37-43. Failures propagate to the test (deterministic mode)."""
    iterations = list(iterations)

    def sink(r):
        assert r.iteration in iterations, f"unexpected iteration {r.iteration}"
        pos = iterations.index(r.iteration)
        got = [float(x) for x in to_host(r.data)]
        assert got == list(expected[pos]), f"iteration {r.iteration}: {got} != {expected[pos]}"
        if seen is not None:
            seen.append(r.iteration)

    return sink
