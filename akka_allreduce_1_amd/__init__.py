"""akka_allreduce_1_amd - MI355X-native threshold allreduce engine.

Same capabilities, actor API and message protocol as the Akka reference
`mike199515/akka-allreduce-1` (master/worker actors, threshold-tolerant pipelined
scatter-reduce + all-gather, bounded-staleness catch-up), rebuilt MI355X-first:
C++ protocol cores and actor runtime (`csrc/core`, `csrc/runtime`), HIP/CDNA4 data
plane kernels (`csrc/hip`), a direct two-shot allreduce over xGMI peer writes, RCCL as
baseline, and a bucketed / backward-overlapped data-parallel gradient reducer.
"""
from __future__ import annotations

try:  # torch first: its bundled HIP runtime must be the one the native module binds to
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None

from ._native import C  # noqa: E402
from .protocol import *  # noqa: E402,F401,F403
from .actors import ActorSystem, make_master, make_worker  # noqa: E402,F401

__version__ = "0.1.0"
