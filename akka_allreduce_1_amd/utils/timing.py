"""Timing helpers for the benchmarks (nccl-tests conventions: algbw = bytes / time,
busbw = algbw * 2 (P - 1) / P)."""
from __future__ import annotations

import math
from typing import Sequence


def percentile(xs: Sequence[float], q: float) -> float:
    if not xs:
        return float("nan")
    s = sorted(xs)
    k = (len(s) - 1) * q / 100.0
    lo, hi = math.floor(k), math.ceil(k)
    return s[lo] if lo == hi else s[lo] + (s[hi] - s[lo]) * (k - lo)


def busbw(algbw: float, world: int) -> float:
    return algbw * 2.0 * (world - 1) / world if world > 1 else 0.0


def summarize(times_ms: Sequence[float]) -> dict:
    return {
        "p50_ms": percentile(times_ms, 50),
        "p10_ms": percentile(times_ms, 10),
        "p90_ms": percentile(times_ms, 90),
        "min_ms": min(times_ms) if times_ms else float("nan"),
        "n": len(times_ms),
    }
