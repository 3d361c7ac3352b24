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


def hbm_bytes(S: int, P: int, algo: str, es: int = 4) -> float:
    """HBM bytes the kernels move when P logical ranks of ONE GPU allreduce S bytes each of an
    `es`-byte element type (every rank's traffic lands in the same HBM; counts checked against
    rocprofv3 PMC FETCH_SIZE / WRITE_SIZE in profiles/pmc_counters.md)."""
    if algo == "ring_native":
        # element-type partials: hop 0 reads in + writes B, hops 1..P-2 read partial + in and
        # write B, the final hop reads 2 B and writes out + fwd, AG hops read B and write out +
        # fwd (the last one out only)
        B = S / P
        return P * B * (6 * P - 4)
    if algo == "ring":
        # per rank, blocks B = S/P: RS hops read in (+ an fp32 partial) and push an fp32 partial
        # (Bp = B * 4 / es: 2 (P - 1) partial transfers), the final hop and the AG hops move
        # E-typed blocks (4 P - 2 of them)
        B = S / P
        return P * (B * (4 * P - 2) + B * 4 / es * (2 * P - 2))
    if algo == "all_to_all":  # S = P blocks per rank: read in + write slab (P-1)/P + read slab + write out
        return P * (2 * S + 2 * S * (P - 1) / P)
    if algo == "reduce_scatter":
        return P * (S + 2 * S * (P - 1) / P + S / P)
    if algo == "all_gather":  # S = the gathered output per rank (input S/P)
        m = S / P
        return P * ((4 * P - 2) * m)
    if algo == "ll":  # read in, write P-1 LL slots (2x), read P-1 LL slots (2x), write out
        return P * (S + 4 * S * (P - 1) + S)
    if algo == "oneshot":
        return P * (S + S * P + S * P + S)  # read in, write P slots, read P slots, write out
    # two-shot: read in + push (P-1)/P, reduce reads S (own input + P-1 slots) and writes S
    # (own output + P-1 peers' R slots), gather reads + writes (P-1)/P
    return P * (S + S * (P - 1) / P + S + S + 2 * S * (P - 1) / P)


def summarize(times_ms: Sequence[float]) -> dict:
    return {
        "p50_ms": percentile(times_ms, 50),
        "p10_ms": percentile(times_ms, 10),
        "p90_ms": percentile(times_ms, 90),
        "min_ms": min(times_ms) if times_ms else float("nan"),
        "n": len(times_ms),
    }
